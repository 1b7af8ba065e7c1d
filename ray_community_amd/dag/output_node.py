"""(reference: ``python/ray/dag/output_node.py``)"""
from .dag_node import MultiOutputNode  # noqa: F401
