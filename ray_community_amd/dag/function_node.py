"""(reference: ``python/ray/dag/function_node.py``)"""
from .dag_node import FunctionNode  # noqa: F401
