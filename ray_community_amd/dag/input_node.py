"""(reference: ``python/ray/dag/input_node.py``)"""
from .dag_node import DAGInputData, InputAttributeNode, InputNode  # noqa: F401
