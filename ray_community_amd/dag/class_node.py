"""(reference: ``python/ray/dag/class_node.py``)"""
from .dag_node import ClassMethodNode, ClassNode  # noqa: F401
