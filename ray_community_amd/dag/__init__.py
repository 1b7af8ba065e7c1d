"""DAG API (reference: ``python/ray/dag/__init__.py``)."""
from .compiled_dag_node import CompiledDAG, CompiledDAGRef
from .dag_node import (ClassMethodNode, ClassNode, DAGInputData, DAGNode, FunctionNode, InputAttributeNode, InputNode,
                       MultiOutputNode)

__all__ = ["DAGNode", "FunctionNode", "ClassNode", "ClassMethodNode", "InputNode", "InputAttributeNode",
           "MultiOutputNode", "DAGInputData", "CompiledDAG", "CompiledDAGRef"]
