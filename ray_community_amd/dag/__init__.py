"""DAG API (reference: ``python/ray/dag/__init__.py``)."""
from .compiled_dag_node import CompiledDAG, CompiledDAGRef
from .dag_node import (ClassMethodNode, ClassNode, DAGInputData, DAGNode, FunctionNode, InputAttributeNode, InputNode,
                       MultiOutputNode)

from .vis import plot
from .torch_tensor import TorchTensorType

# keys the reference stores in DAG node metadata (``dag/constants.py``)
PARENT_CLASS_NODE_KEY = "parent_class_node"
PREV_CLASS_METHOD_CALL_KEY = "prev_class_method_call"
DAGNODE_TYPE_KEY = "__dag_node_type__"

__all__ = ["TorchTensorType", "plot", "PARENT_CLASS_NODE_KEY", "PREV_CLASS_METHOD_CALL_KEY", "DAGNODE_TYPE_KEY", "DAGNode", "FunctionNode", "ClassNode", "ClassMethodNode", "InputNode", "InputAttributeNode",
           "MultiOutputNode", "DAGInputData", "CompiledDAG", "CompiledDAGRef"]
