"""DAG API (reference: ``python/ray/dag/__init__.py``)."""
from .compiled_dag_node import CompiledDAG, CompiledDAGRef
from .dag_node import (ClassMethodNode, ClassNode, DAGInputData, DAGNode, FunctionNode, InputAttributeNode, InputNode,
                       MultiOutputNode)

from .vis import plot
from .torch_tensor import TorchTensorType


def _register_node_module_paths():
    """The reference's per-node-type module paths (``ray.dag.input_node``, ``class_node``,
    ``function_node``, ``output_node``) as aliases of the one module that defines them."""
    import importlib.machinery
    import sys
    import types

    for name, attrs in {"input_node": (InputNode, InputAttributeNode, DAGInputData),
                        "class_node": (ClassNode, ClassMethodNode), "function_node": (FunctionNode,),
                        "output_node": (MultiOutputNode,)}.items():
        m = types.ModuleType(f"{__name__}.{name}", f"ray.dag.{name} import path")
        for a in attrs:
            setattr(m, a.__name__, a)
        m.__all__ = [a.__name__ for a in attrs]
        m.__spec__ = importlib.machinery.ModuleSpec(m.__name__, None)
        sys.modules[m.__name__] = m
        globals()[name] = m


_register_node_module_paths()

# keys the reference stores in DAG node metadata (``dag/constants.py``)
PARENT_CLASS_NODE_KEY = "parent_class_node"
PREV_CLASS_METHOD_CALL_KEY = "prev_class_method_call"
DAGNODE_TYPE_KEY = "__dag_node_type__"

__all__ = ["TorchTensorType", "plot", "PARENT_CLASS_NODE_KEY", "PREV_CLASS_METHOD_CALL_KEY", "DAGNODE_TYPE_KEY", "DAGNode", "FunctionNode", "ClassNode", "ClassMethodNode", "InputNode", "InputAttributeNode",
           "MultiOutputNode", "DAGInputData", "CompiledDAG", "CompiledDAGRef"]
