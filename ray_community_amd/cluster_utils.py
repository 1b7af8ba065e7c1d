"""Multi-node simulation on one machine (reference: ``python/ray/cluster_utils.py``).

Every "node" is a resource pool in the C++ scheduler with its own worker pool; all nodes share
the machine's shm store. Used by tests for placement-group / spread / node-failure behaviour.
"""
from __future__ import annotations

from typing import Dict, List, Optional


class NodeHandle:
    def __init__(self, node_id: str, resources: dict, is_head=False):
        self.node_id = node_id
        self.unique_id = node_id
        self.resources = resources
        self.is_head = is_head
        self.address = "127.0.0.1"
        self.node_ip_address = "127.0.0.1"

    def __repr__(self):
        return f"NodeHandle({self.node_id[:8]}, head={self.is_head})"


class Cluster:
    def __init__(self, initialize_head: bool = False, connect: bool = False, head_node_args: Optional[dict] = None,
                 shutdown_at_exit: bool = True):
        self.head_node: Optional[NodeHandle] = None
        self.worker_nodes: List[NodeHandle] = []
        self._connected = False
        if initialize_head:
            self.add_node(**(head_node_args or {}))
            if connect:
                self.connect()

    @property
    def address(self):
        from ._private.worker import _state

        return _state.get("address")

    def _head(self):
        from ._private.worker import _state

        return _state["head"]

    def add_node(self, wait: bool = True, num_cpus: Optional[float] = 1, num_gpus: Optional[float] = 0,
                 resources: Optional[dict] = None, labels: Optional[dict] = None, object_store_memory=None,
                 _system_config=None, **kwargs) -> NodeHandle:
        from . import _private

        from ._private import worker as w

        res = dict(resources or {})
        if self.head_node is None:
            if not w.is_initialized():
                w.init(num_cpus=num_cpus, num_gpus=num_gpus, resources=res, labels=labels,
                       object_store_memory=object_store_memory, _system_config=_system_config)
            head = self._head()
            self.head_node = NodeHandle(head.head_node_id, head.nodes[head.head_node_id].resources, is_head=True)
            self._connected = True
            return self.head_node
        res["CPU"] = float(num_cpus or 0)
        if num_gpus:
            res["GPU"] = float(num_gpus)
        nid = self._head().add_node(res, labels)
        n = NodeHandle(nid, res)
        self.worker_nodes.append(n)
        return n

    def remove_node(self, node: NodeHandle, allow_graceful: bool = True):
        if node is self.head_node:
            raise ValueError("cannot remove the head node of an in-process cluster")
        self._head().remove_node(node.node_id)
        if node in self.worker_nodes:
            self.worker_nodes.remove(node)

    def connect(self, namespace=None):
        self._connected = True

    def wait_for_nodes(self, timeout: float = 30):
        return True

    @property
    def gcs_address(self) -> Optional[str]:
        """The head's control-plane address (a Unix socket path here, as ``address``)."""
        return self.address

    def remaining_processes_alive(self) -> bool:
        """True while the session's head is up (nodes are virtual: one head process)."""
        from ._private import worker as w

        return w.is_initialized()

    def list_all_nodes(self) -> List[NodeHandle]:
        return ([self.head_node] if self.head_node else []) + list(self.worker_nodes)

    def shutdown(self):
        from ._private import worker as w

        w.shutdown()
        self.head_node = None
        self.worker_nodes = []


class AutoscalingCluster:  # pragma: no cover - cloud autoscaling is out of scope on one MI355X node
    def __init__(self, *a, **k):
        raise NotImplementedError("autoscaling clusters are not supported; use cluster_utils.Cluster")
