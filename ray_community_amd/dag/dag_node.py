"""Lazy task graphs built with ``.bind()`` (reference: ``python/ray/dag/dag_node.py``,
``function_node.py``, ``class_node.py``, ``input_node.py``, ``output_node.py``).

``f.bind(x)`` / ``Cls.bind()`` / ``actor.method.bind(x)`` record a node instead of submitting work.
``dag.execute(*args)`` walks the graph once (each node evaluated at most once per execution, so a
node shared by two consumers runs a single task), submitting tasks/actor calls whose arguments are
the upstream ``ObjectRef``s — the runtime resolves them, nothing is fetched to the driver.
"""
from __future__ import annotations

import uuid
from typing import Any, Callable, Dict, List, Optional, Tuple


def _map_nested(x, fn):
    """Apply ``fn`` to every DAGNode nested in lists/tuples/dicts of ``x``."""
    if isinstance(x, DAGNode):
        return fn(x)
    if isinstance(x, list):
        return [_map_nested(v, fn) for v in x]
    if isinstance(x, tuple):
        return tuple(_map_nested(v, fn) for v in x)
    if isinstance(x, dict):
        return {k: _map_nested(v, fn) for k, v in x.items()}
    return x


def _scan_nodes(x, out: List["DAGNode"]):
    _map_nested(x, lambda n: out.append(n) or n)
    return out


class DAGNode:
    def __init__(self, args: Tuple = (), kwargs: Optional[Dict] = None, options: Optional[Dict] = None,
                 other_args_to_resolve: Optional[Dict] = None):
        self._bound_args = tuple(args)
        self._bound_kwargs = dict(kwargs or {})
        self._bound_options = dict(options or {})
        self._bound_other_args_to_resolve = dict(other_args_to_resolve or {})
        self._stable_uuid = uuid.uuid4().hex
        self.cache_from_last_execute: Dict[str, Any] = {}

    # --------------------------------------------------------------------------- introspection
    def get_args(self) -> Tuple:
        return self._bound_args

    def get_kwargs(self) -> Dict[str, Any]:
        return self._bound_kwargs

    def get_options(self) -> Dict[str, Any]:
        return self._bound_options

    def get_other_args_to_resolve(self) -> Dict[str, Any]:
        return self._bound_other_args_to_resolve

    def get_stable_uuid(self) -> str:
        return self._stable_uuid

    def with_type_hint(self, typ) -> "DAGNode":
        """Mark this node's output type for compiled DAGs, e.g. ``TorchTensorType()``: tensors
        then travel device-to-device (``dag/torch_tensor.py``) instead of through host memory."""
        self._type_hint = typ
        return self

    @property
    def type_hint(self):
        return getattr(self, "_type_hint", None)

    def _children(self) -> List["DAGNode"]:
        out: List[DAGNode] = []
        _scan_nodes(list(self._bound_args), out)
        _scan_nodes(self._bound_kwargs, out)
        _scan_nodes(self._bound_other_args_to_resolve, out)
        seen, uniq = set(), []
        for n in out:
            if id(n) not in seen:
                seen.add(id(n))
                uniq.append(n)
        return uniq

    def _topo(self) -> List["DAGNode"]:
        order: List[DAGNode] = []
        state: Dict[int, int] = {}
        stack = [(self, False)]
        while stack:
            node, done = stack.pop()
            if done:
                if state.get(id(node)) != 2:
                    state[id(node)] = 2
                    order.append(node)
                continue
            if state.get(id(node)) is not None:
                continue
            state[id(node)] = 1
            stack.append((node, True))
            for c in reversed(node._children()):
                if state.get(id(c)) is None:
                    stack.append((c, False))
        return order

    # --------------------------------------------------------------------------- execution
    def apply_recursive(self, fn: Callable[["DAGNode"], Any]) -> Any:
        """Evaluate ``fn`` bottom-up, each node once; ``fn`` sees a node whose children are resolved."""
        cache: Dict[int, Any] = {}
        for node in self._topo():
            resolved = lambda n: cache[id(n)]  # noqa: E731
            cache[id(node)] = fn(node, resolved)
        fn.cache = cache  # type: ignore[attr-defined]
        return cache[id(self)]

    def execute(self, *args, _ray_cache_refs: bool = False, **kwargs):
        def executor(node, resolved):
            a = _map_nested(list(node._bound_args), resolved)
            k = _map_nested(node._bound_kwargs, resolved)
            o = _map_nested(node._bound_other_args_to_resolve, resolved)
            return node._execute_impl(a, k, o, args, kwargs)

        result = self.apply_recursive(executor)
        if _ray_cache_refs:
            self.cache_from_last_execute = {n.get_stable_uuid(): executor.cache[id(n)] for n in self._topo()}
        return result

    def _execute_impl(self, args, kwargs, other, dag_args, dag_kwargs):  # pragma: no cover - abstract
        raise NotImplementedError

    def experimental_compile(self, buffer_size_bytes: Optional[int] = None, enable_asyncio: bool = False,
                             async_max_queue_size: Optional[int] = None, _max_buffered_results: Optional[int] = None):
        from .compiled_dag_node import build_compiled_dag

        return build_compiled_dag(self, buffer_size_bytes, enable_asyncio, _max_buffered_results)

    def clear_cache(self):
        self.cache_from_last_execute = {}

    def get_object_refs_from_last_execute(self) -> Dict[str, Any]:
        """{node stable uuid: its ObjectRef} of the last ``execute(_ray_cache_refs=True)``."""
        return dict(getattr(self, "cache_from_last_execute", {}) or {})

    def apply_functional(self, source_input_list: Any, predictate_fn: Callable, apply_fn: Callable):
        """``apply_fn(x)`` on every element of ``source_input_list`` (a node, or a nested
        list / dict / tuple of them) that ``predictate_fn(x)`` accepts; the structure is kept."""
        def go(x):
            if isinstance(x, (list, tuple)):
                return type(x)(go(v) for v in x)
            if isinstance(x, dict):
                return {k: go(v) for k, v in x.items()}
            return apply_fn(x) if predictate_fn(x) else x
        return go(source_input_list)

    def __reduce__(self):
        raise ValueError("DAGNode cannot be serialized; call .execute() to get ObjectRefs instead.")


class FunctionNode(DAGNode):
    """``remote_fn.bind(...)``."""

    def __init__(self, remote_fn, args, kwargs, options):
        super().__init__(args, kwargs, options)
        self._body = remote_fn

    def _execute_impl(self, args, kwargs, other, dag_args, dag_kwargs):
        return self._body._remote(tuple(args), kwargs, {**self._body._options, **self._bound_options})

    def __str__(self):
        return f"FunctionNode({getattr(self._body, '_name', self._body)})"


class ClassNode(DAGNode):
    """``ActorCls.bind(...)``: creates the actor on execution; ``node.method.bind(...)`` chains calls."""

    def __init__(self, actor_cls, args, kwargs, options):
        super().__init__(args, kwargs, options)
        self._body = actor_cls
        self._cached_handle = None

    def _execute_impl(self, args, kwargs, other, dag_args, dag_kwargs):
        return self._body._remote(tuple(args), kwargs, {**self._body._options, **self._bound_options})

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return _UnboundClassMethod(self, name, {})

    def options(self, **options):
        return ClassNode(self._body, self._bound_args, self._bound_kwargs, {**self._bound_options, **options})


class _UnboundClassMethod:
    def __init__(self, actor, method_name, options):
        self._actor = actor
        self._method_name = method_name
        self._options = options

    def bind(self, *args, **kwargs):
        return ClassMethodNode(self._actor, self._method_name, args, kwargs, self._options)

    def options(self, **options):
        return _UnboundClassMethod(self._actor, self._method_name, {**self._options, **options})


class ClassMethodNode(DAGNode):
    """A method call on an actor: either a live ``ActorHandle`` or a ``ClassNode`` of the same DAG."""

    def __init__(self, actor, method_name, args, kwargs, options):
        other = {"parent_class_node": actor} if isinstance(actor, DAGNode) else {}
        super().__init__(args, kwargs, options, other)
        self._actor = actor
        self._method_name = method_name

    def get_method_name(self) -> str:
        return self._method_name

    def _execute_impl(self, args, kwargs, other, dag_args, dag_kwargs):
        handle = other.get("parent_class_node", self._actor)
        m = getattr(handle, self._method_name)
        if self._bound_options:
            m = m.options(**self._bound_options)
        return m.remote(*args, **kwargs)

    def __str__(self):
        return f"ClassMethodNode({self._method_name})"


class DAGInputData:
    """Arguments of one ``execute`` call (when there is not exactly one positional argument)."""

    def __init__(self, *args, **kwargs):
        self._args = list(args)
        self._kwargs = kwargs

    def __getitem__(self, key):
        if isinstance(key, int):
            return self._args[key]
        return self._kwargs[key]


class InputNode(DAGNode):
    """Placeholder for the arguments of ``dag.execute(...)``; usable as a context manager."""

    def __init__(self, *args, **kwargs):
        if args or kwargs:
            raise ValueError("InputNode() takes no arguments; index or getattr it for multiple inputs.")
        super().__init__()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False

    def __getitem__(self, key):
        return InputAttributeNode(self, key, "__getitem__")

    def __getattr__(self, name):
        if name.startswith("_") or name in ("cache_from_last_execute",):
            raise AttributeError(name)
        return InputAttributeNode(self, name, "__getattr__")

    def _execute_impl(self, args, kwargs, other, dag_args, dag_kwargs):
        if len(dag_args) == 1 and not dag_kwargs:
            return dag_args[0]
        return DAGInputData(*dag_args, **dag_kwargs)


class InputAttributeNode(DAGNode):
    def __init__(self, input_node: InputNode, key, accessor: str):
        super().__init__(other_args_to_resolve={"input": input_node})
        self._key = key
        self._accessor = accessor

    @property
    def key(self):
        return self._key

    def _execute_impl(self, args, kwargs, other, dag_args, dag_kwargs):
        data = other["input"]
        if isinstance(data, DAGInputData):
            return data[self._key]
        if self._accessor == "__getitem__":
            return data[self._key]
        return getattr(data, self._key)


class MultiOutputNode(DAGNode):
    def __init__(self, outputs: List[DAGNode]):
        if not isinstance(outputs, (list, tuple)):
            raise TypeError("MultiOutputNode expects a list of nodes")
        super().__init__(tuple(outputs))

    def _execute_impl(self, args, kwargs, other, dag_args, dag_kwargs):
        return list(args)
