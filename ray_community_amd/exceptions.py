"""Exception hierarchy (reference: ``python/ray/exceptions.py``)."""
from __future__ import annotations

import traceback


class RayError(Exception):
    """Base for all framework errors."""


class CrossLanguageError(RayError):
    pass


class RayTaskError(RayError):
    """A task raised. ``as_instanceof_cause()`` gives an exception that is BOTH a RayTaskError and
    an instance of the original exception class (like the reference's dual inheritance)."""

    def __init__(self, function_name="", traceback_str="", cause=None, proctitle="", pid=None, ip=None,
                 actor_repr=None, actor_id=None):
        self.function_name = function_name
        self.traceback_str = traceback_str
        self.cause = cause
        self.proctitle = proctitle
        self.pid = pid
        self.ip = ip
        self.actor_repr = actor_repr
        self._actor_id = actor_id
        super().__init__(self._msg())

    def _msg(self):
        head = f"{type(self.cause).__name__ if self.cause is not None else 'Error'}: task {self.function_name} failed"
        return f"{head}\n{self.traceback_str}".rstrip()

    def __str__(self):
        return self._msg()

    def as_instanceof_cause(self):
        cause = self.cause
        if cause is None or isinstance(cause, RayTaskError):
            return self
        cls = type(cause)
        if issubclass(RayTaskError, cls):
            return self
        name = f"RayTaskError({cls.__name__})"
        try:
            dual = type(name, (RayTaskError, cls), {"__init__": lambda s, *a, **k: None,
                                                        "__str__": lambda s: RayTaskError._msg(s)})
            inst = dual.__new__(dual)
            inst.function_name = self.function_name
            inst.traceback_str = self.traceback_str
            inst.cause = cause
            inst.proctitle = self.proctitle
            inst.pid = self.pid
            inst.ip = self.ip
            inst.actor_repr = self.actor_repr
            inst._actor_id = self._actor_id
            inst.args = getattr(cause, "args", ())
            try:
                inst.__dict__.update({k: v for k, v in cause.__dict__.items() if k not in inst.__dict__})
            except Exception:
                pass
            return inst
        except TypeError:
            return self

    def __reduce__(self):
        return (RayTaskError, (self.function_name, self.traceback_str, self.cause, self.proctitle, self.pid, self.ip,
                               self.actor_repr, self._actor_id))

    @staticmethod
    def from_exception(e: BaseException, function_name: str, actor_repr=None, actor_id=None):
        tb = "".join(traceback.format_exception(type(e), e, e.__traceback__))
        import os

        try:
            import pickle

            pickle.dumps(e)
            cause = e
        except Exception:
            cause = RuntimeError(f"{type(e).__name__}: {e}")
        return RayTaskError(function_name, tb, cause, pid=os.getpid(), actor_repr=actor_repr, actor_id=actor_id)


class RayActorError(RayError):
    def __init__(self, actor_id=None, error_msg="The actor died unexpectedly before finishing this task.",
                 actor_init_failed=False, preempted=False):
        self.actor_id = actor_id
        self.error_msg = error_msg
        self.actor_init_failed = actor_init_failed
        self.preempted = preempted
        super().__init__(error_msg)

    def __reduce__(self):
        return (type(self), (self.actor_id, self.error_msg, self.actor_init_failed, self.preempted))


class ActorDiedError(RayActorError):
    pass


class ActorUnavailableError(RayActorError):
    pass


class ActorUnschedulableError(RayError):
    pass


class RaySystemError(RayError):
    pass


class WorkerCrashedError(RayError):
    def __init__(self, msg="The worker died unexpectedly while executing this task."):
        super().__init__(msg)


class TaskCancelledError(RayError):
    def __init__(self, task_id=None, error_message=None):
        self.task_id = task_id
        super().__init__(error_message or f"Task {task_id} was cancelled.")

    def __reduce__(self):
        return (type(self), (self.task_id, str(self)))


class GetTimeoutError(RayError, TimeoutError):
    pass


class ObjectLostError(RayError):
    def __init__(self, object_ref_hex="", owner_address="", call_site=""):
        self.object_ref_hex = object_ref_hex
        super().__init__(f"Object {object_ref_hex} is lost.")

    def __reduce__(self):
        return (type(self), (self.object_ref_hex,))


class ObjectFetchTimedOutError(ObjectLostError):
    pass


class ReferenceCountingAssertionError(ObjectLostError):
    pass


class OwnerDiedError(ObjectLostError):
    pass


class ObjectReconstructionFailedError(ObjectLostError):
    pass


class ObjectReconstructionFailedMaxAttemptsExceededError(ObjectReconstructionFailedError):
    pass


class ObjectReconstructionFailedLineageEvictedError(ObjectReconstructionFailedError):
    pass


class ObjectStoreFullError(RayError):
    pass


class OutOfDiskError(RayError):
    pass


class OutOfMemoryError(RayError):
    pass


class NodeDiedError(RayError):
    pass


class PendingCallsLimitExceeded(RayError):
    pass


class TaskUnschedulableError(RayError):
    pass


class TaskPlacementGroupRemoved(RayError):
    pass


class ActorPlacementGroupRemoved(RayError):
    pass


class LocalRayletDiedError(RayError):
    pass


class RuntimeEnvSetupError(RayError):
    def __init__(self, error_message=""):
        super().__init__(error_message)


class AsyncioActorExit(RayError):
    pass


class RayChannelError(RayError):
    pass


class RayChannelTimeoutError(RayChannelError, TimeoutError):
    pass


RAY_EXCEPTION_TYPES = [RayError, RayTaskError, WorkerCrashedError, RayActorError, ObjectStoreFullError, ObjectLostError,
                       GetTimeoutError, TaskCancelledError]


class UserCodeException(RayError):
    """An exception raised by user code (a task / actor body); retry_exceptions looks at its cause."""


class RpcError(RayError):
    """An error of the control-plane RPC layer."""

    def __init__(self, message, rpc_code=None):
        self.message = message
        self.rpc_code = rpc_code

    def __str__(self):
        return self.message


class ObjectFreedError(ObjectLostError):
    """The object was freed explicitly (``ray.internal.free``) while a reference still existed."""


class PlasmaObjectNotAvailable(RayError):
    """An object was not available within the given timeout."""


class ObjectRefStreamEndOfStreamError(RayError):
    """A streaming generator has no more ObjectRefs to hand out."""
