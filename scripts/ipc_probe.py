"""Probe HIP IPC variants between two processes on the MI355X box."""
import ctypes
import os
import pickle
import subprocess
import sys
import time

MODE = sys.argv[1] if len(sys.argv) > 1 else "parent"


def hip():
    return ctypes.CDLL("libamdhip64.so")


if MODE == "child":
    import torch
    from torch.multiprocessing.reductions import reduce_tensor

    t = torch.arange(1 << 20, device="cuda", dtype=torch.float32)
    torch.cuda.synchronize()
    fn, args = reduce_tensor(t)
    args2 = list(args)
    args2[-1] = False
    L = hip()
    h = (ctypes.c_byte * 64)()
    rc = L.hipIpcGetMemHandle(ctypes.byref(h), ctypes.c_void_p(t.data_ptr()))
    payload = {"torch": (fn, args), "torch_nosync": (fn, tuple(args2)), "raw": (bytes(h), rc, t.numel()),
               "pid": os.getpid()}
    sys.stdout.buffer.write(pickle.dumps(payload))
    sys.stdout.flush()
    time.sleep(20)
    sys.exit(0)

p = subprocess.Popen([sys.executable, __file__, "child"], stdout=subprocess.PIPE)
import torch  # noqa: E402

torch.cuda.init()
data = b""
while True:
    chunk = p.stdout.read1(1 << 16) if hasattr(p.stdout, "read1") else p.stdout.read(1 << 16)
    data += chunk
    try:
        payload = pickle.loads(data)
        break
    except Exception:
        if not chunk:
            raise
for key in ("torch", "torch_nosync"):
    fn, args = payload[key]
    try:
        x = fn(*args)
        print(key, "OK", float(x[-1].item()))
    except Exception as e:
        print(key, "FAIL", repr(e)[:200])
raw, rc, n = payload["raw"]
print("raw get rc", rc)
L = hip()
ptr = ctypes.c_void_p()
h = (ctypes.c_byte * 64).from_buffer_copy(raw)
rc2 = L.hipIpcOpenMemHandle(ctypes.byref(ptr), h, ctypes.c_uint(1))
print("raw open rc", rc2, hex(ptr.value or 0))
if rc2 == 0:
    class CAI:
        __cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr.value, False), "version": 2}
    try:
        y = torch.as_tensor(CAI(), device="cuda")
        print("raw tensor OK", float(y[-1].item()), y.is_cuda)
    except Exception as e:
        print("raw tensor FAIL", repr(e)[:200])
p.kill()
