"""Map hipExtStreamCreateWithCUMask bits to XCDs (probe kernel), then time the fused AdamW on a
stream restricted to k CUs per XCD, alone and concurrently with a bf16 GEMM stream (diagnostic)."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    from ray_community_amd.ops._lib import lib

    hip = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so"))
    hip.hipExtStreamCreateWithCUMask.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32,
                                                 ctypes.POINTER(ctypes.c_uint32)]
    hip.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    nw = (ncu + 31) // 32

    def raw_masked(bits):
        m = (ctypes.c_uint32 * nw)()
        for b in bits:
            m[b // 32] |= 1 << (b % 32)
        s = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), nw, m)
        assert rc == 0, rc
        return s.value

    def masked_stream(bits):
        return torch.cuda.ExternalStream(raw_masked(bits))

    out = torch.zeros(2, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    bit_xcc = []
    probe_bits = [int(x) for x in os.environ.get("PROBE_BITS", "0,1,2,3").split(",")]
    for b in probe_bits:  # one short-lived queue at a time
        sp = raw_masked([b])
        lib().rca_probe_hwid(out.data_ptr(), sp)
        assert hip.hipStreamSynchronize(sp) == 0
        bit_xcc.append((b, int(out[0].item()), hex(int(out[1].item()) & 0xffffffff)))
        hip.hipStreamDestroy(sp)
    print("bit -> xcc:", bit_xcc, flush=True)
    if os.environ.get("PROBE_ONLY"):
        return
    # multi-XCC devices deal CU-mask bits round-robin over the XCCs (bit i -> XCC i % 8): the
    # probe's HW_ID words show bits 0, 8, 16, 32, ... landing on distinct CUs of one XCC
    by_xcc = {x: [b for b in range(ncu) if b % 8 == x] for x in range(8)}

    from ray_community_amd.parallel import FlatAdamW
    from ray_community_amd.parallel.flat import FlatParameters

    net = torch.nn.Linear(32768, 32768, bias=False, device="cuda", dtype=torch.bfloat16)  # 1.07 G params
    flat = FlatParameters(net)
    flat.grad.normal_()
    opt = FlatAdamW(flat, lr=1e-4, max_grad_norm=0.0)
    a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
    bm = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)

    def adam_on(st):
        with torch.cuda.stream(st):
            opt.step()

    def timeit(fn, n=3):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t) / n * 1e3

    full = torch.cuda.Stream()
    res = {"adam_full_ms": timeit(lambda: adam_on(full)), "gemm_full_ms": timeit(lambda: a @ bm, 10)}
    xccs = sorted(by_xcc)
    for k in (2, 4, 8):
        bits = [b for x in xccs for b in by_xcc[x][:k]]
        rest = [b for b in range(ncu) if b not in bits]
        sa, sg = masked_stream(bits), masked_stream(rest)
        res[f"adam_{k}perxcd_ms"] = timeit(lambda: adam_on(sa))

        def both():
            with torch.cuda.stream(sg):
                for _ in range(6):
                    a @ bm
            adam_on(sa)

        def gemms_only():
            with torch.cuda.stream(sg):
                for _ in range(6):
                    a @ bm

        res[f"gemm6_rest{k}_ms"] = timeit(gemms_only)
        res[f"both{k}_ms"] = timeit(both)
    res["gemm6_full_ms"] = timeit(lambda: [a @ bm for _ in range(6)])
    print(json.dumps({k: round(v, 2) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
