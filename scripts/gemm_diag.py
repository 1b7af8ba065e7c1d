"""Locate wrong output elements of a hand-GEMM variant: per shape/layout, run it several times
against an fp32 reference and print where (row/col mod the 256 tile, fragment index) and how
often elements are wrong."""
import sys

import torch

sys.path.insert(0, ".")
from ray_community_amd import ops  # noqa: E402

var = int(sys.argv[1]) if len(sys.argv) > 1 else 3
lib = ops._lib.lib()
lib.rca_gemm_set_variant(var)
dev = "cuda"
for (M, N, K) in [(256, 256, 64), (256, 256, 128), (512, 512, 256), (1024, 1024, 1024), (2048, 2048, 4096)]:
    for ak, bk in [(False, False), (False, True), (True, True), (True, False)]:
        torch.manual_seed(0)
        a = torch.randn(K, M, device=dev) if ak else torch.randn(M, K, device=dev)
        b = torch.randn(K, N, device=dev) if bk else torch.randn(N, K, device=dev)
        a, b = a.bfloat16(), b.bfloat16()
        ref = (a.float().t() if ak else a.float()) @ (b.float() if bk else b.float().t())
        bad_total = 0
        masks = []
        base = torch.randn(M, N, device=dev).bfloat16()
        for rep in range(6):
            if rep % 2 == 0:
                out = ops.gemm(a, b, ak, bk)
                r = ref
            else:
                out = base.clone()
                ops.gemm(a, b, ak, bk, out=out, accumulate=True)
                r = ref + base.float()
            torch.cuda.synchronize()
            err = (out.float() - r).abs()
            bad = err > 0.05 * ref.abs().max()
            masks.append(bad)
            bad_total += int(bad.sum())
        if bad_total == 0:
            print(f"{M}x{N}x{K} ak={ak} bk={bk}: ok")
            continue
        m = masks[0]
        for x in masks[1:]:
            m = m | x
        rows = torch.nonzero(m.any(1)).flatten()
        cols = torch.nonzero(m.any(0)).flatten()
        same = all(torch.equal(masks[0], x) for x in masks[1:])
        print(f"{M}x{N}x{K} ak={ak} bk={bk}: bad/run={[int(x.sum()) for x in masks]} deterministic={same} "
              f"rows%256={sorted(set((rows % 256).tolist()))[:40]} cols%256={sorted(set((cols % 256).tolist()))[:40]}",
              flush=True)
