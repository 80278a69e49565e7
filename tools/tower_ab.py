"""Tower (short-K bf16x6) GEMM shapes, tiles from TILES (default 24,34; registered weights, HIP events on the
current stream; `bitwise` compares the first two). Development tool; the r02 resident-B experiment (tile 26,
removed) is recorded under profiles/r02/short_k_bsr/."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar.engine import Context

ctx = Context.get(0)
shapes = [(49152, 288, 96), (49152, 96, 96), (49152, 384, 96), (12288, 576, 192), (12288, 192, 192),
          (12288, 768, 192), (49152, 192, 96), (12288, 384, 192)]
for (M, N, K) in shapes:
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(N, K, device="cuda", generator=g) * 0.03
    ctx.gemm_register_weight(B)
    row = {"M": M, "N": N, "K": K}
    outs = {}
    tiles = [int(t) for t in os.environ.get("TILES", "24,34").split(",")]
    for t in tiles:
        outs[t] = ctx.gemm(A, B, tile=t)
        for _ in range(3):
            ctx.gemm(A, B, tile=t)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            ctx.gemm(A, B, tile=t)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        row[f"t{t}"] = [round(us, 1), round(4 * (M * K + N * K + M * N) / us / 1e6, 2)]
    row["bitwise"] = bool(torch.equal(outs[tiles[0]], outs[tiles[-1]]))
    print(json.dumps(row), flush=True)
    del A, B
