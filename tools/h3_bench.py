"""fp16x3 GEMM microbenchmark over the LG-stage shapes (registered weights), incl. the timing-experiment
variants 37-39 (no loads / no MFMA / no A-split arithmetic; wrong results). Development tool."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar.engine import Context

ctx = Context.get(0)
shapes = [(2048, 3456, 1152), (2048, 1152, 1152), (2048, 4608, 1152), (2048, 1152, 4608), (2048, 1152, 3456),
          (8192, 1152, 1152), (4096, 4608, 1152)]
tiles = [int(t) for t in os.environ.get("TILES", "36,37,38,39").split(",")]
for (M, N, K) in shapes:
    A = torch.rand(M, K, device="cuda") * 2 - 1
    B = torch.rand(N, K, device="cuda") * 2 - 1
    ctx.gemm_register_weight(B)
    row = {"M": M, "N": N, "K": K}
    ref = (A.double() @ B.double().T)
    row["err"] = float((ctx.gemm(A, B, tile=36).double() - ref).abs().max() / ref.abs().max())
    for t in tiles:
        if t in (36, 40) and os.environ.get("ERR", "1") == "1":
            row[f"err{t}"] = float((ctx.gemm(A, B, tile=t).double() - ref).abs().max() / ref.abs().max())
        for _ in range(3):
            ctx.gemm(A, B, tile=t)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 30
        e0.record()
        for _ in range(n):
            ctx.gemm(A, B, tile=t)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        row[f"t{t}"] = f"{us:.1f}us {2 * M * N * K / us / 1e6:.0f}TF"
    print(json.dumps(row), flush=True)
