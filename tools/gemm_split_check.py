"""Accuracy (vs fp64) and speed of the f32-MFMA and bf16x6-split GEMM variants (development tool)."""
import os, sys, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar.engine import Context

ctx = Context.get(0)
tiles = [int(t) for t in os.environ.get("TILES", "2,21,22,23,24,25,26").split(",")]
shapes = [tuple(int(x) for x in sh.split("x")) for sh in os.environ["SHAPES"].split(",")] if os.environ.get("SHAPES") else [(2048, 4608, 1152), (2048, 1152, 4608), (2048, 3456, 1152), (2048, 1152, 1152), (2048, 1024, 4608),
          (8192, 288, 96), (8192, 96, 384), (2048, 576, 192), (49152, 384, 96), (49152, 96, 384)]
keep = []   # registered operands must stay alive while the context lives
for (M, N, K) in shapes:
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(N, K, device="cuda", generator=g) * 0.03
    if os.environ.get("PRE"):
        ctx.gemm_register_weight(B)
    if os.environ.get("APRE"):
        ctx.gemm_register_weight(A)
    keep += [A, B]
    ref = A.double() @ B.double().t()
    scale = (A.double().abs() @ B.double().abs().t())
    row = {"M": M, "N": N, "K": K}
    for t in tiles:
        try:
            C = ctx.gemm(A, B, tile=t)
            err = ((C.double() - ref).abs() / scale).max().item()
            for _ in range(3):
                ctx.gemm(A, B, tile=t)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 20
            e0.record()
            for _ in range(n):
                ctx.gemm(A, B, tile=t)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / n
            row[f"t{t}"] = [round(2 * M * N * K / us / 1e6, 1), float(f"{err:.2e}")]
        except Exception as ex:
            row[f"t{t}"] = str(ex)[:40]
    print(json.dumps(row), flush=True)
