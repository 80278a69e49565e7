"""fp16x3 GEMM microbenchmark over the LG-stage shapes at 2048 tokens per analysis (registered weights, the
engine's tile choice incl. split-K). Development tool: TILES=a,b,... picks the tiles, MROWS scales the rows, tuning
knobs come from VAEVAR_<KEY>. Times one GEMM call (the whole launch sequence: row-scale pass, main kernel, split-K
fixup) with HIP events on the current stream."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar.engine import Context

ctx = Context.get(0)
mult = int(os.environ.get("MROWS", "1"))
shapes = [(2048 * mult, n, k) for n, k in ((3456, 1152), (1152, 1152), (4608, 1152), (1152, 4608), (1152, 3456))]
tot = 0.0
for (M, N, K) in shapes:
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    A = torch.randn(M, K, device="cuda", generator=g)
    B = torch.randn(N, K, device="cuda", generator=g) * 0.03
    ctx.gemm_register_weight(B)
    ref = A.double() @ B.double().T
    scale = A.double().abs() @ B.double().abs().T
    tiles = [int(t) for t in os.environ.get("TILES", "-1").split(",")]
    row = {"M": M, "N": N, "K": K}
    C0 = None
    for t in tiles:
        C = ctx.gemm(A, B, tile=t)
        err = float(((C.double() - ref).abs() / scale).max())
        if C0 is None:
            C0 = C.clone()
        else:
            row[f"t{t}_bitwise_vs_t{tiles[0]}"] = bool(torch.equal(C, C0))
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
        row[f"t{t}"] = [round(us, 1), round(2 * M * N * K / us / 1e6 / 833.3, 3), float('%.2g' % err)]
    print(json.dumps(row), flush=True)
    del A, B
    continue
    C = ctx.gemm(A, B)
    err = float(((C.double() - ref).abs() / scale).max())
    for _ in range(3):
        ctx.gemm(A, B)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 50
    e0.record()
    for _ in range(n):
        ctx.gemm(A, B)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / n
    tot += us
    print(json.dumps({"M": M, "N": N, "K": K, "us": round(us, 2), "tflops": round(2 * M * N * K / us / 1e6, 1),
                      "frac_833": round(2 * M * N * K / us / 1e6 / 833.3, 3), "err": err}), flush=True)
    del A, B
print(json.dumps({"total_us": round(tot, 1)}), flush=True)
