"""Per-workgroup efficiency of the fp16x3 tiles (r06): one-round GEMMs timed with HIP events, STORE epilogue,
registered B (pre-split planes), A split by k_rowsplit (in the event time; run under rocprofv3 --kernel-trace, e.g.
gpu_steps.py ktrace:tools/tile_eff.py, for the GEMM kernels alone).

  tile 48 (256 x 128) at 2048 x 3456 x 1152: 216 workgroups (the qkv GEMM: 40 CUs idle)
  tile 48 (256 x 128) at 2048 x 4096 x 1152: 256 workgroups, the same per-workgroup work
  tile 49 (256 x 144) at 2048 x 4608 x 1152: 256 workgroups, 1.125x the per-workgroup flops
  tile 49 (256 x 144) at 2048 x 3456 x 1152: 192 workgroups

The first two say whether a workgroup runs slower when every CU is busy (clock / L2 share), the second and third the
per-flop cost of the 256 x 144 tile against the 256 x 128 one. Usage: python tools/tile_eff.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch  # noqa: E402

from vaevar.engine import Context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ctx = Context(0)
ctx.set_tuning("small_split", 0)       # data-parallel only: one round of whole-K tiles
ctx.set_tuning("h4_small", 0)
ctx.set_tuning("tail_minkt", 1 << 20)
keep = []


def timed(fn, n):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


out = []
for (M, N, K, tile) in [(2048, 3456, 1152, 48), (2048, 4096, 1152, 48), (2048, 4608, 1152, 49),
                        (2048, 3456, 1152, 49), (2048, 4608, 1152, 48), (4096, 4608, 1152, 49),
                        (4096, 4096, 1152, 48)]:
    g = torch.Generator().manual_seed(M + N + K)
    A = (torch.randn(M, K, generator=g)).cuda()
    B = (torch.randn(N, K, generator=g) * 0.03).cuda()
    ctx.gemm_register_weight(B)
    keep.append(B)
    us = timed(lambda: ctx.gemm(A, B, tile=tile), reps)
    bm, bn = (256, 128) if tile == 48 else (256, 144)
    wgs = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
    rec = {"M": M, "N": N, "K": K, "tile": tile, "workgroups": wgs, "us_per_call": round(us, 2),
           "tflops_fp32eq": round(2.0 * M * N * K / (us * 1e-6) / 1e12, 1),
           "us_per_kt_per_wg_round": round(us / (K // 32) / -(-wgs // 256), 3)}
    out.append(rec)
    print(json.dumps(rec), flush=True)
