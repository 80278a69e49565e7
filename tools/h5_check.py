"""Tile 49 (256 x 144, k_gemm_h5) against tile 48 (all tiles data-parallel: split-K off): bit-identical C on the
LG shapes and ragged edges, and the time per launch of both on the N = 4608 shapes (tile 48 with its default split-K
tail). Usage: python tools/h5_check.py [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch  # noqa: E402

from vaevar.engine import Context  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
keep = []


def mats(M, N, K, seed):
    g = torch.Generator().manual_seed(seed)
    A = (torch.randn(M, K, generator=g) * torch.exp(torch.empty(M, 1).uniform_(-4, 4, generator=g))).cuda()
    B = (torch.randn(N, K, generator=g) * 0.03).cuda()
    return A, B


dp = Context(0)
dp.set_tuning("small_split", 0)
dp.set_tuning("tail_minkt", 1 << 20)
for (M, N, K) in [(2048, 4608, 1152), (2048, 4608, 4608), (777, 300, 96), (2100, 4464, 1152), (256, 144, 32)]:
    A, B = mats(M, N, K, M + N + K)
    dp.gemm_register_weight(B)
    keep.append(B)
    c48 = dp.gemm(A, B, tile=48)
    c49 = dp.gemm(A, B, tile=49)
    ref = (A.double() @ B.double().t())
    err = float((c49.double() - ref).abs().max() / ref.abs().max())
    print(f"{M}x{N}x{K}: tile 49 == tile 48 (DP) {torch.equal(c48, c49)}, max diff {float((c48 - c49).abs().max()):.1e}, "
          f"rel err vs fp64 {err:.1e}", flush=True)

ctx = Context(0)
for (M, N, K) in [(2048, 4608, 1152), (4096, 4608, 1152)]:
    A, B = mats(M, N, K, 11)
    ctx.gemm_register_weight(B)
    keep.append(B)
    out = {}
    for t in (48, 49):
        key = t
        for _ in range(3):
            ctx.gemm(A, B, tile=t)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            ctx.gemm(A, B, tile=t)
        e1.record()
        torch.cuda.synchronize()
        out[key] = e0.elapsed_time(e1) * 1e3 / reps
    fl = 2.0 * M * N * K
    print(f"{M}x{N}x{K}: " + ", ".join(f"{'tile %d' % k} {v:.1f} us "
                                      f"({fl / v / 1e6:.0f} TF)" for k, v in out.items()), flush=True)
    # the k_rowsplit pass alone (A planes), for the main-kernel time

