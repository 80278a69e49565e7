"""Kernel-level numerics on the GPU: the MFMA GEMM and the vector primitives against fp32/fp64
torch CPU references (tolerances written per test)."""
import math

import numpy as np
import pytest
import torch

from conftest import check, check_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from vaevar.engine import Context

    return Context.get(0)


def _ref_gemm(A, B, bias):
    r = A.double() @ B.double().t()
    if bias is not None:
        r = r + bias.double()
    return r


@pytest.mark.parametrize("M,N,K,tile", [
    (256, 96, 96, -1), (2048, 1152, 1152, 0), (2048, 1152, 1152, 4), (2048, 1152, 1152, 2),
    (2048, 3456, 1152, -1), (2048, 1152, 4608, -1), (8192, 288, 96, -1), (100, 70, 64, 2), (130, 200, 32, 0),
    (2048, 1152, 1152, 34), (2048, 1152, 1152, 24), (100, 70, 64, 34), (130, 200, 32, 24), (300, 96, 384, 24),
    (2048, 4608, 1152, 34), (130, 200, 64, 4), (130, 200, 64, 34),
])
def test_gemm_nt(ctx, M, N, K, tile):
    g = torch.Generator().manual_seed(M * 7 + N * 3 + K)
    A = torch.rand(M, K, generator=g) * 2 - 1
    B = torch.rand(N, K, generator=g) * 2 - 1
    bias = torch.rand(N, generator=g) - 0.5
    C = ctx.gemm(A.cuda(), B.cuda(), bias.cuda(), tile=tile).cpu().double()
    ref = _ref_gemm(A, B, bias)
    # exact-f32 MFMA (tiles 0/2/4) and the bf16x6 split (24/34): error ~1e-7 * sum|a*b| per element
    scale = (A.abs().double() @ B.abs().double().t()).max()
    err = (C - ref).abs().max() / scale
    check(f"gemm {M}x{N}x{K} tile {tile} err / max sum|ab|", float(err), 2e-6)


@pytest.mark.parametrize("M,N,K", [(2048, 4608, 1152), (2048, 1152, 4608), (8192, 96, 384), (777, 300, 96)])
def test_gemm_split_accuracy(ctx, M, N, K):
    """bf16x6 split GEMM (tiles 24, 34) vs fp64: element error / sum|a*b| no larger than the exact-f32
    MFMA's on the same operands (x1.5 margin) and below 1e-6; randn operands, weight-like B scale."""
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) * 0.03
    ref = A.double() @ B.double().t()
    scale = A.double().abs() @ B.double().abs().t()
    A, B = A.cuda(), B.cuda()
    e32 = float(((ctx.gemm(A, B, tile=2).cpu().double() - ref).abs() / scale).max())
    for t in (24, 34):
        es = float(((ctx.gemm(A, B, tile=t).cpu().double() - ref).abs() / scale).max())
        print(f"gemm {M}x{N}x{K}: f32 {e32:.2e} split t{t} {es:.2e}")
        check(f"bf16x6 t{t} {M}x{N}x{K} vs fp64", es, min(1e-6, 1.5 * e32))


@pytest.mark.parametrize("M,N,K", [(2048, 4608, 1152), (2048, 1152, 4608), (300, 200, 96), (4096, 384, 1152),
                                   (2048, 3456, 1152)])
def test_gemm_pipelined_registered(ctx, M, N, K):
    """Pipelined 128x128 split kernels (tile 34 bf16x6, 36 fp16x3) and the bf16x6 kernels of 64x64 (24), 128x64 (25) and
    64x64 with three k-tile buffers (26) on a registered weight (pre-split planes), incl. ragged edges and the split-K
    tail: same fp32-level error bound as the other variants."""
    g = torch.Generator().manual_seed(M + 3 * N + 7 * K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) * 0.03
    ref = A.double() @ B.double().t()
    scale = A.double().abs() @ B.double().abs().t()
    Bd = B.cuda()
    ctx.gemm_register_weight(Bd)
    for t in (36, 34, 24, 25, 26):
        C = ctx.gemm(A.cuda(), Bd, tile=t).cpu().double()
        es = float(((C - ref).abs() / scale).max())
        print(f"registered gemm {M}x{N}x{K} t{t}: {es:.2e}")
        check(f"registered gemm {M}x{N}x{K} t{t} vs fp64", es, 1e-6)
    _keep.append(Bd)   # a registered weight must stay alive while the context lives


_keep = []


@pytest.mark.parametrize("tile", [-1, 44, 47, 36])
def test_gemm_h3_tile_unregistered_b(ctx, tile):
    """An fp16x3 tile (or the auto pick) with a B that has no fp16 planes runs the bf16x6 128x128 kernel; its split-K
    tail must be sized for THAT kernel's tiles (256-row tail geometry with 128-row fallback tiles wrote
    past the GEMM workspace at 16384x1152x4608)."""
    M, N, K = 16384, 1152, 4608
    g = torch.Generator().manual_seed(4242)
    A = (torch.rand(M, K, generator=g) * 2 - 1).cuda()
    B = (torch.randn(N, K, generator=g) * 0.03).cuda()
    C = ctx.gemm(A, B, tile=tile).double()
    ref = A.double() @ B.double().t()
    scale = (A.double().abs() @ B.double().abs().t()).max()
    err = float((C - ref).abs().max() / scale)
    print(f"unregistered B, tile {tile}: {err:.2e}")
    check(f"unregistered B tile {tile}", err, 2e-6)


def test_tuning_knobs_per_context():
    """vv_set_tuning / vv_get_tuning: every key round-trips on a fresh context, an unknown key is refused, and a
    routing knob (h3_big = 0: 128x128 fp16x3 tiles; tail_minkt 40: no split-K tail) changes only the kernel, not
    the fp32-level result; a second context on the same device keeps the defaults (knobs are per context)."""
    from vaevar.engine import Context
    from vaevar._lib import VVError

    c1, c2 = Context(0), Context(0)
    for k in Context.TUNING_KEYS:
        v = c1.get_tuning(k)
        alt = {"mlp_hc": 32 if v != 32 else 64, "gattn_qf": 3 - v,
               "fuse_mlp": (v + 1) % 4, "fuse_attn": (v + 1) % 4, "bs_tile": 24 if v != 24 else 27}.get(k, v + 1 if v > 1 or "mink" in k else 1 - v)
        c1.set_tuning(k, alt)
        assert c1.get_tuning(k) == alt
        assert c2.get_tuning(k) == v
        c1.set_tuning(k, v)
    with pytest.raises(VVError):
        c1.set_tuning("no_such_knob", 1)
    # values the dispatch does not accept are refused at vv_set_tuning, not inside a later closure
    for k, bad in (("mlp_hc", 48), ("fuse_attn", 12), ("grid_fused", 3), ("gattn_qf", 0), ("tail_minkt", 0), ("host_wait", 2),
                   ("bs_tile", 0)):
        with pytest.raises(VVError):
            c1.set_tuning(k, bad)
        assert c1.get_tuning(k) != bad
    M, N, K = 2048, 3456, 1152
    g = torch.Generator().manual_seed(99)
    A = (torch.rand(M, K, generator=g) * 2 - 1).cuda()
    B = (torch.randn(N, K, generator=g) * 0.03).cuda()
    c1.gemm_register_weight(B)
    c2.gemm_register_weight(B)
    c1.set_tuning("h3_big", 0)
    c1.set_tuning("tail_minkt", 40)
    ref = A.double() @ B.double().t()
    scale = float((A.double().abs() @ B.double().abs().t()).max())
    for c in (c1, c2):
        err = float((c.gemm(A, B).double() - ref).abs().max()) / scale
        check("routing knobs change only the kernel", err, 1e-6)


@pytest.mark.parametrize("tile", [36, 44, 46, 47, 48])
@pytest.mark.parametrize("M,N,K", [(2048, 1152, 1152), (1000, 520, 4608)])
def test_gemm_split16_dynamic_range(ctx, M, N, K, tile):
    """fp16x3 split (tiles 36 = 128x128, 44 = 256x128 of 8 waves, 46 / 47 the same on 16x16x32 MFMAs) keeps fp32-level error when row magnitudes of A span 2^+-17 and vary along K
    (per-chunk scales), B rows span 2^+-8, with zeros, a zero row and huge/tiny values: no overflow, no flush."""
    g = torch.Generator().manual_seed(M + N + K + 1)
    A = torch.randn(M, K, generator=g) * torch.exp(torch.empty(M, 1).uniform_(-12, 12, generator=g)) \
        * torch.exp(torch.empty(1, K).uniform_(-3, 3, generator=g))
    A[5] = 0.0
    A[:, 7] = 0.0
    A[9, 11] = 3.0e30
    A[10] *= 1e-25
    B = torch.randn(N, K, generator=g) * 0.03 * torch.exp(torch.empty(N, 1).uniform_(-6, 6, generator=g))
    ref = A.double() @ B.double().t()
    scale = (A.double().abs() @ B.double().abs().t()).clamp_min(1e-300)
    Bd = B.cuda()
    ctx.gemm_register_weight(Bd)
    e32 = float(((ctx.gemm(A.cuda(), Bd, tile=2).cpu().double() - ref).abs() / scale).max())
    C = ctx.gemm(A.cuda(), Bd, tile=tile).cpu().double()
    assert torch.isfinite(C).all()
    es = float(((C - ref).abs() / scale).max())
    print(f"split16 (tile {tile}) dynamic range {M}x{N}x{K}: f32 {e32:.2e} split16 {es:.2e}")
    check(f"fp16x3 tile {tile} {M}x{N}x{K} dynamic range vs fp64 (bound min(1e-6, 2x f32 MFMA))", es, min(1e-6, 2.0 * e32))
    assert torch.all(C[5] == 0)
    _keep.append(Bd)


@pytest.mark.parametrize("M,N,K", [(2048, 3456, 1152), (2048, 1152, 4608), (2048, 4608, 1152), (1000, 520, 4608),
                                   (300, 200, 96)])
def test_gemm_h4_bitwise_h3m(ctx, M, N, K):
    """Tile 48 (A split once by k_rowsplit into fp16 planes, both operands staged by LDS-DMA through a 3-stage ring)
    computes the same products in the same order as tile 47 (in-loop split, register staging): C bit-identical,
    including the split-K tail shapes (K 4608 at N 1152, N 4608) and ragged edges."""
    from vaevar.engine import Context

    g = torch.Generator().manual_seed(M + 3 * N + 7 * K)
    A = (torch.randn(M, K, generator=g) * torch.exp(torch.empty(M, 1).uniform_(-4, 4, generator=g))).cuda()
    B = (torch.randn(N, K, generator=g) * 0.03).cuda()
    c = Context(0)  # same split-K chunking for both tiles (tile 48 has its own, lower floor by default)
    c.set_tuning("h4_split_minkt", c.get_tuning("small_split_minkt"))
    c.gemm_register_weight(B)
    c47 = c.gemm(A, B, tile=47)
    c48 = c.gemm(A, B, tile=48)
    check_bitwise(f"tile 48 vs 47 {M}x{N}x{K}", c47, c48)
    _keep.append(B)


@pytest.mark.parametrize("M,N,K", [(2048, 4608, 1152), (2048, 4608, 4608), (777, 300, 96), (2100, 4464, 1152)])
def test_gemm_h5_bitwise_h4(ctx, M, N, K):
    """Tile 49 (256 x 144 tiles) computes every element with tile 48's products in tile 48's order: C bit-identical to
    tile 48 run data-parallel (split-K off), including ragged edges; and the router sends the N = 4608 GEMMs at 2048
    rows (256 tiles of 256 x 144 = one round on 256 CUs; tile 48: 288) to it."""
    from vaevar.engine import Context

    g = torch.Generator().manual_seed(M + 5 * N + 3 * K)
    A = (torch.randn(M, K, generator=g) * torch.exp(torch.empty(M, 1).uniform_(-4, 4, generator=g))).cuda()
    B = (torch.randn(N, K, generator=g) * 0.03).cuda()
    c = Context(0)
    c.set_tuning("small_split", 0)
    c.set_tuning("tail_minkt", 1 << 20)
    c.gemm_register_weight(B)
    c48 = c.gemm(A, B, tile=48)
    c49 = c.gemm(A, B, tile=49)
    check_bitwise(f"tile 49 vs 48 {M}x{N}x{K}", c48, c49)
    _keep.append(B)


def test_reduce_batch_matches_single_calls(ctx):
    """vv_reduce_batch (the L-BFGS mirror's batched scalars): every op equals the one-call-each vv_dot / vv_abssum /
    vv_absmax on the same vectors (same kernels, partial layouts and final reductions), and the appended device doubles
    come back unchanged; bad op codes and too many ops are rejected."""
    from vaevar._lib import VVError

    g = torch.Generator().manual_seed(7)
    n = 1 << 20
    a, b, c = (torch.randn(n, generator=g).cuda() for _ in range(3))
    extra = torch.tensor([1.25, -3.5e7], dtype=torch.float64, device="cuda")
    reqs = [(0, a, b), (1, c, None), (2, b, None), (0, c, c), (2, a, None)]
    got = ctx.reduce_batch(reqs, extra=extra)
    want = [ctx.dot(a, b), ctx.abssum(c), ctx.absmax(b), ctx.dot(c, c), ctx.absmax(a)]
    check_bitwise("reduce_batch vs single calls", got, want + [1.25, -3.5e7])
    with pytest.raises(VVError):
        ctx.reduce_batch([(3, a, None)])
    with pytest.raises(VVError):
        ctx.reduce_batch([(1, a, None)] * 9)
    # r05: all requests in one launch (k_reduce_multi) -- ragged and tiny lengths, the full 8 requests, extras only,
    # and vv_reduce_enqueue's device results, each equal to the one-call-each values
    for m in (1_000_003, 5):
        x, y = a[:m], c[:m]
        reqs = [(0, x, y), (1, x, None), (2, y, None), (0, y, y), (1, y, None), (2, x, None), (0, x, x), (0, y, x)]
        want = [ctx.dot(x, y), ctx.abssum(x), ctx.absmax(y), ctx.dot(y, y), ctx.abssum(y), ctx.absmax(x),
                ctx.dot(x, x), ctx.dot(y, x)]
        check_bitwise(f"reduce_batch 8 requests n={m}", ctx.reduce_batch(reqs), want)
        dev = torch.full((8,), float("nan"), dtype=torch.float64, device="cuda")
        ctx.reduce_enqueue(reqs, dev)
        check_bitwise(f"reduce_enqueue n={m}", dev.cpu().tolist(), want)
    assert ctx.reduce_batch([], extra=extra) == [1.25, -3.5e7]


def test_gemm_rejects_non_library_tiles(ctx):
    """vv_gemm accepts only the library's kernels (tile -1, 0, 2, 4, 24..27, 34, 36, 44, 46, 47, 48, 49): any other hint,
    e.g. the r01 timing experiments 37-39, returns VV_E_ARG instead of running something."""
    from vaevar._lib import VVError

    A = torch.rand(64, 64, device="cuda")
    B = torch.rand(64, 64, device="cuda")
    for t in (1, 3, 21, 28, 35, 37, 38, 39, 40, 41, 42, 45, 50, 1000):
        with pytest.raises(VVError, match="1001"):
            ctx.gemm(A, B, tile=t)
    ref = A.double().cpu() @ B.double().cpu().t()
    for t in (0, 2, 4, 24, 25, 26, 27, 34, 36, 44, 46, 47, 48, 49):
        C = ctx.gemm(A, B, tile=t).cpu().double()
        assert float((C - ref).abs().max()) < 1e-4


@pytest.mark.parametrize("tile", [36, 44, 46, 47, 48])
@pytest.mark.parametrize("M,N,K", [(2048, 1152, 4608), (2048, 4608, 1152), (2048, 1152, 3456)])
def test_gemm_splitk_deterministic(ctx, M, N, K, tile):
    """fp16x3 GEMMs whose tiles are split along K (every tile at N = 1152, the tail at N = 4608): the fixup sums
    the partials in chunk order, so 30 back-to-back launches give bit-identical results at fp32-level error."""
    g = torch.Generator().manual_seed(M + N + K + 7)
    A = torch.randn(M, K, generator=g).cuda()
    B = (torch.randn(N, K, generator=g) * 0.03).cuda()
    ctx.gemm_register_weight(B)
    _keep.append(B)
    first = ctx.gemm(A, B, tile=tile)
    outs = [ctx.gemm(A, B, tile=tile) for _ in range(30)]
    torch.cuda.synchronize()
    check("30 launches differing from the first", sum(0 if torch.equal(o, first) else 1 for o in outs), 0, "==")
    ref = A.double().cpu() @ B.double().cpu().t()
    scale = A.double().abs().cpu() @ B.double().abs().cpu().t()
    check(f"split-K tile {tile} {M}x{N}x{K} vs fp64", float(((first.cpu().double() - ref).abs() / scale).max()), 1e-6)


def test_gemm_math_switch(ctx):
    assert ctx.gemm_math in ("split16", "split", "f32")
    old = ctx.gemm_math
    try:
        for m in ("f32", "split", "split16"):
            ctx.gemm_math = m
            assert ctx.gemm_math == m
    finally:
        ctx.gemm_math = old


def test_gemm_asymmetric_identity(ctx):
    # A = I, asymmetric B catches a transposed C-write (cdna_hip_programming.md §3)
    n = 128
    A = torch.eye(n)
    B = torch.arange(n * n, dtype=torch.float32).reshape(n, n)
    C = ctx.gemm(A.cuda(), B.cuda()).cpu()
    assert torch.equal(C, B.t())


def test_vector_primitives(ctx):
    g = torch.Generator().manual_seed(5)
    n = 1_048_576 + 17
    a = (torch.rand(n, generator=g) * 2 - 1)
    b = (torch.rand(n, generator=g) * 2 - 1)
    da, db = a.cuda(), b.cuda()
    assert abs(ctx.dot(da, db) - float((a.double() * b.double()).sum())) < 1e-6 * n ** 0.5
    assert abs(ctx.abssum(da) - float(a.double().abs().sum())) < 1e-3
    assert ctx.absmax(da) == float(a.abs().max())
    y = db.clone()
    ctx.axpy(y, da, 0.25)
    assert torch.allclose(y.cpu(), b + 0.25 * a, atol=1e-6)
    out = torch.empty_like(da)
    ctx.axpby(out, da, 2.0, db, -1.0)
    assert torch.allclose(out.cpu(), 2 * a - b, atol=1e-6)
    ctx.scale(out, 0.5)
    assert torch.allclose(out.cpu(), a - 0.5 * b, atol=1e-6)


def test_adam_matches_torch(ctx):
    g = torch.Generator().manual_seed(9)
    p0 = torch.rand(4099, generator=g)
    grads = [torch.rand(4099, generator=g) - 0.5 for _ in range(5)]
    pt = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([pt], lr=0.1)
    p = p0.cuda()
    m = torch.zeros_like(p)
    v = torch.zeros_like(p)
    for i, gr in enumerate(grads):
        opt.zero_grad()
        pt.grad = gr.clone()
        opt.step()
        ctx.adam(p, gr.cuda(), m, v, 0.1, 0.9, 0.999, 1e-8, i + 1)
    check("Adam vs torch.optim.Adam (max |diff| - rtol |ref|)", float(((p.cpu() - pt.detach()).abs() - 1e-5 * pt.detach().abs()).max()), 1e-6, "<=")


@pytest.mark.parametrize("src,dst", [((128, 256), (721, 1440)), ((721, 1440), (128, 256)), ((32, 64), (45, 90)),
                                     ((64, 128), (64, 128))])
def test_resample_nearest_matches_interpolate(ctx, src, dst):
    """vv_resample_nearest == F.interpolate(mode='nearest') bit for bit (quirk Q3), and its adjoint == the autograd
    backward of F.interpolate (sums over each source pixel's preimage)."""
    from vaevar.engine import resample_nearest

    g = torch.Generator().manual_seed(sum(src) + sum(dst))
    x = torch.randn(2, 3, *src, generator=g)
    ref = torch.nn.functional.interpolate(x, dst)
    xd = x.cuda().requires_grad_(True)
    out = resample_nearest(ctx, xd, dst)
    check_bitwise(f"nearest {src}->{dst} vs F.interpolate", out.detach().cpu(), ref)
    cot = torch.randn(2, 3, *dst, generator=g)
    out.backward(cot.cuda())
    xr = x.clone().requires_grad_(True)
    torch.nn.functional.interpolate(xr, dst).backward(cot)
    check(f"nearest {src}->{dst} adjoint", float((xd.grad.cpu() - xr.grad).abs().max()) / float(xr.grad.abs().max()), 1e-12, "<=")



def _gelu_ref64(x):
    """nn.GELU() (exact erf form, swinblock.py:13-29) and its derivative in float64."""
    x = x.double()
    cdf = 0.5 * (1.0 + torch.special.erf(x / math.sqrt(2.0)))
    pdf = torch.exp(-0.5 * x * x) / math.sqrt(2.0 * math.pi)
    return x * cdf, cdf + x * pdf


@pytest.mark.parametrize("form", [0, 1])
def test_gelu_device_dense_grid(ctx, form):
    """The branch-free GELU / GELU' of every epilogue (vv_gelu.h: the fitted exp2 form of Phi, v_exp_f32 on the device)
    over 2^21 + 1 points of [-10, 10] and the fitted range's edges, against float64 erf: GELU within 2e-7 max(|x|, 1),
    GELU' within 2e-7 absolute (the verdict's bound; the fit's float32 emulation claims 8.7e-8 |x| / 8.2e-8). Form 0:
    gelu_fast / dgelu_fast (GEMM epilogues), 1: gelu4 / dgelu4 (fused MLP, tile-49 row epilogue). Also +-inf and NaN."""
    xs = torch.linspace(-10.0, 10.0, 2 ** 21 + 1, dtype=torch.float32)
    edge = torch.tensor([0.0, -0.0, 5.75, -5.75, 5.7499995, -5.7500005, 1e-30, -1e-30, 29.9, 30.5, -31.0, 1e4, -1e4],
                        dtype=torch.float32)
    x = torch.cat([xs, edge]).cuda()
    y, dy = ctx.gelu_eval(x, form)
    torch.cuda.synchronize()
    yr, dyr = _gelu_ref64(x.cpu())
    ey = float(((y.cpu().double() - yr).abs() / x.cpu().double().abs().clamp(min=1.0)).max())
    ed = float((dy.cpu().double() - dyr).abs().max())
    print(f"GELU form {form}: max err / max(|x|,1) {ey:.2e}, GELU' max abs err {ed:.2e}")
    check(f"GELU form {form}", ey, 2e-7, "<=")
    check(f"GELU' form {form}", ed, 2e-7, "<=")
    sp = torch.tensor([float("inf"), float("-inf"), float("nan")], device="cuda")
    y, dy = ctx.gelu_eval(sp, form)
    y, dy = y.cpu(), dy.cpu()
    assert y[0] == float("inf") and abs(float(y[1])) < 2e-7 and torch.isnan(y[2])
    assert dy[0] == 1.0 and abs(float(dy[1])) < 2e-7 and torch.isnan(dy[2])


@pytest.mark.parametrize("tile", [0, 24, 36, 48])
def test_gelu_gemm_epilogues_identity(ctx, tile):
    """The GELU / GELU' GEMM epilogues (EPI_GELU: C = gelu(acc + bias), aux = acc + bias; EPI_DGELU: C = acc *
    gelu'(aux)) through identity-B GEMMs over 1,048,576 points of [-10, 10]: GELU of the stored pre-activation within
    2e-7 max(|x|, 1) of float64 erf, the pre-activation bit-identical to the EPI_STORE GEMM of the same tile, and with
    A = 1 (acc = 1 exactly) GELU' of aux within 2e-7."""
    from vaevar.engine import Context

    c = Context(0)
    c.gemm_math = "f32" if tile in (0,) else ("split" if tile == 24 else "split16")
    n = 1024
    eye = torch.eye(n, device="cuda")
    c.gemm_register_weight(eye)
    x = torch.linspace(-10.0, 10.0, n * n, dtype=torch.float32).reshape(n, n)
    x = x[torch.randperm(n, generator=torch.Generator().manual_seed(5))].cuda()  # rows mix magnitudes
    pre = c.gemm(x, eye, tile=tile)
    aux = torch.empty_like(pre)
    yg = c.gemm_epi(x, eye, "gelu", aux=aux, tile=tile)
    ones = torch.ones(n, n, device="cuda")
    yd = c.gemm_epi(ones, eye, "dgelu", aux=x, tile=tile)
    torch.cuda.synchronize()
    check_bitwise(f"tile {tile} GELU epilogue pre-activation vs store epilogue", aux, pre)
    yr, _ = _gelu_ref64(pre.cpu())
    _, dyr = _gelu_ref64(x.cpu())
    ey = float(((yg.cpu().double() - yr).abs() / pre.cpu().double().abs().clamp(min=1.0)).max())
    ed = float((yd.cpu().double() - dyr).abs().max())
    print(f"tile {tile}: GELU epilogue {ey:.2e} (pre-activation vs x {float((pre - x).abs().max()):.1e}), "
          f"GELU' epilogue {ed:.2e}")
    check(f"tile {tile} GELU epilogue", ey, 2e-7, "<=")
    check(f"tile {tile} GELU' epilogue", ed, 2e-7, "<=")
