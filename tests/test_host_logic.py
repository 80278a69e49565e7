"""CPU: host-side logic of the HIP path — the L-BFGS mirror (vaevar/lbfgs.py) against torch.optim.LBFGS,
and Adam, with the device vector primitives replaced by a torch-CPU stand-in of the same contract."""
import numpy as np
import torch


class CpuPrims:
    """Same contract as vaevar.engine.Context's vector primitives (double-accumulated reductions)."""

    def dot(self, a, b):
        return float((a.double() * b.double()).sum())

    def abssum(self, a):
        return float(a.double().abs().sum())

    def absmax(self, a):
        return float(a.abs().max())

    def reduce_batch(self, reqs, extra=None):
        out = [self.dot(a, b) if op == 0 else self.abssum(a) if op == 1 else self.absmax(a) for op, a, b in reqs]
        return out + (extra.tolist() if extra is not None else [])

    def reduce_enqueue(self, reqs, out):
        for i, (op, a, b) in enumerate(reqs):
            out[i] = self.dot(a, b) if op == 0 else self.abssum(a) if op == 1 else self.absmax(a)

    def axpy(self, y, x, alpha):
        y.add_(x, alpha=alpha)

    def axpby(self, out, x, a, y, b):
        out.copy_(a * x + (b * y if y is not None else 0))

    def scale(self, y, alpha):
        y.mul_(alpha)

    def copy(self, dst, src):
        dst.copy_(src)

    def lbfgs_two_loop(self, q, stps, dirs, ro, H_diag):
        # k_twoloop_axpy's arithmetic: fp64-accumulated dot rounded to fp32, times ro[i] in fp32
        f32 = np.float32
        al = [None] * len(stps)
        for i in range(len(stps) - 1, -1, -1):
            al[i] = f32(self.dot(stps[i], q)) * f32(ro[i])
            q.add_(dirs[i], alpha=float(-al[i]))
        q.mul_(float(H_diag))
        for i in range(len(stps)):
            be = f32(self.dot(dirs[i], q)) * f32(ro[i])
            q.add_(stps[i], alpha=float(al[i] - be))

    def adam(self, p, g, m, v, lr, b1, b2, eps, step):
        m.lerp_(g, 1 - b1)
        v.mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** step
        bc2 = 1 - b2 ** step
        p.addcdiv_(m, (v.sqrt() / np.sqrt(bc2)).add_(eps), value=-lr / bc1)


def objective(z):
    # smooth, non-quadratic, well conditioned: sum a_i (z_i - c_i)^2 + 0.1 sum (z_i - c_i)^4 + coupling
    n = z.numel()
    i = torch.arange(n, dtype=torch.float32)
    a = 1.0 + 10.0 * (i % 97)  # condition number ~1e3: 30 iterations stay far from fp32 noise
    c = torch.sin(i * 0.37)
    d = z - c
    return (a * d * d).sum() + 0.1 * (d ** 4).sum() + 0.5 * ((z[1:] - z[:-1]) ** 2).sum()


def test_lbfgs_mirror_matches_torch():
    from vaevar.lbfgs import LBFGS

    n = 4096
    zt = torch.zeros(n, requires_grad=True)
    opt = torch.optim.LBFGS([zt], history_size=10, max_iter=10, line_search_fn="strong_wolfe")

    def closure_t():
        opt.zero_grad()
        f = objective(zt)
        f.backward()
        return f

    zm = torch.zeros(n)
    mir = LBFGS(CpuPrims(), zm, history_size=10, max_iter=10, line_search_fn="strong_wolfe")
    n_eval = [0]

    def closure_m(z, g):
        zz = z.clone().requires_grad_(True)
        f = objective(zz)
        f.backward()
        g.copy_(zz.grad)
        n_eval[0] += 1
        return float(f.detach())

    for _ in range(3):
        opt.step(closure_t)
        mir.step(closure_m)
        st = opt.state[opt._params[0]]
        assert mir.state["n_iter"] == st["n_iter"]
        assert mir.state["func_evals"] == st["func_evals"]
        # same branches taken; iterates agree to fp32 reduction-order noise
        assert torch.allclose(zm, zt.detach(), rtol=1e-4, atol=1e-4), (zm - zt.detach()).abs().max()


def test_lbfgs_batched_scalars_identical():
    """The batched scalar fetches (vv_reduce_batch: gtd_new, |g|_max, |d|_max and the speculative ys, yy after an
    evaluation; gtd and d_norm after the direction) give exactly the iterates, losses and counts of one call per
    scalar, with far fewer host round trips."""
    from vaevar.lbfgs import LBFGS

    class Counting(CpuPrims):
        def __init__(self):
            self.calls = 0

        def dot(self, a, b):
            self.calls += 1
            return super().dot(a, b)

        def abssum(self, a):
            self.calls += 1
            return super().abssum(a)

        def absmax(self, a):
            self.calls += 1
            return super().absmax(a)

        def reduce_batch(self, reqs, extra=None):
            c = self.calls
            out = super().reduce_batch(reqs, extra)
            self.calls = c + 1  # one round trip
            return out

        def lbfgs_two_loop(self, q, stps, dirs, ro, H_diag):
            c = self.calls
            super().lbfgs_two_loop(q, stps, dirs, ro, H_diag)
            self.calls = c  # on the device: no round trip

    def closure_m(z, g):
        zz = z.clone().requires_grad_(True)
        f = objective(zz)
        f.backward()
        g.copy_(zz.grad)
        return float(f.detach())

    runs = []
    for batch in (False, True):
        prims = Counting()
        zm = torch.zeros(4096)
        mir = LBFGS(prims, zm, history_size=10, max_iter=10, line_search_fn="strong_wolfe")
        mir.batch_scalars = batch
        losses = [mir.step(closure_m) for _ in range(3)]
        runs.append((zm, losses, dict(mir.state), prims.calls))
    (z0, l0, s0, c0), (z1, l1, s1, c1) = runs
    assert torch.equal(z0, z1) and l0 == l1
    assert s0["n_iter"] == s1["n_iter"] and s0["func_evals"] == s1["func_evals"]
    print(f"scalar round trips: {c0} one at a time, {c1} batched ({s1['n_iter']} iterations)")
    assert c1 * 2 < c0


def test_lbfgs_speculative_line_search_identical():
    """With queued closures (vaevar.engine.LazyLoss) the mirror also defers gtd / d_norm to the line search's first
    evaluation and discards that evaluation where the reference stops first (gtd > -tolerance_change): iterates,
    losses and every count equal the one-call-per-scalar run; the discarded evaluations are uncounted."""
    from vaevar.lbfgs import LBFGS

    class Lazy:
        def __init__(self, f, counter):
            self.dev = torch.tensor([f, 0.0], dtype=torch.float64)
            self.counter = counter

        def resolve(self, v):
            return float(v[0])

        def discard(self):
            self.counter[0] -= 1

        def __float__(self):
            return float(self.dev[0])

    def make_closure(lazy, counter):
        def closure_m(z, g):
            zz = z.clone().requires_grad_(True)
            f = objective(zz)
            f.backward()
            g.copy_(zz.grad)
            counter[0] += 1
            return Lazy(float(f.detach()), counter) if lazy else float(f.detach())
        return closure_m

    runs = []
    for batch in (False, True):
        cnt = [0]
        zm = torch.zeros(4096)
        mir = LBFGS(CpuPrims(), zm, history_size=10, max_iter=10, line_search_fn="strong_wolfe")
        mir.batch_scalars = batch
        losses = [float(mir.step(make_closure(batch, cnt))) for _ in range(4)]
        # the reference's gtd > -tolerance_change exit (taken before the line search): the speculative run has
        # already evaluated at x + t d and must drop that evaluation
        mir.tolerance_change = 1e9
        losses.append(float(mir.step(make_closure(batch, cnt))))
        runs.append((zm, losses, dict(mir.state), cnt[0]))
    (z0, l0, s0, c0), (z1, l1, s1, c1) = runs
    assert torch.equal(z0, z1) and l0 == l1
    assert s0["n_iter"] == s1["n_iter"] and s0["func_evals"] == s1["func_evals"] and c0 == c1


def test_adam_mirror_matches_torch():
    from vaevar.lbfgs import Adam

    n = 1000
    zt = torch.zeros(n, requires_grad=True)
    opt = torch.optim.Adam([zt], lr=0.1)
    zm = torch.zeros(n)
    mir = Adam(CpuPrims(), zm, lr=0.1)

    def closure_m(z, g):
        zz = z.clone().requires_grad_(True)
        f = objective(zz)
        f.backward()
        g.copy_(zz.grad)
        return float(f.detach())

    for _ in range(20):
        opt.zero_grad()
        objective(zt).backward()
        opt.step()
        mir.step(closure_m)
    assert torch.allclose(zm, zt.detach(), rtol=1e-5, atol=1e-6)


def test_state_files_layout(tmp_path):
    """StateFiles writes/reads data_reader.get_state's file layout (da_4dvar.py:148-166) in CHANNELS order."""
    import datetime as dt
    import os

    from vaevar.cycle import CHANNELS, StateFiles

    t = dt.datetime(2018, 1, 1, 6)
    sf = StateFiles(str(tmp_path), shape=(3, 5))
    x = np.arange(69 * 15, dtype=np.float32).reshape(69, 3, 5)
    sf.put_state(t, x)
    assert os.path.exists(os.path.join(str(tmp_path), "single", "2018", "2018-01-01", "06:00:00-u10.npy"))
    assert os.path.exists(os.path.join(str(tmp_path), "2018", "2018-01-01", "06:00:00-z-50.0.npy"))
    assert os.path.exists(os.path.join(str(tmp_path), "2018", "2018-01-01", "06:00:00-t-1000.0.npy"))
    assert np.array_equal(sf.get_state(t), x)
    assert len(CHANNELS) == 69 and CHANNELS[11] == "z500" and CHANNELS[66] == "t850" and CHANNELS[24] == "q500"


def test_lbfgs_fixed_step_replay():
    """Fixed-step replay: the (t, evals) that torch.optim.LBFGS's _strong_wolfe returned, fed to
    the mirror, reproduce torch's iterates and eval counts without running the mirror's own line search."""
    import torch.optim.lbfgs as tl

    from vaevar.lbfgs import LBFGS

    n = 2048
    zt = torch.zeros(n, requires_grad=True)
    opt = torch.optim.LBFGS([zt], history_size=10, max_iter=10, line_search_fn="strong_wolfe")
    steps, orig = [], tl._strong_wolfe

    def rec(*a, **k):
        out = orig(*a, **k)
        steps.append((float(out[2]), int(out[3])))
        return out

    def closure_t():
        opt.zero_grad()
        f = objective(zt)
        f.backward()
        return f

    tl._strong_wolfe = rec
    try:
        for _ in range(2):
            opt.step(closure_t)
    finally:
        tl._strong_wolfe = orig
    zm = torch.zeros(n)
    mir = LBFGS(CpuPrims(), zm, history_size=10, max_iter=10, line_search_fn="strong_wolfe")
    mir.replay = list(steps)
    calls = [0]

    def closure_m(z, g):
        zz = z.clone().requires_grad_(True)
        f = objective(zz)
        f.backward()
        g.copy_(zz.grad)
        calls[0] += 1
        return float(f.detach())

    for _ in range(2):
        mir.step(closure_m)
    st = opt.state[opt._params[0]]
    assert not mir.replay and len(steps) == st["n_iter"]
    assert mir.state["func_evals"] == st["func_evals"] and mir.state["n_iter"] == st["n_iter"]
    assert calls[0] == 2 + len(steps)  # one evaluation per replayed line search (+ the initial one per step)
    assert torch.allclose(zm, zt.detach(), rtol=1e-4, atol=1e-4)
