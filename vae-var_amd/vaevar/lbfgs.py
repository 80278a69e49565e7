"""On-device L-BFGS with strong-Wolfe line search: a statement-by-statement mirror of
torch.optim.LBFGS (torch/optim/lbfgs.py:12-537, torch 2.10) — the optimiser the reference
constructs as `optim.LBFGS([z], history_size=10, max_iter=10, line_search_fn="strong_wolfe")`
(da_4dvar.py:1240).

Vectors (1,048,576 floats for the 32x128x256 latent) stay in HBM and every vector operation
(dot, axpy, scale, abs-max, abs-sum) is a libvaevar kernel; only scalars come to the host.
Scalar types follow torch's promotion rules (quirk Q7): quantities that are 0-d fp32 tensors in
torch (dot products, ys, ro, H_diag, al, be, gtd, ...) are numpy float32 here (numpy 2 treats
Python floats as weak scalars exactly like torch), the loss is a Python float.

Every closure evaluation is a `yield (z, grad_out)` of the generator `step_gen()` that receives the loss, so B
independent optimisers can be advanced in lockstep over one batched closure (vaevar.da.one_step_da_batch);
`step(closure)` drives the same generator with a plain closure.

Host round trips (r04, `batch_scalars`): torch computes an iteration's scalars one synchronising call at a time
(the loss, gtd_new, |g|_max, |d|_max, ys, yy, gtd, d_norm: eight per iteration). Here the scalars that are
known to be asked for next are computed together, in one vv_reduce_batch round trip: after an evaluation the
loss (a vaevar.engine.LazyLoss from a queued closure), gtd_new = g_new.d, |g_new|_max, |d|_max and -- for the
next iteration, should this step be accepted -- y = g_new - prev_flat_grad, s = t d and their ys, yy; after the
direction, gtd and d_norm. A value is used only if the statement that needs it meets the same tensors (and t):
every scalar is the one the one-at-a-time path computes (same kernels, same inputs), so the trajectory is
unchanged; a speculative y / s that is not used costs two axpby and two dots.
"""
from __future__ import annotations

import os

import numpy as np
import torch

f32 = np.float32


def _is_lazy(res):
    # a queued closure's loss (vaevar.engine.LazyLoss): a device (J_b, J_o) to fetch with the next scalars
    return hasattr(res, "dev") and hasattr(res, "resolve")


def _cubic_interpolate(x1, f1, g1, x2, f2, g2, bounds=None):
    # torch/optim/lbfgs.py:12-37
    if bounds is not None:
        xmin_bound, xmax_bound = bounds
    else:
        xmin_bound, xmax_bound = (x1, x2) if x1 <= x2 else (x2, x1)
    d1 = g1 + g2 - 3 * (f1 - f2) / (x1 - x2)
    d2_square = d1 ** 2 - g1 * g2
    if d2_square >= 0:
        d2 = np.sqrt(d2_square)
        if x1 <= x2:
            min_pos = x2 - (x2 - x1) * ((g2 + d2 - d1) / (g2 - g1 + 2 * d2))
        else:
            min_pos = x1 - (x1 - x2) * ((g1 + d2 - d1) / (g1 - g2 + 2 * d2))
        return min(max(min_pos, xmin_bound), xmax_bound)
    return (xmin_bound + xmax_bound) / 2.0


class LBFGS:
    """torch.optim.LBFGS over one flat fp32 device parameter, vector math in libvaevar.

    closure(z, grad_out) -> float evaluates J at z and writes dJ/dz into grad_out.
    """

    def __init__(self, ctx, z: torch.Tensor, lr=1, max_iter=20, max_eval=None, tolerance_grad=1e-7,
                 tolerance_change=1e-9, history_size=100, line_search_fn=None, device_two_loop=True):
        if max_eval is None:
            max_eval = max_iter * 5 // 4
        self.ctx, self.z = ctx, z
        self.lr, self.max_iter, self.max_eval = lr, max_iter, max_eval
        self.tolerance_grad, self.tolerance_change = tolerance_grad, tolerance_change
        self.history_size, self.line_search_fn = history_size, line_search_fn
        self.device_two_loop = device_two_loop  # False: the two loops with host scalars (one sync per dot)
        # fixed-step replay: a list of (t, ls_func_evals) recorded from the reference's
        # _strong_wolfe calls; each line search then takes the recorded step and eval count instead of searching
        self.replay = None
        self.state = {"func_evals": 0, "n_iter": 0}
        self.batch_scalars = hasattr(ctx, "reduce_batch")  # False: one synchronising call per scalar, as torch
        self._cache = []           # [(op, a, b, value)] from the last vv_reduce_batch
        self._spec = None          # (g, prev_flat_grad, d, t, y, s): y, s computed speculatively
        self._prev_flat_grad = None
        # after the direction (n_iter > 1, queued closures): gtd and d_norm queued on the device instead of fetched,
        # and the line search's first evaluation started before they are known; they come back with that
        # evaluation's scalars, and where the reference would have stopped before it (gtd > -tolerance_change) the
        # evaluation is discarded -- same trajectory, same counts, one round trip less per iteration
        self.speculate = os.environ.get("VAEVAR_LBFGS_SPECULATE", "1") != "0"  # A/B switch
        self._lazy_seen = False
        self._deferred = None      # [(op, a, b)] whose values are queued in self._xbuf[2:]
        self._xbuf = None

    # --- vector helpers ---------------------------------------------------
    def _cached(self, op, a, b):
        for e in self._cache:
            if e[0] == op and e[1] is a and e[2] is b:
                return e[3]
        return None

    def _dot(self, a, b):
        v = self._cached(0, a, b)
        return f32(v) if v is not None else f32(self.ctx.dot(a.view(-1), b.view(-1)))

    def _absmax(self, a):
        v = self._cached(2, a, None)
        return f32(v) if v is not None else f32(self.ctx.absmax(a.view(-1)))

    def _prefetch(self, reqs, lazy=None):
        """One vv_reduce_batch for reqs [(op, a, b)] (+ the lazy loss's J pair); fills the cache; returns the loss
        (float) if lazy was given."""
        vals = self.ctx.reduce_batch([(op, a.view(-1), b.view(-1) if b is not None else None) for op, a, b in reqs],
                                     extra=lazy.dev if lazy is not None else None)
        self._cache = [(op, a, b, v) for (op, a, b), v in zip(reqs, vals)]
        return lazy.resolve(vals[len(reqs):]) if lazy is not None else None

    def _enqueue(self, reqs):
        if self._xbuf is None:
            self._xbuf = torch.empty(2 + 8, dtype=torch.float64, device=self.z.device)
        self.ctx.reduce_enqueue([(op, a.view(-1), b.view(-1) if b is not None else None) for op, a, b in reqs],
                                self._xbuf[2:2 + len(reqs)])
        self._deferred = reqs

    def _loss_of(self, res):
        """The loss a closure returned: a float, or a LazyLoss fetched on its own."""
        return float(res)

    def _after_eval(self, res, g, d, t):
        """The evaluation at z = x + t d returned res (loss) and g: fetch the loss with gtd_new, |g|_max, |d|_max and
        the next iteration's ys, yy (speculative y, s) in one round trip."""
        if not self.batch_scalars:
            return float(res)
        reqs = [(0, g, d), (2, g, None), (2, d, None)]
        self._spec = None
        if self._prev_flat_grad is not None:
            y, s = self._new(), self._new()
            self.ctx.axpby(y, g, 1.0, self._prev_flat_grad, -1.0)
            self.ctx.axpby(s, d, float(t), None, 0.0)
            self._spec = (g, self._prev_flat_grad, d, t, y, s)
            reqs += [(0, y, s), (0, y, y)]
        lazy = res if _is_lazy(res) else None
        if self._deferred is None:
            loss = self._prefetch(reqs, lazy)
            return loss if lazy is not None else float(res)
        # the queued gtd / d_norm come back with this evaluation's scalars (and its J pair, copied beside them)
        dq, self._deferred = self._deferred, None
        k = len(dq)
        self._xbuf[:2].copy_(lazy.dev)
        vals = self.ctx.reduce_batch([(op, a.view(-1), b.view(-1) if b is not None else None) for op, a, b in reqs],
                                     extra=self._xbuf[:2 + k])
        n = len(reqs)
        self._cache = [(op, a, b, v) for (op, a, b), v in zip(reqs, vals[:n])]
        self._cache += [(op, a, b, v) for (op, a, b), v in zip(dq, vals[n + 2:n + 2 + k])]
        return lazy.resolve(vals[n:n + 2])

    def _y_s(self, flat_grad, prev_flat_grad, d, t):
        """y = flat_grad - prev_flat_grad, s = t d (lbfgs.py:397-398): the speculative pair if it was made from the
        same tensors and t."""
        sp = self._spec
        self._spec = None
        if sp is not None and sp[0] is flat_grad and sp[1] is prev_flat_grad and sp[2] is d and sp[3] == t:
            return sp[4], sp[5]
        y = self._new()
        self.ctx.axpby(y, flat_grad, 1.0, prev_flat_grad, -1.0)
        s = self._new()
        self.ctx.axpby(s, d, float(t), None, 0.0)
        return y, s

    def _abssum(self, a):
        v = self._cached(1, a, None)
        return f32(v) if v is not None else f32(self.ctx.abssum(a.view(-1)))

    def _new(self):
        return torch.empty_like(self.z)

    def _add_grad(self, step_size, update):
        self.ctx.axpy(self.z, update, float(step_size))

    def _directional_evaluate(self, x, t, d):
        # lbfgs.py:325-331 (a generator: the evaluation is a yield)
        self._add_grad(t, d)
        g = self._new()
        res = yield self.z, g
        self._last_res = res
        loss = self._after_eval(res, g, d, t)
        self.ctx.copy(self.z, x)
        return loss, g

    def _strong_wolfe(self, x, t, d, f, g, gtd, c1=1e-4, c2=0.9, tolerance_change=1e-9, max_ls=25, exit_tol=None):
        # lbfgs.py:40-209; gtd None: queued (speculate), resolved after the first evaluation, and None is returned
        # where the reference's step() would have stopped on gtd > -exit_tol before calling this search
        g_in = g
        d_norm = self._absmax(d) if gtd is not None else None
        g = g.clone()
        f_new, g_new = yield from self._directional_evaluate(x, t, d)
        if gtd is None:
            gtd = self._dot(g_in, d)
            if gtd > -exit_tol:
                if hasattr(self._last_res, "discard"):
                    self._last_res.discard()
                return None
            d_norm = self._absmax(d)
        ls_func_evals = 1
        gtd_new = self._dot(g_new, d)
        t_prev, f_prev, g_prev, gtd_prev = 0, f, g, gtd
        done = False
        ls_iter = 0
        while ls_iter < max_ls:
            if f_new > (f + c1 * t * gtd) or (ls_iter > 1 and f_new >= f_prev):
                bracket, bracket_f = [t_prev, t], [f_prev, f_new]
                bracket_g, bracket_gtd = [g_prev, g_new.clone()], [gtd_prev, gtd_new]
                break
            if abs(gtd_new) <= -c2 * gtd:
                bracket, bracket_f, bracket_g = [t], [f_new], [g_new]
                done = True
                break
            if gtd_new >= 0:
                bracket, bracket_f = [t_prev, t], [f_prev, f_new]
                bracket_g, bracket_gtd = [g_prev, g_new.clone()], [gtd_prev, gtd_new]
                break
            min_step = t + 0.01 * (t - t_prev)
            max_step = t * 10
            tmp = t
            t = _cubic_interpolate(t_prev, f_prev, gtd_prev, t, f_new, gtd_new, bounds=(min_step, max_step))
            t_prev, f_prev, g_prev, gtd_prev = tmp, f_new, g_new.clone(), gtd_new
            f_new, g_new = yield from self._directional_evaluate(x, t, d)
            ls_func_evals += 1
            gtd_new = self._dot(g_new, d)
            ls_iter += 1
        if ls_iter == max_ls:
            bracket, bracket_f, bracket_g = [0, t], [f, f_new], [g, g_new]

        insuf_progress = False
        low_pos, high_pos = (0, 1) if bracket_f[0] <= bracket_f[-1] else (1, 0)
        while not done and ls_iter < max_ls:
            if abs(bracket[1] - bracket[0]) * d_norm < tolerance_change:
                break
            t = _cubic_interpolate(bracket[0], bracket_f[0], bracket_gtd[0], bracket[1], bracket_f[1],
                                   bracket_gtd[1])
            eps = 0.1 * (max(bracket) - min(bracket))
            if min(max(bracket) - t, t - min(bracket)) < eps:
                if insuf_progress or t >= max(bracket) or t <= min(bracket):
                    if abs(t - max(bracket)) < abs(t - min(bracket)):
                        t = max(bracket) - eps
                    else:
                        t = min(bracket) + eps
                    insuf_progress = False
                else:
                    insuf_progress = True
            else:
                insuf_progress = False
            f_new, g_new = yield from self._directional_evaluate(x, t, d)
            ls_func_evals += 1
            gtd_new = self._dot(g_new, d)
            ls_iter += 1
            if f_new > (f + c1 * t * gtd) or f_new >= bracket_f[low_pos]:
                bracket[high_pos] = t
                bracket_f[high_pos] = f_new
                bracket_g[high_pos] = g_new.clone()
                bracket_gtd[high_pos] = gtd_new
                low_pos, high_pos = (0, 1) if bracket_f[0] <= bracket_f[1] else (1, 0)
            else:
                if abs(gtd_new) <= -c2 * gtd:
                    done = True
                elif gtd_new * (bracket[high_pos] - bracket[low_pos]) >= 0:
                    bracket[high_pos] = bracket[low_pos]
                    bracket_f[high_pos] = bracket_f[low_pos]
                    bracket_g[high_pos] = bracket_g[low_pos]
                    bracket_gtd[high_pos] = bracket_gtd[low_pos]
                bracket[low_pos] = t
                bracket_f[low_pos] = f_new
                bracket_g[low_pos] = g_new.clone()
                bracket_gtd[low_pos] = gtd_new
        t = bracket[low_pos]
        return bracket_f[low_pos], bracket_g[low_pos], t, ls_func_evals

    def step(self, closure):
        """One optimizer step (lbfgs.py:333-535); closure(z, grad_out) -> loss."""
        gen = self.step_gen()
        try:
            req = next(gen)
            while True:
                req = gen.send(closure(*req))
        except StopIteration as e:
            return e.value

    def step_gen(self):
        # lbfgs.py:333-535; every closure evaluation is `loss = yield (z, grad_out)`
        lr, max_iter, max_eval = self.lr, self.max_iter, self.max_eval
        tolerance_grad, tolerance_change = self.tolerance_grad, self.tolerance_change
        state = self.state
        flat_grad = self._new()
        res = yield self.z, flat_grad
        if self.batch_scalars:
            lazy = res if _is_lazy(res) else None
            self._lazy_seen = lazy is not None
            orig_loss = self._prefetch([(2, flat_grad, None)], lazy) if lazy is not None else res
            if lazy is None:
                self._prefetch([(2, flat_grad, None)])
        else:
            orig_loss = res
        orig_loss = float(orig_loss)
        loss = float(orig_loss)
        current_evals = 1
        state["func_evals"] += 1
        opt_cond = self._absmax(flat_grad) <= tolerance_grad
        if opt_cond:
            return orig_loss
        d, t = state.get("d"), state.get("t")
        old_dirs, old_stps, ro = state.get("old_dirs"), state.get("old_stps"), state.get("ro")
        H_diag, prev_flat_grad, prev_loss = state.get("H_diag"), state.get("prev_flat_grad"), state.get("prev_loss")
        n_iter = 0
        while n_iter < max_iter:
            n_iter += 1
            state["n_iter"] += 1
            if state["n_iter"] == 1:
                d = self._new()
                self.ctx.axpby(d, flat_grad, -1.0, None, 0.0)
                old_dirs, old_stps, ro = [], [], []
                H_diag = 1
            else:
                y, s = self._y_s(flat_grad, prev_flat_grad, d, t)
                ys = self._dot(y, s)
                if ys > 1e-10:
                    if len(old_dirs) == self.history_size:
                        old_dirs.pop(0)
                        old_stps.pop(0)
                        ro.pop(0)
                    old_dirs.append(y)
                    old_stps.append(s)
                    ro.append(1.0 / ys)
                    H_diag = ys / self._dot(y, y)
                q = self._new()
                self.ctx.axpby(q, flat_grad, -1.0, None, 0.0)
                if self.device_two_loop:
                    # the two loops below with al / be kept on the device (same fp32 arithmetic, no host sync)
                    self.ctx.lbfgs_two_loop(q, old_stps, old_dirs, ro, H_diag)
                    d = q
                else:
                    num_old = len(old_dirs)
                    if "al" not in state:
                        state["al"] = [None] * self.history_size
                    al = state["al"]
                    for i in range(num_old - 1, -1, -1):
                        al[i] = self._dot(old_stps[i], q) * ro[i]
                        self.ctx.axpy(q, old_dirs[i], float(-al[i]))
                    self.ctx.scale(q, float(H_diag))
                    d = r = q
                    for i in range(num_old):
                        be_i = self._dot(old_dirs[i], r) * ro[i]
                        self.ctx.axpy(r, old_stps[i], float(al[i] - be_i))
            if prev_flat_grad is None:
                prev_flat_grad = flat_grad.clone()
            else:
                self.ctx.copy(prev_flat_grad, flat_grad)
            self._prev_flat_grad = prev_flat_grad
            prev_loss = loss
            deferred = (self.batch_scalars and self.speculate and self._lazy_seen and state["n_iter"] > 1 and
                        not self.replay and self.line_search_fn == "strong_wolfe")
            if deferred:  # gtd and d_norm queued; fetched with the line search's first evaluation
                self._enqueue([(0, flat_grad, d), (2, d, None)])
            elif self.batch_scalars:  # gtd and the line search's d_norm (and the first step's |g|_1) together
                reqs = [(0, flat_grad, d), (2, d, None)] + ([(1, flat_grad, None)] if state["n_iter"] == 1 else [])
                self._prefetch(reqs)
            if state["n_iter"] == 1:
                t = min(1.0, 1.0 / self._abssum(flat_grad)) * lr
            else:
                t = lr
            gtd = None
            if not deferred:
                gtd = self._dot(flat_grad, d)
                if gtd > -tolerance_change:
                    break
            ls_func_evals = 0
            if self.line_search_fn is not None:
                if self.line_search_fn != "strong_wolfe":
                    raise RuntimeError("only 'strong_wolfe' is supported")
                x_init = self.z.clone()
                if self.replay:
                    t, ls_func_evals = self.replay.pop(0)
                    loss, flat_grad = yield from self._directional_evaluate(x_init, t, d)
                else:
                    out = yield from self._strong_wolfe(x_init, t, d, loss, flat_grad, gtd,
                                                        max_ls=max_eval - current_evals, exit_tol=tolerance_change)
                    if out is None:  # the queued gtd > -tolerance_change: the reference stopped before this search
                        break
                    loss, flat_grad, t, ls_func_evals = out
                self._add_grad(t, d)
                opt_cond = self._absmax(flat_grad) <= tolerance_grad
            else:
                self._add_grad(t, d)
                if n_iter != max_iter:
                    flat_grad = self._new()
                    loss = self._loss_of((yield self.z, flat_grad))
                    opt_cond = self._absmax(flat_grad) <= tolerance_grad
                    ls_func_evals = 1
            current_evals += ls_func_evals
            state["func_evals"] += ls_func_evals
            if n_iter == max_iter:
                break
            if current_evals >= max_eval:
                break
            if opt_cond:
                break
            if f32(abs(t)) * self._absmax(d) <= tolerance_change:
                break
            if abs(loss - prev_loss) < tolerance_change:
                break
        state.update(d=d, t=t, old_dirs=old_dirs, old_stps=old_stps, ro=ro, H_diag=H_diag,
                     prev_flat_grad=prev_flat_grad, prev_loss=prev_loss)
        return orig_loss


class Adam:
    """torch.optim.Adam (defaults lr=1e-3, betas=(0.9, 0.999), eps=1e-8; adam.py:34) on libvaevar."""

    def __init__(self, ctx, z, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.ctx, self.z, self.lr, self.betas, self.eps = ctx, z, lr, betas, eps
        self.m = torch.zeros_like(z)
        self.v = torch.zeros_like(z)
        self.t = 0

    def step(self, closure):
        g = torch.empty_like(self.z)
        loss = closure(self.z, g)
        self.t += 1
        self.ctx.adam(self.z, g, self.m, self.v, self.lr, self.betas[0], self.betas[1], self.eps, self.t)
        return loss
