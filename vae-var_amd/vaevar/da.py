"""The vae4dvar analysis step on the HIP engine — mirror of cyclic_4dvar.one_step_DA(..., 'vae4dvar')
(da_4dvar.py:1179-1306). The WRMSE/Bias logging of :1256-1269 runs on the device (vaevar.metrics) when a truth
field and a Metrics object are given.

  z = zeros(1,32,128,256)                                  (:1238)
  LBFGS(history_size=10, max_iter=10, strong_wolfe)        (:1240)
  for kk in range(Nit+1): cal_loss(z) ; lbfgs.step(closure) while kk < Nit   (:1255-1299)
  xa = decoder_hr(z)[0]*stdTr*std + xb                     (:1301-1306)
"""
from __future__ import annotations

import time

import torch

from .engine import DAProblem
from .lbfgs import LBFGS, Adam


def one_step_da(prob: DAProblem, nit: int, history_size: int = 10, max_iter: int = 10, optimizer: str = "lbfgs",
                lr: float | None = None, log_terms: bool = True, log=None, gt=None, metrics=None, replay=None,
                batch_scalars: bool = True):
    """Returns dict(xa, z, J=[(J_b, J_o) per outer pass], n_eval, n_iter, n_discarded (speculative evaluations the
    reference would not have made, not in n_eval but in seconds), seconds); with gt (T,C,Hs,Ws) and a
    vaevar.metrics.Metrics also metrics=[(wrmse[C], bias[C]) per outer pass] of xhat against gt[0] — the
    reference's bg_* (pass 0) and ana_* (pass Nit) entries of metrics_list (:1285-1291)."""
    dev = prob.xb.device
    z = torch.zeros(prob.latent_shape, device=dev, dtype=torch.float32)
    ctx = prob.ctx
    if optimizer == "lbfgs":
        opt = LBFGS(ctx, z, lr=1 if lr is None else lr, history_size=history_size, max_iter=max_iter,
                    line_search_fn="strong_wolfe")
        opt.replay = list(replay) if replay is not None else None  # fixed-step replay of a reference run
        opt.batch_scalars = batch_scalars  # False: one synchronising call per scalar (vaevar/lbfgs.py)
    elif optimizer == "adam":
        opt = Adam(ctx, z, lr=1e-3 if lr is None else lr)
    else:
        raise ValueError(optimizer)

    def closure(zz, g):
        if optimizer == "lbfgs" and batch_scalars:  # queued: the loss comes with the mirror's next scalars
            return prob.closure_lazy(zz, g)
        jb, jo = prob.closure(zz, g)
        return prob.loss_f32(jb, jo)

    js, ms = [], []
    n0 = prob.n_evals
    d0 = prob.n_discarded
    t0 = time.time()
    for kk in range(nit + 1):
        if log_terms:
            jb, jo = prob.closure(z, None)  # cal_loss (:1210-1236): no gradient
            js.append((jb, jo))
            if gt is not None and metrics is not None:
                xhat = prob.trajectory()[0]  # decoder_hr(z)*stdTr*std + xb of this pass (:1256-1258)
                w, b = metrics.wrmse_bias(xhat, gt[0])
                ms.append((w.cpu().numpy(), b.cpu().numpy()))
            if log is not None:
                log(kk, jb, jo)
        if kk < nit:
            opt.step(closure)
    xa = prob.analysis(z)
    torch.cuda.synchronize()
    n_log = (nit + 1) if log_terms else 0
    n_iter = opt.state["n_iter"] if optimizer == "lbfgs" else opt.t
    return {"xa": xa, "z": z, "J": js, "n_eval": prob.n_evals - n0 - n_log, "n_iter": n_iter,
            "n_discarded": prob.n_discarded - d0, "seconds": time.time() - t0, "metrics": ms}


def one_step_da_batch(prob: DAProblem, nit: int, history_size: int = 10, max_iter: int = 10):
    """B independent one_step_DA analyses (da_4dvar.py:1179-1306) in lockstep over one batched closure: each
    analysis b runs its own L-BFGS mirror on its latent z[b]; whenever every unfinished analysis has requested an
    evaluation, ONE vv_closure evaluates all B latents (the GEMMs of the decoder / flow run on B x 2048 rows) and
    each optimiser resumes with its own J and gradient. Analyses that have finished keep their final latent in
    the batch (their results are not used). Returns dict(xa (B,C,Hs,Ws), z, n_eval per analysis, n_iter per
    analysis, batched_evals, seconds)."""
    dev = prob.xb.device
    B = prob.B
    Z = torch.zeros(prob.latent_shape, device=dev, dtype=torch.float32)
    G = torch.empty_like(Z)
    ctx = prob.ctx
    opts = [LBFGS(ctx, Z[b], lr=1, history_size=history_size, max_iter=max_iter, line_search_fn="strong_wolfe")
            for b in range(B)]

    def run(opt):
        for _ in range(nit):
            yield from opt.step_gen()

    t0 = time.time()
    gens = [run(o) for o in opts]
    pending = [None] * B
    active = [True] * B
    n_eval = [0] * B
    for b in range(B):
        try:
            pending[b] = next(gens[b])
        except StopIteration:
            active[b] = False
    batched = 0
    while any(active):
        jb, jo = prob.closure_batch(Z, G)
        batched += 1
        for b in range(B):
            if not active[b]:
                continue
            zb, gb = pending[b]
            ctx.copy(gb, G[b])
            n_eval[b] += 1
            try:
                pending[b] = gens[b].send(prob.loss_f32(jb[b], jo[b]))
            except StopIteration:
                active[b] = False
    xa = prob.analysis(Z)
    torch.cuda.synchronize()
    return {"xa": xa, "z": Z, "n_eval": n_eval, "n_iter": [o.state["n_iter"] for o in opts],
            "batched_evals": batched, "seconds": time.time() - t0}

