"""Host-side costs around the closure (development tool, run on the GPU box).

  python tools/host_probe.py [--T 2] [--n 30]

Times, on the config-3 problem: the host cost of each Python entry point the L-BFGS mirror calls per iteration
(the call alone, the GPU drained before each), the closure's exposed launch latency (a closure started on an
idle GPU and synchronised, minus the back-to-back pipelined closure), and one full L-BFGS step (10 iterations)
against its evaluations x the pipelined closure. Prints one JSON line. Run it under different HIP runtime
environments to A/B the graph submission (e.g. DEBUG_HIP_GRAPH_BATCH_SIZE).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch  # noqa: E402

from vaevar import config as C  # noqa: E402
from vaevar.engine import DAProblem, LGUnet, _stream  # noqa: E402
from vaevar.lbfgs import LBFGS  # noqa: E402
from vaevar.problem import make_problem  # noqa: E402


def host_us(fn, n, drain=True):
    """Median host time of fn() in us, the GPU drained before each call."""
    ts = []
    for _ in range(n):
        if drain:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ts.append(1e6 * (time.perf_counter() - t0))
    torch.cuda.synchronize()
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=2)
    ap.add_argument("--n", type=int, default=30)
    a = ap.parse_args()
    dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
    flow = LGUnet(C.FLOW, 1, a.T - 1).load_synthetic() if a.T > 1 else None
    ctx = dec.ctx
    prob = DAProblem(dec, make_problem(nch=69, Hs=128, Ws=256, T=a.T, seed=20250620), flow=flow)
    z = torch.zeros(prob.latent_shape, device="cuda")
    g = torch.empty_like(z)
    d = torch.randn_like(z)
    for _ in range(3):
        prob.closure_lazy(z, g)
    torch.cuda.synchronize()
    out = {"T": a.T, "env": {k: v for k, v in os.environ.items() if k.startswith(("DEBUG_HIP", "DEBUG_CLR",
                                                                                   "HIP_", "AMD_"))}}
    n = a.n
    out["host_us"] = {
        "stream": host_us(lambda: _stream(), n),
        "empty_like": host_us(lambda: torch.empty_like(z), n),
        "clone": host_us(lambda: z.clone(), n),
        "axpy": host_us(lambda: ctx.axpy(z, d, 0.0), n),
        "copy": host_us(lambda: ctx.copy(g, z), n),
        "axpby": host_us(lambda: ctx.axpby(g, z, 1.0, d, -1.0), n),
        "reduce_batch5_sync": host_us(lambda: ctx.reduce_batch([(0, g, d), (2, g, None), (2, d, None), (0, z, d),
                                                                (0, z, z)]), n),
        "closure_lazy_submit": host_us(lambda: prob.closure_lazy(z, g), n),
    }
    # exposed latency: an idle GPU, one closure, synchronised; vs pipelined back-to-back closures
    ser = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        prob.closure_lazy(z, g)
        torch.cuda.synchronize()
        ser.append(1e3 * (time.perf_counter() - t0))
    ser.sort()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        prob.closure_lazy(z, g)
    torch.cuda.synchronize()
    pipe = 1e3 * (time.perf_counter() - t0) / n
    # GPU-side: events around one closure started on an idle GPU
    ev = []
    for _ in range(n):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        prob.closure_lazy(z, g)
        e1.record()
        torch.cuda.synchronize()
        ev.append(e0.elapsed_time(e1))
    ev.sort()
    out["closure_ms"] = {"serial_median": round(ser[n // 2], 4), "pipelined": round(pipe, 4),
                         "event_median": round(ev[n // 2], 4)}
    # one full L-BFGS step (10 iterations, strong Wolfe) from z = 0, as one_step_da's first outer pass
    zz = torch.zeros_like(z)
    opt = LBFGS(ctx, zz, lr=1, history_size=10, max_iter=10, line_search_fn="strong_wolfe")
    e0 = prob.n_evals
    d0 = prob.n_discarded
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    opt.step(lambda zq, gq: prob.closure_lazy(zq, gq))
    torch.cuda.synchronize()
    wall = 1e3 * (time.perf_counter() - t0)
    ne = prob.n_evals - e0 + prob.n_discarded - d0
    out["lbfgs_step"] = {"ms": round(wall, 3), "evals": ne, "iters": opt.state["n_iter"],
                         "ms_per_eval": round(wall / ne, 4), "overhead_ms_per_eval": round(wall / ne - pipe, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
