"""Same-process A/B of tuning knobs on the full-size closure (development tool, run on the GPU box).

  python tools/knob_ab.py [--T 2] [--grid 721x1440] [--reps 3] [--n 20] SETTING [SETTING ...]

SETTING is `name` (the defaults) or `key=v[,key=v]` (vv_set_tuning keys). Every setting is timed `reps` times,
interleaved (graph replay, `n` closures after 3 warm-ups), then profiled once by HIP events per kernel class (eager
launches). Prints one JSON line per setting: ms per closure (min / median over reps) and the per-class ms / eval.
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
from vaevar.engine import DAProblem, LGUnet  # noqa: E402
from vaevar.problem import make_problem  # noqa: E402


def parse(s):
    if "=" not in s:
        return {}
    return {k: int(v) for k, v in (kv.split("=") for kv in s.split(","))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=2)
    ap.add_argument("--grid", default="128x256")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("settings", nargs="+")
    a = ap.parse_args()
    Hs, Ws = (int(v) for v in a.grid.split("x"))
    dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
    flow = LGUnet(C.FLOW, 1, a.T - 1).load_synthetic() if a.T > 1 else None
    ctx = dec.ctx
    defaults = {k: ctx.get_tuning(k) for k in ctx.TUNING_KEYS}
    prob_np = make_problem(nch=69, Hs=Hs, Ws=Ws, T=a.T, seed=20250620)
    z = torch.zeros(1, 32, 128, 256, device="cuda")
    g = torch.empty_like(z)
    times = {s: [] for s in a.settings}

    def apply(s):
        for k, v in defaults.items():
            ctx.set_tuning(k, v)
        for k, v in parse(s).items():
            ctx.set_tuning(k, v)
        return DAProblem(dec, prob_np, flow=flow)  # bind after the knobs (grid_fused is read at bind)

    for _ in range(a.reps):
        for s in a.settings:
            prob = apply(s)
            for _ in range(3):
                prob.closure(z, g)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.n):
                prob.closure(z, g)
            torch.cuda.synchronize()
            times[s].append(1e3 * (time.perf_counter() - t0) / a.n)
            del prob
    for s in a.settings:
        prob = apply(s)
        prob.closure(z, g)
        ctx.profile_start()
        for _ in range(3):
            prob.closure(z, g)
        pr = ctx.profile_stop()
        t = sorted(times[s])
        print(json.dumps({"setting": s, "T": a.T, "grid": a.grid, "ms_min": t[0], "ms_median": t[len(t) // 2],
                          "ms_all": t, "class_ms_per_eval": {k: round(v["ms"] / 3, 4) for k, v in pr.items()},
                          "class_launches_per_eval": {k: v["launches"] // 3 for k, v in pr.items()}}), flush=True)
        del prob


if __name__ == "__main__":
    main()
