"""Per-workgroup phase clocks of the fused Swin-tower kernels (development tool, run on the GPU box).

  make -C vae-var_amd/csrc BUILD=build_trace EXTRA=-DVV_TRACE OUT=../vaevar/ab/libvaevar_trace.so   (here, on the CPU)
  python tools/tower_trace.py [--grid 128x256] [--T 2]                                             (on the box)

Loads the VV_TRACE build (vv_tower.hip's VV_TR points: wave 0 of every workgroup stores s_memtime at the kernel's
entry, after its prologue, after each weight chunk's second barrier and after each chunk's MFMAs, and at its exit,
plus s_memrealtime and HW_ID / XCC_ID), runs one config-3 closure with the trace buffer set, and prints per kernel
(the last launch of each kind in the closure): the launch's span, workgroup durations, the shader clock implied
by memtime vs realtime, workgroups resident per CU, and the mean cycles per phase.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("VAEVAR_LIB", os.path.join(ROOT, "vae-var_amd", "vaevar", "ab", "libvaevar_trace.so"))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from vaevar import _lib  # noqa: E402
from vaevar import config as C  # noqa: E402
from vaevar.engine import DAProblem, LGUnet  # noqa: E402
from vaevar.problem import make_problem  # noqa: E402

REGIONS = {0: "k_mlp<96> fwd", 1: "k_mlp<96> bwd", 2: "k_ablk_fwd<96>", 3: "k_ablk_bwd<96>",
           4: "k_mlp<192> fwd", 5: "k_mlp<192> bwd", 6: "k_ablk_fwd<192>", 7: "k_ablk_bwd<192>"}
NWG, NS = 2048, 64


def analyse(reg, t):
    live = t[:, 3] != 0
    if not live.any():
        return None
    t = t[live]
    nwg = int(live.sum())
    rt0, rt1 = t[:, 0].astype(np.int64), t[:, 62].astype(np.int64)
    cyc = (t[:, 63] - t[:, 3]).astype(np.int64)
    dur_rt = (rt1 - rt0) * 10.0  # ns (100 MHz)
    span = (rt1.max() - rt0.min()) * 10.0
    hw, xcc = t[:, 1].astype(np.int64), t[:, 2].astype(np.int64)
    cu = ((hw >> 8) & 0xF) | (((hw >> 12) & 1) << 4) | (((hw >> 13) & 0x7) << 5) | ((xcc & 0xF) << 8)
    # residency: for every workgroup, how many workgroups of the same CU overlap its start
    res = []
    for i in range(nwg):
        same = cu == cu[i]
        res.append(int(((rt0[same] <= rt0[i]) & (rt1[same] > rt0[i])).sum()))
    starts = (rt0 - rt0.min()) * 10.0 / 1e3  # us
    ph = {"prologue": float(np.mean(t[:, 4] - t[:, 3]))}
    prev = t[:, 4]
    nch = 0
    for c in range(29):
        a, b = 5 + 2 * c, 6 + 2 * c
        if a >= 62 or not (t[:, a] != 0).all():
            break
        ph[f"c{c:02d}_stage"] = float(np.mean(t[:, a] - prev))
        ph[f"c{c:02d}_work"] = float(np.mean(t[:, b] - t[:, a]))
        prev = t[:, b]
        nch += 1
    if (t[:, 40] != 0).all() and reg in (0, 1, 4, 5):
        ph["after_loop"] = float(np.mean(t[:, 40] - prev))
        prev = t[:, 40]
    ph["epilogue"] = float(np.mean(t[:, 63] - prev))
    stage = sum(v for k, v in ph.items() if k.endswith("_stage"))
    work = sum(v for k, v in ph.items() if k.endswith("_work"))
    return {"kernel": REGIONS[reg], "workgroups": nwg, "span_us": span / 1e3,
            "wg_us_mean": float(np.mean(dur_rt)) / 1e3, "wg_us_min": float(np.min(dur_rt)) / 1e3,
            "wg_us_max": float(np.max(dur_rt)) / 1e3, "wg_cycles_mean": float(np.mean(cyc)),
            "clock_ghz": float(np.mean(cyc / np.maximum(dur_rt, 1.0))),
            "cus_used": int(len(np.unique(cu))), "resident_per_cu_max": int(max(res)),
            "resident_per_cu_mean": float(np.mean(res)),
            "start_us_quantiles": [float(np.quantile(starts, q)) for q in (0, 0.25, 0.5, 0.75, 0.9, 1.0)],
            "chunks": nch, "cycles_stage_total": stage, "cycles_work_total": work,
            "phase_cycles": {k: round(v) for k, v in ph.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=2)
    ap.add_argument("--grid", default="128x256")
    ap.add_argument("--settings", default="", help="key=v,key=v tuning for the traced closure")
    a = ap.parse_args()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.vv_debug_tower_trace.argtypes = [ctypes.c_void_p]
    Hs, Ws = (int(v) for v in a.grid.split("x"))
    dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
    flow = LGUnet(C.FLOW, 1, a.T - 1).load_synthetic() if a.T > 1 else None
    for kv in filter(None, a.settings.split(",")):
        k, v = kv.split("=")
        dec.ctx.set_tuning(k, int(v))
    prob = DAProblem(dec, make_problem(nch=69, Hs=Hs, Ws=Ws, T=a.T, seed=20250620), flow=flow)
    z = torch.zeros(1, 32, 128, 256, device="cuda")
    g = torch.empty_like(z)
    for _ in range(3):
        prob.closure(z, g)
    torch.cuda.synchronize()
    buf = torch.zeros(8 * NWG * NS, dtype=torch.int64, device="cuda")
    assert lib.vv_debug_tower_trace(ctypes.c_void_p(buf.data_ptr())) == 0
    prob.closure(z, g)
    torch.cuda.synchronize()
    assert lib.vv_debug_tower_trace(None) == 0
    t = buf.view(8, NWG, NS).cpu().numpy().view(np.uint64)
    for reg in range(8):
        r = analyse(reg, t[reg])
        if r:
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
