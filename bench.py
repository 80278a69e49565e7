#!/usr/bin/env python3
"""Benchmark of the VAE-Var 4D-Var inner loop on MI355X (BASELINE.json metric).

Workload (N=1): BASELINE config 2 — 3D-Var with the full VAE decoder (nf_model/parameters0_old.yaml,
216M parameters), 69-channel 128x256 state, L-BFGS(history 10, max_iter 10, strong Wolfe) as in
da_4dvar.py:1240, synthetic weights and observations (no checkpoints ship with the reference).

  step   = one outer `lbfgs.step(closure)` (<= 10 L-BFGS iterations, <= 12 closure evaluations);
           --steps 10 is the reference's converged budget for config 2 (Nit 10 x max_iter 10 = 100 iters).
  value  = L-BFGS iterations per second over the whole job (sum over ranks / max time over ranks);
           the analysis decode and the RCCL gather of all analyses to rank 0 are inside the timed region.
  N > 1  = ensemble: rank r runs its own analysis (seed + r), weak scaling, no inner-loop communication.

Prints ONE JSON line on rank 0. See DESIGN.md §Measurement.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK_F32_TFLOPS = 157.3   # MI355X fp32 MFMA dense peak (MI355X_MICROARCH.md, chip-level table)
PEAK_BF16_TFLOPS = 2500.0  # MI355X bf16 MFMA dense peak; the split GEMM spends 6 bf16 products per fp32 product
PEAK_SPLIT_TFLOPS = PEAK_BF16_TFLOPS / 6
PEAK_SPLIT16_TFLOPS = 2500.0 / 3  # fp16 MFMA dense peak (= bf16); the fp16x3 split spends 3 products per fp32 one
PEAK_HBM_GBS = 8000.0     # HBM3E spec
FLOPS_PER_EVAL = {1: 1787.8e9, 2: 3577.0e9, 6: 10733.7e9}  # SURVEY §8 d (input-grad only)

CONFIGS = {
    2: dict(T=1, name="config 2: 3D-Var, full VAE decoder (parameters0_old), 69ch 128x256, 100 L-BFGS iters"),
    3: dict(T=2, name="config 3: 4D-Var, 2-step window with LGUnet flow stand-in, 69ch 128x256, 100 iters"),
    4: dict(T=6, name="config 4: 4D-Var, 6-step window, one analysis per GPU (ensemble)"),
    5: dict(T=2, grid=(721, 1440), name="config 5: 4D-Var at 0.25 deg (69ch 721x1440 state, nearest-interpolated "
                                          "to the 128x256 networks), T=2, 50 iters"),
}


def cpu_baseline(prob_np, evals_per_iter, n_evals, threads):
    """Oracle torch-CPU restatement (oracle/) timed in both SURVEY §8 d modes: weight grads ON (the reference
    computes them, quirk Q5; this is `value`) and OFF (input gradient only, like the HIP path)."""
    from oracle.da_ref import oracle_problem
    from oracle.lgunet_ref import synth_params
    from vaevar import config as C

    torch.set_num_threads(threads)
    p = synth_params(C.DECODER)
    ro = oracle_problem(prob_np, p, C.DECODER)
    z = torch.zeros(1, 32, 128, 256, requires_grad=True)

    def timed(weight_grads):
        for v in p.values():
            v.requires_grad_(weight_grads)
            v.grad = None

        def ev():
            for v in p.values():
                v.grad = None
            z.grad = None
            ro.loss(z).backward()

        ev()  # warm-up
        t0 = time.time()
        for _ in range(n_evals):
            ev()
        return (time.time() - t0) / n_evals

    per_eval = timed(True)
    per_eval_off = timed(False)
    return per_eval, {"value": 1.0 / (per_eval * evals_per_iter), "unit": "L-BFGS iters/s", "cores": threads,
                      "kind": "port",
                      "value_weight_grads_off": 1.0 / (per_eval_off * evals_per_iter),
                      "sample": f"{n_evals} closure evaluations (J + dJ/dz) of config 2 at z=0 on {threads} host "
                                f"threads after 1 warm-up, per mode: weight grads on (reference-faithful, `value`) "
                                f"{per_eval:.3f} s/eval, off {per_eval_off:.3f} s/eval; iters/s = 1/(s_per_eval x "
                                f"{evals_per_iter:.3f} evals per iteration of the GPU run)"}


def gemm_traffic(kernel):
    """HBM bytes per launch of `kernel` ("k_gemm_h3" or "all") from the committed rocprofv3 --pmc passes
    (FETCH_SIZE x2 + WRITE_SIZE, gfx950 corrections, tools/pmc_traffic.py) of `bench.py --config 2`; PMC counters
    cannot be read live."""
    path = os.path.join(ROOT, "profiles", "r01", "gemm_traffic.json")
    try:
        with open(path) as f:
            return json.load(f)[kernel]["hbm_bytes_per_launch"]
    except (OSError, KeyError, ValueError, TypeError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10, help="outer L-BFGS steps (Nit)")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-evals", type=int, default=3)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-profile", action="store_true", help="skip the HIP-event per-kernel-class profile")
    args = ap.parse_args()

    from vaevar import config as C
    from vaevar import ensemble
    from vaevar.da import one_step_da
    from vaevar.engine import DAProblem, LGUnet
    from vaevar.lbfgs import LBFGS
    from vaevar.problem import make_problem

    rank, size, local = ensemble.init()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    T = CONFIGS[args.config]["T"]
    dec = LGUnet(C.DECODER, 1, 1, device=local).load_synthetic()
    flow = LGUnet(C.FLOW, 1, T - 1, device=local).load_synthetic() if T > 1 else None
    Hs, Ws = CONFIGS[args.config].get("grid", (128, 256))
    prob_np = make_problem(nch=69, Hs=Hs, Ws=Ws, T=T, seed=20250620 + rank)
    prob = DAProblem(dec, prob_np, flow=flow, device=local)

    # warm-up: W outer steps of a throw-away analysis (same path, same shapes)
    if args.warmup > 0:
        one_step_da(prob, nit=args.warmup, log_terms=False)
    torch.cuda.synchronize()
    prof = (rank == 0) and not args.no_profile

    ensemble.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = one_step_da(prob, nit=args.steps, log_terms=False)
    xs = ensemble.gather_analyses(res["xa"])
    torch.cuda.synchronize()
    ensemble.barrier()
    elapsed = time.perf_counter() - t0
    if prof:
        # per-kernel-class HIP-event profile of the same work (a second pass of the same analysis, so the
        # event records do not perturb the timed region above)
        prob.ctx.profile_start()
        res_p = one_step_da(prob, nit=args.steps, log_terms=False)
        torch.cuda.synchronize()
        pr = prob.ctx.profile_stop()
        prof_elapsed = res_p["seconds"]
    t_max = ensemble.reduce_scalar(elapsed, "max", dev)
    iters = ensemble.reduce_scalar(res["n_iter"], "sum", dev)
    evals = ensemble.reduce_scalar(res["n_eval"], "sum", dev)

    # J before / after (not timed)
    j_end = prob.closure(res["z"], None)
    z0 = torch.zeros_like(res["z"])
    j_0 = prob.closure(z0, None)

    if rank != 0:
        return
    out = {
        "metric": "4D-Var inner-loop iters/sec + wall-clock to convergence, 69ch 128×256 state",
        "value": iters / t_max,
        "unit": "L-BFGS iters/s",
        "n_gpus": size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * t_max / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": CONFIGS[args.config]["name"], "analyses": size, "T": T, "outer_steps": args.steps,
                   "parallelism": "ensemble: 1 independent analysis per GPU, RCCL gather of xa at the end"},
        "wall_clock_to_convergence_s": t_max,
        "iters": iters,
        "evals": evals,
        "evals_per_s": evals / t_max,
        "ms_per_eval": 1e3 * t_max * size / max(evals, 1),
        "J_start": j_0[0] + j_0[1],
        "J_final": j_end[0] + j_end[1],
        "timed_region": "the Nit outer lbfgs.step calls + the analysis decode (+ the gather at N>1); the "
                        "per-outer-pass logging evaluation cal_loss and WRMSE/Bias (da_4dvar.py:1256-1269, SURVEY "
                        "§8 a3) is not run in it: 1 forward per outer pass, reported here as excluded",
    }
    flops_eval = FLOPS_PER_EVAL.get(T)
    if prof:
        math = prob.ctx.gemm_math
        g16, g6 = pr["gemm16"], pr["gemm"]
        allg = {k: g16[k] + g6[k] for k in ("ms", "flops", "bytes", "launches")}
        if math == "split16":
            dom, peak, tkey = g16, PEAK_SPLIT16_TFLOPS, "k_gemm_h3"
            kname = ("k_rowscale + k_gemm_h3 (+ split-K fixup): every GEMM launch that ran the fp16x3 kernel in a "
                     "HIP-event-profiled repeat of the timed analysis")
            desc = ("fp16x3 split: fp32 operands scaled per row by 2^e and split into 2 fp16 planes, 3 "
                    "v_mfma_f32_32x32x16_f16 products per fp32 product; peak = 2.5 PF fp16 dense / 3")
        elif math == "split":
            dom, peak, tkey = allg, PEAK_SPLIT_TFLOPS, "all"
            kname = "every GEMM launch (k_gemm_bs*) of a HIP-event-profiled repeat of the timed analysis"
            desc = "bf16x6 split (fp32 operands as 3 bf16 planes, 6 v_mfma_f32_32x32x16_bf16 products; peak = 2.5 PF / 6)"
        else:
            dom, peak, tkey = allg, PEAK_F32_TFLOPS, "all"
            kname = "every GEMM launch (k_gemm_nt) of a HIP-event-profiled repeat of the timed analysis"
            desc = "exact f32 MFMA (v_mfma_f32_32x32x2_f32; peak 157.3 TF)"
        ach = dom["flops"] / max(dom["ms"] * 1e-3, 1e-12) / 1e12
        n = max(dom["launches"], 1)
        all_ach = allg["flops"] / max(allg["ms"] * 1e-3, 1e-12) / 1e12
        out["roofline"] = {"bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s",
                           "frac": ach / peak, "traffic": gemm_traffic(tkey),
                           "kernel": kname, "gemm_math": desc,
                           "frac_of_f32_mfma_peak": ach / PEAK_F32_TFLOPS,
                           "launches": dom["launches"], "avg_launch_us": 1e3 * dom["ms"] / n,
                           "flops_per_launch": dom["flops"] / n,
                           "algorithmic_bytes_per_launch": dom["bytes"] / n,
                           "share_of_gemm_time": dom["ms"] / max(allg["ms"], 1e-12),
                           "all_gemm": {"achieved": all_ach, "launches": allg["launches"],
                                        "avg_launch_us": 1e3 * allg["ms"] / max(allg["launches"], 1),
                                        "frac_of_f32_mfma_peak": all_ach / PEAK_F32_TFLOPS},
                           "traffic_source": "profiles/r01/gemm_traffic.json: rocprofv3 --pmc FETCH_SIZE / "
                                             "WRITE_SIZE passes of bench.py (tools/pmc_traffic.py)"}
        busy = sum(v["ms"] for v in pr.values())
        out["kernel_time_ms"] = {k: round(v["ms"], 3) for k, v in pr.items()}
        out["kernel_launches"] = {k: v["launches"] for k, v in pr.items()}
        out["gpu_busy_frac"] = busy / (1e3 * prof_elapsed)
        if flops_eval:
            out["eval_roofline_frac"] = (flops_eval / (PEAK_F32_TFLOPS * 1e12)) / (t_max * size / max(evals, 1))
    if size == 1 and not args.no_cpu_baseline and args.config == 2:
        evals_per_iter = evals / max(iters, 1)
        per_eval, cb = cpu_baseline(prob_np, evals_per_iter, args.cpu_evals, args.cpu_threads)
        out["cpu_baseline"] = cb
        out["cpu_wall_clock_to_convergence_s_extrapolated"] = per_eval * evals
        out["speedup_vs_cpu"] = out["value"] / cb["value"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
