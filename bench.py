#!/usr/bin/env python3
"""Benchmark of the VAE-Var 4D-Var inner loop on MI355X (BASELINE.json metric: inner-loop iterations/s and
wall-clock to the converged analysis, 69ch 128x256 state).

Workload (default, r05): BASELINE config 3 — the metric's own config: 4D-Var with a 2-step window (da_win = 2:
the full VAE decoder, nf_model/parameters0_old.yaml, 216M parameters, plus one step of the LGUnet flow stand-in in
the loss, da_4dvar.py:1183-1208), 69-channel 128x256 state, L-BFGS(history 10, max_iter 10, strong Wolfe) as
da_4dvar.py:1240, Nit = 10 outer passes (the reference's budget: <= 100 iterations), synthetic weights and
observations (no checkpoints ship with the reference). `--config 2|4|5` selects the other BASELINE configs
(Nit 10 / 10 / 5); every line carries the others as sub-records (config2 = 3D-Var, the r01-r04 headline).

  step   = one converged analysis (one_step_DA 'vae4dvar', da_4dvar.py:1179-1306): z = 0, Nit outer lbfgs.step
           calls, the analysis decode; at N > 1 plus the RCCL gather of every rank's analysis to rank 0
  value  = L-BFGS iterations per second over the whole job (iterations summed over ranks / max time over ranks)
  N > 1  = ensemble: rank r runs its own analysis (seed + r), weak scaling, no inner-loop
           communication. `--gpus N` without WORLD_SIZE spawns the N ranks itself (before any GPU call); under
           torch.distributed.run WORLD_SIZE must equal --gpus.
  config4 = every line also carries BASELINE config 4 (T = 6 window, one analysis per GPU, the RCCL gather),
           timed on its own after the main region, so its analyses/s can be compared across N as well.
  --batch B = B independent analyses per GPU advanced in lockstep over ONE batched closure per evaluation (the
           decoder / flow GEMMs on B x 2048 rows, vaevar.da.one_step_da_batch); value counts every analysis.

Prints ONE JSON line on rank 0. See DESIGN.md §6.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
sys.path.insert(0, ROOT)

PEAK_F32_TFLOPS = 157.3    # MI355X exact-f32 MFMA dense peak (MI355X_MICROARCH.md, chip-level table)
PEAK_16_TFLOPS = 2500.0    # MI355X bf16 / fp16 MFMA dense peak
PEAK_SPLIT16_TFLOPS = PEAK_16_TFLOPS / 3  # fp16x3 split: 3 fp16 MFMA products per fp32 product
PEAK_SPLIT_TFLOPS = PEAK_16_TFLOPS / 6    # bf16x6 split: 6 bf16 MFMA products per fp32 product
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E peak (MI355X_MICROARCH.md)
FLOPS_PER_EVAL = {1: 1787.8e9, 2: 3577.0e9, 6: 10733.7e9}  # SURVEY §8 d (input-grad only)
METRIC = "4D-Var inner-loop iters/sec + wall-clock to convergence, 69ch 128×256 state"

CONFIGS = {
    2: dict(T=1, nit=10, name="config 2: 3D-Var, full VAE decoder (parameters0_old), 69ch 128x256, L-BFGS Nit 10 "
                             "(<= 100 iterations) per analysis"),
    3: dict(T=2, nit=10, name="config 3: 4D-Var, 2-step window with the LGUnet flow stand-in, 69ch 128x256, Nit 10"),
    4: dict(T=6, nit=10, name="config 4: 4D-Var, 6-step window (5 flow steps), 69ch 128x256, Nit 10, one analysis "
                             "per GPU + RCCL gather"),
    5: dict(T=2, nit=5, grid=(721, 1440), name="config 5: 4D-Var at 0.25 deg (69ch 721x1440 state, nearest-"
                                               "interpolated to the 128x256 networks), T=2, Nit 5 (<= 50 iterations)"),
}


# ---------------------------------------------------------------------------------------------------------------
# launch
def spawn(n: int, argv) -> int:
    """Start N ranks of this script (before this process touches the GPU) and return rank 0's exit code."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    codes = [p.wait() for p in procs]
    bad = [c for c in codes if c != 0]
    return bad[0] if bad else 0


def physical_cores():
    """(physical cores among the CPUs this process may run on, those CPUs, the OMP_NUM_THREADS share if set)."""
    cpus = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    cores = set()
    for c in cpus:
        try:
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/core_id") as f:
                core = f.read().strip()
            with open(f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id") as f:
                pkg = f.read().strip()
            cores.add((pkg, core))
        except OSError:
            cores.add(("?", str(c)))
    share = os.environ.get("OMP_NUM_THREADS")
    return len(cores), len(cpus), int(share) if share and share.isdigit() else None


def cgroup_cpu_quota():
    """CPUs' worth of time the process's cgroup may use (cgroup v2 cpu.max 'quota period'), or None if unlimited."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        return None


# ---------------------------------------------------------------------------------------------------------------
# CPU baseline: the oracle restatement (oracle/, a torch-CPU port of the reference path) on the host cores
def cpu_baseline(prob_np, T, evals_per_iter, gpu_evals_per_analysis, evals, threads, cores_note, all_cores=None):
    """The oracle closure (J + dJ/dz) timed on `threads` host threads, weight grads on (as the reference computes
    them, quirk Q5) and off (the cheapest faithful CPU formulation: only dJ/dz is used); with `all_cores` also one
    bounded sample at every physical core of the process's affinity. Returns (s/eval with grads on, record)."""
    import torch

    from oracle.da_ref import oracle_problem
    from oracle.lgunet_ref import synth_params
    from vaevar import config as C

    p = synth_params(C.DECODER)
    fp = synth_params(C.FLOW) if T > 1 else None
    ro = oracle_problem(prob_np, p, C.DECODER, fp, C.FLOW if T > 1 else None)
    z = torch.zeros(1, 32, 128, 256, requires_grad=True)
    params = list(p.values()) + (list(fp.values()) if fp else [])

    def timed(weight_grads, n, nthreads):
        torch.set_num_threads(nthreads)
        for v in params:
            v.requires_grad_(weight_grads)
            v.grad = None

        def ev():
            for v in params:
                v.grad = None
            z.grad = None
            ro.loss(z).backward()

        ev()  # warm-up
        t0 = time.time()
        for _ in range(n):
            ev()
        return (time.time() - t0) / n

    per_eval = timed(True, evals, threads)
    per_off = timed(False, evals, threads)
    out = {"value": 1.0 / (per_eval * evals_per_iter), "unit": "L-BFGS iters/s", "cores": threads, "kind": "port",
           "value_weight_grads_off": 1.0 / (per_off * evals_per_iter), "s_per_eval": per_eval,
           "s_per_eval_weight_grads_off": per_off,
           "wall_clock_to_convergence_s_extrapolated": per_eval * gpu_evals_per_analysis}
    sample = (f"T={T}: {evals} closure evaluation(s) (J + dJ/dz) at z=0 after 1 warm-up on {threads} host threads "
              f"({cores_note}), weight grads on as the reference computes them (quirk Q5): {per_eval:.3f} s/eval; "
              f"off: {per_off:.3f} s/eval")
    if all_cores and all_cores > threads:
        per_all = timed(True, 1, all_cores)
        out["value_all_cores"] = 1.0 / (per_all * evals_per_iter)
        out["cores_all"] = all_cores
        quota = cgroup_cpu_quota()
        sample += (f"; all {all_cores} physical cores: 1 evaluation after 1 warm-up, {per_all:.3f} s/eval"
                   + (f" (the cgroup CPU quota is {quota:.0f} CPUs, so {all_cores} threads oversubscribe it"
                      + (": slower than the share" if per_all > per_eval else "") + ")" if quota else ""))
        out["cgroup_cpu_quota"] = quota
        torch.set_num_threads(threads)
    out["sample"] = sample + (f"; iters/s = 1 / (s_per_eval x {evals_per_iter:.3f} evals per iteration of the GPU "
                              f"run)")
    return per_eval, out


def grid_cost_s(prob_np, T, threads, reps=1):
    """Seconds per oracle closure evaluation of everything that scales with the state grid (the decoder_hr / integrate
    nearest interpolations, the misfit J_o over T x 69 x Hs x Ws and their backward) with the two networks replaced by
    trivial maps of the same shapes: the grid-dependent part of one evaluation, for extrapolating a 721x1440 CPU
    closure from a measured 128x256 one without a minutes-long oracle run."""
    import torch

    from oracle.da_ref import RefProblem

    torch.set_num_threads(threads)
    dec = lambda z: torch.cat([z, z, z[:, :5]], 1) * 0.01     # (1,32,128,256) -> (1,69,128,256)
    flow = (lambda x: torch.cat([x, x], 1)) if T > 1 else None
    rp = RefProblem(prob_np, dec, (128, 256), flow)
    z = torch.zeros(1, 32, 128, 256, requires_grad=True)

    def ev():
        z.grad = None
        rp.loss(z).backward()

    ev()
    t0 = time.time()
    for _ in range(reps):
        ev()
    return (time.time() - t0) / reps


def cpu_convergence_measured():
    """The measured full CPU convergence of config 2 (tools/cpu_convergence.py on the GPU box's host cores: the
    oracle restatement + torch.optim.LBFGS, Nit 10, weight grads on), committed under profiles/ (SURVEY §8 d)."""
    for rnd in ("r02",):
        try:
            with open(os.path.join(ROOT, "profiles", rnd, "cpu_convergence_c2.jsonl")) as f:
                rows = [json.loads(l) for l in f if l.strip().startswith("{")]
            r = [x for x in rows if x.get("cpu_convergence")][-1]
            return {"wall_clock_s": r["wall_clock_s"], "iters": r["iters"], "evals": r["evals"],
                    "threads": r["threads"], "source": f"profiles/{rnd}/cpu_convergence_c2.jsonl (tools/cpu_convergence.py)"}
        except (OSError, ValueError, KeyError, IndexError):
            continue
    return None


def sc4dvar_line(dev_index: int):
    """the sc4dvar mode (da_4dvar.py:1064-1177) on the same state (69ch 128x256): one Nit = 10 analysis
    of LBFGS(10, max_iter 5) over the B-matrix transform closure, timed after a warm-up analysis."""
    import torch

    from vaevar.problem import make_problem
    from vaevar.sc4dvar import BMatrix, Sc4dvarProblem, one_step_sc4dvar

    bm = BMatrix.from_npz(os.path.join(ROOT, "tests", "golden", "bq_info_lr.npz"))
    prob = Sc4dvarProblem(bm, make_problem(nch=69, Hs=128, Ws=256, T=1, seed=20250620), device=dev_index)
    one_step_sc4dvar(prob, nit=10, log_terms=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = one_step_sc4dvar(prob, nit=10, log_terms=False)
    dt = time.perf_counter() - t0
    return {"workload": "sc4dvar (static B: SHT correlation, balance, vertical EOFs, winds), 69ch 128x256, T=1, "
                        "Nit 10 x LBFGS max_iter 5", "iters_per_s": res["n_iter"] / dt, "wall_clock_s": dt,
            "iters": res["n_iter"], "evals": res["n_eval"], "ms_per_eval": 1e3 * dt / max(res["n_eval"], 1)}


def gemm_rocprof(key="gemm16_avg_us_per_call"):
    """Average rocprofv3 --kernel-trace --stats duration per fp16x3 GEMM call (main kernel + row scales + split-K
    fixup, tools/rocprof_gemm_summary.py) from the latest committed profile of `bench.py` itself."""
    for rnd in ("r06", "r05"):  # the latest profile of the default command (config 3); r01-r04 profiled config 2
        path = os.path.join(ROOT, "profiles", rnd, "gemm_rocprof_summary.json")
        try:
            with open(path) as f:
                return float(json.load(f)[key]), f"profiles/{rnd}/gemm_rocprof_summary.json"
        except (OSError, KeyError, ValueError, TypeError):
            continue
    return None, None


def gemm_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc passes of `bench.py` (FETCH_SIZE x2 +
    WRITE_SIZE with the gfx950 corrections, tools/pmc_traffic.py); PMC counters cannot be read live."""
    for rnd in ("r06", "r05"):
        path = os.path.join(ROOT, "profiles", rnd, "gemm_traffic.json")
        try:
            with open(path) as f:
                d = json.load(f)
            rec = d.get(kernel) or (d.get("k_gemm_h3") if kernel == "fp16x3" else None)
            return rec["hbm_bytes_per_launch"], f"profiles/{rnd}/gemm_traffic.json"
        except (OSError, KeyError, ValueError, TypeError):
            continue
    return None, None


PMC_CLASSES = {"fp16x3": ("k_gemm_h4", "k_gemm_h5"), "tower": ("k_mlp", "k_ablk"), "bf16x6": ("k_gemm_bs",)}


def pmc_mfma():
    """MFMA busy fraction and held clock per kernel class from the committed rocprofv3 --pmc passes
    (tools/pmc_mfma.py: SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE, SQ_INSTS_MFMA, SQ_BUSY_CYCLES, one pass each, over
    config-3 closures), weighted by each kernel's share of the class's time; PMC counters cannot be read live."""
    for rnd in ("r06",):
        path = os.path.join(ROOT, "profiles", rnd, "pmc_mfma.json")
        try:
            with open(path) as f:
                pm = json.load(f)
            ks = pm["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        out = {}
        for cls, pre in PMC_CLASSES.items():
            rows = [r for k, r in ks.items() if k.split("<")[0].split("::")[-1].startswith(pre) and "mfma_busy" in r]
            w = [r["duration_us_median"] * r["dispatches_per_pass"] for r in rows]
            if not rows or sum(w) <= 0:
                continue
            avg = lambda key: sum(r.get(key, 0.0) * x for r, x in zip(rows, w)) / sum(w)
            out[cls] = {"mfma_busy": avg("mfma_busy"), "mfma_busy_active_cus": avg("mfma_busy_active_cus"),
                        "mfma_rate_of_spec": avg("mfma_rate_of_spec"), "grbm_clock_ghz": avg("held_clock_ghz"),
                        "kernels": len(rows)}
        lg = pm.get("long_gemm", {})
        if lg:
            out["long_gemm"] = {k: {"shape": v.get("shape"), "duration_us": v.get("duration_us_median"),
                                    "held_clock_ghz": v.get("held_clock_ghz"), "mfma_busy": v.get("mfma_busy")}
                                for k, v in lg.items()}
        if out:
            out["source"] = (f"profiles/{rnd}/pmc_mfma.json (tools/pmc_mfma.py: one rocprofv3 --pmc pass per counter + "
                             "--kernel-trace over config-3 closures; busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 "
                             "x 1024 SIMDs), clock = GRBM_GUI_ACTIVE / 8 / duration; time-weighted over the class)")
            return out
    return None


def grid_roofline(prof):
    """Config 5's HBM roofline (SURVEY §8 d: 2.006 GB of state fields per evaluation at 721x1440, T = 2): the misfit
    class of an event-profiled analysis (k_misfit_grid, one pass over xb / yo / H / R per slot, and its network-grid
    adjoint k_misfit_net_bwd) — algorithmic bytes over the summed launch durations, against 8 TB/s — with the
    rocprofv3 average of k_misfit_grid and its PMC traffic from the committed profile."""
    pr, secs, evals = prof
    m = pr["misfit"]
    ach = m["bytes"] / max(m["ms"] * 1e-3, 1e-12) / 1e9
    rec = {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
           "kernel": "the config-5 state-grid misfit class: k_misfit_grid (x, J partials, the up-sampling adjoint of "
                     "H(x-yo)/R onto the network grid, the next flow input, in one pass) + k_misfit_net_bwd",
           "launches": m["launches"], "ms_per_eval": m["ms"] / max(evals, 1),
           "algorithmic_bytes_per_eval": m["bytes"] / max(evals, 1),
           "survey_bytes_per_eval": 2.006e9, "evals_profiled": evals,
           "floor_ms_per_eval_at_peak": 2.006e9 / (PEAK_HBM_GBS * 1e9) * 1e3}
    for rnd in ("r05",):
        try:
            with open(os.path.join(ROOT, "profiles", rnd, "grid_roofline.json")) as f:
                d = json.load(f)
            rec["rocprof"] = d.get("rocprof")
            rec["traffic"] = d.get("traffic_bytes_per_eval")
            rec["traffic_source"] = f"profiles/{rnd}/grid_roofline.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes)"
        except (OSError, ValueError):
            rec["traffic"] = None
    return rec


# ---------------------------------------------------------------------------------------------------------------
# per-rank workloads
class GpuAnalyses:
    """One rank's share: the HIP engine (libvaevar) on cuda:LOCAL_RANK; `batch` analyses per GPU run in lockstep
    over one batched closure (vaevar.da.one_step_da_batch) when batch > 1."""

    def __init__(self, cfg_id: int, rank: int, local: int, batch: int = 1):
        import torch

        from vaevar import config as C
        from vaevar.engine import DAProblem, LGUnet
        from vaevar.problem import make_problem

        self.torch = torch
        local = local % max(torch.cuda.device_count(), 1)  # ranks beyond the visible GPUs share them (tests)
        torch.cuda.set_device(local)
        self.dev = torch.device("cuda", local)
        self.cfg = CONFIGS[cfg_id]
        self.T, self.nit, self.batch = self.cfg["T"], self.cfg["nit"], batch
        self.dec = LGUnet(C.DECODER, batch, 1, device=local).load_synthetic()
        self.flow = None
        Hs, Ws = self.cfg.get("grid", (128, 256))
        probs = [make_problem(nch=69, Hs=Hs, Ws=Ws, T=self.T, seed=20250620 + rank * batch + b) for b in range(batch)]
        self.prob_np = probs[0]
        if self.T > 1:
            self.flow = LGUnet(C.FLOW, batch, self.T - 1, device=local).load_synthetic()
        self.prob = DAProblem(self.dec, probs if batch > 1 else probs[0], flow=self.flow, device=local)
        self.ctx = self.prob.ctx
        self._C, self._DAProblem, self._LGUnet, self._make_problem = C, DAProblem, LGUnet, make_problem
        self.rank, self.local = rank, local

    def analysis(self):
        """One step: the rank's `batch` analyses to convergence; (xa of every analysis, iterations, evaluations)."""
        from vaevar.da import one_step_da, one_step_da_batch

        if self.batch == 1:
            res = one_step_da(self.prob, nit=self.nit, log_terms=False)
            return res["xa"], res["n_iter"], res["n_eval"]
        res = one_step_da_batch(self.prob, nit=self.nit)
        return res["xa"], sum(res["n_iter"]), sum(res["n_eval"])

    def sync(self):
        self.torch.cuda.synchronize()

    def discarded(self):
        """speculative evaluations the L-BFGS mirror ran and discarded so far (vaevar/lbfgs.py; in the timed region)"""
        return getattr(self.prob, "n_discarded", 0)

    def rebind(self, cfg_id: int):
        """Re-bind this rank to BASELINE config `cfg_id`'s problems (T from CONFIGS, T - 1 flow slots, the same decoder);
        returns the analysis runner (used for the config-3 / 4 / 5 sub-records)."""
        cfg = CONFIGS[cfg_id]
        T = cfg["T"]
        flow = self._LGUnet(self._C.FLOW, self.batch, T - 1, device=self.local).load_synthetic() if T > 1 else None
        Hs, Ws = cfg.get("grid", (128, 256))
        ps = [self._make_problem(nch=69, Hs=Hs, Ws=Ws, T=T, seed=20250620 + self.rank * self.batch + b)
              for b in range(self.batch)]
        self.prob = self._DAProblem(self.dec, ps if self.batch > 1 else ps[0], flow=flow, device=self.local)
        self.prob_np = ps[0]
        self.flow, self.T, self.nit = flow, T, cfg["nit"]
        return self.analysis


class SelftestAnalyses:
    """--selftest: a stand-in analysis with known outputs (CPU, no GPU) that exercises the launch, the gloo/RCCL
    collectives, the gather and the JSON aggregation of this script (tests/test_bench_launch.py)."""

    def __init__(self, cfg_id: int, rank: int, local: int, batch: int = 1):
        import torch

        self.torch, self.rank, self.batch = torch, rank, batch
        self.T, self.nit = CONFIGS[cfg_id]["T"], CONFIGS[cfg_id]["nit"]

    def analysis(self):
        time.sleep(0.01 * (1 + self.rank))
        shape = (69, 128, 256) if self.batch == 1 else (self.batch, 69, 128, 256)
        return self.torch.full(shape, float(self.rank)), self.batch * (97 + self.rank), self.batch * (110 + self.rank)

    def sync(self):
        pass

    def discarded(self):
        return 0

    def rebind(self, cfg_id: int):
        return self.analysis


def thread_cpu():
    """{tid: (thread name, CPU seconds)} of this process's threads (/proc/self/task/*/stat utime + stime)."""
    tick = os.sysconf("SC_CLK_TCK") if hasattr(os, "sysconf") else 100
    out = {}
    try:
        for tid in os.listdir("/proc/self/task"):
            try:
                with open(f"/proc/self/task/{tid}/stat") as f:
                    s = f.read()
            except OSError:
                continue
            name = s[s.index("(") + 1:s.rindex(")")]
            fl = s[s.rindex(")") + 2:].split()
            out[tid] = (name, (int(fl[11]) + int(fl[12])) / tick)
    except OSError:
        pass
    return out


class ThreadSampler:
    """VV_THREAD_SAMPLE=1: every 20 ms, each thread's scheduler state, kernel wait channel and current syscall
    (/proc/self/task/*/{stat,wchan,syscall}), to name what a busy HIP-runtime thread is doing."""

    def __init__(self):
        import threading
        from collections import Counter, defaultdict

        self.stats = defaultdict(lambda: {"n": 0, "R": 0, "wchan": Counter(), "syscall": Counter()})
        self.stop = threading.Event()
        self.t = threading.Thread(target=self.run, daemon=True)

    def run(self):
        while not self.stop.wait(0.02):
            try:
                tids = os.listdir("/proc/self/task")
            except OSError:
                continue
            for tid in tids:
                try:
                    with open(f"/proc/self/task/{tid}/stat") as f:
                        st = f.read()
                    state = st[st.rindex(")") + 2]
                    with open(f"/proc/self/task/{tid}/wchan") as f:
                        wc = f.read().strip() or "0"
                    with open(f"/proc/self/task/{tid}/syscall") as f:
                        sc = f.read().split()[0]
                except (OSError, IndexError):
                    continue
                r = self.stats[tid]
                r["n"] += 1
                r["R"] += state == "R"
                r["wchan"][wc] += 1
                r["syscall"][sc] += 1

    def summary(self):
        out = {}
        for tid, r in self.stats.items():
            out[tid] = {"running_frac": round(r["R"] / max(r["n"], 1), 3), "wchan": r["wchan"].most_common(2),
                        "syscall": r["syscall"].most_common(2)}
        return out


def thread_cpu_delta(before, after, seconds, sampled=None):
    """Per-thread CPU over an interval, as fractions of one CPU, the busiest first (threads named by their comm and
    whether they are the main thread)."""
    main = str(os.getpid())
    rows = []
    for tid, (name, cs) in after.items():
        d = cs - before.get(tid, (name, 0.0))[1]
        if d > 0:
            rows.append({"thread": name + (" (main)" if tid == main else ""), "cpu_frac": round(d / max(seconds, 1e-9), 3)})
            if sampled and tid in sampled:
                rows[-1].update(sampled[tid])
    rows.sort(key=lambda r: -r["cpu_frac"])
    return rows[:8]


def timed_analyses(w, ensemble, steps, dev):
    """Barrier + sync, `steps` analyses (each gathered to rank 0 at N > 1), sync + barrier; max time over ranks."""
    ensemble.barrier()
    w.sync()
    sampler = ThreadSampler() if os.environ.get("VV_THREAD_SAMPLE") == "1" else None
    if sampler:
        sampler.t.start()
    th0 = thread_cpu()
    t0 = time.perf_counter()
    c0 = time.process_time()
    d0 = w.discarded()
    iters = evals = 0
    shapes = None
    for _ in range(steps):
        xa, it, ev = w.analysis()
        xs = ensemble.gather_analyses(xa)
        iters, evals = iters + it, evals + ev
        shapes = [tuple(x.shape) for x in xs] if xs is not None else None
    w.sync()
    ensemble.barrier()
    el = time.perf_counter() - t0
    cpu = time.process_time() - c0  # host CPU seconds of this rank (all its threads) over the timed region
    if sampler:
        sampler.stop.set()
        sampler.t.join()
    threads = thread_cpu_delta(th0, thread_cpu(), el, sampler.summary() if sampler else None)
    disc = w.discarded() - d0
    return (ensemble.reduce_scalar(el, "max", dev), ensemble.reduce_scalar(iters, "sum", dev),
            ensemble.reduce_scalar(evals, "sum", dev), shapes,
            (ensemble.reduce_scalar(cpu, "max", dev), ensemble.reduce_scalar(cpu, "sum", dev), threads),
            ensemble.reduce_scalar(disc, "sum", dev))


def sub_record(w, cid, ensemble, dev, size, batch, profile=False):
    """BASELINE config `cid` on this rank's GPU: a warm-up analysis (graph capture), then one timed analysis per rank
    with the RCCL gather, max time over ranks (the same timed-region rules as the main line); with `profile` (rank 0)
    one more analysis under the HIP-event profiler, outside the timed region."""
    run = w.rebind(cid)
    w.sync()
    run()
    ensemble.barrier()
    w.sync()
    t0 = time.perf_counter()
    d0 = w.discarded()
    xa, it, ev = run()
    xs = ensemble.gather_analyses(xa)
    w.sync()
    ensemble.barrier()
    t = ensemble.reduce_scalar(time.perf_counter() - t0, "max", dev)
    it = ensemble.reduce_scalar(it, "sum", dev)
    ev = ensemble.reduce_scalar(ev, "sum", dev)
    disc = ensemble.reduce_scalar(w.discarded() - d0, "sum", dev)
    prof = None
    if profile:
        w.ctx.profile_start()
        tp = time.perf_counter()
        _, _, ev_p = run()
        w.sync()
        prof = (w.ctx.profile_stop(), time.perf_counter() - tp, ev_p)
    return {"workload": CONFIGS[cid]["name"], "T": CONFIGS[cid]["T"], "n_gpus": size, "analyses_per_gpu": batch,
            "analyses": size * batch, "analyses_per_s": size * batch / t, "iters_per_s": it / t,
            "wall_clock_s": t, "iters": it, "evals": ev, "ms_per_eval": 1e3 * t * size / max(ev, 1),
            "discarded_speculative_evals": disc,
            "gathered": [list(x.shape) for x in xs] if xs is not None else None,
            "_prob_np": getattr(w, "prob_np", None), "_prof": prof,
            "timed_region": f"barrier + sync, one config-{cid} analysis per rank, RCCL gather of the analyses to rank 0, "
                            "sync + barrier; max over ranks"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed analyses per rank (each = Nit outer L-BFGS passes)")
    ap.add_argument("--warmup", type=int, default=1, help="untimed analyses per rank before the timed ones")
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-evals", type=int, default=None, help="timed CPU closure evaluations (default by config)")
    ap.add_argument("--no-profile", action="store_true", help="skip the HIP-event per-kernel-class profile")
    ap.add_argument("--no-config2", action="store_true", help="skip the config-2 (T=1, 3D-Var) line section")
    ap.add_argument("--no-config3", action="store_true", help="skip the config-3 (T=2) line section")
    ap.add_argument("--no-config4", action="store_true", help="skip the config-4 (T=6) line section")
    ap.add_argument("--no-config5", action="store_true", help="skip the config-5 (721x1440, T=2) line section")
    ap.add_argument("--no-exact-f32", action="store_true", help="skip the exact-f32 GEMM analysis")
    ap.add_argument("--no-sc4dvar", action="store_true", help="skip the sc4dvar (SURVEY §8 f4) section")
    ap.add_argument("--batch", type=int, default=1, help="independent analyses per GPU, evaluated in one batched "
                                                         "closure (B x 2048-row GEMMs)")
    ap.add_argument("--selftest", action="store_true", help="CPU stand-in analyses (tests the launch/aggregation)")
    args = ap.parse_args()

    world = os.environ.get("WORLD_SIZE")
    if world is None and args.gpus > 1:
        sys.exit(spawn(args.gpus, sys.argv[1:]))
    if world is not None and int(world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")

    import torch  # noqa: F401  (after the spawn: the parent of N ranks never touches the GPU)

    from vaevar import ensemble

    rank, size, local = ensemble.init("gloo" if args.selftest else None)
    Runner = SelftestAnalyses if args.selftest else GpuAnalyses
    w = Runner(args.config, rank, local, args.batch)
    dev = None if args.selftest else w.dev

    for _ in range(args.warmup):
        w.analysis()
    t_max, iters, evals, shapes, host_cpu, discarded = timed_analyses(w, ensemble, args.steps, dev)

    prof = None
    exact = None
    if not args.selftest:
        w.sync()
        if rank == 0 and not args.no_profile:
            # per-kernel-class HIP-event profile of one more analysis of the same problem (outside the timed region,
            # so the event records do not perturb it; the closure launches eagerly while events are recorded)
            w.ctx.profile_start()
            t0 = time.perf_counter()
            w.analysis()
            w.sync()
            prof = (w.ctx.profile_stop(), time.perf_counter() - t0)
        if rank == 0 and not args.no_exact_f32:
            old = w.ctx.gemm_math
            w.ctx.gemm_math = "f32"
            w.analysis()  # warm-up (graph capture) in this arithmetic
            t0 = time.perf_counter()
            _, it_f, ev_f = w.analysis()
            w.sync()
            exact = (it_f / (time.perf_counter() - t0), it_f, ev_f)
            w.ctx.gemm_math = old

    # J before / after of the main problem (not timed)
    j_info = None
    if not args.selftest:
        from vaevar.da import one_step_da, one_step_da_batch

        # analysis 0 of this rank
        if w.batch == 1:
            res = one_step_da(w.prob, nit=w.nit, log_terms=False)
        else:
            res = one_step_da_batch(w.prob, nit=w.nit)
        j_end = w.prob.closure_batch(res["z"], None)
        j_0 = w.prob.closure_batch(torch.zeros_like(res["z"]), None)
        j_info = (float(j_0[0][0] + j_0[1][0]), float(j_end[0][0] + j_end[1][0]))

    # the other BASELINE configs (2: T = 1, 3: T = 2, 4: T = 6, 5: 721x1440, T = 2) as sub-records of every line, each
    # timed on its own after the main region (warm-up analysis for the graph capture, then one timed analysis per rank
    # + the gather); config 5 also gets an event-profiled repeat on rank 0 for its HBM roofline (the grid kernels)
    main_prob_np = getattr(w, "prob_np", None)
    subs = {}
    for cid, skip in ((2, args.no_config2), (3, args.no_config3), (4, args.no_config4), (5, args.no_config5)):
        if skip or args.config == cid:
            continue
        subs[cid] = sub_record(w, cid, ensemble, dev, size, args.batch,
                               profile=cid == 5 and rank == 0 and not args.selftest and not args.no_profile)

    sc4 = None
    if rank == 0 and not args.selftest and not args.no_sc4dvar:
        sc4 = sc4dvar_line(w.local)

    if rank != 0:
        ensemble.barrier()
        return
    cfg = CONFIGS[args.config]
    per_analysis = t_max / max(args.steps, 1)
    out = {
        "metric": METRIC,
        "value": iters / t_max,
        "unit": "L-BFGS iters/s",
        "n_gpus": size,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1e3 * per_analysis,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32 (GEMMs: fp16x3 split, fp32-level error)",
        "data": "synthetic (counter-hash RNG weights and observations; the reference ships no checkpoints)",
        "config": {"workload": cfg["name"], "analyses_per_gpu": args.batch, "T": cfg["T"], "nit": cfg["nit"],
                   "parallelism": f"ensemble: {size * args.batch} independent analyses, {args.batch} per GPU "
                                  f"({'one batched closure' if args.batch > 1 else 'one closure each'}), RCCL gather "
                                  "of xa per step"},
        "wall_clock_to_convergence_s": per_analysis,
        "iters": iters,
        "evals": evals,
        "discarded_speculative_evals": discarded,
        "iters_per_analysis": iters / (size * args.steps * args.batch),
        "evals_per_s": evals / t_max,
        "ms_per_eval": 1e3 * t_max * size / max(evals, 1),
        "analyses_per_s": size * args.batch * args.steps / t_max,
        "gathered": [list(s) for s in shapes] if shapes else None,
        # host CPU the ranks' Python drivers (L-BFGS mirror, launches, syncs) use in the timed region: at 8 ranks on
        # one node, 8 x cpu_frac_max_rank CPUs against the box's CPU quota
        "host_cpu": {"cpu_s_max_rank": host_cpu[0], "cpu_s_all_ranks": host_cpu[1],
                     "cpu_frac_max_rank": host_cpu[0] / max(t_max, 1e-12),
                     "cpus_busy_all_ranks": host_cpu[1] / max(t_max, 1e-12),
                     "threads_rank0": host_cpu[2],
                     "host_wait": (w.ctx.get_tuning("host_wait") if not args.selftest else None)},
        "timed_region": f"barrier + sync, {args.steps} step(s) of {args.batch} analyses per rank (z = 0, Nit = {cfg['nit']} outer lbfgs.step "
                        "calls, the analysis decode, at N > 1 the RCCL gather of every analysis to rank 0), sync + "
                        "barrier; max over ranks. The per-outer-pass logging evaluation cal_loss and WRMSE/Bias "
                        "(da_4dvar.py:1256-1269, SURVEY §8 a3; 1 forward per pass) is not run in it",
    }
    out["headline_config"] = (f"BASELINE config {args.config} (" + {2: "vae4dvar, da_win=1: 3D-Var with the full VAE "
                              "decoder, the da_4dvar_script.sh default window", 3: "vae4dvar, da_win=2: 4D-Var with the "
                              "flow stand-in, 69ch 128x256: the config the metric names", 4: "vae4dvar, da_win=6",
                              5: "vae4dvar, da_win=2 at 721x1440"}[args.config]
                              + "); `value` measures this config. The 3D-Var (da_win = 1) figure is `value_3dvar` "
                              "(the config2 sub-record, r01-r04's headline)")
    out["discarded_speculative_evals_note"] = (
        "evaluations the L-BFGS mirror started speculatively (the line search's first, queued before gtd is known) and "
        "discarded where the reference stops on gtd > -tolerance_change: not in `evals`, their time is in the timed region")
    if 3 in subs:
        out["value_4dvar"] = subs[3]["iters_per_s"]
    elif args.config == 3:
        out["value_4dvar"] = out["value"]
    if 2 in subs:
        out["value_3dvar"] = subs[2]["iters_per_s"]
    elif args.config == 2:
        out["value_3dvar"] = out["value"]
    if j_info:
        out["J_start"], out["J_final"] = j_info
    if exact:
        out["exact_f32"] = {"value": exact[0], "unit": "L-BFGS iters/s", "iters": exact[1], "evals": exact[2],
                            "note": "one analysis with every GEMM on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32), "
                                    "rank 0, timed on its own"}
    for cid, rec in subs.items():
        out[f"config{cid}"] = rec
    if sc4:
        out["sc4dvar"] = sc4
    if prof is not None:
        pr, prof_s = prof
        math = w.ctx.gemm_math
        g16, g6 = pr["gemm16"], pr["gemm"]
        allg = {k: g16[k] + g6[k] for k in ("ms", "flops", "bytes", "launches")}
        if math == "split16":
            dom, peak, tkey = g16, PEAK_SPLIT16_TFLOPS, "fp16x3"
            kname = ("the fp16x3 GEMM class: k_gemm_h4 / k_gemm_h5 (tiles 48 / 49, LDS-DMA on pre-split planes) / k_gemm_h3(m) with "
                     "their split-K fixups and the A split / row-scale passes: every GEMM launch that ran an fp16x3 "
                     "kernel in a HIP-event-profiled repeat of one timed analysis")
            desc = ("fp16x3 split: fp32 operands scaled per row by 2^e and split into 2 fp16 planes, 3 "
                    "fp16 MFMA products (v_mfma_f32_16x16x32_f16) per fp32 product; peak = 2.5 PF fp16 dense / 3")
        elif math == "split":
            dom, peak, tkey = allg, PEAK_SPLIT_TFLOPS, "all"
            kname = "every GEMM launch of a HIP-event-profiled repeat of one timed analysis"
            desc = "bf16x6 split (6 v_mfma_f32_32x32x16_bf16 products per fp32 product; peak = 2.5 PF / 6)"
        else:
            dom, peak, tkey = allg, PEAK_F32_TFLOPS, "all"
            kname = "every GEMM launch (k_gemm_nt) of a HIP-event-profiled repeat of one timed analysis"
            desc = "exact f32 MFMA (v_mfma_f32_32x32x2_f32; peak 157.3 TF)"
        ach = dom["flops"] / max(dom["ms"] * 1e-3, 1e-12) / 1e12
        n = max(dom["launches"], 1)
        traffic, tsrc = gemm_traffic(tkey)
        out["roofline"] = {"bound": "mfma", "achieved": ach, "peak": peak, "unit": "TFLOP/s", "frac": ach / peak,
                           "traffic": traffic, "kernel": kname, "gemm_math": desc,
                           "launches": dom["launches"], "avg_launch_us": 1e3 * dom["ms"] / n,
                           "flops_per_launch": dom["flops"] / n, "algorithmic_bytes_per_launch": dom["bytes"] / n,
                           "share_of_gemm_time": dom["ms"] / max(allg["ms"], 1e-12),
                           "traffic_source": (f"{tsrc}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py "
                                              "(tools/pmc_traffic.py)") if tsrc else None}
        if math == "split16":
            us, src = gemm_rocprof()
            if us:
                # the same flops per call over the per-kernel rocprof durations (no inter-kernel gaps inside a call)
                out["roofline"]["rocprof"] = {"avg_call_us": us, "achieved": dom["flops"] / n / (us * 1e-6) / 1e12,
                                              "frac": dom["flops"] / n / (us * 1e-6) / 1e12 / peak,
                                              "source": f"{src} (rocprofv3 --kernel-trace --stats of bench.py)"}
            pm = pmc_mfma()
            if pm:
                if "fp16x3" in pm:
                    # MFMA-pipe busy cycles over the class's dispatches: of their active cycles (GRBM_GUI_ACTIVE, which
                    # over-counts dispatches this short, so a lower bound) and of the 2.4 GHz spec rate
                    out["roofline"]["mfma_busy"] = pm["fp16x3"]["mfma_busy"]
                    out["roofline"]["mfma_busy_active_cus"] = pm["fp16x3"]["mfma_busy_active_cus"]
                    out["roofline"]["mfma_rate_of_spec"] = pm["fp16x3"]["mfma_rate_of_spec"]
                lg = pm.get("long_gemm", {}).get("tile48")
                if lg and lg.get("held_clock_ghz"):
                    # the clock the chip holds under the tile-48 main loop (a ~2 ms dispatch of the same kernel: the
                    # GRBM clock is exact there), the fp16 peak at that clock and the class's fraction of it
                    out["roofline"]["held_clock_ghz"] = lg["held_clock_ghz"]
                    out["roofline"]["peak_at_held_clock"] = peak * lg["held_clock_ghz"] / 2.4
                    out["roofline"]["frac_of_held_clock_peak"] = ach / out["roofline"]["peak_at_held_clock"]
                out["roofline"]["pmc"] = pm
            # the other GEMM class (bf16x6, short-K Swin-tower linears) against its own peak
            g6a = g6["flops"] / max(g6["ms"] * 1e-3, 1e-12) / 1e12
            out["roofline"]["bf16x6_class"] = {"achieved": g6a, "peak": PEAK_SPLIT_TFLOPS,
                                               "frac": g6a / PEAK_SPLIT_TFLOPS, "launches": g6["launches"]}
        busy = sum(v["ms"] for v in pr.values())
        out["kernel_time_ms"] = {k: round(v["ms"], 3) for k, v in pr.items()}
        out["kernel_launches"] = {k: v["launches"] for k, v in pr.items()}
        out["profiled_analysis_s"] = prof_s
        # kernel busy time of the eager, event-profiled repeat over that repeat's own wall time
        out["profiled_busy_frac"] = busy / (1e3 * prof_s)
        fe = FLOPS_PER_EVAL.get(cfg["T"])
        if fe:
            # whole-evaluation roofline (SURVEY §8 d) against the peak of the arithmetic actually used
            ms_eval = 1e3 * t_max * size / max(evals, 1)
            pk = {"split16": PEAK_SPLIT16_TFLOPS, "split": PEAK_SPLIT_TFLOPS}.get(math, PEAK_F32_TFLOPS)
            out["eval_roofline"] = {"achieved_tflops": fe / (ms_eval * 1e-3) / 1e12, "peak": pk,
                                    "frac": fe / (ms_eval * 1e-3) / 1e12 / pk}
    if size == 1 and not args.no_cpu_baseline and not args.selftest:
        # CPU baselines (rank 0, N = 1): the main config (if the oracle closure finishes in seconds there: T <= 2 on the
        # 128x256 grid) and the config-3 sub-record at the box's thread share; config 4 extrapolated from both
        pc, ncpu, share = physical_cores()
        threads = min(pc, share) if share else pc
        note = (f"{pc} physical cores on the {ncpu} CPUs of this process's affinity"
                + (f", OMP_NUM_THREADS share {share}" if share else ""))
        per_eval_T = {}
        if cfg["T"] <= 2 and "grid" not in cfg:
            evals_per_iter = evals / max(iters, 1)
            n_cpu = args.cpu_evals or (3 if cfg["T"] == 1 else 2)
            per_eval, cb = cpu_baseline(main_prob_np, cfg["T"], evals_per_iter, evals / max(args.steps * args.batch, 1),
                                        n_cpu, threads, note, all_cores=pc if args.batch == 1 else None)
            per_eval_T[cfg["T"]] = per_eval
            out["cpu_baseline"] = cb
            out["cpu_wall_clock_to_convergence_s_extrapolated"] = cb.pop("wall_clock_to_convergence_s_extrapolated")
            out["speedup_vs_cpu"] = out["value"] / cb["value"]
            if "value_all_cores" in cb and cb["value_all_cores"] > cb["value"]:
                # only a faster all-cores run is a baseline; an oversubscribed (slower) one would inflate the ratio
                out["speedup_vs_cpu_all_cores"] = out["value"] / cb["value_all_cores"]
            meas = cpu_convergence_measured() if args.config == 2 and args.batch == 1 else None
            if meas:
                out["cpu_convergence_measured"] = meas
                out["wall_clock_speedup_vs_cpu_measured"] = meas["wall_clock_s"] / per_analysis
        for cid, rec in subs.items():
            Tc = CONFIGS[cid]["T"]
            if Tc > 2 or "grid" in CONFIGS[cid] or rec.get("_prob_np") is None:
                continue
            epi = rec["evals"] / max(rec["iters"], 1)
            per_eval, cb = cpu_baseline(rec["_prob_np"], Tc, epi, rec["evals"] / max(rec["analyses"], 1),
                                        args.cpu_evals or (3 if Tc == 1 else 2), threads, note)
            per_eval_T[Tc] = per_eval
            if cid == 2 and args.batch == 1:
                meas = cpu_convergence_measured()
                if meas:
                    rec["cpu_convergence_measured"] = meas
                    rec["wall_clock_speedup_vs_cpu_measured"] = meas["wall_clock_s"] / rec["wall_clock_s"] * rec["analyses"]
            rec["cpu_baseline"] = cb
            rec["speedup_vs_cpu"] = rec["iters_per_s"] / cb["value"]
            rec["wall_clock_speedup_vs_cpu"] = (cb["wall_clock_to_convergence_s_extrapolated"] * rec["analyses"]
                                                / rec["wall_clock_s"])
        if 2 in per_eval_T and 5 in subs and subs[5].get("_prob_np") is not None:
            # config 5 (721x1440, T = 2): the measured 128x256 T = 2 closure + the measured grid-dependent part at
            # 721x1440 minus the same at 128x256 (grid_cost_s); one full oracle evaluation there takes minutes
            rec = subs[5]
            from vaevar.problem import make_problem

            small = make_problem(nch=69, Hs=128, Ws=256, T=2, seed=20250620)
            g_big, g_small = grid_cost_s(rec["_prob_np"], 2, threads), grid_cost_s(small, 2, threads)
            s5 = per_eval_T[2] + g_big - g_small
            epi = rec["evals"] / max(rec["iters"], 1)
            rec["cpu_baseline"] = {"value": 1.0 / (s5 * epi), "unit": "L-BFGS iters/s", "cores": threads,
                                   "kind": "port (extrapolated)", "s_per_eval": s5,
                                   "wall_clock_to_convergence_s_extrapolated": s5 * rec["evals"] / max(rec["analyses"], 1),
                                   "sample": f"not run at 721x1440: s/eval = s(T=2, 128x256, measured above) + grid "
                                             f"part at 721x1440 - grid part at 128x256 = {per_eval_T[2]:.3f} + "
                                             f"{g_big:.3f} - {g_small:.3f} (grid part: the oracle closure's nearest "
                                             f"interpolations and misfit with the networks replaced by trivial maps, "
                                             f"1 evaluation after 1 warm-up each, {threads} threads)"}
            rec["speedup_vs_cpu"] = rec["iters_per_s"] / rec["cpu_baseline"]["value"]
        if 1 in per_eval_T and 2 in per_eval_T and 4 in subs:
            # per evaluation: decoder (T = 1) + (T - 1) flow steps, each step's cost = s(T=2) - s(T=1)
            a, b = per_eval_T[1], per_eval_T[2] - per_eval_T[1]
            rec = subs[4]
            s6 = a + 5 * b
            epi = rec["evals"] / max(rec["iters"], 1)
            rec["cpu_baseline"] = {"value": 1.0 / (s6 * epi), "unit": "L-BFGS iters/s", "cores": threads,
                                   "kind": "port (extrapolated)", "s_per_eval": s6,
                                   "wall_clock_to_convergence_s_extrapolated": s6 * rec["evals"] / max(rec["analyses"], 1),
                                   "sample": f"not run at T=6: s/eval(T=6) = s(T=1) + 5 x (s(T=2) - s(T=1)) = {a:.3f} + "
                                             f"5 x {b:.3f} from the two measured oracle closures above (weight grads "
                                             f"on, {threads} threads)"}
            rec["speedup_vs_cpu"] = rec["iters_per_s"] / rec["cpu_baseline"]["value"]
    if 5 in subs and subs[5].get("_prof") is not None:
        subs[5]["roofline_hbm"] = grid_roofline(subs[5]["_prof"])
    for rec in subs.values():
        rec.pop("_prob_np", None)
        rec.pop("_prof", None)
    print(json.dumps(out), flush=True)
    ensemble.barrier()


if __name__ == "__main__":
    main()
