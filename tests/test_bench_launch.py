"""CPU: bench.py's multi-rank path as the driver runs it — `bench.py --gpus 2` spawns its own two ranks (no
WORLD_SIZE), they meet over gloo, every rank's analysis is gathered to rank 0, time is the max over ranks and
iterations the sum — with the --selftest stand-in analysis (known outputs) in place of the GPU engine; and (GPU)
the same launch over the real engine."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _run(*extra, env=None):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + list(extra)
    e = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=e)
    return p


def test_bench_spawns_its_ranks():
    p = _run("--gpus", "2", "--selftest", "--steps", "2", "--warmup", "1")
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout  # one JSON line, from rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    # stand-in analysis of rank r: 97 + r iterations, 110 + r evaluations; 2 steps each
    assert out["iters"] == 2 * (97 + 98) and out["evals"] == 2 * (110 + 111)
    assert out["gathered"] == [[69, 128, 256], [69, 128, 256]]
    assert out["value"] == out["iters"] / (out["ms_per_step"] * 1e-3 * out["steps"])
    assert out["config"]["T"] == 2  # the default workload is config 3, the metric's 4D-Var config (r05)
    for cid in (2, 4, 5):  # every BASELINE config other than the main one is a sub-record of the line
        c = out[f"config{cid}"]
        assert c["n_gpus"] == 2 and c["gathered"] == [[69, 128, 256], [69, 128, 256]] and c["iters"] == 97 + 98
    for k in ("metric", "unit", "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out


def test_bench_spawns_eight_ranks():
    """Config 4's layout (8 analyses, one per GPU of a node) on CPU: `bench.py --gpus 8` spawns 8 ranks over gloo;
    rank 0 receives 8 (69, 128, 256) analyses per step, the iterations are summed over the ranks, the time is the
    slowest rank's (the stand-in analysis of rank r sleeps 10 (1 + r) ms, so rank 7 sets it), and the host-CPU record
    covers all ranks."""
    p = _run("--gpus", "8", "--selftest", "--steps", "2", "--warmup", "1", env={"OMP_NUM_THREADS": "1"})
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8
    assert out["iters"] == 2 * sum(97 + r for r in range(8)) and out["evals"] == 2 * sum(110 + r for r in range(8))
    assert out["gathered"] == [[69, 128, 256]] * 8
    assert out["ms_per_step"] >= 80.0  # max over ranks: rank 7's 80 ms stand-in
    assert out["value"] == out["iters"] / (out["ms_per_step"] * 1e-3 * out["steps"])
    c4 = out["config4"]
    assert c4["n_gpus"] == 8 and c4["analyses"] == 8 and c4["gathered"] == [[69, 128, 256]] * 8
    assert c4["iters"] == sum(97 + r for r in range(8)) and c4["wall_clock_s"] >= 0.08
    hc = out["host_cpu"]
    assert hc["cpu_s_all_ranks"] >= hc["cpu_s_max_rank"] > 0


def test_bench_world_size_must_match():
    p = _run("--gpus", "2", "--selftest", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0 and "WORLD_SIZE" in p.stderr


@pytest.mark.gpu
def test_bench_two_ranks_product_path():
    """The product path with two ranks: `bench.py --gpus 2` spawns two processes that each run a full config-3
    analysis (the default workload: T = 2) on libvaevar (here both on the box's one GPU, over gloo since RCCL refuses
    two ranks per device), gather both analyses to rank 0, take the max time and sum the iterations (G13: J falls to
    0.41 of its start over the budget)."""
    p = _run("--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--no-profile", "--no-exact-f32",
             "--no-config2", "--no-config4", "--no-config5", "--no-sc4dvar", env={"VAEVAR_DIST_BACKEND": "gloo"})
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    print({k: out[k] for k in ("n_gpus", "iters", "evals", "value", "gathered", "J_start", "J_final")})
    assert out["n_gpus"] == 2 and out["gathered"] == [[69, 128, 256], [69, 128, 256]]
    assert 150 <= out["iters"] <= 200 and out["J_final"] < 0.5 * out["J_start"]
