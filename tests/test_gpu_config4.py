"""BASELINE config 4's 6-step assimilation window (T = 6: the decoder plus five integrate steps of the flow model
inside the loss, da_4dvar.py:1183-1208, :666-681) on the GPU through the C-ABI.

  G12 (tests/golden/g12_tiny_4dvar_t6.npz, oracle/make_golden.py): the reference's own networks_old.LGUnet_all tiny
      decoder + tiny flow and torch.optim.LBFGS: one closure, and one outer pass (Nit = 1) with every line search's
      (t, evals) recorded for the fixed-step replay.
  full size: the 216M-parameter decoder and flow stand-in at 69x128x256, T = 6 (5 flow slots of saved activations),
      one closure against the oracle restatement on the host CPU (pinned to the reference by G12/G5b/G6).
Tolerances: one evaluation rel <= 1e-5 (tiny) / 1e-4 (full); after L-BFGS iterations J and xa
rel <= 1e-3. "rel" = max|a-b| / max|b|.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLD, check, note

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def _tiny_t6():
    from vaevar import config as C
    from vaevar.engine import DAProblem, LGUnet
    from vaevar.problem import make_problem

    dec = LGUnet(C.TINY, 1, 1).load_synthetic()
    flow = LGUnet(C.TINY_FLOW, 1, 5).load_synthetic()
    p = make_problem(nch=4, Hs=32, Ws=64, T=6, seed=779, obs_frac=0.1)
    return DAProblem(dec, p, flow=flow), p


def test_tiny_t6_closure_g12():
    g = np.load(os.path.join(GOLD, "g12_tiny_4dvar_t6.npz"))
    prob, _ = _tiny_t6()
    z = torch.from_numpy(g["z"]).cuda()
    grad = torch.empty_like(z)
    jb, jo = prob.closure(z, grad)
    e = (abs(jb - g["J_b"]) / g["J_b"], abs(jo - g["J_o"]) / g["J_o"], rel(grad.cpu(), g["grad"]))
    print(f"G12 tiny 4D-Var T=6 closure: J_b {e[0]:.2e} J_o {e[1]:.2e} grad {e[2]:.2e}")
    check("G12 J_b", e[0], 5e-8)
    check("G12 J_o", e[1], 5e-7)
    check("G12 grad", e[2], 1e-5)
    # the trajectory x_t of the five integrate steps is kept per slot
    assert prob.trajectory().shape == (6, 4, 32, 64)


@pytest.mark.parametrize("mode", ["free", "replay"])
def test_tiny_t6_lbfgs_g12(mode):
    """One outer L-BFGS pass (10 iterations) at T = 6 against the reference modules + torch.optim.LBFGS."""
    from vaevar.da import one_step_da

    g = np.load(os.path.join(GOLD, "g12_tiny_4dvar_t6.npz"))
    prob, _ = _tiny_t6()
    replay = [(float(t), int(n)) for t, n in zip(g["ls_t"], g["ls_evals"])] if mode == "replay" else None
    res = one_step_da(prob, nit=1, replay=replay)
    J = np.array([a + b for a, b in res["J"]])
    Jr = g["J"].sum(1)
    xa = res["xa"].cpu().numpy()
    e_j = float(np.abs(J - Jr).max() / np.abs(Jr).max())
    e_x = float(np.linalg.norm(xa - g["xa"]) / np.linalg.norm(g["xa"]))
    print(f"G12 T=6 L-BFGS {mode}: J {J.tolist()} vs {Jr.tolist()} (rel {e_j:.1e}), xa rel-L2 {e_x:.1e}, "
          f"evals {res['n_eval']} (ref {int(g['n_eval'])}), iters {res['n_iter']} (ref {int(g['n_iter'])})")
    check(f"G12 T=6 L-BFGS {mode} J per pass (max)", e_j, 2e-5)
    check(f"G12 T=6 L-BFGS {mode} xa rel-L2", e_x, 2e-6)
    if mode == "free":
        assert res["n_iter"] == int(g["n_iter"])


def test_full_t6_closure_vs_oracle():
    """Config-4 shapes: full decoder + flow stand-in, 69x128x256, T = 6, one closure vs the oracle on CPU."""
    from oracle.da_ref import oracle_problem
    from oracle.lgunet_ref import synth_params
    from vaevar import config as C
    from vaevar.engine import DAProblem, LGUnet
    from vaevar.problem import make_problem
    from vaevar.synth import smooth_field

    p = make_problem(nch=69, Hs=128, Ws=256, T=6, seed=20250624, obs_frac=0.02)
    dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
    flow = LGUnet(C.FLOW, 1, 5).load_synthetic()
    prob = DAProblem(dec, p, flow=flow)
    z = torch.from_numpy(0.3 * smooth_field(1202, (1, 32, 128, 256)))
    g = torch.empty(1, 32, 128, 256, device="cuda")
    jb, jo = prob.closure(z.cuda(), g)
    xs = prob.trajectory().cpu()
    torch.set_num_threads(16)
    ro = oracle_problem(p, synth_params(C.DECODER), C.DECODER, synth_params(C.FLOW), C.FLOW)
    zr = z.clone().requires_grad_(True)
    rb, rob = ro.loss_terms(zr)
    (rb + rob).backward()
    with torch.no_grad():
        xr = ro.trajectory(z)
    e_j = abs(jo - float(rob)) / abs(float(rob))
    e_g = rel(g.cpu(), zr.grad)
    e_x = [rel(xs[t], xr[t]) for t in range(6)]
    print(f"config-4 T=6 closure: J_o {jo:.6e} (oracle {float(rob):.6e}, rel {e_j:.2e}), grad rel {e_g:.2e}, "
          f"x_t rel {['%.1e' % v for v in e_x]}")
    check("config-4 T=6 closure J_o", e_j, 1e-7)
    check("config-4 T=6 closure dJ/dz", e_g, 2e-5)
    check("config-4 T=6 closure x_t (max over t)", max(e_x), 1e-6)


@pytest.mark.parametrize("mode", ["free", "replay"])
def test_config4_trajectory_g16(mode):
    """BASELINE config 4's window at full size (216M-parameter decoder + the flow stand-in, T = 6: five integrate steps
    in the loss, 69x128x256) over the bench's full budget, Nit = 10 outer passes (r05; 97 L-BFGS iterations, 111
    evaluations; r04: Nit 3) against G16: the reference's networks_old modules + torch.optim.LBFGS on CPU
    (oracle/make_golden.py --g16, da_4dvar.py:1183-1208, :1238-1299). Bounds: SURVEY c6's 1e-3 on J, or twice the
    reference's own summation-order drift on this trajectory where that is larger (g16_sensitivity.npz: the same run
    on 4 threads, free-running and replayed along G16's line searches, oracle/g10_sensitivity.py --case g16); xa
    rel-L2 1e-3 free (r06: ~30x what the HIP path achieves, profiles/r06/parity_margins.jsonl; c6: 1e-2), 2e-4
    replayed, |xa-xb|^2 2e-3 free and replayed."""
    from vaevar import config as C
    from vaevar.da import one_step_da
    from vaevar.engine import DAProblem, LGUnet
    from vaevar.problem import make_problem

    g = np.load(os.path.join(GOLD, "g16_config4_trajectory.npz"))
    dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
    flow = LGUnet(C.FLOW, 1, 5).load_synthetic()
    prob_np = make_problem(nch=69, Hs=128, Ws=256, T=6, seed=20250620)
    prob = DAProblem(dec, prob_np, flow=flow)
    replay = [(float(t), int(n)) for t, n in zip(g["ls_t"], g["ls_evals"])] if mode == "replay" else None
    res = one_step_da(prob, nit=int(g["nit"]), replay=replay)
    J = np.array([a + b for a, b in res["J"]])
    Jr = g["J"].sum(1)
    e_pass = np.abs(J - Jr) / np.abs(Jr)
    xa = res["xa"].cpu().numpy().reshape(-1).astype(np.float64)
    e_x = float(np.linalg.norm(xa[g["idx_xa"]] - g["xa_sample"]) / np.linalg.norm(g["xa_sample"]))
    dx = float(((xa - prob_np["xb"].reshape(-1).astype(np.float64)) ** 2).sum())
    e_dx = abs(dx - float(g["dxa_sumsq"])) / float(g["dxa_sumsq"])
    sens = np.load(os.path.join(GOLD, "g16_sensitivity.npz"))
    print(f"G16 config 4 ({mode}): J per pass rel {['%.1e' % v for v in e_pass]}; xa rel-L2 {e_x:.1e}; "
          f"|xa-xb|^2 rel {e_dx:.1e}; iters {res['n_iter']} (ref {int(g['n_iter'])}), evals {res['n_eval']} "
          f"(ref {int(g['n_eval'])}); reference drift free {float(sens['free_rel'][-1]):.1e} replay "
          f"{float(sens['replay_rel'].max()):.1e}")
    for i, v in enumerate(e_pass):
        note(f"G16 {mode} J rel, pass {i}", v)
    if mode == "replay":
        check("G16 replay J per pass (max)", e_pass.max(), max(1e-3, 2 * float(sens["replay_rel"].max())))
        check("G16 replay xa rel-L2", e_x, 2e-4)  # r06: 1e-3 -> 2e-4 (achieved 2.7e-5, parity_margins.jsonl)
        check("G16 replay |xa-xb|^2", e_dx, 2e-3)
    else:
        check("G16 free final J", e_pass[-1], max(1e-3, 2 * float(sens["free_rel"][-1])))
        check("G16 free xa rel-L2", e_x, 1e-3)
        check("G16 free |xa-xb|^2", e_dx, 2e-3)
