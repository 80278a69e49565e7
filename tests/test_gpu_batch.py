"""B independent analyses per GPU in one launch sequence ("batching several analyses per GPU"):
the decoder / flow GEMMs run on B x tokens rows, the misfit per analysis, each analysis with its own L-BFGS.

  tiny networks: no GEMM of the tiny config splits K, so every output element is summed in the same order at
      B = 1 and B = 2 -> the batched closure and the batched L-BFGS trajectories equal B = 1 runs BIT FOR BIT.
  full networks: at B = 1 the chip is filled by splitting K of the 2048-row LG GEMMs; at B > 1 the rows fill it and
      the split is dropped, so results differ at fp32 rounding level (bounded here at ~5x the measured difference, profiles/r06/parity_margins.jsonl).
"""
import numpy as np
import pytest
import torch

from conftest import check, check_bitwise

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def _tiny(B, T):
    from vaevar import config as C
    from vaevar.engine import LGUnet

    dec = LGUnet(C.TINY, B, 1).load_synthetic()
    flow = LGUnet(C.TINY_FLOW, B, T - 1).load_synthetic() if T > 1 else None
    return dec, flow


def _tiny_probs(T):
    from vaevar.problem import make_problem

    return [make_problem(nch=4, Hs=32, Ws=64, T=T, seed=780 + b, obs_frac=0.1) for b in range(2)]


@pytest.mark.parametrize("T", [1, 3])
def test_tiny_batch2_closure_bitwise(T):
    from vaevar.engine import DAProblem
    from vaevar.synth import smooth_field

    probs = _tiny_probs(T)
    z = torch.from_numpy(0.3 * smooth_field(1301, (2, 4, 32, 64), sigma=2.0)).cuda()
    dec2, flow2 = _tiny(2, T)
    pb = DAProblem(dec2, probs, flow=flow2)
    g2 = torch.empty_like(z)
    jb2, jo2 = pb.closure_batch(z, g2)
    x2 = pb.trajectory()
    assert x2.shape == (2, T, 4, 32, 64)
    dec1, flow1 = _tiny(1, T)
    for b in range(2):
        p1 = DAProblem(dec1, probs[b], flow=flow1)
        g1 = torch.empty(1, 4, 32, 64, device="cuda")
        jb1, jo1 = p1.closure(z[b:b + 1].contiguous(), g1)
        check_bitwise(f"B=2 vs B=1 T={T} analysis {b} J", (jb1, jo1), (jb2[b], jo2[b]))
        check_bitwise(f"B=2 vs B=1 T={T} analysis {b} dJ/dz", g1[0], g2[b])
        check_bitwise(f"B=2 vs B=1 T={T} analysis {b} x_t", p1.trajectory(), x2[b])


def test_tiny_batch2_lbfgs_bitwise():
    """Two analyses advanced in lockstep over the batched closure follow exactly the trajectories they follow alone."""
    from vaevar.da import one_step_da, one_step_da_batch
    from vaevar.engine import DAProblem

    probs = _tiny_probs(2)
    dec2, flow2 = _tiny(2, 2)
    res = one_step_da_batch(DAProblem(dec2, probs, flow=flow2), nit=2)
    dec1, flow1 = _tiny(1, 2)
    for b in range(2):
        r1 = one_step_da(DAProblem(dec1, probs[b], flow=flow1), nit=2, log_terms=False)
        assert r1["n_iter"] == res["n_iter"][b] and r1["n_eval"] == res["n_eval"][b]
        check_bitwise(f"batched L-BFGS analysis {b} xa", r1["xa"], res["xa"][b])
    assert res["batched_evals"] == max(res["n_eval"])


def test_full_batch2_closure_vs_single():
    """Full decoder + flow stand-in, 69x128x256, T = 2, B = 2 vs two B = 1 closures."""
    from vaevar import config as C
    from vaevar.engine import DAProblem, LGUnet
    from vaevar.problem import make_problem
    from vaevar.synth import smooth_field

    probs = [make_problem(nch=69, Hs=128, Ws=256, T=2, seed=20250700 + b) for b in range(2)]
    z = torch.from_numpy(0.3 * smooth_field(1302, (2, 32, 128, 256))).cuda()
    dec2 = LGUnet(C.DECODER, 2, 1).load_synthetic()
    flow2 = LGUnet(C.FLOW, 2, 1).load_synthetic()
    pb = DAProblem(dec2, probs, flow=flow2)
    g2 = torch.empty_like(z)
    jb2, jo2 = pb.closure_batch(z, g2)
    xa2 = pb.analysis(z).cpu()
    del pb, dec2, flow2
    dec1 = LGUnet(C.DECODER, 1, 1).load_synthetic()
    flow1 = LGUnet(C.FLOW, 1, 1).load_synthetic()
    for b in range(2):
        p1 = DAProblem(dec1, probs[b], flow=flow1)
        g1 = torch.empty(1, 32, 128, 256, device="cuda")
        jb1, jo1 = p1.closure(z[b:b + 1].contiguous(), g1)
        e = (abs(jb1 - jb2[b]) / jb1, abs(jo1 - jo2[b]) / jo1, rel(g2[b].cpu(), g1[0].cpu()),
             rel(xa2[b], p1.analysis(z[b:b + 1].contiguous()).cpu()))
        print(f"full B=2 vs B=1, analysis {b}: J_b {e[0]:.1e} J_o {e[1]:.1e} grad {e[2]:.1e} xa {e[3]:.1e}")
        check(f"full B=2 vs B=1 analysis {b} J_b", e[0], 1e-12, "<=")
        check(f"full B=2 vs B=1 analysis {b} J_o", e[1], 5e-8)
        check(f"full B=2 vs B=1 analysis {b} dJ/dz", e[2], 1e-5)
        check(f"full B=2 vs B=1 analysis {b} xa", e[3], 5e-7)
