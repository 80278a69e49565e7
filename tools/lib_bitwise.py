"""Dev tool: dump the config-2 decoder forward, the closure J and dJ/dz at a fixed z with the library named by
VAEVAR_LIB, to compare two builds bit for bit: python tools/lib_bitwise.py out.npz"""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
sys.path.insert(0, ROOT)
from vaevar import config as C
from vaevar.engine import DAProblem, LGUnet
from vaevar.problem import make_problem
from vaevar.synth import smooth_field

dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
z = torch.from_numpy(0.3 * smooth_field(11, (1, 32, 128, 256), sigma=2.0)).cuda()
out = dec.forward_raw(z).cpu().numpy()
prob = DAProblem(dec, make_problem(nch=69, Hs=128, Ws=256, T=1, seed=20250620))
g = torch.empty_like(z)
jb, jo = prob.closure(z, g)
np.savez(sys.argv[1], out=out, j=np.array([jb, jo]), g=g.cpu().numpy())
if len(sys.argv) > 2:
    r = np.load(sys.argv[2])
    for k in ("out", "j", "g"):
        a, b = np.load(sys.argv[1])[k], r[k]
        print(k, "bitwise" if np.array_equal(a, b) else f"DIFF max {np.abs(a - b).max():.3e} n {(a != b).sum()}")
