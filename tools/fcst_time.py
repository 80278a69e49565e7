"""Time the 0.25-degree forecast integrate(x, LGUnet_all_1, 1) on the HIP engine (dev tool).
Synthetic weights; prints per-forecast time and the per-kernel-class split."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar import config as C
from vaevar.engine import LGUnet, integrate
from vaevar.synth import smooth_field

cfg = C.FCST if not os.environ.get("MID") else C.MID_FCST
t0 = time.time()
m = LGUnet(cfg, 1, 1).load_synthetic()
print(f"model built + synthetic weights {time.time() - t0:.1f}s, workspace {m.workspace_bytes() / 1e9:.1f} GB",
      flush=True)
Cs = C.in_channels(cfg)
H, W = cfg["img_size"]
x = torch.from_numpy(smooth_field(11, (Cs, H, W))).cuda()
mean = torch.zeros(Cs)
std = torch.ones(Cs)
out = integrate(m, x, mean, std)
torch.cuda.synchronize()
n = int(os.environ.get("N", "2"))
t0 = time.time()
for _ in range(n):
    integrate(m, x, mean, std, out=out)
torch.cuda.synchronize()
dt = (time.time() - t0) / n
print(f"forecast {H}x{W}: {dt * 1e3:.1f} ms", flush=True)
m.ctx.profile_start()
integrate(m, x, mean, std, out=out)
pr = m.ctx.profile_stop()
print({k: round(v["ms"], 2) for k, v in pr.items()}, "gemm TF",
      round(pr["gemm"]["flops"] / max(pr["gemm"]["ms"], 1e-9) / 1e9, 1), flush=True)
print("finite", bool(torch.isfinite(out).all()), float(out.abs().max()))
