"""Time vv_attention_global (the flash MFMA kernel of the 0.25-degree global LG window) on the 16,200-token,
6-head, head_dim-192 shape (dev tool); prints us per call and the fp16x3 MFMA fraction of the 2.5 PF peak."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar.engine import Context

ctx = Context.get(0)
N, C, H = int(os.environ.get("N", "16200")), 1152, 6
qkv = torch.randn(N, 3 * C, device="cuda")
qkv[:, :C] *= 192 ** -0.5
for _ in range(2):
    ctx.attention_global(qkv, H)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
n = 10
e0.record()
for _ in range(n):
    ctx.attention_global(qkv, H)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / n
fl = 2 * 2 * N * N * C  # QK^T and PV, fp32-equivalent
print(json.dumps({"N": N, "us": round(us, 1), "tflops_fp32eq": round(fl / us / 1e6, 1),
                  "frac_of_fp16x3_peak": round(fl / us / 1e6 / 833.3, 3)}), flush=True)
