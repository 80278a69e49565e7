"""Quick timing of the full-size vae4dvar closure (development tool)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "vae-var_amd"))
import torch
from vaevar import config as C
from vaevar.engine import LGUnet, DAProblem
from vaevar.problem import make_problem

T = int(os.environ.get("T", "1"))
dec = LGUnet(C.DECODER, 1, 1).load_synthetic()
flow = LGUnet(C.FLOW, 1, max(T - 1, 1)).load_synthetic() if T > 1 else None
print("workspace GB", dec.workspace_bytes() / 1e9, flush=True)
prob = DAProblem(dec, make_problem(T=T), flow=flow)
z = torch.zeros(1, 32, 128, 256, device="cuda")
g = torch.empty_like(z)
for i in range(3):
    prob.closure(z, g)
torch.cuda.synchronize()
n = 10
t0 = time.time()
for i in range(n):
    prob.closure(z, g)
torch.cuda.synchronize()
dt = (time.time() - t0) / n
fl = 1787.8e9 * (1 if T == 1 else (T * 1.0))
print(f"closure T={T}: {dt*1e3:.2f} ms/eval  -> {1787.8e9*T/dt/1e12:.1f} TFLOP/s algorithmic", flush=True)
x = torch.randn(1, 32, 128, 256, device="cuda")
out = dec.forward_raw(x)
torch.cuda.synchronize()
t0 = time.time()
for i in range(n):
    dec.forward_raw(x, out=out)
torch.cuda.synchronize()
dt = (time.time() - t0) / n
print(f"decoder fwd: {dt*1e3:.2f} ms -> {892.1e9/dt/1e12:.1f} TFLOP/s", flush=True)
