"""Library GEMM ceilings on the box: torch (hipBLASLt) bf16 / fp32 / tf32-off matmul TF on given shapes (dev tool)."""
import os, sys, json
import torch

shapes = [tuple(int(x) for x in sh.split("x")) for sh in os.environ.get(
    "SHAPES", "8192x8192x8192,2048x4608x1152,2048x1152x1152,2048x1152x4608").split(",")]
torch.backends.cuda.matmul.allow_tf32 = False
for (M, N, K) in shapes:
    row = {"M": M, "N": N, "K": K}
    for name, dt in (("bf16", torch.bfloat16), ("fp16", torch.float16), ("fp32", torch.float32)):
        A = torch.randn(M, K, device="cuda").to(dt)
        B = torch.randn(N, K, device="cuda").to(dt)
        for _ in range(3):
            A @ B.t()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n):
            A @ B.t()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / n
        row[name] = round(2 * M * N * K / us / 1e6, 1)
    print(json.dumps(row), flush=True)
