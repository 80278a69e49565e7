"""Dev probe: library fp16 GEMM speed on the LG shapes with the 3-product split folded into K (A' = [Ah Ah Al],
B' = [Bh Bl Bh], K' = 3K), to size a hipBLASLt path against k_gemm_h3."""
import json, torch
shapes = [(2048, 3456, 1152), (2048, 1152, 1152), (2048, 4608, 1152), (2048, 1152, 4608), (2048, 1152, 3456)]
for (M, N, K) in shapes:
    A = torch.randn(M, 3 * K, device="cuda", dtype=torch.float16)
    B = torch.randn(N, 3 * K, device="cuda", dtype=torch.float16)
    row = {"M": M, "N": N, "K": K}
    for name, f in (("f16_out16", lambda: A @ B.t()),
                    ("f16_out32", lambda: torch.ops.aten._scaled_mm if False else torch.mm(A, B.t(), out_dtype=torch.float32) if hasattr(torch, "float32") else None)):
        try:
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(30):
                f()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 30
            row[name] = f"{us:.1f}us {2 * M * N * K / us / 1e6:.0f}TF-equiv"
        except Exception as ex:
            row[name] = f"err {type(ex).__name__}: {str(ex)[:80]}"
    print(json.dumps(row), flush=True)
