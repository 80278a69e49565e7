"""Dev probe: what the library GEMMs reach on the tower shapes (bf16 with the 6 split products folded into K,
fp32 output; plain fp32), next to a same-size elementwise write -- sizes the headroom of tiles 24 / 26."""
import json, torch
shapes = [(49152, 288, 96), (49152, 384, 96), (12288, 576, 192), (12288, 768, 192)]


def tm(f, n=30):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


for (M, N, K) in shapes:
    row = {"M": M, "N": N, "K": K}
    A6 = torch.randn(M, 6 * K, device="cuda", dtype=torch.bfloat16)
    B6 = torch.randn(N, 6 * K, device="cuda", dtype=torch.bfloat16)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(N, K, device="cuda")
    C = torch.empty(M, N, device="cuda")
    try:
        row["bf16x6K_out32_us"] = round(tm(lambda: torch.mm(A6, B6.t(), out_dtype=torch.float32)), 1)
    except Exception as ex:
        row["bf16x6K_out32_us"] = f"err {str(ex)[:60]}"
    row["bf16x6K_out16_us"] = round(tm(lambda: A6 @ B6.t()), 1)
    row["f32_us"] = round(tm(lambda: torch.mm(A, B.t(), out=C)), 1)
    row["fill_C_us"] = round(tm(lambda: C.fill_(1.0)), 1)
    row["copy_A_to_C_us"] = round(tm(lambda: C.view(-1)[: A.numel()].copy_(A.view(-1))), 1)
    print(json.dumps(row), flush=True)
