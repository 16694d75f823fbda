"""dgrad GEMM layout probe: dx = dy · W with W [N, K] as stored (torch.mm(dy, W)) vs with a
transposed copy Wt [K, N] (torch.mm(dy, Wt.t()): both operands reduction-contiguous, the
forward's layout). GPT-2 124M shapes, M = 65536 tokens, bf16, one MI355X."""
import json, torch

def t_ms(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n

M = 65536
for name, N, K in [("qkv", 2304, 768), ("proj", 768, 768), ("fc", 3072, 768), ("fc2", 768, 3072), ("lm_head", 50304, 768)]:
    dy = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    wt = w.t().contiguous()
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    out = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    fl = 2 * M * N * K
    r = {"shape": name}
    r["dgrad_W_TF"] = fl / t_ms(lambda: torch.mm(dy, w, out=out)) / 1e9
    r["dgrad_Wt_TF"] = fl / t_ms(lambda: torch.mm(dy, wt.t(), out=out)) / 1e9
    o2 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    r["fwd_TF"] = fl / t_ms(lambda: torch.mm(x, w.t(), out=o2)) / 1e9
    r["transpose_ms"] = t_ms(lambda: wt.copy_(w.t()))
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) and k != "transpose_ms" else (round(v, 4) if isinstance(v, float) else v)) for k, v in r.items()}), flush=True)
    del dy, w, wt, x, out, o2
