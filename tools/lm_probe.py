import sys, json, torch
sys.path.insert(0, ".")
from tools.gemm_probe import bench
T, V, C = 65536, 50304, 1024
d = torch.device("cuda")
dy = torch.randn(T, V, device=d, dtype=torch.bfloat16)
x = torch.randn(T, C, device=d, dtype=torch.bfloat16)
out = {}
out["mm_us"] = bench(lambda: dy.t() @ x, iters=5, warm=2)
for s in (2, 4, 8):
    ds = dy.view(s, T // s, V).transpose(1, 2)
    xs = x.view(s, T // s, C)
    out[f"split{s}_us"] = bench(lambda: torch.sum(torch.bmm(ds, xs), 0), iters=5, warm=2)
xt = x.t().contiguous()
out["mm_xt_us"] = bench(lambda: torch.mm(dy.t(), x), iters=5, warm=2)
out["mmT_us"] = bench(lambda: torch.mm(xt, dy).t(), iters=5, warm=2)  # dW^T = X^T dY
fl = 2 * T * V * C
print(json.dumps({k: (round(v, 1), round(fl / (v * 1e-6) / 1e12)) for k, v in out.items()}))
