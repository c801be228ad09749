"""Memory-bound kernel probe at the GPT-2-medium B=64 shapes: achieved TB/s, numerics vs fp32.

    python tools/elt_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def load_alt(path):
    """Load another build of the extension (A/B against the in-tree one)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("_pdo_hip", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def ln_bwd_ab(mods):
    dev = torch.device("cuda")
    N, C = 65536, 1024
    g = torch.Generator(device=dev).manual_seed(1)
    h = torch.randn(N, C, device=dev, generator=g).bfloat16()
    r = torch.randn(N, C, device=dev, generator=g).bfloat16()
    w = (1 + 0.1 * torch.randn(C, device=dev, generator=g)).bfloat16()
    b = (0.1 * torch.randn(C, device=dev, generator=g)).bfloat16()
    rb = (0.1 * torch.randn(C, device=dev, generator=g)).bfloat16()
    dy = torch.randn(N, C, device=dev, generator=g).bfloat16()
    _, y, mean, rstd = mods[0].add_layernorm_fwd(h, r, w, b, 1e-5, rb)
    outs = [mm.layernorm_bwd_add(dy, h, w, mean, rstd, r, True) for mm in mods]
    diff = max((a.float() - c.float()).abs().max().item() for a, c in zip(outs[0], outs[-1]))
    ts = {i: [] for i in range(len(mods))}
    for _ in range(5):
        for i, mm in enumerate(mods):
            ts[i].append(bench(lambda: mm.layernorm_bwd_add(dy, h, w, mean, rstd, r, True)))
    nb = N * C * 2 * 4  # dy, h, dres read + dx write
    for i in ts:
        t = sorted(ts[i])[2]
        print(json.dumps({"ln_bwd_build": i, "us": round(t, 1), "TBps": round(nb / t / 1e6, 2), "maxdiff_vs_0": diff}))


def main():
    from paddle_operator_amd import _native, ops
    m = _native.require_hip()
    if len(sys.argv) > 1:
        ln_bwd_ab([m, load_alt(sys.argv[1])])
        return
    dev = torch.device("cuda")
    N, F = 65536, 4096
    g = torch.Generator(device=dev).manual_seed(0)
    x = (2 * torch.randn(N, F, device=dev, generator=g)).bfloat16()
    b = (0.5 * torch.randn(F, device=dev, generator=g)).bfloat16()
    dy = torch.randn(N, F, device=dev, generator=g).bfloat16()
    # fp32 reference on a slice
    xs = x[:4096].float().requires_grad_()
    yr = ops.ref_bias_gelu(xs, b.float())
    yr.backward(dy[:4096].float())
    variants = [0, 1, 2, 3] if hasattr(m, "set_gelu_variant") else [None]
    res = {}
    for v in variants:
        if v is not None:
            m.set_gelu_variant(v)
        y = m.bias_gelu_fwd(x, b)
        dx, db = m.bias_gelu_bwd(dy, x, b)
        res[v] = {"fwd_err": ((y[:4096].float() - yr).abs().max() / yr.abs().max()).item(),
                  "bwd_err": ((dx[:4096].float() - xs.grad).abs().max() / xs.grad.abs().max()).item(),
                  "fwd": [], "bwd": []}
    for _ in range(5):
        for v in variants:
            if v is not None:
                m.set_gelu_variant(v)
            res[v]["fwd"].append(bench(lambda: m.bias_gelu_fwd(x, b)))
            res[v]["bwd"].append(bench(lambda: m.bias_gelu_bwd(dy, x, b)))
    nb = N * F * 2
    yc = torch.empty_like(x)
    cp = sorted(bench(lambda: yc.copy_(x)) for _ in range(5))[2]
    print(json.dumps({"copy_us": round(cp, 1), "copy_TBps": round(2 * nb / cp / 1e6, 2)}))
    for v in variants:
        f, bw = sorted(res[v]["fwd"])[2], sorted(res[v]["bwd"])[2]
        print(json.dumps({"variant": v, "fwd_us": round(f, 1), "fwd_TBps": round(2 * nb / f / 1e6, 2),
                          "bwd_us": round(bw, 1), "bwd_TBps": round(3 * nb / bw / 1e6, 2),
                          "fwd_err": res[v]["fwd_err"], "bwd_err": res[v]["bwd_err"]}))


if __name__ == "__main__":
    main()
