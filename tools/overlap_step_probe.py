#!/usr/bin/env python3
"""The GPT-2-medium training step with "all-reduce-like" kernels beside it — the
N > 1 situation rehearsed on one GPU.  When the weight gradient of fc2 in every
``--every``-th block is ready (the hook BucketedDDP uses to launch a bucket),
a kernel that holds one CU for ≈ ``--hold-us`` is launched on a side stream
after an event on the compute stream, as an RCCL all-reduce is.  Interleaved
rounds of: no side kernels, side kernels with gemm_nt4's static tile order,
side kernels with the dynamic order (what BucketedDDP selects for multi-rank
jobs).  ms/step per configuration.

    python tools/overlap_step_probe.py [--steps 10] [--rounds 2] [--every 2] [--hold-us 300]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--every", type=int, default=2)
    ap.add_argument("--hold-us", type=float, default=300.0)
    ap.add_argument("--side-priority", type=int, default=0,
                    help="side stream priority (0 default, -1 high: ProcessGroupNCCL's is_high_priority_stream)")
    a = ap.parse_args()
    import torch
    from paddle_operator_amd import _native
    from paddle_operator_amd.models.gpt2 import GPT2Config
    from paddle_operator_amd.train import GPT2Trainer
    m = _native.require_hip()
    dev = torch.device("cuda", 0)
    tr = GPT2Trainer(GPT2Config.named("gpt2-medium"), 64, 1024, dev)
    bf = dict(device=dev, dtype=torch.bfloat16)

    def hog_of(th):
        hy, hx, ho = torch.randn(th, 256, **bf), torch.randn(th, 256, **bf), torch.empty(256, 256, **bf)
        return lambda: m.gemm_dw(hy, hx, ho, False, 1)

    def once(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3

    t4 = once(hog_of(4096))
    hog = hog_of(max(256, int(4096 * a.hold_us / t4) // 128 * 128))
    side = torch.cuda.Stream(dev, priority=a.side_priority)
    active = [False]
    launched = [0]

    def ready_hook(p):
        if not active[0]:
            return
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            hog()
        launched[0] += 1

    # the fc2 (fc_proj) weight of every --every-th block: its dW is the last
    # gradient of the block's MLP, where a bucket boundary often falls
    params = [p for n, p in tr.model.named_parameters()
              if n.endswith("fc_proj.weight") and int(n.split(".")[1]) % a.every == 0]
    for p in params:
        prev = getattr(p, "_pdo_ready", None)

        def hook(q, prev=prev):
            if prev is not None:
                prev(q)
            ready_hook(q)
        p._pdo_ready = hook

    def run(cfg):
        active[0] = cfg != "none"
        m.gemm_nt4_dynamic(1 if cfg == "dynamic" else 0)
        for _ in range(2):
            tr.step()
        torch.cuda.synchronize()
        launched[0] = 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.steps):
            tr.step()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.steps, launched[0] / a.steps

    res = {c: [] for c in ("none", "static", "dynamic")}
    per = {}
    for _ in range(a.rounds):
        for c in res:
            ms, n = run(c)
            res[c].append(round(ms, 3))
            per[c] = n
    m.gemm_nt4_dynamic(0)
    print(json.dumps({"side_priority": a.side_priority, "hooked_params": len(params), "side_kernels_per_step": per, "hold_us": a.hold_us,
                      "ms_per_step": res, "median": {c: statistics.median(v) for c, v in res.items()}}))


if __name__ == "__main__":
    main()
