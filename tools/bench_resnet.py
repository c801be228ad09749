"""ResNet-50 training throughput (img/s) on one GPU — BASELINE configs 2/3/5 workload.

    python tools/bench_resnet.py [--batch 256] [--steps 20] [--warmup 10] [--graph]

--graph: the step captured once into a HIP graph (ResNetTrainer(graph=True)),
replayed behind a fresh batch draw.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    import torch
    from paddle_operator_amd.workloads.resnet import ResNetTrainer
    if os.environ.get("BENCH_GAP_FRAMEWORK") == "1":  # A/B: the framework's average pool (and its backward copies)
        import torch.nn.functional as F

        from paddle_operator_amd import ops
        ops.global_avg_pool = lambda x: torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
    if os.environ.get("BENCH_CONV_DIRECT_NCHW") == "1":  # A/B: the round-5-earlier direct-write rule for conv weights
        from paddle_operator_amd.ops import core as ops_core
        from paddle_operator_amd.ops import resnet as ops_resnet
        ops_resnet._direct_cl_ok = lambda p: (ops_core._direct_ok(p) and p.grad.dtype == torch.float32
                                              and p.grad.is_contiguous(memory_format=torch.channels_last))
    if os.environ.get("BENCH_WT1X1_PERCALL") == "1":  # A/B: a transpose per 1×1 input gradient (pre round 6)
        from paddle_operator_amd.ops import resnet as ops_resnet
        from paddle_operator_amd.ops.core import transpose
        ops_resnet._wt_1x1 = lambda ctx, wb, K, C: transpose(wb.view(K, C))
    t0 = time.time()
    tr = ResNetTrainer(a.batch, "cuda:0", graph=a.graph)
    for _ in range(a.warmup):
        tr.step()
    torch.cuda.synchronize()
    t_warm = time.time() - t0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        loss = tr.step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.steps
    print(json.dumps({"metric": "ResNet-50 train img/s (bf16 autocast, channels_last)", "value": round(a.batch / ms * 1e3, 1),
                      "ms_per_step": round(ms, 2), "batch": a.batch, "graph": tr._graph is not None, "warmup_s": round(t_warm, 1),
                      "loss": float(loss.detach()), "miopen_find_mode": os.environ.get("MIOPEN_FIND_MODE", "default")}))


if __name__ == "__main__":
    main()
