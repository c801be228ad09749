#!/usr/bin/env python3
"""ResNet-50 step: whole-step HIP graph replay vs eager, in lockstep.

Two trainers from the same seed (PDO_RESNET_GRAPH=0 / 1) step side by side;
after every step prints the loss of each and the relative difference of the
parameter arena, the momentum buffer and the BatchNorm buffers.

    python tools/resnet_graph_probe.py [--batch 16] [--steps 8]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    import torch

    from paddle_operator_amd.workloads.resnet import ResNetTrainer

    tr = []
    for g in (0, 1, 0):  # the second eager trainer: run-to-run spread of the eager path itself
        os.environ["PDO_RESNET_GRAPH"] = str(g)
        torch.manual_seed(0)
        tr.append(ResNetTrainer(a.batch, "cuda:0"))

    def rel(p, q):
        return float((p.float() - q.float()).norm() / (q.float().norm() + 1e-30))

    def bufs(t):
        return torch.cat([b.float().reshape(-1) for b in t.model.buffers()])

    for s in range(a.steps):
        losses = []
        for t in tr:  # one trainer at a time: they share the ops' scratch buffers
            losses.append(float(t.step()))
            torch.cuda.synchronize()
        rec = {"step": s + 1, "loss_eager": losses[0], "loss_graph": losses[1], "loss_eager2": losses[2]}
        for name, i in (("graph", 1), ("eager2", 2)):
            pa, pb = dict(tr[i].model.named_parameters()), dict(tr[0].model.named_parameters())
            per = sorted(((rel(pa[n], pb[n]), n) for n in pb), reverse=True)
            live = torch.zeros(tr[0].flat.numel, dtype=torch.bool, device=tr[0].flat.params.device)
            for sl in tr[0].flat.slots:
                live[sl.offset:sl.offset + sl.numel] = True
            rec[name] = {"params_live": rel(tr[i].flat.params[live], tr[0].flat.params[live]),
                         "nan_live": int(torch.isnan(tr[i].flat.params[live]).sum()),
                         "nan_pad": int(torch.isnan(tr[i].flat.params[~live]).sum()),
                         "worst": [(round(e, 5), n) for e, n in per[:4]],
                         "bn_bufs": rel(bufs(tr[i]), bufs(tr[0]))}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
