#!/usr/bin/env python3
"""Where the ResNet-50 HIP path departs from fp32: per-block forward outputs
and the stem's input gradient of three runs on the same weights and batch —

* ``hip``: the production HIP path (bf16 shadow weights + autocast, fused ops);
* ``fw``:  the framework ops in bf16 on the GPU (``PDO_OPS=torch``, autocast);
* ``ref``: the framework ops in fp32 on the CPU —

printed as relative L2 errors against ``ref`` (tests/test_workloads_gpu.py::
test_resnet50_width_hip_vs_fp32 is the pass/fail form).

    python tools/resnet_anchor_probe.py [--batch 16] [--res 128] [--zero-init]
"""
import argparse
import copy
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--res", type=int, default=128)
    ap.add_argument("--zero-init", action="store_true", help="keep bn3's zero γ (the training recipe)")
    ap.add_argument("--bn3", type=float, default=0.0, help="bn3 γ drawn from [bn3/2, 3·bn3/2] (0: as the others)")
    a = ap.parse_args()
    import torch
    import torch.nn.functional as F

    from paddle_operator_amd import ops
    from paddle_operator_amd.models.resnet import resnet50
    from paddle_operator_amd.parallel.flat import FlatParams

    torch.manual_seed(0)
    ref = resnet50()
    if not a.zero_init:
        for m in ref.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                torch.nn.init.uniform_(m.weight, 0.5, 1.5)
                torch.nn.init.uniform_(m.bias, -0.1, 0.1)
        if a.bn3 > 0:
            for blk in ref.modules():
                if hasattr(blk, "bn3"):
                    torch.nn.init.uniform_(blk.bn3.weight, 0.5 * a.bn3, 1.5 * a.bn3)
    dev = torch.device("cuda", 0)
    hip = copy.deepcopy(ref).to(dev).to(memory_format=torch.channels_last)
    fw = copy.deepcopy(ref).to(dev).to(memory_format=torch.channels_last)
    flat = FlatParams(hip, dtype=torch.float32, device=dev, bucket_bytes=25 << 20)
    flat.enable_shadow(torch.bfloat16)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(a.batch, 3, a.res, a.res, generator=g)
    y = torch.randint(0, 1000, (a.batch,), generator=g)

    def run(m, xin, yy):
        acts = {}
        hooks = []
        names = ["layer1", "layer2", "layer3", "layer4"]
        for ln in names:
            for i, blk in enumerate(getattr(m, ln)):
                hooks.append(blk.register_forward_hook(
                    lambda mod, inp, out, k=f"{ln}.{i}": acts.__setitem__(k, out.detach().float().cpu())))
        h = ops.conv_bn_relu_maxpool(m.conv1, m.bn1, xin)
        h.retain_grad()
        acts["stem"] = h.detach().float().cpu()
        z = m.layer4(m.layer3(m.layer2(m.layer1(h))))
        logits = m.fc(torch.flatten(F.adaptive_avg_pool2d(z, 1), 1))
        loss = F.cross_entropy(logits.float(), yy)
        loss.backward()
        for hk in hooks:
            hk.remove()
        acts["logits"] = logits.detach().float().cpu()
        return acts, h.grad.float().cpu(), float(loss)

    xh = x.to(dev, torch.bfloat16).contiguous(memory_format=torch.channels_last)
    flat.zero_grad()
    with flat.shadow_scope(), torch.autocast("cuda", dtype=torch.bfloat16):
        A_h, G_h, L_h = run(hip, xh, y.to(dev))
    os.environ["PDO_OPS"] = "torch"
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16):
            A_f, G_f, L_f = run(fw, xh, y.to(dev))
    finally:
        os.environ["PDO_OPS"] = "hip"
    A_r, G_r, L_r = run(ref, x, y)

    def rel(p, q):
        return round(float((p - q).norm() / (q.norm() + 1e-12)), 4)

    for k in A_r:
        print(json.dumps({"point": k, "hip": rel(A_h[k], A_r[k]), "fw_bf16": rel(A_f[k], A_r[k]),
                          "ref_norm": round(float(A_r[k].norm()), 2)}))
    print(json.dumps({"point": "dstem", "hip": rel(G_h, G_r), "fw_bf16": rel(G_f, G_r)}))
    print(json.dumps({"loss": {"hip": L_h, "fw_bf16": L_f, "ref": L_r}}))
    rp = dict(ref.named_parameters())
    fp = dict(fw.named_parameters())
    worst = sorted(((rel(p.grad.float().cpu(), rp[n].grad), rel(fp[n].grad.float().cpu(), rp[n].grad), n)
                    for n, p in hip.named_parameters()), reverse=True)[:12]
    for eh, ef, n in worst:
        print(json.dumps({"grad": n, "hip": eh, "fw_bf16": ef}))


if __name__ == "__main__":
    main()
