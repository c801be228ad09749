"""Run only the attention kernels (for rocprofv3 --pmc passes): fwd and bwd at the GPT-2-medium shape."""
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))


def main():
    from paddle_operator_amd import _native
    m = _native.require_hip()
    B, S, H, D = int(sys.argv[1]) if len(sys.argv) > 1 else 64, 1024, 16, 64
    which = sys.argv[2] if len(sys.argv) > 2 else "both"
    dev = torch.device("cuda")
    qkv = torch.randn(B, S, 3 * H * D, device=dev, dtype=torch.bfloat16)
    dout = torch.randn(B, S, H * D, device=dev, dtype=torch.bfloat16)
    o, lse = m.attn_fwd(qkv, H)
    for _ in range(5):
        if which in ("fwd", "both"):
            o, lse = m.attn_fwd(qkv, H)
        if which in ("bwd", "both"):
            m.attn_bwd(dout, qkv, o, lse, H)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
