"""Fused ops for the flagship workloads (HIP kernels in ``csrc/hip``).

* ``ops.core``   — dispatch, fp32 references, arena gradient hand-off,
  ``linear``, the batched Wᵀ and deferred column sums;
* ``ops.gpt2``   — LayerNorm, MLP, attention, LM head + cross-entropy, embedding;
* ``ops.resnet`` — convolutions, BatchNorm, the stem;
* ``ops.optim``  — the fused flat AdamW.

Every op has a HIP path (GPU tensors; a missing extension raises) and a plain
PyTorch fp32 reference (CPU, and the oracle of the numerics tests).
"""
from .core import (  # noqa: F401
    _HIP_DW, _NT_ALL, _arena_grads, _direct_ok, _fwd_gemm, _input_grad, _signal_ready, _splitk, _weight_grad,
    _weight_grad_lib, _workspace, deferred_reductions, flush_deferred, linear, ref_attention, ref_bias_gelu,
    ref_cross_entropy, ref_layer_norm, transpose, use_hip)
from .gpt2 import (  # noqa: F401
    _LMHeadXentFn, _LM_CHUNK, _QKV_FUSED, _RES_EPI, _XENT_FUSED, _NT_GELU, _NT_DGELU, _NT_GD, add_layer_norm,
    attention, bias_gelu, cross_entropy, embedding, layer_norm, layer_norm_res, linear_add_layer_norm, lm_head_xent, mlp, mlp_add_layer_norm,
    qkv_attention)
from .resnet import (  # noqa: F401
    _BNActBNResFn, _BNLink, _BNReluPoolFn, _CompactGradLink, _ResMaskLink, _StemFn, _BN_FUSED, _DS_FUSED,
    _GEMM_BN_STATS, _BN_LINK, _BN_LINK_USED, _DS_COMPACT, _DS_COMPACT_USED, _HIP_CONV, _HIP_STEM, _RES_MASK,
    _RES_MASK_USED, _STEM_POOL, _apply_bitmask, _stem_ok, bn_act, conv1x1, conv_bn_act, conv_bn_ds_act,
    conv_bn_relu_maxpool, global_avg_pool,
    max_pool_3x3s2)

__all__ = [
    "layer_norm", "layer_norm_res", "add_layer_norm", "bias_gelu", "attention", "cross_entropy",
    "embedding", "ref_layer_norm", "ref_bias_gelu", "ref_attention",
    "ref_cross_entropy", "use_hip", "linear", "mlp", "qkv_attention", "lm_head_xent",
    "conv_bn_act", "conv_bn_ds_act", "bn_act", "deferred_reductions",
]
