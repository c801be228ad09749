"""paddle_operator_amd — an MI355X-native distributed-training job framework.

Capabilities of lfeng-nl/paddle-operator (a Kubernetes operator for the
``PaddleJob`` CRD, see ``/root/reference/controllers/paddlejob_controller.go``)
re-designed MI355X-first:

* ``api``        — PaddleJob schema (batch.paddlepaddle.org/v1), CRD generation.
* ``controller`` — Python driver of the native C++ planner / local cluster
                   backend (``csrc/core``), reconcile semantics of the reference.
* ``kv``         — client for ``pdo-kv``, the native etcd-v3-subset store.
* ``launch``     — ``pdo-launch``: the in-container PyTorch-ROCm launcher that
                   turns the Paddle env contract into an RCCL process group.
* ``parallel``   — bucketed RCCL data parallel, parameter server, elastic.
* ``models``     — GPT-2(-medium), ResNet-50, wide&deep workloads.
* ``ops``        — hand-written HIP/CDNA4 kernels (``csrc/hip``) with PyTorch
                   fp32 reference implementations used for CPU and numerics tests.
* ``utils``      — topology (rocm_smi), device affinity, checkpointing, metrics.
"""

__version__ = "0.1.0"
