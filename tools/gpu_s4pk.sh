#!/bin/bash
# packed-fp32 GEMM epilogues: GPU tests, per-shape probe and in-step A/B (ab/base.so vs ab/pk.so)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-s4pk}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_nt_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu_so_ab.sh python tools/nt4_probe.py --shapes fc1_fwd,fc2_dx --impls 0,1 --rounds 3 > $O/probe.txt || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
bash tools/gpu_so_ab.sh python tools/train_probe.py --dist --steps 20 --warmup 3 > $O/step_gelu0.txt || { cat $O/step_gelu0.txt; exit 1; }
cat $O/step_gelu0.txt
bash tools/gpu_so_ab.sh env PDO_NT_GELU=1 python tools/train_probe.py --dist --steps 20 --warmup 3 > $O/step_gelu1.txt || { cat $O/step_gelu1.txt; exit 1; }
cat $O/step_gelu1.txt
