#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_ops_gpu.py -x -v -k "gemm_dw or splitk or arena or gpt2_tiny or linear" --timeout 120 --timeout-method thread > gpurun_out/dw_test.log 2>&1 &&
timeout -k 10 300 python -u tools/dw_probe.py --pdo-only > gpurun_out/dw_probe.log 2>&1
