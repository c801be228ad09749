#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gemm_nt_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/nt_test.log 2>&1 &&
timeout -k 10 300 python -u tools/nt_probe.py > gpurun_out/nt_probe.log 2>&1
