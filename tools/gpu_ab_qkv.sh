#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/b_q1.json 2> gpurun_out/b_q.err &&
PDO_QKV_FUSED=0 timeout -k 10 300 python bench.py > gpurun_out/b_q0.json 2>> gpurun_out/b_q.err &&
timeout -k 10 300 python bench.py > gpurun_out/b_q1b.json 2>> gpurun_out/b_q.err
