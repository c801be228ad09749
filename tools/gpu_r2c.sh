#!/bin/bash
# round-2 GPU session C: GPU-warm slots (ready p50), GPU test subset, launched bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2c; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 400 python -u -m pytest tests/test_rccl_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest_rccl.log 2>&1 || { tail -60 $O/pytest_rccl.log; exit 1; }
tail -12 $O/pytest_rccl.log
timeout -k 10 300 python bench.py --ready-only --ready-trials 10 > $O/ready_warm.json 2> $O/ready_warm.err || { tail -60 $O/ready_warm.err; exit 1; }
cat $O/ready_warm.json
timeout -k 10 300 python bench.py --ready-only --ready-trials 10 --no-warm-slots > $O/ready_nowarm.json 2> $O/ready_nowarm.err || { tail -60 $O/ready_nowarm.err; exit 1; }
cat $O/ready_nowarm.json
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --compat-trials 3 > $O/bench.json 2> $O/bench.err || { tail -60 $O/bench.err; exit 1; }
cat $O/bench.json
