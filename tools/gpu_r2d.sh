#!/bin/bash
# round-2 GPU session D: full GPU suite with the 4-wave gemm_nt default, launched bench
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2d; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -80 $O/pytest_gpu.log; exit 1; }
tail -5 $O/pytest_gpu.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -60 $O/bench.err; exit 1; }
cat $O/bench.json
