#!/bin/bash
# round-2 GPU session C: persistent GEMM numerics + timing; RCCL init breakdown
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2c; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gemm_pnt_gpu.py -x -v --timeout 120 --timeout-method thread > $O/pytest_pnt.log 2>&1 || { tail -60 $O/pytest_pnt.log; exit 1; }
tail -3 $O/pytest_pnt.log
timeout -k 10 400 python tools/pnt_probe.py --rounds 3 --iters 20 > $O/pnt_probe.jsonl 2> $O/pnt_probe.err || { tail -30 $O/pnt_probe.err; exit 1; }
cat $O/pnt_probe.jsonl
NCCL_DEBUG=INFO NCCL_DEBUG_TIMESTAMP_LEVELS=ALL timeout -k 10 120 python tools/rccl_init_probe.py > $O/rccl_init.json 2> $O/rccl_init.err || { tail -30 $O/rccl_init.err; exit 1; }
cat $O/rccl_init.json
timeout -k 10 120 python tools/rccl_init_probe.py >> $O/rccl_init.json 2>/dev/null; tail -1 $O/rccl_init.json
