#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && MIOPEN_FIND_MODE=FAST timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_resnet -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_resnet.py --steps 5 --warmup 3 > $GRAFT_REPO_ROOT/gpurun_out/prof_resnet.log 2>&1
