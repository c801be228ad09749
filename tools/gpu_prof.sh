#!/bin/bash
# kernel-trace profile of the headline bench (summary → gpurun_out/prof_<tag>)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-cur}; MB=${MB:-64}
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG -o run -- python3 $GRAFT_REPO_ROOT/bench.py --micro-batch $MB --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log 2>&1
