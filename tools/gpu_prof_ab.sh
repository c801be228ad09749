#!/bin/bash
# kernel-trace profiles of the headline bench under two env settings (A: default, B: $B_ENV)
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_A -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_A.log 2>&1 &&
env $B_ENV true && export $B_ENV && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_B -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_B.log 2>&1
