#!/bin/bash
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && PDO_ROCTX=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats -d $R/gpurun_out/prof_roctx -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_roctx.log 2>&1
