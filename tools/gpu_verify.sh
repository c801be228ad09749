#!/bin/bash
# One GPU call: kernel tests, smoke, headline bench, roctx+kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
cd /tmp && PDO_ROCTX=1 timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --stats -d $R/gpurun_out/prof_roctx -o run -- python3 $R/bench.py --steps 3 --warmup 2 > $R/gpurun_out/prof_roctx.log 2>&1
