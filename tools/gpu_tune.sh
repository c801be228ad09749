#!/bin/bash
# retune the shipped TunableOp table for the current GEMM set, re-bench with it, profile
set -o pipefail
mkdir -p gpurun_out
MB=${MB:-32}
export PDO_TUNE_MS=${PDO_TUNE_MS:-60}
PDO_TUNE_GEMMS=1 PDO_TUNE_OUT=$GRAFT_REPO_ROOT/gpurun_out/tune0.csv timeout -k 10 900 python bench.py --micro-batch $MB --steps 2 --warmup 1 > gpurun_out/tune_run.log 2>&1 || { tail -20 gpurun_out/tune_run.log; exit 1; }
python tools/merge_tune.py gpurun_out/tune0.csv paddle_operator_amd/tuning/tunableop_gpt2-medium_b${MB}_gfx950.csv || exit 1
cp paddle_operator_amd/tuning/tunableop_gpt2-medium_b${MB}_gfx950.csv gpurun_out/merged_b${MB}.csv
timeout -k 10 300 python bench.py --micro-batch $MB --steps 10 --warmup 3 > gpurun_out/bench_tuned.jsonl 2> gpurun_out/bench_tuned.err || { tail -20 gpurun_out/bench_tuned.err; exit 1; }
cat gpurun_out/bench_tuned.jsonl
if [ -n "$PROF" ]; then
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r1c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --micro-batch $MB --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_r1c.log 2>&1) || exit 1
fi
