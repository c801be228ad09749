#!/bin/bash
# one GPU session: numerics tests → bench (hip ops) → kernel-trace profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MB=${MB:-16}
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for mb in $MB; do
  timeout -k 10 300 python bench.py --micro-batch $mb --steps 10 --warmup 3 >> gpurun_out/bench_hip.jsonl 2>> gpurun_out/bench_hip.err || { tail -20 gpurun_out/bench_hip.err; exit 1; }
done
cat gpurun_out/bench_hip.jsonl
if [ -n "$PROF" ]; then
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_hip -o run -- python3 $GRAFT_REPO_ROOT/bench.py --micro-batch 16 --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_hip.log 2>&1) || exit 1
fi
if [ -n "$TUNE" ]; then
  export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$GRAFT_REPO_ROOT/gpurun_out/tunableop_results%d.csv PYTORCH_TUNABLEOP_VERBOSE=1
  timeout -k 10 900 python bench.py --micro-batch $TUNE --steps 10 --warmup 3 >> gpurun_out/bench_tune.jsonl 2> gpurun_out/bench_tune.err || { tail -20 gpurun_out/bench_tune.err; exit 1; }
  export PYTORCH_TUNABLEOP_TUNING=0
  timeout -k 10 300 python bench.py --micro-batch $TUNE --steps 10 --warmup 3 >> gpurun_out/bench_tune.jsonl 2>> gpurun_out/bench_tune.err || exit 1
  cat gpurun_out/bench_tune.jsonl
fi
if [ -n "$RESNET" ]; then
  timeout -k 10 400 python -m paddle_operator_amd.launch --workload resnet50 --batch $RESNET --steps 30 --log-every 10 > gpurun_out/resnet50.log 2>&1 || { tail -30 gpurun_out/resnet50.log; exit 1; }
  grep -E "PDO_READY|PDO_DONE|step" gpurun_out/resnet50.log
fi
