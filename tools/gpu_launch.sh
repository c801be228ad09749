#!/bin/bash
# launch-latency on one GPU: compat / fast / fast+zygote, noop + resnet50 ranks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench_launch.py --ranks 1 --trials ${TRIALS:-5} --workload noop > gpurun_out/launch_noop.jsonl 2> gpurun_out/launch_noop.err || { tail -30 gpurun_out/launch_noop.err; exit 1; }
cat gpurun_out/launch_noop.jsonl
timeout -k 10 500 python bench_launch.py --ranks 1 --trials 3 --workload resnet50 --modes fast,fast+zygote > gpurun_out/launch_resnet.jsonl 2> gpurun_out/launch_resnet.err || { tail -30 gpurun_out/launch_resnet.err; exit 1; }
cat gpurun_out/launch_resnet.jsonl
