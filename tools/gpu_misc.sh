#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/lt_probe.py > gpurun_out/lt_probe.log 2>&1 || { tail -20 gpurun_out/lt_probe.log; exit 1; }
cat gpurun_out/lt_probe.log
# multi-rank GPU rehearsal: 2 ranks on the one GPU over gloo (RCCL needs one GPU per rank)
PDO_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --micro-batch 8 > gpurun_out/bench_gloo2.log 2>&1 || { tail -30 gpurun_out/bench_gloo2.log; exit 1; }
grep metric gpurun_out/bench_gloo2.log
