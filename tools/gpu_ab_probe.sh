#!/bin/bash
# A/B the in-process GPT-2-medium step over env settings on one box:
#   gpu_ab_probe.sh "A=0" "A=1" ...   (2 interleaved rounds; STEPS env, default 20)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-20}
for round in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python tools/train_probe.py --dist --steps $STEPS --warmup 3 > gpurun_out/abp.json 2> gpurun_out/abp.err || { tail -30 gpurun_out/abp.err; exit 1; }
    echo "$round [$cfg] $(tail -1 gpurun_out/abp.json)"
  done
done
