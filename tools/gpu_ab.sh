#!/bin/bash
# A/B the headline bench over env settings on one box: gpu_ab.sh "A=0" "A=1" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-10}
for round in 1 2; do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python bench.py --steps $STEPS --warmup 3 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -30 gpurun_out/ab.err; exit 1; }
    echo "$round [$cfg] $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['value'], d['ms_per_step'])")"
  done
done
