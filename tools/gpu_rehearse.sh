#!/bin/bash
# multi-rank launched GPU path rehearsed on ONE GPU (ranks share it over gloo): gpu_rehearse.sh NAME [N...]
set -o pipefail
O=gpurun_out/${1:-rehearse}; mkdir -p $O; shift
export TMPDIR=/tmp
for n in ${@:-2}; do
  PDO_BENCH_LOG_TAIL=20000 timeout -k 10 420 python bench.py --gpus $n --rehearse-shared-gpu --micro-batch ${MB:-32} --steps 2 --warmup 1 --ready-trials 2 --timeout 200 > $O/n$n.json 2> >(tee $O/n$n.err >&2) || { echo "N=$n failed"; exit 1; }
  cat $O/n$n.json
done
