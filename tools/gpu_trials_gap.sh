#!/bin/bash
# Does the number of ready trials before the bench job change its step time?
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PDO_BENCH_PS=1
for n in 1 10 1 10; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ready-trials $n > gpurun_out/t.json 2> gpurun_out/t$n.err || { tail -20 gpurun_out/t$n.err; exit 1; }
  echo "trials=$n $(python -c "import json;d=json.loads(open('gpurun_out/t.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])")"
  grep descendant gpurun_out/t$n.err
done
