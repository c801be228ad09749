#!/bin/bash
# Launched-rank vs in-process step time on one box (where do the ms go?)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
v() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(d.get('value', d.get('tokens_per_s')), d.get('ms_per_step'))" "$1"; }
for round in 1 2; do
  timeout -k 10 300 python tools/train_probe.py --dist --steps 20 --warmup 5 > gpurun_out/g.json 2> gpurun_out/g.err || { tail -20 gpurun_out/g.err; exit 1; }
  echo "$round in-process $(v gpurun_out/g.json)"
  for flags in "" "--no-warm-slots" "--no-zygote"; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --ready-trials 1 $flags > gpurun_out/g.json 2> gpurun_out/g.err || { tail -20 gpurun_out/g.err; exit 1; }
    echo "$round launched [$flags] $(v gpurun_out/g.json)"
  done
done
