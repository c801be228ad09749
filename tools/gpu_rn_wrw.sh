#!/bin/bash
# ResNet-50 A/B: MIOpen's GTC NHWC weight-gradient solver (atomic split-K: zero-fill + cast passes) on / off
set -o pipefail
O=gpurun_out/${1:-rnwrw}; mkdir -p $O
export TMPDIR=/tmp
for round in 1 2; do
  timeout -k 10 300 python tools/bench_resnet.py --steps 20 --warmup 10 > $O/on_$round.json 2> $O/on_$round.err || { tail -20 $O/on_$round.err; exit 1; }
  echo "$round on  $(tail -1 $O/on_$round.json)"
  MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 timeout -k 10 300 python tools/bench_resnet.py --steps 20 --warmup 10 > $O/off_$round.json 2> $O/off_$round.err || { tail -20 $O/off_$round.err; exit 1; }
  echo "$round off $(tail -1 $O/off_$round.json)"
done
