#!/bin/bash
# A/B built extension variants on one box: ab/<name>.so are copied in turn over
# paddle_operator_amd/_pdo_hip.so and "$@" is run with each (2 interleaved rounds);
# the tree's own .so is restored at the end.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cp paddle_operator_amd/_pdo_hip.so gpurun_out/.tree_hip.so
rc=0
for round in 1 2; do
  for v in ab/*.so; do
    cp "$v" paddle_operator_amd/_pdo_hip.so
    out=$(timeout -k 10 300 "$@" 2> gpurun_out/so_ab.err) || { rc=$?; tail -20 gpurun_out/so_ab.err; break 2; }
    echo "$round $(basename "$v" .so) $out"
  done
done
cp gpurun_out/.tree_hip.so paddle_operator_amd/_pdo_hip.so
rm -f gpurun_out/.tree_hip.so
exit $rc
