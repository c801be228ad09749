#!/bin/bash
# per-kernel A/B of built extension variants in the training step: each ab/<name>.so
# under rocprofv3 --kernel-trace; prints the summary rows matching $MATCH (default attn_)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/soprof; mkdir -p $O
export TMPDIR=/tmp
MATCH=${MATCH:-attn_}
cp $R/paddle_operator_amd/_pdo_hip.so $O/.tree_hip.so
rc=0
for v in $R/ab/*.so; do
  n=$(basename $v .so)
  cp $v $R/paddle_operator_amd/_pdo_hip.so
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$n -o run -- python3 $R/tools/train_probe.py --dist --steps 4 --warmup 2 > $O/$n.log 2>&1) || { rc=$?; tail -20 $O/$n.log; break; }
  echo "== $n $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log)"
  python3 $R/tools/prof_summary.py $(find $O/$n -name '*.db' | head -1) --steps 6 --top 40 | grep -E "$MATCH"
done
cp $O/.tree_hip.so $R/paddle_operator_amd/_pdo_hip.so
exit $rc
