#!/bin/bash
# per-kernel in-step times (rocprofv3 --kernel-trace --stats) for env settings: gpu_env_kprof.sh NAME "A=1" "A=2" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; shift
cd /tmp
export TMPDIR=/tmp
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p$i -o run -- python3 $R/tools/train_probe.py --dist --steps 5 --warmup 2 > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  DB=$(find $O/p$i -name '*.db' | head -1)
  python3 $R/tools/prof_summary.py $DB --steps 7 --top 12 > $O/s$i.md
  rm -rf $O/p$i
  echo "[$cfg] $(grep tokens_per_s $O/p$i.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  grep -E "gemm_nt4|Cijk|gemm_dw4|attn_fwd" $O/s$i.md | cut -c1-160
done
