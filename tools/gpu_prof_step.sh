#!/bin/bash
# kernel-trace profile of the GPT-2-medium step (in-process, RCCL world 1): gpu_prof_step.sh NAME
set -o pipefail
N=${1:-step}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$N; mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/train_probe.py --dist --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
python3 $R/tools/prof_summary.py $(find $O/prof -name '*.db' | head -1) --steps 5 --top 32 > $O/summary.md
grep tokens_per_s $O/prof.log | tail -1
cat $O/summary.md | head -45
