#!/bin/bash
# kernel-trace profile of the ResNet-50 step (in-process, batch 256): gpu_prof_resnet.sh NAME
set -o pipefail
N=${1:-rn}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$N; mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/bench_resnet.py --steps 5 --warmup 3 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
DB=$(find $O/prof -name '*.db' | head -1)
python3 $R/tools/prof_summary.py $DB --steps 8 --top 30 > $O/summary.md
python3 $R/tools/prof_shapes.py $DB --match bn_ --steps 8 > $O/bn_shapes.md
tail -2 $O/prof.log
head -40 $O/summary.md
cat $O/bn_shapes.md
