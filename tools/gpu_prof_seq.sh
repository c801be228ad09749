#!/bin/bash
# kernel-trace profile of the GPT-2-medium step + the last step's kernel sequence and device-idle gaps: gpu_prof_seq.sh NAME
set -o pipefail
N=${1:-seq}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$N; mkdir -p $O
cd /tmp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/train_probe.py --dist --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
DB=$(find $O/prof -name '*.db' | head -1)
python3 $R/tools/prof_summary.py $DB --steps 5 --top 40 > $O/summary.md
python3 $R/tools/prof_sequence.py $DB --last 1078 --list > $O/sequence.md
grep tokens_per_s $O/prof.log | tail -1
head -12 $O/sequence.md
rm -rf $O/prof
