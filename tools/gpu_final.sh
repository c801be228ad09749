#!/bin/bash
# end-of-session validation: pytest -m gpu, smoke(), launched bench, then the step kernel table (gpu_final.sh NAME)
set -o pipefail
N=${1:-final}
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$N; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -80 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -40 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -60 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/tools/train_probe.py --dist --steps 7 --warmup 2 > $O/prof.log 2>&1 || { tail -30 $O/prof.log; exit 1; }
DB=$(find $O/prof -name '*.db' | head -1)
python3 $R/tools/prof_summary.py $DB --steps 7 --top 32 > $O/summary.md
rm -rf $O/prof
grep tokens_per_s $O/prof.log | tail -1
head -30 $O/summary.md
