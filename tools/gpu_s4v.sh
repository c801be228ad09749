#!/bin/bash
# validation after the bootstrap store change: GPU suite, smoke, launched bench, 2-rank shared-GPU rehearsal
set -o pipefail
O=gpurun_out/${1:-s4v}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -40 $O/bench.err; exit 1; }
cat $O/bench.json
MB=16 bash tools/gpu_rehearse.sh $(basename $O)_reh 2 3
