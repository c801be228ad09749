#!/bin/bash
# GPU visibility modes: GPU suite, launched bench with all-visible (default) and isolate, 2-rank rehearsal
set -o pipefail
O=gpurun_out/${1:-s4vis}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_all.json 2> $O/bench_all.err || { tail -40 $O/bench_all.err; exit 1; }
cat $O/bench_all.json
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 --gpu-visibility isolate > $O/bench_iso.json 2> $O/bench_iso.err || { tail -40 $O/bench_iso.err; exit 1; }
cat $O/bench_iso.json
MB=16 bash tools/gpu_rehearse.sh $(basename $O)_reh 2
