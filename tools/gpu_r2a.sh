#!/bin/bash
# round-2 GPU session A: GPU tests (incl. RCCL/IPC) → launched bench → RCCL sweep →
# kernel trace of a DDP-enabled step at world 1 (RCCL bucket kernels) → same-GPU 2-rank probe
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2a; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 --compat-trials 3 > $O/bench.json 2> $O/bench.err || { tail -80 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 bin/pdo-allreduce-bench --gpus 1 --min 1M --max 1G --iters 20 > $O/allreduce_bf16.jsonl 2>&1 || { cat $O/allreduce_bf16.jsonl | tail; exit 1; }
timeout -k 10 300 bin/pdo-allreduce-bench --gpus 1 --min 1M --max 1G --iters 20 --dtype f32 > $O/allreduce_f32.jsonl 2>&1 || exit 1
cd /tmp && PDO_DDP_ALWAYS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_ddp -o run -- python3 $R/tools/train_probe.py --dist --batch 64 --steps 3 --warmup 2 > $O/prof_ddp.log 2>&1 || { tail -30 $O/prof_ddp.log; exit 1; }
cd $R
DB=$(find $O/prof_ddp -name '*results.db' | head -1)
python tools/prof_summary.py $DB --steps 5 --title "GPT-2-medium B64 DDP(world1, RCCL) r2a" > $O/prof_ddp_summary.md 2>&1
python tools/overlap_summary.py $DB --title "GPT-2-medium B64, PDO_DDP_ALWAYS=1 world 1" > $O/overlap.md 2>&1

timeout -k 10 150 python tools/rccl_same_gpu_probe.py > $O/same_gpu.json 2>&1; echo "same_gpu rc=$?"; tail -3 $O/same_gpu.json
