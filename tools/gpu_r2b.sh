#!/bin/bash
# round-2 GPU session B: per-shape GEMM table (gemm_nt vs hipBLASLt, gemm_dw),
# ready-latency breakdown + RCCL init env A/B, rccl-trace availability
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r2b; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python tools/nt_probe.py --iters 20 > $O/nt_probe.jsonl 2> $O/nt_probe.err || { tail -30 $O/nt_probe.err; exit 1; }
cat $O/nt_probe.jsonl
timeout -k 10 300 python tools/dw_probe.py --pdo-only > $O/dw_probe.jsonl 2> $O/dw_probe.err || { tail -30 $O/dw_probe.err; exit 1; }
cat $O/dw_probe.jsonl
timeout -k 10 300 python bench.py --ready-only --ready-trials 10 > $O/ready_default.json 2> $O/ready_default.err || { tail -40 $O/ready_default.err; exit 1; }
cat $O/ready_default.json
NCCL_IB_DISABLE=1 RCCL_MSCCL_ENABLE=0 RCCL_MSCCLPP_ENABLE=0 NCCL_NET_PLUGIN=none timeout -k 10 300 python bench.py --ready-only --ready-trials 10 > $O/ready_env1.json 2> $O/ready_env1.err || { tail -40 $O/ready_env1.err; exit 1; }
cat $O/ready_env1.json
cd /tmp && PDO_DDP_ALWAYS=1 timeout -k 10 300 rocprofv3 --kernel-trace --rccl-trace --stats -d $O/prof_rccl -o run -- python3 $R/tools/train_probe.py --dist --model gpt2 --batch 8 --seq 1024 --steps 2 --warmup 1 > $O/prof_rccl.log 2>&1; echo "rccl-trace rc=$?"
find $O/prof_rccl -name '*.db' | head; tail -5 $O/prof_rccl.log
