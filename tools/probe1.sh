#!/bin/bash
# first GPU probe: environment + torch-ops baseline of the GPT-2-medium step
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
(rocm-smi --showtopo; rocm-smi; rocminfo | grep -E "Marketing|gfx|Compute Unit" | head -20) > gpurun_out/env.txt 2>&1 || true
timeout -k 10 300 python -c "import torch;print(torch.cuda.get_device_properties(0))" >> gpurun_out/env.txt 2>&1 || exit 1
for mb in 8 16 32; do
  timeout -k 10 300 python bench.py --ops torch --micro-batch $mb --steps 6 --warmup 3 >> gpurun_out/probe1.jsonl 2>> gpurun_out/probe1.err || exit 1
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_torch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --ops torch --micro-batch 16 --steps 3 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_torch.log 2>&1 || exit 1
