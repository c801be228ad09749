#!/bin/bash
# gemm_nt4 grouped tile order A/B (PDO_NT_GROUP_M) on the GPT-2 NT shapes, then the numerics tests with the winner
set -o pipefail
O=gpurun_out/${1:-groupm}; mkdir -p $O
export TMPDIR=/tmp
for round in 1 2; do
  for g in 1 4 8 16; do
    PDO_NT_GROUP_M=$g timeout -k 10 300 python tools/nt4_probe.py --shapes wide_plain,fc2_dx,fc1_fwd,qkv_fwd,fc2_fwd --impls 1 --rounds 1 > $O/g${g}_$round.txt 2>&1 || { tail -20 $O/g${g}_$round.txt; exit 1; }
    echo "$round g=$g $(grep -o '"shape": "[a-z0-9_]*"\|"nt1_us": [0-9.]*' $O/g${g}_$round.txt | paste -s -d' ')"
  done
done
PDO_NT_GROUP_M=${G:-8} timeout -k 10 300 python -u -m pytest tests/test_gemm_nt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
