#!/bin/bash
# ResNet-50 on one MI355X: BN kernel numerics, fused-vs-MIOpen BN img/s, MIOpen
# find-db capture (→ paddle_operator_amd/tuning/miopen), kernel profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O/miopen
export MIOPEN_USER_DB_PATH=$O/miopen
cd $R
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -m gpu -q -k bn > $O/t_bn.log 2>&1 &&
PDO_BN_FUSED=1 timeout -k 10 400 python tools/bench_resnet.py --steps 20 --warmup 5 > $O/rn_fused1_cold.json 2> $O/rn_fused1_cold.err &&
PDO_BN_FUSED=0 timeout -k 10 400 python tools/bench_resnet.py --steps 20 --warmup 5 > $O/rn_fused0.json 2> $O/rn_fused0.err &&
PDO_BN_FUSED=1 timeout -k 10 300 python tools/bench_resnet.py --steps 20 --warmup 5 > $O/rn_fused1_warm.json 2> $O/rn_fused1_warm.err &&
cd /tmp && export TMPDIR=/tmp && PDO_BN_FUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_rn -o run -- python3 $R/tools/bench_resnet.py --steps 5 --warmup 3 > $O/prof_rn.log 2>&1
rc=$?
cat $O/rn_*.json
exit $rc
