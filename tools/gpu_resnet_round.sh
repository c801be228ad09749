#!/bin/bash
# ResNet-50 on one MI355X: BN kernel numerics, fused-vs-MIOpen BN img/s (shipped
# MIOpen find-db), kernel profile.  CAPTURE_DB=1 records a fresh find-db into
# gpurun_out/miopen instead (→ paddle_operator_amd/tuning/miopen).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
if [ "${CAPTURE_DB:-0}" = 1 ]; then mkdir -p $O/miopen; export MIOPEN_USER_DB_PATH=$O/miopen; fi
cd $R
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -m gpu -q -k "bn or maxpool" > $O/t_bn.log 2>&1 &&
PDO_BN_FUSED=1 timeout -k 10 300 python tools/bench_resnet.py --steps 20 --warmup 5 > $O/rn_fused1.json 2> $O/rn_fused1.err &&
PDO_BN_FUSED=0 timeout -k 10 400 python tools/bench_resnet.py --steps 20 --warmup 5 > $O/rn_fused0.json 2> $O/rn_fused0.err &&
cd /tmp && export TMPDIR=/tmp && PDO_BN_FUSED=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_rn -o run -- python3 $R/tools/bench_resnet.py --steps 5 --warmup 3 > $O/prof_rn.log 2>&1
rc=$?
tail -3 $O/t_bn.log
cat $O/rn_*.json
exit $rc
