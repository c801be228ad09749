#!/bin/bash
# PMC passes over gemm_nt impl 0 vs impl 1 on one shape (N K as args)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/nt4pmc; mkdir -p $O
cd /tmp
N=${1:-1024}; K=${2:-4096}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum"
for impl in 0 3; do
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    D=$O/i${impl}_p$i
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $D -o run -- python3 $R/tools/nt_only.py $N $K 3 $impl > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $(find $O -path "*i${impl}_p*" -name '*.db') --filter pdo > $O/summary_i$impl.txt 2>&1
  cat $O/summary_i$impl.txt
done
