#!/bin/bash
# PMC passes over gemm_nt vs hipBLASLt (one pass per counter group) on two shapes
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ntpmc; mkdir -p $O
cd /tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
for S in "1024 4096" "3072 1024"; do
  set -- $S
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    D=$O/n$1k$2_p$i
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $D -o run -- python3 $R/tools/nt_only.py $1 $2 3 > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
  done
  python3 $R/tools/pmc_summary.py $(find $O -path "*n$1k$2_p*" -name '*.db') > $O/summary_n$1k$2.txt 2>&1
  cat $O/summary_n$1k$2.txt
done
