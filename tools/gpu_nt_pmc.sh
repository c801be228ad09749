#!/bin/bash
# PMC passes over gemm_nt vs hipBLASLt (one pass per counter group)
set -o pipefail
mkdir -p gpurun_out
cd /tmp
R=$GRAFT_REPO_ROOT
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  (timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/ntpmc$i -o run -- python3 $R/tools/nt_only.py 1024 4096 3 > $R/gpurun_out/ntpmc$i.log 2>&1) || { tail -20 $R/gpurun_out/ntpmc$i.log; exit 1; }
done
