#!/bin/bash
# PMC passes: gemm_nt4 (impl 1) and hipBLASLt side by side on one shape (default: the wide K=1024 shape)
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${3:-widepmc}; mkdir -p $O
cd /tmp
N=${1:-4096}; K=${2:-1024}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"
P3="SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_WR SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  D=$O/p$i
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d $D -o run -- python3 $R/tools/nt_only.py $N $K 3 1 > $D.log 2>&1 || { tail -20 $D.log; exit 1; }
done
python3 $R/tools/pmc_summary.py $(find $O -name '*.db') > $O/summary.txt 2>&1
cat $O/summary.txt
find $O -name '*.db' -delete
