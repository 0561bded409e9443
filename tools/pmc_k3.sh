#!/bin/bash
# PMC passes on K3 (tools/k3_only.py, res-64 B4 f8, self-replace on): bash tools/pmc_k3.sh OUTDIR
set -e
out=$1; mkdir -p $out
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES"
C="FETCH_SIZE"
D="WRITE_SIZE"
for p in A B C D; do
  timeout -s KILL 90 rocprofv3 --pmc ${!p} --kernel-trace --output-format csv -d $out/$p -o run -- python3 tools/k3_only.py 5 > $out/$p.log 2>&1
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $out/T -o run -- python3 tools/k3_only.py 20 > $out/T.log 2>&1
