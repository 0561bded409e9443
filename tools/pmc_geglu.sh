#!/bin/bash
# PMC passes on the fused K10 GEGLU projection (tools/geglu_only.py) -> OUTDIR/{A,B,C}
#   bash tools/pmc_geglu.sh OUTDIR M K INNER
set -e
out=$1; shift; mkdir -p $out
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES"
C="SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES SQ_WAVE_CYCLES"
for p in A B C; do
  timeout -s KILL 90 rocprofv3 --pmc ${!p} --kernel-trace --output-format csv -d $out/$p -o run -- python3 tools/geglu_only.py "$@" 5 > $out/$p.log 2>&1
done
