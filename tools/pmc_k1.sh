#!/bin/bash
# PMC passes on K1 (tools/k1_only.py) for the variants given: bash tools/pmc_k1.sh OUTDIR VAR...
set -e
out=$1; shift; mkdir -p $out
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES"
for v in "$@"; do
  for p in A B; do
    VP2P_K1_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc ${!p} --kernel-trace --output-format csv -d $out/v${v}_$p -o run -- python3 tools/k1_only.py 5 > $out/v${v}_$p.log 2>&1
  done
done
