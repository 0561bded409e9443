#!/bin/bash
# rocprofv3 kernel trace + one SQ/GRBM PMC pass of the d = 160 K1 launches (resident kernel and the
# one-set kernel, VP2P_K1_D160=0).
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k1d160p}
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 1 0; do
  VP2P_K1_D160=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_T$v -o run -- \
    python3 tools/k1_d160_only.py 20 > gpurun_out/${tag}_T$v.log 2>&1 || exit 1
  VP2P_K1_D160=$v timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT \
    --kernel-trace --output-format csv -d gpurun_out/${tag}_P$v -o run -- python3 tools/k1_d160_only.py 5 > gpurun_out/${tag}_P$v.log 2>&1 || exit 1
done
rm -f gpurun_out/${tag}_T*/run_kernel_trace.csv
echo done
