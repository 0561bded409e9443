#!/bin/bash
# PMC of tools/k2_bench.py's kernels: wave-cycle split and instruction-cache behaviour.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/k2pmc
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAVES \
  --kernel-trace --output-format csv -d gpurun_out/k2pmc/A -o run -- python3 tools/k2_bench.py --iters 5 > gpurun_out/k2pmc/A.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS \
  --kernel-trace --output-format csv -d gpurun_out/k2pmc/B -o run -- python3 tools/k2_bench.py --iters 5 > gpurun_out/k2pmc/B.log 2>&1 || exit 1
echo ok
