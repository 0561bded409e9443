#!/bin/bash
# Round 4: the whole GPU suite on the product library.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
VP2P_PARITY_REPORT=$PWD/gpurun_out/r04h_parity.jsonl timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=25 \
  > gpurun_out/r04h_gpu_suite.log 2>&1
rc=$?; tail -5 gpurun_out/r04h_gpu_suite.log; exit $rc
