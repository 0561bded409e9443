#!/bin/bash
# The whole GPU suite on the product library (+ the parity report of every recorded test).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
VP2P_PARITY_REPORT=$PWD/gpurun_out/suite_parity.jsonl timeout -k 10 1080 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread --durations=25 \
  > gpurun_out/suite_gpu_suite.log 2>&1
rc=$?; tail -5 gpurun_out/suite_gpu_suite.log; exit $rc
