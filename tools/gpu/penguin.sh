#!/bin/bash
# configs[2] against the reference fixture: single-rank fp32 / bf16 and the 4-rank sharded layout.
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-penguin}
mkdir -p gpurun_out
VP2P_PARITY_REPORT=$PWD/gpurun_out/${tag}_parity.jsonl timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread \
  tests/test_reference_gpu.py tests/test_frame_parallel.py -k "penguin" --durations=5 > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -8 gpurun_out/${tag}_tests.log; exit $rc
