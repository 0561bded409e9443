#!/bin/bash
# K1 d = 160 one-set geometry A/B (tools/k1_d160_ab.py) + the K1 kernel tests on the product form.
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k1d160}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "frame_attention" \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -u tools/k1_d160_ab.py gpurun_out/${tag}_ab.jsonl || exit 1
echo done
