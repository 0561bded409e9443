#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_unet_gpu.py -k inference_mode \
  > gpurun_out/r04j_infmode.log 2>&1; tail -4 gpurun_out/r04j_infmode.log | cut -c1-400
bash tools/miopen_cache.sh gpurun_out/kcache
