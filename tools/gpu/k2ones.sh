#!/bin/bash
# K2 ones-row A/B: the K2 kernel tests and the reference edit tests under the variant library, then
# k2_bench (producer timing) with the product library and the variant, two rounds.
# usage: tools/gpu/k2ones.sh TAG VARIANT.so
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k2ones}; var=$(realpath $2)
mkdir -p gpurun_out
VP2P_LIB=$var timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_reference_gpu.py \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
K2AB_PRODUCER=1 bash tools/gpu/k2_ab.sh gpurun_out/${tag}.jsonl video-p2p_amd/lib/libvp2p_hip.so $var > /dev/null || exit 1
echo done
