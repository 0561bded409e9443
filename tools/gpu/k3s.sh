#!/bin/bash
# K3s: the GPU tests of K3 (stream vs short kernel vs oracle), then the timing A/B (ring depths), then
# (if built) lab builds without stores (diag1) / without DMA (diag4).
#   bash tools/gpu/k3s.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k3s}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "temporal" \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
timeout -k 10 300 python -u tools/k3_stream_ab.py gpurun_out/${tag}_ab.jsonl || exit 1
for d in 1 4; do
  L=$PWD/video-p2p_amd/lib/diag/libvp2p_k3diag$d.so
  [ -f $L ] || continue
  K3AB_MODES=3 K3AB_SHAPES=1 VP2P_LIB=$L timeout -k 10 120 python -u tools/k3_stream_ab.py gpurun_out/${tag}_d$d.jsonl || exit 1
done
echo done
