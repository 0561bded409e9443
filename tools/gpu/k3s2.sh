#!/bin/bash
# K3s lab runs: producer-before-launch timing of the product (short vs ring 2/3/4), the contiguous item
# order, the no-store / no-DMA builds, and the flushed-cache form of the product.
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k3s}
mkdir -p gpurun_out
export K3AB_SHAPES=1
timeout -k 10 200 python -u tools/k3_stream_ab.py gpurun_out/${tag}_ab.jsonl || exit 1
K3AB_PRODUCER=0 timeout -k 10 200 python -u tools/k3_stream_ab.py gpurun_out/${tag}_flush.jsonl || exit 1
for n in k3order k3diag1 k3diag4; do
  K3AB_MODES=0,2,3,4 VP2P_LIB=$PWD/video-p2p_amd/lib/diag/libvp2p_$n.so timeout -k 10 200 python -u tools/k3_stream_ab.py gpurun_out/${tag}_$n.jsonl || exit 1
done
echo done
