#!/bin/bash
# K3s timing diagnostics: the product stream (ring 3) against lab builds without stores / compute / DMA.
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k3diag}
mkdir -p gpurun_out
export K3AB_MODES=3 K3AB_SHAPES=1
timeout -k 10 120 python -u tools/k3_stream_ab.py gpurun_out/${tag}_prod.jsonl || exit 1
for d in 1 2 3 4; do
  VP2P_LIB=$PWD/video-p2p_amd/lib/diag/libvp2p_k3diag$d.so timeout -k 10 120 python -u tools/k3_stream_ab.py gpurun_out/${tag}_d$d.jsonl || exit 1
done
echo done
