#!/bin/bash
# Round 4: K1 pipelined kernel (SETS=3) vs x2f timing at res-64 / res-32.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/k1_lab.py gpurun_out/r04b_k1_ab.jsonl video-p2p_amd/lib/lab/libvp2p_x2f.so \
  video-p2p_amd/lib/lab/libvp2p_pp3.so
