#!/bin/bash
# Round 4, K1 pipelined kernel: parity of the lab builds on the frame-attention kernel tests, then
# the res-64 / res-32 timing A/B against x2f.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for v in pp3 pp4; do
  VP2P_LIB=$PWD/video-p2p_amd/lib/lab/libvp2p_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_kernels_gpu.py -k "frame_attention" > gpurun_out/r04a_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -3 gpurun_out/r04a_tests_$v.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u tools/k1_lab.py gpurun_out/r04a_k1_ab.jsonl video-p2p_amd/lib/lab/libvp2p_x2f.so \
  video-p2p_amd/lib/lab/libvp2p_pp3.so video-p2p_amd/lib/lab/libvp2p_pp4.so
