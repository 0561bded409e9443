#!/bin/bash
# Round 4: K1 pipelined variants (3 sets x 4 waves, 2 sets x 8 waves): kernel tests, then timing vs x2f.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for v in pp3w4 pp2w8; do
  VP2P_LIB=$PWD/video-p2p_amd/lib/lab/libvp2p_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_kernels_gpu.py -k "frame_attention" > gpurun_out/r04d_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -2 gpurun_out/r04d_tests_$v.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python -u tools/k1_lab.py gpurun_out/r04d_k1_ab.jsonl video-p2p_amd/lib/lab/libvp2p_x2f.so \
  video-p2p_amd/lib/lab/libvp2p_pp3w4.so video-p2p_amd/lib/lab/libvp2p_pp2w8.so
