#!/bin/bash
# Round 4: issue microbenchmark; K1 pipelined variants with part of the exps as a packed polynomial.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/issue_bench > gpurun_out/r04f_issue_bench.jsonl || exit 1
cat gpurun_out/r04f_issue_bench.jsonl
L=video-p2p_amd/lib/lab
for v in pp2w8p12 pp2w8p55 pp3w4p12; do
  VP2P_LIB=$PWD/$L/libvp2p_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_kernels_gpu.py -k "frame_attention" > gpurun_out/r04f_tests_$v.log 2>&1
  rc=$?; echo "tests $v rc=$rc"; tail -1 gpurun_out/r04f_tests_$v.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u tools/k1_lab.py gpurun_out/r04f_k1_ab.jsonl $L/libvp2p_x2f.so $L/libvp2p_pp2w8.so \
  $L/libvp2p_pp2w8p12.so $L/libvp2p_pp2w8p55.so $L/libvp2p_pp3w4p12.so
