#!/bin/bash
# Round 4: the 64-row K10 tile (small clips): conv tests, then the small-shape A/B against split-K.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py \
  > gpurun_out/r04g_conv_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r04g_conv_tests.log; [ $rc -ne 0 ] && exit $rc
L=video-p2p_amd/lib/lab
for v in $PWD/video-p2p_amd/lib/libvp2p_hip.so $L/libvp2p_k10s256.so $L/libvp2p_k10noshort.so; do
  VP2P_LIB=$v timeout -k 10 200 python -u tools/k10_small_bench.py gpurun_out/r04g_k10_small.jsonl > /dev/null || exit 1
done

# K10 diagnostics: the same launches without the main-loop DMA (1) and without DMA or barriers (3)
for v in $PWD/video-p2p_amd/lib/libvp2p_hip.so $L/libvp2p_k10diag1.so $L/libvp2p_k10diag3.so; do
  VP2P_LIB=$v timeout -k 10 200 python -u tools/k10_bench.py gpurun_out/r04g_k10_diag.jsonl > /dev/null || exit 1
done
echo diag done
