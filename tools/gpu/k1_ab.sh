#!/bin/bash
# K1 kernel tests, then the K1 A/B (tools/k1_lab.py) of the product library against lab builds in
# video-p2p_amd/lib/ab/, then the LDS-conflict / MFMA PMC pass of the product K1.
#   bash tools/gpu/k1_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k1ab}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "frame_attention" \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 400 python -u tools/k1_lab.py gpurun_out/${tag}.jsonl video-p2p_amd/lib/libvp2p_hip.so video-p2p_amd/lib/ab/*.so || exit 1
export TMPDIR=/tmp
P="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/${tag}_pmc -o run -- \
  python3 tools/k1_only.py 5 > gpurun_out/${tag}_pmc.log 2>&1 || exit 1
echo done
