#!/bin/bash
# One LDS/issue PMC pass of K1 (tools/k1_only.py) per library: the product and video-p2p_amd/lib/ab/*.so.
#   bash tools/gpu/k1_pmc_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k1pmc}
mkdir -p gpurun_out
export TMPDIR=/tmp
P="SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
for lib in video-p2p_amd/lib/libvp2p_hip.so video-p2p_amd/lib/ab/*.so; do
  n=$(basename $lib .so)
  VP2P_LIB=$PWD/$lib timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/${tag}_$n -o run -- \
    python3 tools/k1_only.py 5 > gpurun_out/${tag}_$n.log 2>&1 || exit 1
  python3 tools/pmc_summary.py frame_attn_kernel_pp gpurun_out/${tag}_$n | sed "s/^/$n /"
done
