#!/bin/bash
# Round 4: PMC passes (tools/pmc_k1.sh) on the x2f and pp3 K1 builds + the gfx950 counter list.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r04c_counters.txt 2>&1
for v in x2f pp3; do
  VP2P_LIB=$PWD/video-p2p_amd/lib/lab/libvp2p_$v.so bash tools/pmc_k1.sh gpurun_out/r04c_pmc_$v || exit 1
done
python tools/pmc_summary.py frame_attn gpurun_out/r04c_pmc_x2f/A gpurun_out/r04c_pmc_x2f/B gpurun_out/r04c_pmc_x2f/C > gpurun_out/r04c_pmc_summary.txt
python tools/pmc_summary.py frame_attn gpurun_out/r04c_pmc_pp3/A gpurun_out/r04c_pmc_pp3/B gpurun_out/r04c_pmc_pp3/C >> gpurun_out/r04c_pmc_summary.txt
cat gpurun_out/r04c_pmc_summary.txt
