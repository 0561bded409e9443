#!/bin/bash
# Kernel-level split of tools/k2_bench.py (v3 / v3e / LocalBlend reduce per case) under rocprofv3.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/k2prof -o run -- \
  python3 tools/k2_bench.py --iters 20 > gpurun_out/k2prof.json 2> gpurun_out/k2prof.err || exit 1
python3 tools/trace_by_shape.py gpurun_out/k2prof/run_kernel_trace.csv > gpurun_out/k2prof_shapes.txt || exit 1
rm -f gpurun_out/k2prof/run_kernel_trace.csv
grep -i "cross\|lb_reduce\|kv_prep" gpurun_out/k2prof_shapes.txt
