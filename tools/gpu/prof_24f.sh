#!/bin/bash
# Kernel stats of one timed edit at configs[1] (rabbit, 8 frames) and configs[2] (penguin, 24 frames)
# on the same box: why per-launch efficiency differs between the two.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "rabbit 8" "penguin 24"; do
  set -- $cfg
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/p24_$1 -o run -- \
    python3 bench.py --edit $1 --frames $2 --steps 1 --warmup 1 --extras none --no-cpu-baseline \
    > gpurun_out/p24_$1.json 2> gpurun_out/p24_$1.err || exit 1
  tail -1 gpurun_out/p24_$1.json | cut -c1-160
done
python3 tools/trace_by_shape.py gpurun_out/p24_rabbit/run_kernel_trace.csv gpurun_out/p24_penguin/run_kernel_trace.csv > gpurun_out/p24_compare.txt || exit 1
rm -f gpurun_out/p24_*/run_kernel_trace.csv
head -60 gpurun_out/p24_compare.txt
