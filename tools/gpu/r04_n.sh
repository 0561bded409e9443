#!/bin/bash
# Round 4: plain projections all on K10 vs the chooser's table, in the 8-frame bench; then the small clips.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for m in table k10; do
  VP2P_LINEAR=$m timeout -k 10 300 python -u bench.py --extras none --no-cpu-baseline > gpurun_out/r04n_bench_$m.json \
    2> gpurun_out/r04n_bench_$m.err || exit 1
  tail -1 gpurun_out/r04n_bench_$m.json | cut -c1-160
done
bash tools/gpu/r04_m.sh
