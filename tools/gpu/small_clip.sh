#!/bin/bash
# Small-clip edit times (1 / 2 / 3 frames, eager and per-step HIP graphs) + the 1-frame kernel stats.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
for f in 1 2 3; do for g in 0 1; do
  timeout -k 10 240 python -u bench.py --frames $f --graphs $g --steps 2 --warmup 1 --extras none --no-cpu-baseline \
    --no-events > gpurun_out/sc_f${f}_g${g}.json 2> gpurun_out/sc_f${f}_g${g}.err || exit 1
  tail -1 gpurun_out/sc_f${f}_g${g}.json | cut -c1-220
done; done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sc_prof -o run -- \
  python3 bench.py --frames 1 --graphs 1 --steps 1 --warmup 1 --extras none --no-cpu-baseline --no-events \
  > gpurun_out/sc_prof.json 2> gpurun_out/sc_prof.err || exit 1
python3 tools/trace_by_shape.py gpurun_out/sc_prof/run_kernel_trace.csv > gpurun_out/sc_prof_shapes.txt || exit 1
rm -f gpurun_out/sc_prof/run_kernel_trace.csv
echo done
