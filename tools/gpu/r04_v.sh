#!/bin/bash
# Round 4: bench line + kernel stats after the GEGLU epilogue and the fused norm2 statistics.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r04v_bench.json 2> gpurun_out/r04v_bench.err || exit 1
tail -1 gpurun_out/r04v_bench.json | cut -c1-200
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04v_prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/r04v_bench_profiled.json 2> gpurun_out/r04v_prof.err || exit 1
rm -f gpurun_out/r04v_prof/run_kernel_trace.csv
echo done
