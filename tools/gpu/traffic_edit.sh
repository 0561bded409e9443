#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of every kernel of a 5-DDIM-step configs[1] edit (bench.py), by launch
# shape -> gpurun_out/traffic_edit/summary.txt   (tools/traffic_by_kernel.py)
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/traffic_edit
mkdir -p $out
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $out/$c -o run -- \
    python3 -u bench.py --steps 1 --warmup 0 --ddim-steps 5 --extras none --no-cpu-baseline > $out/$c.log 2>&1 || { tail -5 $out/$c.log; exit 1; }
done
python3 tools/traffic_by_kernel.py $out/FETCH_SIZE/run_counter_collection.csv $out/WRITE_SIZE/run_counter_collection.csv 60 > $out/summary.txt || exit 1
rm -f $out/*/run_counter_collection.csv $out/*/run_kernel_trace.csv
head -70 $out/summary.txt
