#!/bin/bash
# Small-clip edit times (SC_FRAMES, default 1 2 3; eager and per-step HIP graphs) + the kernel trace of
# one graphed SC_PROF_FRAMES-frame edit (default 1), per launch shape.
# usage: tools/gpu/small_clip.sh [TAG]
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-sc}
mkdir -p gpurun_out
for f in ${SC_FRAMES:-1 2 3}; do for g in 0 1; do
  timeout -k 10 240 python -u bench.py --frames $f --graphs $g --steps 2 --warmup 1 --extras none --no-cpu-baseline \
    --no-events > gpurun_out/${tag}_f${f}_g${g}.json 2> gpurun_out/${tag}_f${f}_g${g}.err || exit 1
  tail -1 gpurun_out/${tag}_f${f}_g${g}.json | cut -c1-220
  python3 -c "
import json
d=json.loads(open('gpurun_out/${tag}_f${f}_g${g}.json').read().strip().splitlines()[-1])
print(json.dumps({'frames': $f, 'graphs': $g, 'ms_per_edit': d['ms_per_step'], 'value': d['value']}))" >> gpurun_out/${tag}.jsonl || exit 1
done; done
export TMPDIR=/tmp
pf=${SC_PROF_FRAMES:-1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --frames $pf --graphs 1 --steps 1 --warmup 1 --extras none --no-cpu-baseline --no-events \
  > gpurun_out/${tag}_prof.json 2> gpurun_out/${tag}_prof.err || exit 1
python3 tools/trace_by_shape.py gpurun_out/${tag}_prof/run_kernel_trace.csv > gpurun_out/${tag}_f${pf}_by_shape.txt || exit 1
rm -f gpurun_out/${tag}_prof/run_kernel_trace.csv
echo done
