#!/bin/bash
# One round checkpoint on the product tree: the GPU suite (+ parity report), the default bench line,
# and the rocprofv3 kernel stats of a 1-step bench.   bash tools/gpu/round.sh TAG [suite|nosuite]
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-round}; what=${2:-suite}
mkdir -p gpurun_out
if [ "$what" = suite ]; then
  VP2P_PARITY_REPORT=$PWD/gpurun_out/${tag}_parity.jsonl timeout -k 10 1000 python -u -m pytest tests -m gpu -v \
    --timeout 600 --timeout-method thread --durations=25 > gpurun_out/${tag}_suite.log 2>&1
  rc=$?; tail -3 gpurun_out/${tag}_suite.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
tail -1 gpurun_out/${tag}_bench.json | cut -c1-400
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/${tag}_profiled.json 2> gpurun_out/${tag}_prof.err || exit 1
rm -f gpurun_out/${tag}_prof/run_kernel_trace.csv
python tools/prof_summary.py gpurun_out/${tag}_prof gpurun_out/${tag}_kernel_stats.txt > /dev/null || exit 1
head -25 gpurun_out/${tag}_kernel_stats.txt
echo done
