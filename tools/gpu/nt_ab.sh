#!/bin/bash
# Null-text (configs[3]) after a change: the backward GPU tests, then the nulltext bench line at
# DDIM_STEPS steps and its kernel stats.   bash tools/gpu/nt_ab.sh TAG [DDIM_STEPS]
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-nt}; n=${2:-10}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_backward_gpu.py \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -3 gpurun_out/${tag}_tests.log
A="--mode nulltext --steps 1 --warmup 1 --ddim-steps $n --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $A > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
tail -1 gpurun_out/${tag}_bench.json | cut -c1-300
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py $A > gpurun_out/${tag}_profiled.json 2> gpurun_out/${tag}_prof.err || exit 1
rm -f gpurun_out/${tag}_prof/run_kernel_trace.csv
python tools/prof_summary.py gpurun_out/${tag}_prof gpurun_out/${tag}_kernel_stats.txt > /dev/null || exit 1
head -30 gpurun_out/${tag}_kernel_stats.txt
echo done
