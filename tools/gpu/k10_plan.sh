#!/bin/bash
# K10 launch plans at the small-clip shapes: the conv tests, then tools/k10_plan_sweep.py (frames $SWEEP_FRAMES).
# usage: [SWEEP_FRAMES=..] [SWEEP_LINEAR="frames"] tools/gpu/k10_plan.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k10plan}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 600 python -u tools/k10_plan_sweep.py gpurun_out/${tag}.jsonl ${SWEEP_FRAMES:-1 2 3} > gpurun_out/${tag}_sweep.log 2>&1 \
  || { tail -20 gpurun_out/${tag}_sweep.log; exit 1; }
if [ -n "$SWEEP_LINEAR" ]; then
  timeout -k 10 600 python -u tools/k10_plan_sweep.py gpurun_out/${tag}_linear.jsonl --linear $SWEEP_LINEAR \
    > gpurun_out/${tag}_linear.log 2>&1 || { tail -20 gpurun_out/${tag}_linear.log; exit 1; }
fi
echo done
