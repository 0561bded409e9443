#!/bin/bash
# The small-clip row counts for the projection table: conv tests, tools/linear_choose.py on M 256..49152
# merged into round 5's measurement (rules written in this tree), then the 1 / 3-frame edits.
# usage: tools/gpu/linear_small.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-linsmall}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 600 python -u tools/linear_choose.py gpurun_out/${tag}_linear_choose.jsonl --write \
  --from profiles/r05_linear_choose.jsonl --ms 256,768,1024,3072,12288,49152 > gpurun_out/${tag}_choose.log 2>&1 \
  || { tail -20 gpurun_out/${tag}_choose.log; exit 1; }
tail -1 gpurun_out/${tag}_choose.log | cut -c1-400
SC_FRAMES="1 3" SC_PROF_FRAMES=3 bash tools/gpu/small_clip.sh ${tag}_sc || exit 1
echo done
