#!/bin/bash
# K2 v3d: the K2 kernel tests and the reference cross-attention tests, then k2_bench (producer timing)
# with v3d (default) and v3 (VP2P_K2_V3D=0), two rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k2d}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "cross" \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
for rnd in 0 1; do
  for v in 0 1; do
    VP2P_K2_V3D=$v timeout -k 10 180 python -u tools/k2_bench.py --iters 60 --producer 1 > gpurun_out/${tag}.tmp || exit 1
    python3 -c "
import json
for l in open('gpurun_out/${tag}.tmp'):
    d=json.loads(l); d['v3d']=$v; d['round']=$rnd; print(json.dumps(d))" >> gpurun_out/${tag}.jsonl || exit 1
  done
done
echo done
