#!/bin/bash
# Whole-edit A/B of a runtime switch: bench.py with VAR=1 / VAR=0 alternating, two rounds per frame count.
# usage: tools/gpu/env_ab.sh TAG VAR "FRAMES..."     (8 frames: the default bench config)
set -o pipefail
cd "$(dirname "$0")/../.."
tag=$1; var=$2; frames=${3:-"1 3"}
mkdir -p gpurun_out
for f in $frames; do for r in 0 1; do for v in 1 0; do
  extra=""; [ "$f" = 8 ] || extra="--no-events"
  env $var=$v timeout -k 10 300 python -u bench.py --frames $f --steps 2 --extras none --no-cpu-baseline $extra \
    > gpurun_out/${tag}_f${f}_v${v}_$r.json 2> gpurun_out/${tag}_f${f}_v${v}_$r.err || { tail -20 gpurun_out/${tag}_f${f}_v${v}_$r.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(json.dumps({'frames': $f, '$var': $v, 'round': $r, 'value': d['value'], 'ms_per_edit': d['ms_per_step']}))" \
    gpurun_out/${tag}_f${f}_v${v}_$r.json | tee -a gpurun_out/${tag}.jsonl
done; done; done
echo done
