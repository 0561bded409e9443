#!/bin/bash
# K2 A/B: tools/k2_bench.py under each lab library in turn (two rounds), one process per library.
# usage: [K2AB_PRODUCER=1] tools/gpu/k2_ab.sh OUT.jsonl lib1.so lib2.so ...
set -o pipefail
cd "$(dirname "$0")/../.."
out=$1; shift
mkdir -p gpurun_out
for rnd in 0 1; do
  for lib in "$@"; do
    VP2P_LIB=$(realpath $lib) timeout -k 10 180 python -u tools/k2_bench.py --iters 100 --producer ${K2AB_PRODUCER:-0} > gpurun_out/k2ab.tmp || exit 1
    python3 -c "
import json,sys
for l in open('gpurun_out/k2ab.tmp'):
    d=json.loads(l); d['lib']='$(basename $lib)'; d['round']=$rnd; print(json.dumps(d))" | tee -a $out || exit 1
  done
done
