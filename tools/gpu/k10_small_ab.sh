#!/bin/bash
# K10 small-clip shapes: tools/k10_small_bench.py on the product library and every lib/ab/*.so.
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k10small}
mkdir -p gpurun_out
for r in 0 1; do
  for lib in video-p2p_amd/lib/libvp2p_hip.so video-p2p_amd/lib/ab/*.so; do
    VP2P_LIB=$PWD/$lib timeout -k 10 200 python -u tools/k10_small_bench.py gpurun_out/$tag.jsonl > /dev/null 2>&1 || exit 1
  done
done
grep '"linear"' gpurun_out/$tag.jsonl | python3 -c "
import json,sys,collections
b=collections.defaultdict(dict)
for l in sys.stdin:
    d=json.loads(l); k=tuple(d['shape']); b[k][d['lib']]=min(b[k].get(d['lib'],9),d['ms'])
for k,v in b.items(): print(k, v)"
