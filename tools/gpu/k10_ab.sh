#!/bin/bash
# K10 A/B: tools/k10_bench.py on the product library and every video-p2p_amd/lib/ab/*.so (or lib/$K10AB_DIR),
# two rounds.
#   bash tools/gpu/k10_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-k10ab}
mkdir -p gpurun_out
for r in 0 1; do
  for lib in video-p2p_amd/lib/libvp2p_hip.so video-p2p_amd/lib/${K10AB_DIR:-ab}/*.so; do
    VP2P_LIB=$PWD/$lib timeout -k 10 200 python -u tools/k10_bench.py gpurun_out/$tag.jsonl > gpurun_out/${tag}_last.log 2>&1 || { tail -20 gpurun_out/${tag}_last.log; exit 1; }
  done
done
python3 - gpurun_out/$tag.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
best = collections.defaultdict(dict)
for r in rows:
    k = (r["op"], tuple(r["shape"]))
    best[k][r["lib"]] = min(best[k].get(r["lib"], 1e9), r["ms"])
libs = sorted({r["lib"] for r in rows})
print("op shape " + " ".join(libs))
for k, v in best.items():
    print(k[0], list(k[1]), " ".join(f"{v.get(l, 0):.4f}" for l in libs))
PY
