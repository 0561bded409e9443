# CF 3 (wide tile, 32-channel K-steps, 4-stage ring): conv tests forced deep + timing A/B vs wide
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VP2P_CONV_TILE=deep timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
    > gpurun_out/r03q_conv.log 2>&1 || { tail -40 gpurun_out/r03q_conv.log; exit 1; }
tail -1 gpurun_out/r03q_conv.log
for t in wide deep wide deep; do
  VP2P_CONV_TILE=$t timeout -k 10 180 python tools/k10_bench.py gpurun_out/r03q_k10_ab.jsonl > /dev/null
done
python - <<'PY'
import json
from collections import defaultdict
d = defaultdict(list); s = defaultdict(set)
for l in open("gpurun_out/r03q_k10_ab.jsonl"):
    r = json.loads(l); k = (r["op"], tuple(r["shape"])); d[(k, r["lib"].split(":")[1])].append(r["ms"]); s[k].add(r["sum"])
for k in sorted(set(k for k, _ in d)):
    a, b = min(d[(k, "wide")]), min(d[(k, "deep")])
    print(k, "wide %.4f deep %.4f ratio %.3f" % (a, b, b / a), "bit-equal" if len(s[k]) == 1 else "SUMS DIFFER")
PY
