# K3 with all 8 heads of a token block in one workgroup: K3 tests, A/B vs 4 heads, bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VP2P_K3_WPB=8 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_longclip_gpu.py -k "temporal" \
    > gpurun_out/r03x_k3.log 2>&1 || { tail -40 gpurun_out/r03x_k3.log; exit 1; }
tail -1 gpurun_out/r03x_k3.log
for w in 4 8 4 8; do
  VP2P_K3_WPB=$w timeout -k 10 120 python tools/k3_wpb_bench.py gpurun_out/r03x_k3_ab.jsonl > /dev/null
done
python - <<'PY'
import json
from collections import defaultdict
d = defaultdict(list); s = defaultdict(set)
for l in open("gpurun_out/r03x_k3_ab.jsonl"):
    r = json.loads(l); k = (r["C"], r["self_replace"]); d[(k, r["wpb"])].append(r["us"]); s[k].add(r["sum"])
for k in sorted(set(k for k, _ in d)):
    a, b = min(d[(k, "4")]), min(d[(k, "8")])
    print(k, "wpb4 %.1f wpb8 %.1f ratio %.3f" % (a, b, b / a), "bit-equal" if len(s[k]) == 1 else "SUMS DIFFER")
PY
VP2P_K3_WPB=8 VP2P_PARITY_REPORT=gpurun_out/r03x_parity.jsonl timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_reference_gpu.py -k "edit_vs_reference and bf16 and not penguin24" > gpurun_out/r03x_ref.log 2>&1 || { tail -30 gpurun_out/r03x_ref.log; exit 1; }
tail -1 gpurun_out/r03x_ref.log
for w in 8 4; do
  VP2P_K3_WPB=$w timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/r03x_bench_$w.json 2> gpurun_out/r03x_bench.err
  echo "wpb=$w $(cut -c1-150 gpurun_out/r03x_bench_$w.json)"
done
