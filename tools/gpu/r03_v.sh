# GEGLU fused-vs-unfused table re-measured with the register epilogue; GEGLU / 1x1 tile A/B; bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/geglu_choose.py gpurun_out/r03v_geglu_choose.jsonl > gpurun_out/r03v_geglu.out 2>&1 || { tail -20 gpurun_out/r03v_geglu.out; exit 1; }
python - <<'PY'
import json
rows = [json.loads(l) for l in open("gpurun_out/r03v_geglu_choose.jsonl")]
print(len(rows), "keys;", sum(r["new"] != r["old"] for r in rows), "flipped")
for r in rows:
    if r["new"] != r["old"] or "(32," in r["key"]:
        print(r)
PY
for t in 128 auto 128 auto; do
  VP2P_CONV_TILE=$t timeout -k 10 180 python tools/k10_bench.py gpurun_out/r03v_k10_ab.jsonl > /dev/null
done
grep -E "geglu|linear" gpurun_out/r03v_k10_ab.jsonl | cut -c1-160
