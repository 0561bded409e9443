# K7: 8 rows in flight per thread vs 4 (old build), GN bench + norm tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 env VP2P_LIB=$R/video-p2p_amd/lib/lab/libvp2p_gnold.so python tools/gn_bench.py gpurun_out/gn_aj_old.jsonl > /dev/null
timeout -k 10 200 python tools/gn_bench.py gpurun_out/gn_aj_new.jsonl > /dev/null
python - <<'PY'
import json
o=[json.loads(l) for l in open("gpurun_out/gn_aj_old.jsonl")]; n=[json.loads(l) for l in open("gpurun_out/gn_aj_new.jsonl")]
for a,b in zip(o,n):
    print(a["C"],a["H"],a["silu"],"stats",a["stats_us"],"->",b["stats_us"],"apply_stats",a["apply_stats_us"],"->",b["apply_stats_us"],"apply_old",a["apply_old_us"],"->",b["apply_old_us"])
PY
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_gpu.py > gpurun_out/tests_aj.log 2>&1 || { tail -20 gpurun_out/tests_aj.log; exit 1; }
tail -1 gpurun_out/tests_aj.log
