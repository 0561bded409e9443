# K10: conv tests, then per-shape A/B of the 32x32x16 layout ("p" column) vs VP2P_CONV_MM=16 ("g")
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/t14.log 2>&1
tail -2 gpurun_out/t14.log
timeout -k 10 200 python tools/conv_bench.py > gpurun_out/conv_p.jsonl  # default: MM32
VP2P_CONV_MM=16 timeout -k 10 200 python tools/conv_bench.py > gpurun_out/conv_g.jsonl
python - <<'PY'
import json
a=[json.loads(l) for l in open("gpurun_out/conv_g.jsonl")]; b=[json.loads(l) for l in open("gpurun_out/conv_p.jsonl")]
for x,y in zip(a,b):
    if "k10_ms" in x: print(x["x"], x["cout"], x["k"], x["stride"], x["calls"], "g", x["k10_tflops"], "p", y["k10_tflops"], "lib", x["tflops"])
PY
