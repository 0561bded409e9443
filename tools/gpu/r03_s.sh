# GroupNorm predicated tails (stats + apply), device timestep cache: norm/unet/backward tests,
# GN microbench A/B against the previous library, default bench x2
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_norm_gpu.py tests/test_unet_gpu.py \
    tests/test_backward_gpu.py tests/test_frame_parallel.py > gpurun_out/r03s_tests.log 2>&1 || { tail -40 gpurun_out/r03s_tests.log; exit 1; }
tail -1 gpurun_out/r03s_tests.log
for l in base new base new; do
  if [ $l = base ]; then export VP2P_LIB=$GRAFT_REPO_ROOT/tools/libvp2p_hip_base.so; else unset VP2P_LIB; fi
  timeout -k 10 180 python tools/gn_bench.py gpurun_out/r03s_gn_$l.jsonl > /dev/null
done
unset VP2P_LIB
python - <<'PY'
import json
for l in ("base", "new"):
    for line in open(f"gpurun_out/r03s_gn_{l}.jsonl"):
        print(l, line.strip()[:300])
PY
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/r03s_bench_$i.json 2> gpurun_out/r03s_bench.err
  echo "bench $(cut -c1-160 gpurun_out/r03s_bench_$i.json)"
done
