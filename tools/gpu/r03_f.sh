# K10 256-row / 3-stage tile: conv tests, bit-equality + timing A/B vs the 128-row tile, default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
    tests/test_reference_gpu.py -k "not edit_vs_reference" > gpurun_out/r03f_tests.log 2>&1 || { tail -40 gpurun_out/r03f_tests.log; exit 1; }
tail -3 gpurun_out/r03f_tests.log
for t in 128 256 auto; do
  VP2P_CONV_TILE=$t timeout -k 10 180 python tools/k10_bench.py gpurun_out/r03f_k10_ab.jsonl > /dev/null
done
cat gpurun_out/r03f_k10_ab.jsonl
timeout -k 10 600 python bench.py --extras none > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err
cat gpurun_out/r03f_bench.json
