# K10 wide tile: conv tests forced wide + timing A/B; rabbit8 edit parity on the regenerated fixture
# (default tile choice, wide auto for 3x3 Cout % 320); default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
VP2P_CONV_TILE=wide timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
    > gpurun_out/r03n_tests.log 2>&1 || { tail -40 gpurun_out/r03n_tests.log; exit 1; }
tail -2 gpurun_out/r03n_tests.log
for t in 128 wide 128 wide; do
  VP2P_CONV_TILE=$t timeout -k 10 180 python tools/k10_bench.py gpurun_out/r03n_k10_ab.jsonl > /dev/null
done
cat gpurun_out/r03n_k10_ab.jsonl
VP2P_PARITY_REPORT=gpurun_out/r03n_parity.jsonl timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_reference_gpu.py \
    -k "rabbit8" > gpurun_out/r03n_rabbit.log 2>&1 || { tail -40 gpurun_out/r03n_rabbit.log; exit 1; }
tail -5 gpurun_out/r03n_rabbit.log
cat gpurun_out/r03n_parity.jsonl
timeout -k 10 600 python bench.py > gpurun_out/r03n_bench.json 2> gpurun_out/r03n_bench.err
cat gpurun_out/r03n_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03n_prof -o r03n -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --extras none --no-events > gpurun_out/r03n_prof_bench.json 2> gpurun_out/r03n_prof_bench.err
cat gpurun_out/r03n_prof_bench.json
