# full GPU suite on the current tree (rabbit8 edit parity excluded: its fixture is being
# regenerated), smoke, default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T) $(tail -c 200 gpurun_out/r03l_suite.log | tr -d '\n' | tail -c 60)"; done ) &
HB=$!
VP2P_PARITY_REPORT=gpurun_out/r03l_parity.jsonl timeout -k 10 800 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests \
    -k "not rabbit8" --durations=15 > gpurun_out/r03l_suite.log 2>&1 || { kill $HB; tail -40 gpurun_out/r03l_suite.log; exit 1; }
kill $HB
tail -20 gpurun_out/r03l_suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03l_smoke.txt 2>&1
cat gpurun_out/r03l_smoke.txt | grep -v amdgpu.ids
timeout -k 10 600 python bench.py > gpurun_out/r03l_bench.json 2> gpurun_out/r03l_bench.err
cat gpurun_out/r03l_bench.json
