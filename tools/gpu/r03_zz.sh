# committed round-3 tree: full GPU suite, smoke, default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T) $(tail -c 120 gpurun_out/r03zz_suite.log 2>/dev/null | tr -d '\n' | tail -c 60)"; done ) &
HB=$!
trap "kill $HB" EXIT
VP2P_PARITY_REPORT=gpurun_out/r03zz_parity.jsonl timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    --durations=10 > gpurun_out/r03zz_suite.log 2>&1 || { tail -40 gpurun_out/r03zz_suite.log; exit 1; }
tail -3 gpurun_out/r03zz_suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03zz_smoke.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03zz_smoke.txt | tail -2
timeout -k 10 600 python bench.py > gpurun_out/r03zz_bench.json 2> gpurun_out/r03zz_bench.err
cut -c1-300 gpurun_out/r03zz_bench.json
