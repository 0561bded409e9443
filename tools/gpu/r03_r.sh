# full GPU suite on the current tree (context K/V cache, linear rules, wide GEGLU), smoke, A/B of the
# context cache, default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T) $(tail -c 120 gpurun_out/r03r_suite.log 2>/dev/null | tr -d '\n' | tail -c 60)"; done ) &
HB=$!
trap "kill $HB" EXIT
VP2P_PARITY_REPORT=gpurun_out/r03r_parity.jsonl timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    --durations=15 > gpurun_out/r03r_suite.log 2>&1 || { tail -40 gpurun_out/r03r_suite.log; exit 1; }
tail -22 gpurun_out/r03r_suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03r_smoke.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03r_smoke.txt | tail -3
for c in 1 0 1 0; do
  VP2P_CTX_CACHE=$c timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/r03r_bench_c$c.json 2> gpurun_out/r03r_bench.err
  echo "ctx_cache=$c $(cut -c1-160 gpurun_out/r03r_bench_c$c.json)"
  cat gpurun_out/r03r_bench_c$c.json >> gpurun_out/r03r_bench_ab.jsonl
done
