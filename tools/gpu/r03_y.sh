# last tree: full GPU suite + smoke; K10 tile A/B for the GEGLU / 1x1 shapes (256 x 160 vs auto)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T) $(tail -c 120 gpurun_out/r03y_suite.log 2>/dev/null | tr -d '\n' | tail -c 60)"; done ) &
HB=$!
trap "kill $HB" EXIT
VP2P_PARITY_REPORT=gpurun_out/r03y_parity.jsonl timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests \
    --durations=10 > gpurun_out/r03y_suite.log 2>&1 || { tail -40 gpurun_out/r03y_suite.log; exit 1; }
tail -3 gpurun_out/r03y_suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03y_smoke.txt 2>&1
grep -v amdgpu.ids gpurun_out/r03y_smoke.txt | tail -2
for t in 256 auto 256 auto; do
  VP2P_CONV_TILE=$t timeout -k 10 180 python tools/k10_bench.py gpurun_out/r03y_k10_ab.jsonl > /dev/null
done
grep -E "geglu|linear" gpurun_out/r03y_k10_ab.jsonl | cut -c1-140
