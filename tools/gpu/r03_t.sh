# round-3 tree: same-box A/B of the device timestep cache, default bench (all lines), rocprofv3
# kernel stats of one edit, configs[2] (penguin 24 frames) and configs[3] (null-text) lines
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
for c in 1 0 1 0; do
  VP2P_T_CACHE=$c timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/r03t_tc$c.json 2> gpurun_out/r03t.err
  echo "t_cache=$c $(cut -c1-150 gpurun_out/r03t_tc$c.json)"
  cat gpurun_out/r03t_tc$c.json >> gpurun_out/r03t_tcache_ab.jsonl
done
timeout -k 10 600 python bench.py > gpurun_out/r03t_bench.json 2> gpurun_out/r03t_bench.err
cut -c1-400 gpurun_out/r03t_bench.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03t_prof -o r03t -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --extras none --no-events > gpurun_out/r03t_prof_bench.json 2> gpurun_out/r03t_prof.err
cut -c1-200 gpurun_out/r03t_prof_bench.json
find gpurun_out/r03t_prof -name "*stats*"
timeout -k 10 400 python bench.py --edit penguin --frames 24 --no-cpu-baseline --extras none > gpurun_out/r03t_penguin24.json 2> gpurun_out/r03t_p24.err
cut -c1-300 gpurun_out/r03t_penguin24.json
timeout -k 10 300 python bench.py --mode nulltext --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r03t_nulltext.json 2> gpurun_out/r03t_nt.err
cut -c1-300 gpurun_out/r03t_nulltext.json
