# host floor: eager vs HIP-graph replay edits at 1, 2, 8 frames (one process, N=1)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for f in 1 2 8; do
  for g in 0 1; do
    timeout -k 10 300 python bench.py --frames $f --graphs $g --steps 3 --warmup 1 --extras none --no-cpu-baseline --no-events \
      > gpurun_out/r03g_f${f}_g${g}.json 2> gpurun_out/r03g_f${f}_g${g}.err
    python -c "import json,sys; d=json.load(open('gpurun_out/r03g_f${f}_g${g}.json')); print(json.dumps({'frames': $f, 'graphs': $g, 'ms_per_edit': d['ms_per_step'], 'frames_per_s': d['value'], 'finite': d['output_finite']}))" | tee -a gpurun_out/r03g_host_floor.jsonl
  done
done
