# configs[2] on one GPU with the final code: penguin-run refine edit, 24 frames
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 700 python bench.py --edit penguin --frames 24 --steps 1 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/bench_penguin24_am.json 2> gpurun_out/bench_penguin24_am.err
cut -c1-400 gpurun_out/bench_penguin24_am.json
