# configs[3] official mode on one GPU with the final code: DDIM inversion + null-text optimisation, 50 steps
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python bench.py --mode nulltext --ddim-steps 50 --steps 1 --warmup 1 > gpurun_out/bench_nulltext_an.json 2> gpurun_out/bench_nulltext_an.err
cut -c1-500 gpurun_out/bench_nulltext_an.json
