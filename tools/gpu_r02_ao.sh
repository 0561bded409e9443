# configs[4] long clip on one GPU with the final code: 128 frames 768^2 sparse-causal attention (K1)
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python bench.py --mode k1long --steps 3 --warmup 1 > gpurun_out/bench_k1long_ao.json 2> gpurun_out/bench_k1long_ao.err
cut -c1-600 gpurun_out/bench_k1long_ao.json
