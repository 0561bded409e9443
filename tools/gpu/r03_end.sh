# records on the committed tree: configs[4] long clip (attn1 at 128 frames 768^2), HIP-graph bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --mode k1long --no-cpu-baseline > gpurun_out/r03end_k1long.json 2> gpurun_out/r03end_k1long.err
cut -c1-400 gpurun_out/r03end_k1long.json
timeout -k 10 400 python bench.py --graphs 1 --no-cpu-baseline --extras none > gpurun_out/r03end_graphs.json 2> gpurun_out/r03end_graphs.err
cut -c1-200 gpurun_out/r03end_graphs.json
timeout -k 10 400 python bench.py --no-cpu-baseline --extras none > gpurun_out/r03end_eager.json 2> gpurun_out/r03end_eager.err
cut -c1-200 gpurun_out/r03end_eager.json
