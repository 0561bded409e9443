# bench line + kernel-trace stats of the same command + K1/K2 PMC passes (traffic, waits)
set -e
R=$GRAFT_REPO_ROOT
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_h -o run -- python3 $R/bench.py --steps 2 --warmup 1 --extras none --no-cpu-baseline > $R/gpurun_out/prof_h.out 2>&1
cd $R
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/k1pmc/f -o run -- python3 tools/k1_only.py 5 > gpurun_out/k1pmc_f.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/k1pmc/w -o run -- python3 tools/k1_only.py 5 > gpurun_out/k1pmc_w.log 2>&1
python tools/pmc_traffic.py gpurun_out/k1pmc/f/run_counter_collection.csv gpurun_out/k1pmc/w/run_counter_collection.csv frame_attn_kernel_x2f gpurun_out/k1_pmc_traffic.json 188743680 32,4096,320
bash tools/pmc_k2.sh $R/gpurun_out/k2pmc_v2f 30
python tools/pmc_summary.py cross_attn_kernel_v2 gpurun_out/k2pmc_v2f/A gpurun_out/k2pmc_v2f/B gpurun_out/k2pmc_v2f/C gpurun_out/k2pmc_v2f/D > gpurun_out/k2pmc_v2f.txt 2>&1 || true
