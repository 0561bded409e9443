# bench line + kernel-trace stats + K1 traffic/PMC with the folded-max K1
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 500 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_p.json 2> gpurun_out/bench_p.err
cat gpurun_out/bench_p.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_p -o run -- python3 $R/bench.py --steps 2 --warmup 1 --extras none --no-cpu-baseline > $R/gpurun_out/prof_p.out 2>&1
cd $R
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/k1pmc_p/f -o run -- python3 tools/k1_only.py 5 > gpurun_out/k1pmc_pf.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/k1pmc_p/w -o run -- python3 tools/k1_only.py 5 > gpurun_out/k1pmc_pw.log 2>&1
python tools/pmc_traffic.py gpurun_out/k1pmc_p/f/run_counter_collection.csv gpurun_out/k1pmc_p/w/run_counter_collection.csv frame_attn_kernel_x2f gpurun_out/k1_pmc_traffic.json 188743680 32,4096,320
