# round-2 v7: full GPU suite + smoke + bench line + kernel-trace stats + K1 traffic (FETCH/WRITE passes)
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/suite_ag.log 2>&1 || { tail -30 gpurun_out/suite_ag.log; exit 1; }
tail -2 gpurun_out/suite_ag.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_ag.log 2>&1
tail -2 gpurun_out/smoke_ag.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_ag.json 2> gpurun_out/bench_ag.err
cut -c1-400 gpurun_out/bench_ag.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_ag -o run -- python3 $R/bench.py --steps 2 --warmup 1 --extras none --no-cpu-baseline > $R/gpurun_out/prof_ag.out 2>&1
cd $R
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/k1pmc_ag/f -o run -- python3 tools/k1_only.py 5 > gpurun_out/k1pmc_agf.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/k1pmc_ag/w -o run -- python3 tools/k1_only.py 5 > gpurun_out/k1pmc_agw.log 2>&1
python tools/pmc_traffic.py gpurun_out/k1pmc_ag/f/run_counter_collection.csv gpurun_out/k1pmc_ag/w/run_counter_collection.csv frame_attn_kernel_x2f gpurun_out/k1_pmc_traffic.json 188743680 32,4096,320
