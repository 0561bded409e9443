# full GPU suite + smoke + bench line + kernel-trace stats (round-2 v4)
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/suite_x.log 2>&1 || { tail -30 gpurun_out/suite_x.log; exit 1; }
tail -2 gpurun_out/suite_x.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_x.log 2>&1
tail -2 gpurun_out/smoke_x.log
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_x.json 2> gpurun_out/bench_x.err
cat gpurun_out/bench_x.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_x -o run -- python3 $R/bench.py --steps 2 --warmup 1 --extras none --no-cpu-baseline > $R/gpurun_out/prof_x.out 2>&1
