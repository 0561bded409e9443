# full GPU suite + smoke
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t15.log 2>&1
tail -3 gpurun_out/t15.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 200 python tools/linear_bench.py > gpurun_out/linear_fast.jsonl 2>/dev/null
