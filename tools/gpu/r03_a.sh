# round 3 baseline on the current tree: GPU suite (minus the end-to-end edits, whose fixtures are being
# regenerated), smoke, kernel microbench, default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    -k "not test_edit_vs_reference_pipeline" > gpurun_out/r03a_suite.log 2>&1 || { tail -40 gpurun_out/r03a_suite.log; exit 1; }
tail -3 gpurun_out/r03a_suite.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03a_smoke.txt 2>&1
cat gpurun_out/r03a_smoke.txt
timeout -k 10 120 python tools/kbench.py > gpurun_out/r03a_kbench.jsonl
timeout -k 10 500 python bench.py > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
cat gpurun_out/r03a_bench.json
