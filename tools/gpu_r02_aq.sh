# K2 v3 with the 77-token specialisation: timing (kbench, k2_bench), K2 tests, reference parity
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python tools/kbench.py > gpurun_out/kbench_aq.jsonl
grep cross gpurun_out/kbench_aq.jsonl
timeout -k 10 200 python tools/k2_bench.py > gpurun_out/k2_aq.jsonl
cat gpurun_out/k2_aq.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_reference_gpu.py tests/test_dropin_gpu.py > gpurun_out/tests_aq.log 2>&1 || { tail -30 gpurun_out/tests_aq.log; exit 1; }
tail -2 gpurun_out/tests_aq.log
