# K7 GroupNorm: finalize + apply_stats vs per-block merge; norm + backward tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python tools/gn_bench.py gpurun_out/gn_w.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_norm_gpu.py tests/test_backward_gpu.py > gpurun_out/tests_w.log 2>&1
tail -3 gpurun_out/tests_w.log
