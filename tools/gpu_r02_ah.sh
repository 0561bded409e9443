# plain K = 320 projections on K10 (attn2 to_q, proj_in at res-64): A/B, parity tests, bench line
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python tools/linear_plain_ab.py gpurun_out/linear_plain_ah.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_reference_gpu.py tests/test_unet_gpu.py tests/test_dropin_gpu.py tests/test_backward_gpu.py > gpurun_out/tests_ah.log 2>&1 || { tail -30 gpurun_out/tests_ah.log; exit 1; }
tail -2 gpurun_out/tests_ah.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/bench_ah.json 2> gpurun_out/bench_ah.err
cut -c1-300 gpurun_out/bench_ah.json
