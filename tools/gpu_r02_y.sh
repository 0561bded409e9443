# two-source (cat-free) up-block resnets: unit tests, model parity tests, bench line
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_norm_gpu.py tests/test_conv_gpu.py tests/test_reference_gpu.py tests/test_unet_gpu.py > gpurun_out/tests_y.log 2>&1 || { tail -30 gpurun_out/tests_y.log; exit 1; }
tail -2 gpurun_out/tests_y.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/bench_y.json 2> gpurun_out/bench_y.err
cat gpurun_out/bench_y.json
