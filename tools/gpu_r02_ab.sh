# host-overhead trims (raw stream handle, one K|V GEMM): small-frame bench, drop-in + reference tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 python bench.py --frames 1 --steps 2 --warmup 1 --extras none --no-cpu-baseline --no-events > gpurun_out/hb_ab_f1.json 2>/dev/null
timeout -k 10 200 python bench.py --frames 2 --steps 2 --warmup 1 --extras none --no-cpu-baseline --no-events > gpurun_out/hb_ab_f2.json 2>/dev/null
cut -c1-200 gpurun_out/hb_ab_f1.json gpurun_out/hb_ab_f2.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dropin_gpu.py tests/test_reference_gpu.py tests/test_kernels_gpu.py tests/test_frame_parallel.py > gpurun_out/tests_ab.log 2>&1 || { tail -30 gpurun_out/tests_ab.log; exit 1; }
tail -2 gpurun_out/tests_ab.log
