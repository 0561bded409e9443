# frame-sharded backward (null-text over 2 ranks, gloo-staged on the one GPU) + the other sharded GPU tests
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_frame_parallel.py \
    tests/test_backward_gpu.py --durations=10 > gpurun_out/r03h_tests.log 2>&1 || { tail -60 gpurun_out/r03h_tests.log; exit 1; }
tail -25 gpurun_out/r03h_tests.log
