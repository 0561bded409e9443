# K10 fused-upsample buffer path (old vs new build) + K1 double-buffer: conv and kernel GPU tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 env VP2P_LIB=$R/video-p2p_amd/lib/lab/libvp2p_base.so python tools/conv_up_bench.py gpurun_out/conv_up_r.jsonl
timeout -k 10 120 python tools/conv_up_bench.py gpurun_out/conv_up_r.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_kernels_gpu.py > gpurun_out/tests_r.log 2>&1
tail -3 gpurun_out/tests_r.log
