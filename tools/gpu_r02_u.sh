# K1 mixed 32x32 / 16x16x32 PV tiles at d = 40: lab A/B vs the double-buffered build, then K1 tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
L=video-p2p_amd/lib/lab
timeout -k 10 300 python -u tools/k1_lab.py gpurun_out/k1_lab_u.jsonl $L/libvp2p_dbuf.so $L/libvp2p_mix.so > gpurun_out/k1_lab_u.log 2>&1
cat gpurun_out/k1_lab_u.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "frame" > gpurun_out/tests_u.log 2>&1
tail -3 gpurun_out/tests_u.log
