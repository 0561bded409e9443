# K10 epilogue A/B: old (lab dbuf), new erf only (lab base), new erf + transposed-tile epilogue (product)
set -e
R=$GRAFT_REPO_ROOT
cd $R
L=$R/video-p2p_amd/lib/lab
for lib in $L/libvp2p_dbuf.so $L/libvp2p_base.so $R/video-p2p_amd/lib/libvp2p_hip.so; do
  timeout -k 10 150 env VP2P_LIB=$lib python tools/k10_bench.py gpurun_out/k10_t.jsonl > /dev/null
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py > gpurun_out/tests_t.log 2>&1
tail -2 gpurun_out/tests_t.log
