# K3 1-D XCD-remapped grid vs the 2-D grid at the UNet's fused-qkv layout; K3 tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
for rnd in 1 2; do
  timeout -k 10 120 env VP2P_LIB=$R/video-p2p_amd/lib/lab/libvp2p_k3old.so python tools/k3_views.py gpurun_out/k3_af.jsonl
  timeout -k 10 120 python tools/k3_views.py gpurun_out/k3_af.jsonl
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k temporal > gpurun_out/tests_af.log 2>&1 || { tail -30 gpurun_out/tests_af.log; exit 1; }
tail -2 gpurun_out/tests_af.log
