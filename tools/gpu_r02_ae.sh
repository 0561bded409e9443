# K2 edit launches: unconditional half on v3 (v1 only for the edited half) vs all-v1; K2 + drop-in + reference tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 200 env VP2P_K2=v1 python tools/k2_bench.py > gpurun_out/k2_ae_v1.jsonl
timeout -k 10 200 python tools/k2_bench.py > gpurun_out/k2_ae_v3.jsonl
cat gpurun_out/k2_ae_v1.jsonl gpurun_out/k2_ae_v3.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_dropin_gpu.py tests/test_reference_gpu.py > gpurun_out/tests_ae.log 2>&1 || { tail -30 gpurun_out/tests_ae.log; exit 1; }
tail -2 gpurun_out/tests_ae.log
