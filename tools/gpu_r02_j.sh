# K1 folded-max (pre-scaled q) kernel: timing/accuracy both conventions, kernel tests, reference parity
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 python tools/k1_modes.py gpurun_out/k1_modes_j.jsonl > /dev/null
timeout -k 10 120 python tools/k1_modes.py gpurun_out/k1_modes_j.jsonl > /dev/null
cat gpurun_out/k1_modes_j.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > gpurun_out/t11.log 2>&1
tail -2 gpurun_out/t11.log
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_reference_gpu.py > gpurun_out/t12.log 2>&1
tail -2 gpurun_out/t12.log
