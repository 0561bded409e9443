# K2 v2: parity tests, then the v1/v2 timing A/B on the same box
set -e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "cross" -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/t4.log 2>&1
VP2P_K2=v1 timeout -k 10 120 python tools/k2_bench.py > gpurun_out/k2_v1.jsonl
timeout -k 10 120 python tools/k2_bench.py > gpurun_out/k2_v2.jsonl
VP2P_K2=v1 timeout -k 10 120 python tools/k2_bench.py > gpurun_out/k2_v1b.jsonl
timeout -k 10 120 python tools/k2_bench.py > gpurun_out/k2_v2b.jsonl
