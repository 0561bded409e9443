set -e
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "cross" -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/t7.log 2>&1
timeout -k 10 120 python tools/k2_bench.py > gpurun_out/k2_v2d.jsonl
VP2P_K2=v1 timeout -k 10 120 python tools/k2_bench.py > gpurun_out/k2_v1d.jsonl
timeout -k 10 120 python tools/k2_bench.py > gpurun_out/k2_v2e.jsonl
