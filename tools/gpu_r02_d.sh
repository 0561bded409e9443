# K1 d=80 x2f + K2 v2 (non-edit launches) parity, then A/B timings on the same box
set -e
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_reference_gpu.py -k "frame or cross or transformer" -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/t5.log 2>&1
for i in 1 2; do
  VP2P_K1_D80=1set VP2P_K2=v1 timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_old_$i.jsonl
  timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_new_$i.jsonl
done
timeout -k 10 120 python tools/k2_bench.py > gpurun_out/k2_v2c.jsonl
