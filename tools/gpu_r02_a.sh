# round-2 GPU check: multi-rank layout tests, kernel tests, then the bench at N=1 with every extra line
set -e
timeout -k 10 400 python -u -m pytest tests/test_frame_parallel.py tests/test_kernels_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/t2.log 2>&1
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_a.json 2> gpurun_out/bench_a.err
bash tools/hb_small_frames.sh
