# round-2 GPU check b: long-clip temporal kernel, drop-in surface, then a kernel trace of a 1-frame edit
set -e
export VP2P_PARITY_REPORT=$PWD/gpurun_out/parity_b.jsonl
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py::test_temporal_attention_p2p tests/test_unet_gpu.py tests/test_dropin_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/t3.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_f1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --frames 1 --steps 1 --warmup 1 --extras none --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_f1.out 2>&1
