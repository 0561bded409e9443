# K1 folded-max / staggered variants: interleaved per-process A/B + the K1 GPU tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
for rep in 1 2; do
  for m in 0 1 2 3; do
    VP2P_K1_MODE=$m timeout -k 10 120 python tools/k1_modes.py gpurun_out/k1_modes_i.jsonl > /dev/null
  done
done
cat gpurun_out/k1_modes_i.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_reference_gpu.py -k "frame" > gpurun_out/t10.log 2>&1
tail -3 gpurun_out/t10.log
