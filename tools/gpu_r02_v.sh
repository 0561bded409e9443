# K2 v3 (K/V in LDS, 4 waves/SIMD) vs v2 / v1 on the non-edit launches; K2 kernel tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
for k in v1 v2 v3; do
  timeout -k 10 120 env VP2P_K2=$k python tools/kbench.py > gpurun_out/kbench_v_$k.jsonl
done
grep cross gpurun_out/kbench_v_v1.jsonl gpurun_out/kbench_v_v2.jsonl gpurun_out/kbench_v_v3.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "cross" > gpurun_out/tests_v.log 2>&1
tail -3 gpurun_out/tests_v.log
