# K10 wide tile (256 x 320, CF 2): conv tests under VP2P_CONV_TILE=wide, bit-equality + timing A/B
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VP2P_CONV_TILE=wide timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
    > gpurun_out/r03m_tests.log 2>&1 || { tail -40 gpurun_out/r03m_tests.log; exit 1; }
tail -2 gpurun_out/r03m_tests.log
for t in 128 wide 128 wide; do
  VP2P_CONV_TILE=$t timeout -k 10 180 python tools/k10_bench.py gpurun_out/r03m_k10_ab.jsonl > /dev/null
done
cat gpurun_out/r03m_k10_ab.jsonl
