# K10 alpha epilogue + wide 1x1 + projections through ops.linear: conv/linear tests, linear chooser,
# model-level parity, rabbit8 bf16 edit parity, default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
    > gpurun_out/r03o_conv.log 2>&1 || { tail -40 gpurun_out/r03o_conv.log; exit 1; }
tail -2 gpurun_out/r03o_conv.log
timeout -k 10 400 python -u tools/linear_choose.py gpurun_out/r03o_linear.jsonl > gpurun_out/r03o_linear.out 2>&1 || { tail -20 gpurun_out/r03o_linear.out; exit 1; }
tail -1 gpurun_out/r03o_linear.out
VP2P_PARITY_REPORT=gpurun_out/r03o_parity.jsonl timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_reference_gpu.py tests/test_unet_gpu.py tests/test_dropin_gpu.py -k "not (edit_vs_reference and fp32) and not penguin24" > gpurun_out/r03o_ref.log 2>&1 || { tail -40 gpurun_out/r03o_ref.log; exit 1; }
tail -3 gpurun_out/r03o_ref.log
grep final_psnr gpurun_out/r03o_parity.jsonl | cut -c1-300
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r03o_bench.json 2> gpurun_out/r03o_bench.err
cat gpurun_out/r03o_bench.json | cut -c1-1500
