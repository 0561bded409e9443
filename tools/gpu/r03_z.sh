# block residual adds on the output projections' K10 epilogue: model/edit parity tests, A/B bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VP2P_PARITY_REPORT=gpurun_out/r03z_parity.jsonl timeout -k 10 700 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_reference_gpu.py tests/test_unet_gpu.py tests/test_dropin_gpu.py tests/test_frame_parallel.py tests/test_graph_gpu.py \
    tests/test_ctx_cache_gpu.py -k "not (edit_vs_reference and fp32) and not penguin24" > gpurun_out/r03z_tests.log 2>&1 || { tail -40 gpurun_out/r03z_tests.log; exit 1; }
tail -1 gpurun_out/r03z_tests.log
grep final_psnr gpurun_out/r03z_parity.jsonl | cut -c1-140
for c in 1 0 1 0; do
  VP2P_FUSE_OUT_RES=$c timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/r03z_b$c.json 2> gpurun_out/r03z.err
  echo "fuse_out_res=$c $(cut -c1-150 gpurun_out/r03z_b$c.json)"
  cat gpurun_out/r03z_b$c.json >> gpurun_out/r03z_ab.jsonl
done
