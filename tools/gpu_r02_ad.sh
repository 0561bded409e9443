# K10 3x3 conv PMC (res-64 320 -> 320, B4 f8): what limits the GEMM core
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/pmc_conv.sh gpurun_out/conv_pmc 32 320 64 320
python tools/pmc_summary.py conv_kernel_g gpurun_out/conv_pmc/A gpurun_out/conv_pmc/B gpurun_out/conv_pmc/C > gpurun_out/conv_pmc.txt 2>&1 || true
cat gpurun_out/conv_pmc.txt
timeout -k 10 200 python bench.py --frames 2 --steps 2 --warmup 1 --extras none --no-cpu-baseline --no-events > gpurun_out/hb_ad_f2.json 2>/dev/null
cut -c1-200 gpurun_out/hb_ad_f2.json
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_norm_gpu.py tests/test_unet_gpu.py > gpurun_out/tests_ad.log 2>&1 || { tail -30 gpurun_out/tests_ad.log; exit 1; }
tail -2 gpurun_out/tests_ad.log
