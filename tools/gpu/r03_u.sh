# GEGLU epilogue from the accumulators (DPP pair exchange, ABI 13): conv tests under every tile,
# model-level parity, GEGLU timing, PMC, default bench
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in auto 128 256 wide; do
  VP2P_CONV_TILE=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py -k "geglu or linear" \
      > gpurun_out/r03u_conv_$t.log 2>&1 || { tail -40 gpurun_out/r03u_conv_$t.log; exit 1; }
  echo "$t $(tail -1 gpurun_out/r03u_conv_$t.log)"
done
VP2P_PARITY_REPORT=gpurun_out/r03u_parity.jsonl timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_reference_gpu.py tests/test_unet_gpu.py -k "not (edit_vs_reference and fp32) and not penguin24" > gpurun_out/r03u_ref.log 2>&1 || { tail -40 gpurun_out/r03u_ref.log; exit 1; }
tail -1 gpurun_out/r03u_ref.log
grep final_psnr gpurun_out/r03u_parity.jsonl | cut -c1-120
for t in auto auto; do
  VP2P_CONV_TILE=$t timeout -k 10 180 python tools/k10_bench.py gpurun_out/r03u_k10.jsonl > /dev/null
done
grep geglu gpurun_out/r03u_k10.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/pmc_geglu.sh gpurun_out/r03u_pmc_geglu 131072 320 1280
python tools/pmc_summary.py conv_kernel gpurun_out/r03u_pmc_geglu/A gpurun_out/r03u_pmc_geglu/B | grep -E "VALU|MFMA|duration|WAIT_ANY|WAVE_CYCLES"
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/r03u_bench_$i.json 2> gpurun_out/r03u_bench.err
  echo "bench $(cut -c1-150 gpurun_out/r03u_bench_$i.json)"
done
