# linear rules (K10 for measured-faster projections) + wide GEGLU: tests, same-box A/B bench, GEGLU A/B + PMC
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
( while true; do sleep 60; echo "[heartbeat] $(date +%T)"; done ) &
HB=$!
trap "kill $HB" EXIT
VP2P_CONV_TILE=wide timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_conv_gpu.py \
    > gpurun_out/r03p_conv.log 2>&1 || { tail -40 gpurun_out/r03p_conv.log; exit 1; }
tail -1 gpurun_out/r03p_conv.log
VP2P_PARITY_REPORT=gpurun_out/r03p_parity.jsonl timeout -k 10 600 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
    tests/test_reference_gpu.py tests/test_unet_gpu.py tests/test_dropin_gpu.py tests/test_graph_gpu.py -k "not (edit_vs_reference and fp32) and not penguin24" > gpurun_out/r03p_ref.log 2>&1 || { tail -40 gpurun_out/r03p_ref.log; exit 1; }
tail -1 gpurun_out/r03p_ref.log
grep final_psnr gpurun_out/r03p_parity.jsonl | cut -c1-200
for m in table library table library; do
  VP2P_LINEAR=$m timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > gpurun_out/r03p_bench_$m.json 2> gpurun_out/r03p_bench.err
  echo "$m $(cut -c1-200 gpurun_out/r03p_bench_$m.json)"
  cat gpurun_out/r03p_bench_$m.json >> gpurun_out/r03p_bench_ab.jsonl
done
for t in 128 wide 128 wide; do
  VP2P_CONV_TILE=$t timeout -k 10 180 python tools/k10_bench.py gpurun_out/r03p_k10_ab.jsonl > /dev/null
done
grep geglu gpurun_out/r03p_k10_ab.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/pmc_geglu.sh gpurun_out/r03p_pmc_geglu 131072 320 1280
ls gpurun_out/r03p_pmc_geglu/*
