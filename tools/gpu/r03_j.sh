# K2 v3 staged Q/O rows (VP2P_K2_V3=2): kernel + drop-in + transformer parity, A/B vs mode 0;
# kernel-time profile of 1- and 2-frame edits (the per-rank work at N = 8)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VP2P_K2_V3=2 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py \
    tests/test_dropin_gpu.py tests/test_reference_gpu.py -k "cross or dropin or transformer3d or controlled" \
    > gpurun_out/r03j_tests.log 2>&1 || { tail -40 gpurun_out/r03j_tests.log; exit 1; }
tail -2 gpurun_out/r03j_tests.log
for m in 0 2 0 2; do
  VP2P_K2_V3=$m timeout -k 10 120 python tools/k2_bench.py | sed "s/^/{\"v3mode\": $m, \"r\": /; s/$/}/" >> gpurun_out/r03j_k2_ab.jsonl
done
cat gpurun_out/r03j_k2_ab.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r03j_prof_f$f -o run -- python3 bench.py --frames $f --graphs 1 --steps 1 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/r03j_f$f.json 2> gpurun_out/r03j_f$f.err
  find /tmp/r03j_prof_f$f -name "*kernel_stats.csv" -exec cp {} gpurun_out/r03j_f${f}_kernel_stats.csv \;
done
ls gpurun_out | grep r03j
