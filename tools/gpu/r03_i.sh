# K2 v3: 2-deep Q prefetch and workgroups-per-CU A/B (bit-equal checksums); K2 kernel tests;
# kernel-time profile of a 1-frame and a 2-frame edit (graph replay) -- the per-rank work at N = 8
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "cross" \
    > gpurun_out/r03i_tests.log 2>&1 || { tail -40 gpurun_out/r03i_tests.log; exit 1; }
tail -2 gpurun_out/r03i_tests.log
VP2P_K2_PF=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "cross" \
    > gpurun_out/r03i_tests_pf2.log 2>&1 || { tail -40 gpurun_out/r03i_tests_pf2.log; exit 1; }
tail -2 gpurun_out/r03i_tests_pf2.log
for pf in 1 2; do for wg in 4 6 8 12; do
  VP2P_K2_PF=$pf VP2P_K2_WGCU=$wg timeout -k 10 120 python tools/k2_bench.py | sed "s/^/{\"pf\": $pf, \"wgcu\": $wg, \"r\": /; s/$/}/" >> gpurun_out/r03i_k2_ab.jsonl
done; done
cat gpurun_out/r03i_k2_ab.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03i_prof_f$f -o run -- python3 bench.py --frames $f --graphs 1 --steps 1 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/r03i_f$f.json 2>/dev/null
done
ls -R gpurun_out/r03i_prof_f1 | head
