# parity tests of the new fixtures + K2 (v3 1-D XCD-grouped grid, v3e edited half): tests, A/B timing, PMC
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export VP2P_PARITY_REPORT=gpurun_out/r03c_parity.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_longclip_gpu.py tests/test_vae_gpu.py "tests/test_backward_gpu.py::test_null_optimization_vs_reference" \
    "tests/test_reference_gpu.py::test_edit_vs_reference_pipeline[car2-dtype0-100.0]" \
    "tests/test_reference_gpu.py::test_edit_vs_reference_pipeline[car2-dtype1-45.0]" \
    tests/test_kernels_gpu.py tests/test_dropin_gpu.py \
    --durations=20 > gpurun_out/r03c_tests.log 2>&1 || { tail -60 gpurun_out/r03c_tests.log; exit 1; }
tail -25 gpurun_out/r03c_tests.log
for cfg in "3d v1" "1d v1" "1d v3"; do
  set -- $cfg
  VP2P_K2_GRID=$1 VP2P_K2_EDIT=$2 timeout -k 10 120 python tools/k2_bench.py | sed "s/^/{\"grid\": \"$1\", \"edit\": \"$2\", \"r\": /; s/$/}/" >> gpurun_out/r03c_k2_ab.jsonl
done
cat gpurun_out/r03c_k2_ab.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for st in 3 30; do
  for c in FETCH_SIZE WRITE_SIZE "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
    tag=$(echo $c | cut -c1-8)
    timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r03c_pmc_k2_s${st}_${tag} -o run -- python3 tools/k2_only.py 5 4096 320 $st > /dev/null 2>&1
  done
done
ls -R gpurun_out | grep -c csv
