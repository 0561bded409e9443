# new parity tests: long clip (configs[4] size), null-text vs the reference fixture, car2 edit with
# non-trivial masks (K6 mask output), VAE decode raise
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export VP2P_PARITY_REPORT=gpurun_out/r03b_parity.jsonl
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_longclip_gpu.py tests/test_vae_gpu.py "tests/test_backward_gpu.py::test_null_optimization_vs_reference" \
    "tests/test_reference_gpu.py::test_edit_vs_reference_pipeline[car2-dtype0-100.0]" \
    "tests/test_reference_gpu.py::test_edit_vs_reference_pipeline[car2-dtype1-45.0]" \
    --durations=20 > gpurun_out/r03b_tests.log 2>&1 || { tail -60 gpurun_out/r03b_tests.log; exit 1; }
tail -30 gpurun_out/r03b_tests.log
