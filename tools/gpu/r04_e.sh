#!/bin/bash
# Round 4: MFMA / v_exp / VALU co-issue microbenchmark (tools/issue_bench.hip), then the kernel tests on
# the cleaned-up library (A/B switches and rejected variants removed).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 120 tools/issue_bench > gpurun_out/r04e_issue_bench.jsonl || exit 1
cat gpurun_out/r04e_issue_bench.jsonl
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_conv_gpu.py > gpurun_out/r04e_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r04e_tests.log; exit $rc
