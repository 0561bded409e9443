set -e
export VP2P_PARITY_REPORT=$PWD/gpurun_out/parity_g.jsonl
rm -f $VP2P_PARITY_REPORT
timeout -k 10 600 python -u -m pytest tests/test_reference_gpu.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/t8.log 2>&1
