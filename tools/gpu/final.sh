#!/bin/bash
# The round's measurement set on one box: the default bench line, rocprofv3 kernel stats of a 1-step
# bench, K1 (res-64 pp kernel) PMC passes + HBM traffic, K3 (res-64 stream) HBM traffic + SQ pass.
#   bash tools/gpu/final.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-fin}
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
tail -1 gpurun_out/${tag}_bench.json | cut -c1-300
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/${tag}_profiled.json 2> gpurun_out/${tag}_prof.err || exit 1
rm -f gpurun_out/${tag}_prof/run_kernel_trace.csv
python tools/prof_summary.py gpurun_out/${tag}_prof gpurun_out/${tag}_kernel_stats.txt > /dev/null || exit 1
bash tools/pmc_k1.sh gpurun_out/${tag}_pmc_k1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${tag}_k1_$c -o run -- \
    python3 tools/k1_only.py 5 > gpurun_out/${tag}_k1_$c.log 2>&1 || exit 1
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${tag}_k3_$c -o run -- \
    python3 tools/k3_only.py 5 > gpurun_out/${tag}_k3_$c.log 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT \
  --kernel-trace --output-format csv -d gpurun_out/${tag}_k3_sq -o run -- python3 tools/k3_only.py 5 > gpurun_out/${tag}_k3_sq.log 2>&1 || exit 1
python tools/pmc_traffic.py $(ls gpurun_out/${tag}_k1_FETCH_SIZE/*counter_collection.csv) $(ls gpurun_out/${tag}_k1_WRITE_SIZE/*counter_collection.csv) \
  frame_attn_kernel_pp gpurun_out/${tag}_k1_traffic.json 188743680 32,4096,320 || exit 1
python tools/pmc_traffic.py $(ls gpurun_out/${tag}_k3_FETCH_SIZE/*counter_collection.csv) $(ls gpurun_out/${tag}_k3_WRITE_SIZE/*counter_collection.csv) \
  temporal_attn_stream gpurun_out/${tag}_k3_traffic.json 293601280 32,4096,320 || exit 1
cat gpurun_out/${tag}_k1_traffic.json gpurun_out/${tag}_k3_traffic.json
head -30 gpurun_out/${tag}_kernel_stats.txt
echo done
