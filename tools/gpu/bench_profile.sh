#!/bin/bash
# The bench line (product, and the x2f lab library as the K1 A/B baseline on the same box),
# its rocprofv3 kernel stats, and K1 PMC passes (SQ A/B/C, FETCH/WRITE).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bp_bench.json 2> gpurun_out/bp_bench.err || exit 1
tail -1 gpurun_out/bp_bench.json | cut -c1-200
X2F=$PWD/video-p2p_amd/lib/lab/libvp2p_x2f.so     # tools/lab_build.sh x2f frame_attn -DVP2P_K1_LAB_X2F=1
if [ -f $X2F ]; then
  VP2P_LIB=$X2F timeout -k 10 300 python -u bench.py --extras none --no-cpu-baseline \
    > gpurun_out/bp_bench_x2f.json 2> gpurun_out/bp_bench_x2f.err || exit 1
  tail -1 gpurun_out/bp_bench_x2f.json | cut -c1-200
fi
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bp_prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --extras none --no-cpu-baseline > gpurun_out/bp_bench_profiled.json 2> gpurun_out/bp_prof.err || exit 1
rm -f gpurun_out/bp_prof/run_kernel_trace.csv
bash tools/pmc_k1.sh gpurun_out/bp_pmc_k1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/bp_pmc_$c -o run -- \
    python3 tools/k1_only.py 5 > gpurun_out/bp_pmc_$c.log 2>&1 || exit 1
done
du -sh gpurun_out
echo done
