#!/bin/bash
# Round 4: the bench line, its rocprofv3 kernel stats, and K1 PMC passes (SQ A/B/C, FETCH/WRITE).
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r04i_bench.json 2> gpurun_out/r04i_bench.err || exit 1
tail -1 gpurun_out/r04i_bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04i_prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 > gpurun_out/r04i_bench_profiled.json 2> gpurun_out/r04i_prof.err || exit 1
bash tools/pmc_k1.sh gpurun_out/r04i_pmc_k1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r04i_pmc_$c -o run -- \
    python3 tools/k1_only.py 5 > gpurun_out/r04i_pmc_$c.log 2>&1 || exit 1
done
echo done
