#!/bin/bash
# configs[3] (official mode: DDIM inversion + null-text optimisation) -- where its time goes.
#   bash tools/gpu/nulltext_prof.sh TAG [DDIM_STEPS]
# 1. the bench's nulltext line at DDIM_STEPS (default 10) DDIM steps x 10 Adam iterations;
# 2. rocprofv3 kernel stats of the same command (total kernel time vs wall: GPU-busy fraction);
# 3. cProfile of the host side of the same command.
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-nt}; n=${2:-10}
mkdir -p gpurun_out
A="--mode nulltext --steps 1 --warmup 1 --ddim-steps $n --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $A > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
tail -1 gpurun_out/${tag}_bench.json | cut -c1-300
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- \
  python3 bench.py $A > gpurun_out/${tag}_profiled.json 2> gpurun_out/${tag}_prof.err || exit 1
rm -f gpurun_out/${tag}_prof/run_kernel_trace.csv
python tools/prof_summary.py gpurun_out/${tag}_prof gpurun_out/${tag}_kernel_stats.txt > /dev/null || exit 1
head -45 gpurun_out/${tag}_kernel_stats.txt
timeout -k 10 300 python -u -c "
import cProfile, pstats, io, sys
sys.argv = ['bench.py'] + '$A'.split()
sys.path.insert(0, '.')
import bench
pr = cProfile.Profile(); pr.enable(); bench.main(); pr.disable()
s = io.StringIO(); st = pstats.Stats(pr, stream=s).sort_stats('tottime'); st.print_stats(40)
st.sort_stats('cumulative').print_stats(40)
open('gpurun_out/${tag}_host_profile.txt', 'w').write(s.getvalue())
" > gpurun_out/${tag}_host.log 2>&1 || exit 1
echo done
