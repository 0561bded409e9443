#!/bin/bash
# Small-clip A/B on one box: 1- and 3-frame graphed edits on the product library and every
# video-p2p_amd/lib/ab/*.so, two rounds.   bash tools/gpu/sc_ab.sh TAG
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-scab}
mkdir -p gpurun_out
for r in 0 1; do
  for lib in video-p2p_amd/lib/libvp2p_hip.so video-p2p_amd/lib/ab/*.so; do
    n=$(basename $lib .so)
    for f in 1 3; do
      VP2P_LIB=$PWD/$lib timeout -k 10 240 python -u bench.py --frames $f --graphs 1 --steps 2 --warmup 1 --extras none \
        --no-cpu-baseline --no-events > gpurun_out/${tag}_${n}_f${f}_$r.json 2> gpurun_out/${tag}_${n}_f${f}_$r.err || exit 1
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'f'+sys.argv[3], sys.argv[4], d['ms_per_step'])" \
        gpurun_out/${tag}_${n}_f${f}_$r.json $n $f $r | tee -a gpurun_out/${tag}.txt
    done
  done
done
