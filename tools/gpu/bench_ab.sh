#!/bin/bash
# Whole-edit A/B on one box: bench.py (no extras) alternating the product library and every
# video-p2p_amd/lib/$AB_DIR/*.so (default ab; "diag" is uploaded, "ab" is not), two rounds.
#   [AB_DIR=diag] bash tools/gpu/bench_ab.sh TAG [bench args]
set -o pipefail
cd "$(dirname "$0")/../.."
tag=${1:-benchab}; shift
mkdir -p gpurun_out
for r in 0 1; do
  for lib in video-p2p_amd/lib/libvp2p_hip.so video-p2p_amd/lib/${AB_DIR:-ab}/*.so; do
    n=$(basename $lib .so)
    VP2P_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --extras none --no-cpu-baseline "$@" \
      > gpurun_out/${tag}_${n}_$r.json 2> gpurun_out/${tag}_${n}_$r.err || { tail -20 gpurun_out/${tag}_${n}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), (d.get('attention') or {}).get('mfma_util'))" \
      gpurun_out/${tag}_${n}_$r.json $n $r | tee -a gpurun_out/${tag}.txt
  done
done
