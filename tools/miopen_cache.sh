#!/bin/bash
# Fill MIOpen's user find/perf database and compiled-kernel cache for every convolution the tests and
# the bench run on MIOpen (the fp32 edits: all convolutions, at 2 / 8 / 24 frames; bf16: conv_in /
# conv_out), starting from the in-tree ones, into OUTDIR; then copy OUTDIR/*.txt to miopen_db/ and
# OUTDIR/kcache/*.ukdb to miopen_db/kcache/.   bash tools/miopen_cache.sh OUTDIR   (on the MI355X)
# Without the find entries MIOpen searches every applicable solver (naive ones included) at the first
# call of each new shape: 11-35 s per 24-frame fp32 shape (profiles/r04_fp32_conv_probe.jsonl).
set -o pipefail
out=$1; mkdir -p $out/kcache
cp miopen_db/*.txt $out/ && cp miopen_db/kcache/*.ukdb $out/kcache/ 2>/dev/null
export MIOPEN_USER_DB_PATH=$(cd $out && pwd) MIOPEN_CUSTOM_CACHE_DIR=$(cd $out/kcache && pwd)
# a heartbeat under gpurun_out while one long test runs silently (each step below has its own limit)
(while true; do date >> $out.heartbeat; sleep 50; done) & hb=$!
timeout -k 10 1000 python -u -m pytest tests/test_reference_gpu.py -k "edit_vs_reference_pipeline and fp32" -v \
  --timeout 900 --timeout-method thread --durations=5 > $out.log 2>&1; rc=$?
tail -12 $out.log
if [ $rc -eq 0 ]; then timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 > $out.bench.json 2>&1; rc=$?; fi
kill $hb
ls -la $out $out/kcache
exit $rc
