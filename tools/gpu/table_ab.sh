#!/bin/bash
# Whole-edit A/B of two kernel-choice tables on one box: the tracked miopen_db/kernel_choices.json
# against miopen_db/kernel_choices_new.json (swapped in on the box's copy), two rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
cp miopen_db/kernel_choices.json gpurun_out/kc_old.json
for r in 0 1; do
  for t in old new; do
    if [ $t = new ]; then cp miopen_db/kernel_choices_new.json miopen_db/kernel_choices.json; else cp gpurun_out/kc_old.json miopen_db/kernel_choices.json; fi
    timeout -k 10 300 python -u bench.py --extras none --no-cpu-baseline > gpurun_out/tab_${t}_$r.json 2> gpurun_out/tab_${t}_$r.err || { tail -20 gpurun_out/tab_${t}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/tab_${t}_$r.json $t $r | tee -a gpurun_out/table_ab.txt
  done
done
cp gpurun_out/kc_old.json miopen_db/kernel_choices.json
