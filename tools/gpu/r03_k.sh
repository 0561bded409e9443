# TunableOp (warm-operand tuning) vs hipBLASLt heuristic on the 8-frame edit
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 800 python tools/tune_gemms.py gpurun_out/tunableop_warm.csv 2> gpurun_out/r03k_tune.err | tee gpurun_out/r03k_tune.jsonl
wc -l gpurun_out/tunableop_warm.csv
