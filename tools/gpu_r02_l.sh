# K1 fold: double-buffered (default) vs single-buffered x2f form, interleaved; K1 kernel tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
for rep in 1 2; do
  timeout -k 10 120 python tools/k1_modes.py gpurun_out/k1_modes_l_db.jsonl > /dev/null
  VP2P_K1_FOLD=x2f timeout -k 10 120 python tools/k1_modes.py gpurun_out/k1_modes_l_x2f.jsonl > /dev/null
done
grep '"prescaled": true' gpurun_out/k1_modes_l_db.jsonl gpurun_out/k1_modes_l_x2f.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k frame > gpurun_out/t13.log 2>&1
tail -2 gpurun_out/t13.log
