# session 2 start: graph-replay bit-equality, K1 grid A/B (+PMC traffic), default bench on the rebuilt tree
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_graph_gpu.py \
    > gpurun_out/r03e_graph.log 2>&1 || { tail -40 gpurun_out/r03e_graph.log; exit 1; }
tail -3 gpurun_out/r03e_graph.log
for g in bh hf; do
  VP2P_K1_GRID=$g timeout -k 10 120 python tools/kbench.py | grep frame | sed "s/^/{\"k1grid\": \"$g\", \"r\": /; s/$/}/" >> gpurun_out/r03e_k1_ab.jsonl
done
cat gpurun_out/r03e_k1_ab.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for g in bh hf; do
  for c in FETCH_SIZE WRITE_SIZE; do
    VP2P_K1_GRID=$g timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/r03e_pmc_k1_${g}_$c -o run -- python3 tools/k1_only.py 5 > /dev/null 2>&1
  done
done
for g in bh hf; do for c in FETCH_SIZE WRITE_SIZE; do echo "$g $c"; python tools/pmc_summary.py "x2f" gpurun_out/r03e_pmc_k1_${g}_$c; done; done
timeout -k 10 600 python bench.py > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err
cat gpurun_out/r03e_bench.json
