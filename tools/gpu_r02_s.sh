# K10 GEGLU epilogue with the branch-free erf: old (lab dbuf build) vs new; GEGLU tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 env VP2P_LIB=$R/video-p2p_amd/lib/lab/libvp2p_dbuf.so python tools/geglu_bench.py > gpurun_out/geglu_s_old.jsonl
timeout -k 10 120 python tools/geglu_bench.py > gpurun_out/geglu_s_new.jsonl
cat gpurun_out/geglu_s_old.jsonl gpurun_out/geglu_s_new.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_gpu.py tests/test_norm_gpu.py tests/test_reference_gpu.py -k "geglu or transformer or Transformer" > gpurun_out/tests_s.log 2>&1
tail -3 gpurun_out/tests_s.log
