# conv_in / conv_out on K10 (channel padding): host profile at 1 frame, small-frame bench, UNet parity tests
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python tools/host_profile.py 1 gpurun_out/host_profile_aa.txt > gpurun_out/host_profile_aa.log 2>&1
timeout -k 10 200 python bench.py --frames 1 --steps 2 --warmup 1 --extras none --no-cpu-baseline --no-events > gpurun_out/hb_aa_f1.json 2>/dev/null
timeout -k 10 200 python bench.py --frames 2 --steps 2 --warmup 1 --extras none --no-cpu-baseline --no-events > gpurun_out/hb_aa_f2.json 2>/dev/null
cut -c1-250 gpurun_out/hb_aa_f1.json gpurun_out/hb_aa_f2.json
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_reference_gpu.py tests/test_unet_gpu.py > gpurun_out/tests_aa.log 2>&1 || { tail -30 gpurun_out/tests_aa.log; exit 1; }
tail -2 gpurun_out/tests_aa.log
