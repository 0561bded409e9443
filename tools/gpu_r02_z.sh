# host-side profile at small frame counts (where the launch rate limits the step time)
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python tools/host_profile.py 1 gpurun_out/host_profile_z.txt > gpurun_out/host_profile_z.log 2>&1
timeout -k 10 200 python bench.py --frames 1 --steps 2 --warmup 1 --extras none --no-cpu-baseline --no-events > gpurun_out/hb_z_f1.json 2>/dev/null
timeout -k 10 200 python bench.py --frames 2 --steps 2 --warmup 1 --extras none --no-cpu-baseline --no-events > gpurun_out/hb_z_f2.json 2>/dev/null
cat gpurun_out/hb_z_f1.json gpurun_out/hb_z_f2.json | cut -c1-300
