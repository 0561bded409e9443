# VAE parity, then PMC passes on K2 v2 (no-edit launch, res-64)
set -e
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py -x -v --timeout 200 --timeout-method thread -m gpu > gpurun_out/t6.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash tools/pmc_k2.sh $GRAFT_REPO_ROOT/gpurun_out/k2pmc_v2 30
python tools/pmc_summary.py cross_attn_kernel_v2 gpurun_out/k2pmc_v2/A gpurun_out/k2pmc_v2/B gpurun_out/k2pmc_v2/C gpurun_out/k2pmc_v2/D > gpurun_out/k2pmc_v2.txt 2>&1 || true
