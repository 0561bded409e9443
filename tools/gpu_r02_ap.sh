# K2 v3 PMC (res-64 non-edit launch, step 30) and the K2 v1/v3 edit launch (step 3)
set -e
R=$GRAFT_REPO_ROOT
cd $R
bash tools/pmc_k2.sh gpurun_out/k2pmc_v3 30
python tools/pmc_summary.py cross_attn_kernel_v3 gpurun_out/k2pmc_v3/A gpurun_out/k2pmc_v3/B gpurun_out/k2pmc_v3/C gpurun_out/k2pmc_v3/D > gpurun_out/k2pmc_v3.txt 2>&1 || true
cat gpurun_out/k2pmc_v3.txt
