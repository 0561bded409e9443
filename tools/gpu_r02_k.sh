# K1 folded-max PMC passes (3 x 5 dispatches)
set -e
R=$GRAFT_REPO_ROOT
cd $R
export TMPDIR=/tmp
bash tools/pmc_k1.sh gpurun_out/k1pmc_fold
python tools/pmc_summary.py frame_attn_kernel_x2f gpurun_out/k1pmc_fold/A gpurun_out/k1pmc_fold/B gpurun_out/k1pmc_fold/C > gpurun_out/k1pmc_fold.txt 2>&1 || true
cat gpurun_out/k1pmc_fold.txt
