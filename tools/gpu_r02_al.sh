# final tree: full GPU suite + smoke
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/suite_al.log 2>&1 || { tail -30 gpurun_out/suite_al.log; exit 1; }
tail -2 gpurun_out/suite_al.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_al.log 2>&1
tail -2 gpurun_out/smoke_al.log
