# K1 lab: iglp_opt(0) and s_setprio(1) on the folded d = 40 loop vs the product build
set -e
R=$GRAFT_REPO_ROOT
cd $R
L=video-p2p_amd/lib/lab
timeout -k 10 300 python -u tools/k1_lab.py gpurun_out/k1_lab_ak.jsonl $L/libvp2p_base.so $L/libvp2p_iglp0.so $L/libvp2p_prio1.so > gpurun_out/k1_lab_ak.log 2>&1
python - <<'PY'
import json
for l in open("gpurun_out/k1_lab_ak.jsonl"):
    r=json.loads(l); print(r["round"], r["lib"], r["d"], r["ms_median"], r["tflops"], r["abs_sum"])
PY
