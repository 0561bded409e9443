# K1 lab A/B: base vs double-buffered LDS vs scheduling fences
set -e
R=$GRAFT_REPO_ROOT
cd $R
L=video-p2p_amd/lib/lab
timeout -k 10 400 python -u tools/k1_lab.py gpurun_out/k1_lab_q.jsonl $L/libvp2p_base.so $L/libvp2p_dbuf.so $L/libvp2p_sched.so $L/libvp2p_dbufsched.so > gpurun_out/k1_lab_q.log 2>&1
cat gpurun_out/k1_lab_q.log
