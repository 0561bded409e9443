# the attn_temp qkv projection (N = 960) on K10 vs hipBLASLt
set -e
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 120 env VP2P_LINEAR_K10_MAX_N=960 python tools/linear_plain_ab.py gpurun_out/linear_plain_ai.jsonl 131072x320x960 16384x320x640
