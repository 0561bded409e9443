#!/bin/bash
# PMC of the K10 shapes that carry most of the edit's conv / projection time: the wide 3x3 conv
# (64^2, 320 -> 320, B f = 32), the res-32 3x3 (640 -> 640), and the K10s streams (K = N = 320
# residual / plain, the N = 2560 GEGLU), each as its own target (tools/conv_only.py /
# tools/gemm_only.py) in five passes: A/B/C (wave-cycle split, MFMA busy, LDS), F (FETCH_SIZE),
# W (WRITE_SIZE).  Summaries -> gpurun_out/k10pmc/summary.txt, traffic -> gpurun_out/k10pmc/*.json
#   [K10PMC_SET=small] bash tools/gpu/k10_pmc.sh
set -o pipefail
cd "$(dirname "$0")/../.."
out=gpurun_out/k10pmc
mkdir -p $out
export TMPDIR=/tmp
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES"
C="SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES SQ_WAVE_CYCLES"
F="FETCH_SIZE"
W="WRITE_SIZE"
run() {  # name kernel_substr alg_bytes cmd...
  local name=$1 sub=$2 alg=$3; shift 3
  for p in A B C F W; do
    timeout -s KILL 60 rocprofv3 --pmc ${!p} --kernel-trace --output-format csv -d $out/$name/$p -o run -- "$@" \
      > $out/$name/$p.log 2>&1 || { echo "$name pass $p failed"; tail -5 $out/$name/$p.log; return 1; }
  done
  { echo "## $name ($*)"; python3 tools/pmc_summary.py "$sub" $out/$name/A $out/$name/B $out/$name/C; } >> $out/summary.txt || return 1
  python3 tools/pmc_traffic.py $out/$name/F/run_counter_collection.csv $out/$name/W/run_counter_collection.csv \
    "$sub" $out/$name.json $alg || return 1
  echo "$name ok"
}
rm -f $out/summary.txt
if [ "$K10PMC_SET" = small ]; then   # the 3-frame clip's 64^2 convs: the 192 x 320 tile vs 128 x 160 (VP2P_K10_PLAN=0,1)
  mkdir -p $out/m320 $out/g320 $out/m960 $out/g960
  run m320 "conv_kernel_m<3" $((2 * (12*4096*320*3 + 320*320*9))) python3 tools/conv_only.py 12 320 64 320 5 &&
  VP2P_K10_PLAN=0,1 run g320 "conv_kernel_g<3" $((2 * (12*4096*320*3 + 320*320*9))) python3 tools/conv_only.py 12 320 64 320 5 &&
  run m960 "conv_kernel_m<3" $((2 * (12*4096*(960+320*2) + 320*960*9))) python3 tools/conv_only.py 12 960 64 320 5 &&
  VP2P_K10_PLAN=0,1 run g960 "conv_kernel_g<3" $((2 * (12*4096*(960+320*2) + 320*960*9))) python3 tools/conv_only.py 12 960 64 320 5 &&
  echo all-ok
  exit $?
fi
mkdir -p $out/c3 $out/c3r32 $out/sres $out/splain $out/sgeglu
# algorithmic bytes: x + W + residual in, y out (bf16)
run c3 "conv_kernel_w<3" $((2 * (32*4096*320*3 + 320*320*9))) python3 tools/conv_only.py 32 320 64 320 5 &&
run c3r32 "conv_kernel_w<3" $((2 * (32*1024*640*3 + 640*640*9))) python3 tools/conv_only.py 32 640 32 640 5 &&
run sres "conv_kernel_k320" $((2 * (131072*320*3 + 320*320))) python3 tools/gemm_only.py residual 131072 320 320 5 &&
run splain "conv_kernel_k320" $((2 * (131072*320*2 + 320*320))) python3 tools/gemm_only.py plain 131072 320 320 5 &&
run sgeglu "conv_kernel_k320" $((2 * (131072*320 + 131072*1280 + 2560*320))) python3 tools/gemm_only.py geglu 131072 320 2560 5 &&
echo all-ok
