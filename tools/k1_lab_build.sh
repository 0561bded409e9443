#!/bin/bash
# Build K1 A/B variants of libvp2p_hip.so into video-p2p_amd/lib/lab/ (the product objects plus
# frame_attn.o / frame_attn_pp.o compiled with the given -D switches).
# usage: tools/k1_lab_build.sh NAME [-DFLAG=1 ...]
set -e
cd "$(dirname "$0")/../video-p2p_amd"
name=$1; shift
mkdir -p build/lab lib/lab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -fno-honor-nans"
/opt/rocm/bin/hipcc $F "$@" -c csrc/frame_attn.hip -o build/lab/frame_attn_$name.o
/opt/rocm/bin/hipcc $F -mllvm -amdgpu-mfma-vgpr-form "$@" -c csrc/frame_attn_pp.hip -o build/lab/frame_attn_pp_$name.o
objs=$(ls build/*.o | grep -v "frame_attn.o\|frame_attn_pp.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/lab/frame_attn_$name.o build/lab/frame_attn_pp_$name.o \
  -o lib/lab/libvp2p_$name.so
echo built lib/lab/libvp2p_$name.so
