#!/bin/bash
# Build an A/B variant of libvp2p_hip.so into video-p2p_amd/lib/lab/libvp2p_NAME.so (or lib/$LABDIR): the product
# objects, with csrc/SRC.hip recompiled under the given -D switches (plus the Makefile's per-file flags).
# usage: tools/lab_build.sh NAME SRC [-DFLAG=1 ...]     (SRC: conv, norm, cross_attn, ...)
set -e
cd "$(dirname "$0")/../video-p2p_amd"
name=$1; src=$2; shift 2
out=${LABDIR:-lab}        # lib/lab is not uploaded by gpurun; LABDIR=diag builds into lib/diag (uploaded)
mkdir -p build/lab lib/$out
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include"
case $src in
  frame_attn) F="$F -fno-honor-nans" ;;
  frame_attn_pp) F="$F -fno-honor-nans -mllvm -amdgpu-mfma-vgpr-form" ;;
esac
/opt/rocm/bin/hipcc $F "$@" -c csrc/$src.hip -o build/lab/${src}_$name.o
objs=$(ls build/*.o | grep -v "^build/$src.o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $objs build/lab/${src}_$name.o -o lib/$out/libvp2p_$name.so
echo built lib/$out/libvp2p_$name.so
