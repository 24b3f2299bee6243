#!/bin/bash
# Build a variant libvqa.so in which only the listed sources get extra compile flags (the other objects are the
# product build's, with the Makefile's flags). Usage: tools/mkvar.sh NAME "EXTRA FLAGS" src1.hip [src2.hip ...]  ->  variants/NAME.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; FLAGS=$2; shift 2
C=vae-based-music--deep-generative-models_amd/csrc
B=vae-based-music--deep-generative-models_amd/build
VB=build_var_$NAME
mkdir -p $VB variants
make -s -C $C >/dev/null
objs=""
for o in $B/*.o; do
  src=$(basename $o .o).hip
  if [[ " $* " == *" $src "* ]]; then
    sched=""; [[ $src == vqa_resblock.hip ]] && sched="-mllvm -amdgpu-sched-strategy=max-memory-clause"
    /opt/rocm/bin/hipcc $FLAGS $sched -Xclang -target-feature -Xclang -packed-fp32-ops --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function \
      -Iinclude -mllvm -amdgpu-mfma-vgpr-form=1 -c $C/$src -o $VB/$(basename $o) 2> >(grep -v 'packed-fp32-ops' >&2) &
    objs="$objs $VB/$(basename $o)"
  else
    objs="$objs $o"
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o variants/$NAME.so $objs
echo "variants/$NAME.so"
