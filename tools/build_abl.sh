#!/bin/bash
# Build ablation variants of the library into abl/libabl_<NAME>.so (timing experiments only).
# NAME is a macro (-DMGX_ABL_NAME=1) or NAME=VALUE for a plain -D (e.g. MGX_FB=16 -> libabl_MGX_FB_16.so).
cd "$(dirname "$0")/.." && mkdir -p abl
for v in "$@"; do
  case $v in
    *=*) def="-D$v"; tag=$(echo $v | tr '=' '_') ;;
    *) def="-DMGX_ABL_$v=1"; tag=$v ;;
  esac
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -mllvm -disable-machine-licm \
    $def -shared -o abl/libabl_$tag.so -x hip meyda_amd/csrc/kernels.hip meyda_amd/csrc/plan.cpp &
done
wait
