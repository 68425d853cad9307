#!/bin/bash
# Build ablation variants of the library into abl/libabl_<NAME>.so (timing experiments only).
cd "$(dirname "$0")/.." && mkdir -p abl
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -mllvm -disable-machine-licm \
    -DMGX_ABL_$v=1 -shared -o abl/libabl_$v.so -x hip meyda_amd/csrc/kernels.hip meyda_amd/csrc/plan.cpp &
done
wait
