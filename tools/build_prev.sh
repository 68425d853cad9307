#!/bin/bash
# Build ab/libabl_PREV.so (ab/ travels to the GPU box; abl/ does not) from kernels.hip at a git revision (default HEAD) for A/B timing.
cd "$(dirname "$0")/.." && mkdir -p ab
git show ${1:-HEAD}:meyda_amd/csrc/kernels.hip > meyda_amd/csrc/.prev_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -mllvm -disable-machine-licm \
  -shared -o ab/libabl_PREV.so -x hip meyda_amd/csrc/.prev_kernels.hip meyda_amd/csrc/plan.cpp
rc=$?; rm -f meyda_amd/csrc/.prev_kernels.hip; exit $rc
