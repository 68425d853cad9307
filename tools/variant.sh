#!/bin/bash
# Build the current tree's library with extra compile flags into ab/lib_NAME.so (A/B variants for
# tools/ab_libs.py; the tree's own library is untouched).  usage: tools/variant.sh NAME [-DFLAG ...]
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-result \
  -mllvm -disable-machine-licm "$@" -shared -o ab/lib_$name.so -x hip \
  meyda_amd/csrc/kernels.hip meyda_amd/csrc/plan.cpp meyda_amd/csrc/group.cpp -ldl 2>&1 | grep -v hip-link || true
test -f ab/lib_$name.so
