#!/bin/bash
# Build the library as it was at git revision REV into ab/lib_NAME.so (the baseline of an A/B timing with
# tools/ab_libs.py; the tree is untouched).  usage: tools/build_rev.sh REV NAME
set -e
cd "$(dirname "$0")/.."
rev=$1; name=$2
tmp=$(mktemp -d)
git archive "$rev" meyda_amd/csrc include | tar -x -C "$tmp"
mkdir -p ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -Wall -Wno-unused-result \
  -mllvm -disable-machine-licm -I "$tmp/meyda_amd/csrc" -I "$tmp/include" -shared -o ab/lib_$name.so -x hip \
  "$tmp/meyda_amd/csrc/kernels.hip" "$tmp/meyda_amd/csrc/plan.cpp" "$tmp/meyda_amd/csrc/group.cpp" -ldl 2>&1 | grep -v hip-link || true
rm -rf "$tmp"
test -f ab/lib_$name.so && echo "built ab/lib_$name.so from $rev"
