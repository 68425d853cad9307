#!/bin/bash
# Device assembly of kernels.hip (optionally with -D flags) and per-kernel VALU op histograms.
# ./tools/isa.sh OUT.s [-DMACRO ...]
cd "$(dirname "$0")/.."
out=$1; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -mllvm -disable-machine-licm \
  "$@" -x hip --cuda-device-only -S -o "$out" meyda_amd/csrc/kernels.hip
