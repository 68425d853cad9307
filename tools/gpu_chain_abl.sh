#!/bin/bash
# Where the reference-order MFCC's extra time goes (MGX_FLAG_MFCC_REFERENCE, the CHAIN kernels) at N = 1024, all
# features: the default plan, the reference-order plan, and reference-order builds with one part skipped
# (tools/ablate.py patches, copied to ab/lib_x_*.so; their outputs are wrong by design, timing only), one process,
# 7 interleaved rounds (tools/ab_libs.py). Output: gpurun_out/chain_abl.log
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
args="default=base reference=base:2"
for v in chain_none chain_norows chain_nofence no_ln no_dct chain_none_no_ln_no_dct; do args="$args $v=ab/lib_x_$v.so:2"; done
timeout -k 10 400 python tools/ab_libs.py --n ${N:-1024} --rounds 7 $args > gpurun_out/chain_abl.log 2>&1 || { tail -20 gpurun_out/chain_abl.log; exit 1; }
grep -v amdgpu.ids gpurun_out/chain_abl.log
