#!/bin/bash
# Timing ablations of the current tree (tools/ablate.py variants), interleaved in one process.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/ablations
mkdir -p $O && cd $R
for cfg in "1024 262144" "512 262144"; do
  n=${cfg% *}; f=${cfg#* }
  echo "== N=$n"
  timeout -k 10 300 python tools/ab_libs.py --rounds 5 --n $n --frames $f BASE=base mom_dpp=abl/libabl_mom_dpp.so no_amp=abl/libabl_no_amp.so no_dct=abl/libabl_no_dct.so no_frame_load=abl/libabl_no_frame_load.so no_ln=abl/libabl_no_ln.so no_loud2=abl/libabl_no_loud2.so no_mel=abl/libabl_no_mel.so no_phase2=abl/libabl_no_phase2.so no_prefix=abl/libabl_no_prefix.so no_scalars=abl/libabl_no_scalars.so no_window_load=abl/libabl_no_window_load.so twuni=abl/libabl_twuni.so > $O/abl_$n.log 2>&1 || { tail -20 $O/abl_$n.log; exit 1; }
  grep -v amdgpu.ids $O/abl_$n.log
done
