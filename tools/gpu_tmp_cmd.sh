#!/bin/bash
# Scratch GPU command of the current experiment (kept for the record of what ran).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/stag && mkdir -p $O && cd $R
timeout -k 10 300 python tools/ab_libs.py --rounds 7 base=base st1=abl/libabl_st1.so st2=abl/libabl_st2.so st4=abl/libabl_st4.so > $O/ab.log 2>&1
rc=$?; grep median $O/ab.log; exit $rc
