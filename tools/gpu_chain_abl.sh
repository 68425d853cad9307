#!/bin/bash
# Where the paired-chain (MGX_FLAG_MFCC_REFERENCE) kernel's extra time goes: timing ablations in one
# process (chains skipped / row stores skipped / the fence dropped) and the HBM traffic per launch.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/chain_abl
mkdir -p $O && cd $R
timeout -k 10 300 python tools/ab_libs.py --n 1024 --rounds 5 REF_G=base:2 NONE=ab/libabl_chain_none.so:2 NOROWS=ab/libabl_chain_norows.so:2 NOFENCE=ab/libabl_chain_nofence.so:2 DEF=base > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
BUDGET_TAG=chain_pmc BUDGET_SETS="FETCH_SIZE|WRITE_SIZE|SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
  BUDGET_VARIANTS="DEF=base REF_G=base:2 NONE=ab/libabl_chain_none.so:2 NOROWS=ab/libabl_chain_norows.so:2" bash tools/gpu_budget.sh
