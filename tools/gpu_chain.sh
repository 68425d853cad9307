#!/bin/bash
# MGX_FLAG_MFCC_REFERENCE as mel chains: parity tests, then the cost against the default plan.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/${CHAIN_TAG:-chain}
mkdir -p $O && cd $R
echo "[chain] tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_mfcc_chain.py tests/test_gpu_parity.py -k "chain or reference" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
echo "[chain] cost"
MGX_GRID_CAP=print timeout -k 10 300 python tools/mfcc_cost.py --n 1024 512 256 > $O/cost_all.log 2>&1 || { tail -20 $O/cost_all.log; exit 1; }
cat $O/cost_all.log | grep -v amdgpu.ids
timeout -k 10 300 python tools/mfcc_cost.py --n 1024 512 --features c4 > $O/cost_c4.log 2>&1 || { tail -20 $O/cost_c4.log; exit 1; }
grep -v amdgpu.ids $O/cost_c4.log
echo "[chain] ablation: the chains skipped"
MEYDA_AMD_LIB=$R/abl/libabl_chain_none.so timeout -k 10 300 python tools/mfcc_cost.py --n 1024 512 --rounds 5 > $O/cost_none.log 2>&1 || { tail -20 $O/cost_none.log; exit 1; }
grep -v amdgpu.ids $O/cost_none.log
