#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in base ONE_PASS NO_REDUCE NO_PHASE2; do
  if [ $v = base ]; then unset MEYDA_AMD_LIB; else export MEYDA_AMD_LIB=$PWD/abl/libabl_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python tools/prof_variants.py 1024 2>&1 | grep -E "faithful/(centroid|all|time)|fast/(centroid|all)" || exit 1
done
