#!/bin/bash
# A/B timing of alternative library builds: ./tools/gpu_ab.sh base NT ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "$@"; do
  if [ $v = base ]; then unset MEYDA_AMD_LIB; else export MEYDA_AMD_LIB=$PWD/abl/libabl_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python tools/prof_variants.py ${VARIANT_NS:-1024} 2>&1 | grep -E "faithful/(time_only|centroid|spectral\+loud|mfcc|all)|fast/(centroid|all)" || exit 1
done
