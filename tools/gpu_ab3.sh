#!/bin/bash
# A/B timing (tools/ab_libs.py) of the given variants at N = 1024, 2048 and 512.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd $R
for cfg in "1024 262144" "2048 131072" "512 262144"; do
  set -- $cfg "${@:3}"
  break
done
for cfg in "1024 262144" "2048 131072" "512 262144"; do
  n=${cfg% *}; f=${cfg#* }
  echo "== N=$n frames=$f"
  timeout -k 10 200 python tools/ab_libs.py --rounds 7 --n $n --frames $f $VARIANTS || exit $?
done
