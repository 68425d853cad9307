#!/bin/bash
# List the PMC counters rocprofv3 offers on this GPU (for choosing --pmc sets).
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p $R/gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --list-avail > $R/gpurun_out/pmc_avail.txt 2>&1
grep -c "" $R/gpurun_out/pmc_avail.txt
