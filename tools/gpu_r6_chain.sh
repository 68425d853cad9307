#!/bin/bash
# Round 6, after the cheaper pow023 (loudness) and the reference-order MFCC's fast log (ref_ln): the -m gpu suite,
# then launch times against the round-start library (ab/lib_r6a.so, tools/build_rev.sh), outputs compared bit for
# bit, at the headline and in reference order (flag 2); then the reference-order MFCC's cost ladder with the fixed
# chain ablation (tools/ablate.py chain_none now skips both chain forms) and its PMC instruction budget.
# Results in gpurun_out/r6c/.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r6c
mkdir -p $O && cd $R
step() { echo "[r6c] $1 $(date +%T)"; }
step mfma_order
timeout -k 10 120 tools/ubench/mfma_f64_order | tee $O/mfma_order.log || exit 1
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step ab_default
timeout -k 10 300 python tools/ab_libs.py --n 1024 --rounds 7 --compare old=ab/lib_r6a.so new=base > $O/ab_default.log 2>&1 || { tail -20 $O/ab_default.log; exit 1; }
grep -v amdgpu.ids $O/ab_default.log
timeout -k 10 300 python tools/ab_libs.py --n 2048 --rounds 5 --compare old=ab/lib_r6a.so new=base > $O/ab_2048.log 2>&1 || { tail -20 $O/ab_2048.log; exit 1; }
grep -v amdgpu.ids $O/ab_2048.log
step ab_reference
timeout -k 10 300 python tools/ab_libs.py --n 1024 --rounds 7 --compare old=ab/lib_r6a.so:2 new=base:2 > $O/ab_ref.log 2>&1 || { tail -20 $O/ab_ref.log; exit 1; }
grep -v amdgpu.ids $O/ab_ref.log
step chain_ladder
args="default=base reference=base:2 c_nochains=ab/lib_r6_c_nochains.so:2 c_norows=ab/lib_r6_c_norows.so:2 c_nolndct=ab/lib_r6_c_nolndct.so:2 c_skel=ab/lib_r6_c_skel.so:2 d_skel=ab/lib_r6_d_skel.so"
timeout -k 10 500 python tools/ab_libs.py --n 1024 --rounds 7 $args > $O/chain_ab.log 2>&1 || { tail -20 $O/chain_ab.log; exit 1; }
grep -v amdgpu.ids $O/chain_ab.log
step chain_pmc
BUDGET_TAG=r6c/chain_budget BUDGET_VARIANTS="old=ab/lib_r6a.so $args" timeout -k 10 600 $R/tools/gpu_budget.sh > $O/chain_budget.log 2>&1 || { tail -20 $O/chain_budget.log; exit 1; }
cat $O/chain_budget/budget.txt
step rehearsal
run() {  # port tag args...
  local port=$1 tag=$2; shift 2
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 2 --allow-shared-gpu --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/$tag.log 2>&1
}
summ() { tail -1 $O/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gather']; c=d['c5']; print('$1', 'shards', round(d['value']/1e6,1), 'M/s gather', g.get('status'), round((g.get('value') or 0)/1e6,1), 'vs_shards', round(g.get('vs_shards') or 0,3), 'ms/step', round(g.get('ms_per_step') or 0,3), '| c5 value', round((c.get('value') or 0)/1e6,1), 'shards_value', round(c['shards_value']/1e6,1), 'vs', round(c['gather'].get('vs_shards') or 0,3))"; }
rm -f /tmp/r6trace_*
port=29561
for mode in sync_copy lag_copy lag_zero; do
  port=$((port+1))
  ( export MGX_GROUP_TRANSPORT=ipc MGX_GROUP_TRACE=/tmp/r6trace_$mode
    case $mode in sync_copy) export MGX_IPC_SYNC=1 MGX_IPC_COPY=1;; lag_copy) export MGX_IPC_COPY=1;; esac
    run $port ipc_$mode ) || { tail -30 $O/ipc_$mode.log; exit 1; }
  summ ipc_$mode
  echo "-- $mode"; python3 tools/gather_trace.py /tmp/r6trace_$mode --last 20
done
cp /tmp/r6trace_* $O/ 2>/dev/null
step done
