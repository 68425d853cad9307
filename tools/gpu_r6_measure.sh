#!/bin/bash
# Round-6 measurements in one GPU call (results in gpurun_out/r6m/):
#  1. the group tests (the IPC hand-over now runs one chunk behind extraction);
#  2. the two-rank cross-process rehearsal of the gather (bench.py under torchrun, MGX_GROUP_TRANSPORT=ipc), with
#     the hand-over traced (MGX_GROUP_TRACE) -- round 5's synchronous hand-over (MGX_IPC_SYNC=1) first, then the
#     lagged one -- and tools/gather_trace.py's split of each;
#  3. the reference-order MFCC's cost, item by item: launch times of the CHAIN kernel with its parts removed one after
#     another (tools/ablate.py builds copied to ab/lib_r6_*.so; outputs wrong by design), the default kernel's own
#     skeleton beside it, then the PMC instruction budget of the same variants;
#  4. the launch overlap of consecutive steps (tools/step_overlap.py).
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/r6m
mkdir -p $O && cd $R
step() { echo "[r6m] $1 $(date +%T)"; }
step group_tests
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 160 --timeout-method thread -p no:cacheprovider > $O/group_tests.log 2>&1 || { tail -30 $O/group_tests.log; exit 1; }
tail -1 $O/group_tests.log
run() {  # port tag args...
  local port=$1 tag=$2; shift 2
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 2 --allow-shared-gpu --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/$tag.log 2>&1
}
summ() { tail -1 $O/$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); g=d['gather']; c=d['c5']; print('$1', 'shards', round(d['value']/1e6,1), 'M/s gather', g.get('status'), round((g.get('value') or 0)/1e6,1), 'vs_shards', round(g.get('vs_shards') or 0,3), 'ms/step', round(g.get('ms_per_step') or 0,3), '| c5 value', round((c.get('value') or 0)/1e6,1), 'shards_value', round(c['shards_value']/1e6,1), 'vs', round(c['gather'].get('vs_shards') or 0,3))"; }
step rehearsal_sync
rm -f /tmp/r6trace_sync.* /tmp/r6trace_lag.*
MGX_GROUP_TRANSPORT=ipc MGX_IPC_SYNC=1 MGX_GROUP_TRACE=/tmp/r6trace_sync run 29541 ipc_sync || { tail -30 $O/ipc_sync.log; exit 1; }
summ ipc_sync
step rehearsal_lag
MGX_GROUP_TRANSPORT=ipc MGX_GROUP_TRACE=/tmp/r6trace_lag run 29542 ipc_lag || { tail -30 $O/ipc_lag.log; exit 1; }
summ ipc_lag
cp /tmp/r6trace_sync.* /tmp/r6trace_lag.* $O/ 2>/dev/null
echo "sync (round 5's hand-over), N=1024 gather phase then C5:"; python3 tools/gather_trace.py /tmp/r6trace_sync --last 20
echo "lagged:"; python3 tools/gather_trace.py /tmp/r6trace_lag --last 20
step chain_ab
args="default=base reference=base:2 c_nochains=ab/lib_r6_c_nochains.so:2 c_norows=ab/lib_r6_c_norows.so:2 c_skel=ab/lib_r6_c_skel.so:2 c_nolndct=ab/lib_r6_c_nolndct.so:2 c_plain=ab/lib_r6_c_plain.so:2 d_skel=ab/lib_r6_d_skel.so"
timeout -k 10 500 python tools/ab_libs.py --n 1024 --rounds 7 $args > $O/chain_ab.log 2>&1 || { tail -20 $O/chain_ab.log; exit 1; }
grep -v amdgpu.ids $O/chain_ab.log
step chain_pmc
BUDGET_TAG=r6m/chain_budget BUDGET_VARIANTS="$args" timeout -k 10 600 $R/tools/gpu_budget.sh > $O/chain_budget.log 2>&1 || { tail -20 $O/chain_budget.log; exit 1; }
cat $O/chain_budget/budget.txt
cd $R
step overlap
timeout -k 10 300 python tools/step_overlap.py > $O/overlap.log 2>&1 || { tail -20 $O/overlap.log; exit 1; }
grep -v amdgpu.ids $O/overlap.log | tail -12
step done
