#!/bin/bash
# The driver's multi-GPU command line, rehearsed on a one-GPU box with two ranks sharing the
# device: the torchrun / gloo control path without the gather, then WITH the gather through the
# cross-process IPC test transport (MGX_GROUP_TRANSPORT=ipc: every chunk crosses the process
# boundary through hipIpc-mapped transfer buffers; RCCL itself refuses two ranks on one device),
# then the same gather with a forced failure, which must exit non-zero after the line.
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/dist
mkdir -p $O && cd $R
run() {  # port tag args...
  local port=$1 tag=$2; shift 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port \
    bench.py --gpus 2 --allow-shared-gpu "$@" > $O/$tag.log 2>&1
}
run 29533 nogather --steps 20 --warmup 5 --no-gather || { tail -20 $O/nogather.log; exit 1; }
tail -1 $O/nogather.log | cut -c1-300
MGX_GROUP_TRANSPORT=ipc run 29534 ipc --steps 20 --warmup 5 || { tail -30 $O/ipc.log; exit 1; }
tail -1 $O/ipc.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({k: d['gather'].get(k) for k in ('status','value','vs_shards','ms_per_step','rccl_comm','transport','finite_last_frames')})); print('c5', json.dumps({k: d['c5']['gather'].get(k) for k in ('status','value','vs_shards','ms_per_step')}))"
# a peer that never posts: the root's wait passes its deadline, the line is printed, the run exits 3
MGX_GROUP_TRANSPORT=ipc MGX_IPC_TIMEOUT_S=5 MGX_IPC_FAIL_RANK=1 run 29535 ipcfail --steps 5 --warmup 2 --no-c5 --gather-timeout 30
rc=$?; echo "forced gather failure: torchrun rc=$rc (non-zero wanted); ranks' exit codes:"; grep -oE "exitcode *: *-?[0-9]+" $O/ipcfail.log | sort | uniq -c
grep -m1 '^{"metric"' $O/ipcfail.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('line printed; gather:', d['gather']['status'][:200])"
[ $rc -ne 0 ] || exit 1
