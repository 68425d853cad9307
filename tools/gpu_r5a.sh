set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r5a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "alternate or destroy_right or small_host" > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -3 $O/t.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']); print(json.dumps(d['roofline_fp64'])); print(json.dumps(d['cpu_baseline'].get('all_cores'))); print(json.dumps(d['c4'].get('mfcc_exact'))); print(json.dumps(d['c5'].get('mfcc_exact'))); print(json.dumps(d.get('latency')))"
