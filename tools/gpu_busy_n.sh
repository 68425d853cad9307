#!/bin/bash
# VALU-busy fraction and instruction mix per frame of the all-feature kernel at several N (rocprofv3 --pmc
# passes, kernel-trace only, over tools/pmc_probe.py: 262,144 frames, 3 launches): is the launch bound by VALU
# issue at each N, or waiting? usage: tools/gpu_busy_n.sh [N ...]   Output: gpurun_out/busy_n/summary.txt
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O=$R/gpurun_out/busy_n
mkdir -p $O && cd /tmp && export TMPDIR=/tmp
NS="${*:-2048 1024 512}"
for n in $NS; do
  i=0
  for ctrs in "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE" \
              "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64"; do
    i=$((i + 1))
    PROBE_SET=all PROBE_N=$n timeout -s KILL 90 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv \
      -d $O/n$n/p$i -o run -- python3 $R/tools/pmc_probe.py > $O/n$n.p$i.log 2>&1 || { echo "pmc failed n=$n pass $i"; exit 1; }
  done
done
python3 - "$O" $NS > $O/summary.txt <<'PY'
import collections, csv, glob, sys
O, ns = sys.argv[1], sys.argv[2:]
F = 262144
for n in ns:
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{O}/n{n}/*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if "extract_kernel" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    c = {k: sum(v) / len(v) for k, v in agg.items()}
    kcyc = c["GRBM_GUI_ACTIVE"] / 8.0
    simds = 1024
    print(f"N={n}: valu_busy {4 * c['SQ_ACTIVE_INST_VALU'] / (kcyc * simds):.3f}  any_busy {4 * c['SQ_ACTIVE_INST_ANY'] / (kcyc * simds):.3f}"
          f"  lds_busy {4 * c['SQ_ACTIVE_INST_LDS'] / (kcyc * simds):.3f}  waves/SIMD(avg over kernel) {c['SQ_WAVE_CYCLES'] / (kcyc * simds):.2f}"
          f"  wait_any/wave_cycles {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}  wait_inst_any/wave_cycles {c['SQ_WAIT_INST_ANY'] / c['SQ_WAVE_CYCLES']:.3f}")
    print("   per frame: " + "  ".join(f"{k.replace('SQ_INSTS_', '')} {c[k] / F:.1f}" for k in sorted(c) if k.startswith("SQ_INSTS")))
    print("   kernel cycles (GRBM_GUI_ACTIVE / 8) %.0f = %.3f ms at 2.4 GHz" % (kcyc, kcyc / 2.4e6))
PY
cat $O/summary.txt
