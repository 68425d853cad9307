#!/usr/bin/env python3
"""Benchmark of the meyda hot path on MI355X.

Metric (BASELINE.json): audio frames/sec at bufferSize=1024 with all features, on
1/2/4/8 GPUs, and the fraction of the HBM roofline.

A "step" is one fused extraction launch over one batch of 262,144 synthetic frames
of 1024 float32 samples per GPU (BASELINE config C3/C4 size), computing every
per-frame feature: rms, energy, zcr, spectralCentroid/Flatness/Slope/Rolloff/
Spread/Skewness/Kurtosis, loudness (24 specific + total), perceptualSpread,
perceptualSharpness, mfcc (13 coefficients of the reference's 26 mel bands).
Inputs are generated in HBM before the timed region. Consecutive steps alternate
between two streams and two output sets, as a caller streaming batches runs them: one
launch's drain (its last waves leaving the SIMDs) overlaps the next launch's start.

Multi-GPU (--gpus N): one process per GPU under torchrun (the driver's launch; --gpus must
equal WORLD_SIZE), or one process driving devices 0..N-1 without it; never fewer GPUs than
asked (the run fails instead). Each rank extracts its own 262,144-frame shard of one global
stream (weak scaling). The run is measured twice: the shards alone, then the steps through
the library's multi-device group (include/meyda_gpu.h, mgx_group_create_rank /
mgx_group_create), which gathers every rank's per-frame feature records to rank 0 over
xGMI with RCCL point-to-point transfers, chunked so that chunk i's transfer overlaps chunk
i+1's extraction. `value` is the shards' rate: frames are independent (src/meyda.js:69-91),
so the path partitions with no data-path collective; the gather-inclusive rate of the same
run is `gather.value` (the north star's RCCL gather, timed inside its steps), with the
gather's status if it fails or passes its deadline. (Rank 0's inbound xGMI bounds that rate:
7 peers x 52 MB of records per 262,144-frame step.) The RCCL communicator's own view (ranks, rank, device) and every
rank's GPU (uuid, PCI bus) are in the line. torch.distributed (gloo) is only the control
plane: the RCCL id broadcast, barriers and the max-over-ranks elapsed time.

Config C5 (BASELINE.json configs[4]: bufferSize=2048, all features incl. MFCC, 262,144
frames per GPU -- 2,097,152 at 8 GPUs -- with the RCCL gather) is the `c5` field of every
line: its shards' rate, and at N > 1 its gather-inclusive rate, `vs_shards` and the
communicator's view (at N = 1 the gather is reported as skipped).

A gather that fails or passes its deadline leaves `value` (the shards) measured: rank 0
still prints the line with the gather's status, then the process exits with status 3 -- a
broken RCCL path is a failed run. --allow-gather-failure (a shards-only run) exits 0 instead.
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from meyda_amd import capi  # noqa: E402

FEATURES = capi.ALL_FEATURES  # 13 scalars + loudness.specific(24) + mfcc(13)
OUT_FLOATS = 3 + 7 + 25 + 2 + 13  # per frame, f32 outputs
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
C5_N = 2048  # BASELINE.json configs[4]
C3_FEATURES = [f for f in FEATURES if f not in ("rms", "energy", "zcr", "mfcc")]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs of the job (default: the torchrun world size, else 1). Under torchrun it must equal "
                         "WORLD_SIZE; without torchrun, N > 1 drives devices 0..N-1 from this one process")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed launches before the warmup steps, until the GPU clock has ramped "
                         "(3 warmup launches alone leave the first timed steps ~8%% slow)")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=262144, help="frames per GPU per step")
    ap.add_argument("--precision", default="faithful", choices=["faithful", "fast"])
    ap.add_argument("--single-stream", action="store_true",
                    help="every step on one stream (no pipelining): a rocprofv3 --stats run of this command then "
                         "averages whole, non-overlapping launches (profiles/*_kernel_stats.csv)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    ap.add_argument("--cpu-seconds", type=float, default=6.0,
                    help="CPU baseline: seconds of the multi-thread run of the headline set (1 thread and the C "
                         "port: a third; each other config: half)")
    ap.add_argument("--no-fast", action="store_true", help="N = 1: skip the fp32-butterfly mode beside the faithful one")
    ap.add_argument("--no-c3", action="store_true", help="N = 1: skip the config C3 feature set (spectral* + loudness)")
    ap.add_argument("--no-c2", action="store_true", help="N = 1: skip config C2 (N = 512, amplitude + centroid)")
    ap.add_argument("--no-c4", action="store_true", help="N = 1: skip config C4 exactly (40 mel bands, 13 MFCC)")
    ap.add_argument("--no-c5", action="store_true", help="skip config C5 (bufferSize 2048, all features, + gather)")
    ap.add_argument("--c5-frames", type=int, default=262144, help="C5 frames per GPU per step")
    ap.add_argument("--no-mfcc-exact", action="store_true",
                    help="N = 1: skip the reference-order MFCC (MGX_FLAG_MFCC_REFERENCE) timing")
    ap.add_argument("--no-latency", action="store_true",
                    help="N = 1: skip the per-call get() / streaming latency of the JS facade (node)")
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: time the shards alone, without the RCCL gather to rank 0")
    ap.add_argument("--chunks", type=int, default=0, help="N > 1: gather pipeline depth (0 = automatic)")
    ap.add_argument("--gather-timeout", type=float, default=60.0,
                    help="N > 1: deadline (s) of each gather phase; past it rank 0 reports the shards alone")
    ap.add_argument("--allow-gather-failure", action="store_true",
                    help="N > 1: exit 0 even when a gather failed or timed out (the line still reports the "
                         "shards and the gather's status); by default such a run exits with status 3")
    ap.add_argument("--strict-gather", action="store_true", help=argparse.SUPPRESS)  # the default since round 5
    ap.add_argument("--allow-shared-gpu", action="store_true",
                    help="rehearsal only: ranks may share a GPU (RCCL refuses that, so no gather)")
    ap.add_argument("--no-every-output", action="store_true",
                    help="N = 1: skip the secondary timing with every output (spectra too) and 40 mel bands")
    ap.add_argument("--no-pmc", action="store_true",
                    help="N = 1: skip the live rocprofv3 --pmc passes (HBM traffic, VALU instruction mix)")
    return ap.parse_args(argv)


CPU_THREADS = 16  # the GPU box's CPU share per GPU (os.cpu_count() there is the whole machine)


def cpu_port_c(n, seconds, threads):
    """Secondary: the C restatement (oracle/meyda_oracle.c) on the same cores."""
    from oracle import oracle
    oracle.lib()
    per = 256
    x = oracle.synth_frames(capi_seed(), 0, per * threads, n)

    def work(i):
        done = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            oracle.extract(x[i * per:(i + 1) * per])
            done += per
        return done, time.perf_counter() - t0

    with cf.ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        res = list(ex.map(work, range(threads)))
        wall = time.perf_counter() - t0
    return {"value": sum(r[0] for r in res) / wall, "unit": "frames/s", "cores": threads, "kind": "port-c"}


# The CPU baseline of every GPU config ("on the same seeded synthetic batches and
# feature sets as each GPU config"): oracle/js/bench_cpu.js feature sets
CPU_SETS = {"c2": (512, "c2", "amplitudeSpectrum + spectralCentroid"),
            "c3": (1024, "c3", "spectral* + loudness + perceptual"),
            "c4": (1024, "c4", "40-band mel + 13 MFCC"),
            "c5": (C5_N, "all", "all features incl. 26-band MFCC")}


def node_cpu(n, seconds, threads, fset="all", timeout_extra=120):
    import subprocess
    js = os.path.join(ROOT, "oracle", "js", "bench_cpu.js")
    r = subprocess.run(["node", js, str(n), str(seconds), str(threads), "reference", fset], capture_output=True,
                       text=True, timeout=timeout_extra + 4 * seconds, check=True)
    return json.loads(r.stdout.strip().splitlines()[-1])


def cpu_quota():
    """CPUs this process's cgroup may use (cpu.max / cfs quota), or None without a quota."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_baseline(n, seconds):
    """The reference's Node/jsfft CPU path as the build's JavaScript restatement
    (oracle/js/meyda_cpu.js, bit-exact to the reference's golden outputs), in the
    reference's per-buffer structure, timed on this host with 1 and CPU_THREADS
    worker_threads on the seeded stream; the C port beside it. The
    other configs' feature sets ride along in `configs` (C1 as µs per get() call)."""
    import shutil
    threads = min(CPU_THREADS, os.cpu_count() or 1)
    out = {"unit": "frames/s", "kind": "js-restatement"}
    if shutil.which("node"):
        one = node_cpu(n, max(1.0, seconds / 3), 1)
        many = node_cpu(n, seconds, threads)
        out.update({"value": many["value"], "cores": threads, "cpu_model": many["cpu_model"],
                    "logical_cpus": many["logical_cpus"], "node": many["node"], "one_thread": one["value"],
                    "sample": "%d frames (N=%d, all features, seeded noise, the reference's per-buffer structure) "
                              "over %.1f s on %d worker_threads; 1 thread: %.0f frames/s"
                              % (many["frames"], n, many["seconds"], threads, one["value"])})
        # also os.cpus().length worker_threads -- the whole host, beyond this GPU's share
        allc = os.cpu_count() or threads
        try:
            aff = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            aff = allc
        quota = cpu_quota()
        try:
            a = node_cpu(n, seconds, allc, timeout_extra=300)
            out["all_cores"] = {"value": a["value"], "unit": "frames/s", "cores": allc, "schedulable_cpus": aff,
                                "cgroup_cpu_quota": quota, "kind": "js-restatement",
                                "sample": "%d frames (N=%d, all features) over %.1f s on %d worker_threads "
                                          "(os.cpus().length; %d CPUs in this process's affinity mask, cgroup CPU quota %s: "
                                          "threads beyond the quota time-share it, each paying its own JIT warm-up)"
                                          % (a["frames"], n, a["seconds"], allc, aff,
                                             "%.1f CPUs" % quota if quota else "none")}
        except Exception as e:  # a report, never the measurement itself
            out["all_cores"] = {"value": None, "cores": allc, "note": "failed: %r" % (e,)}
        cfgs = {}
        for key, (cn, fset, what) in CPU_SETS.items():
            try:
                m = node_cpu(cn, max(1.0, seconds / 2), threads, fset)
                o = node_cpu(cn, max(0.5, seconds / 6), 1, fset)
                cfgs[key] = {"value": m["value"], "unit": "frames/s", "cores": threads, "one_thread": o["value"],
                             "kind": "js-restatement",
                             "sample": "%d frames (N=%d, %s, seeded noise) over %.1f s on %d worker_threads"
                                       % (m["frames"], cn, what, m["seconds"], threads)}
            except Exception as e:  # a report, never the measurement itself
                cfgs[key] = {"value": None, "note": "failed: %r" % (e,)}
        try:
            c1 = node_cpu(512, 2.0, 1, "c1")
            cfgs["c1"] = {"value": c1["us_per_call"], "unit": "us per get(['rms','spectralCentroid']) call",
                          "calls": c1["calls"], "cores": 1, "kind": "js-restatement",
                          "sample": "sound1.wav frame 0 (tests/golden, N=512): window, FFT, amplitude, rms and "
                                    "centroid per call, median of %d calls" % c1["calls"]}
        except Exception as e:
            cfgs["c1"] = {"value": None, "note": "failed: %r" % (e,)}
        out["configs"] = cfgs
    else:  # no Node on this host: the C port stands in
        out.update({"kind": "port", "value": None, "note": "node not found"})
    out["port_c"] = cpu_port_c(n, max(1.0, seconds / 3), threads)
    if out.get("value") is None:
        out["value"] = out["port_c"]["value"]
        out["cores"] = threads
    return out


def latency_js():
    """The real-time path through the product's own JS facade over the N-API addon
    (tools/latency.js): C1's get(['rms','spectralCentroid']) per call -- launched per call (`c1`) and
    served by the resident workgroup (`c1_resident`, options.resident / MGX_FLAG_RESIDENT), back to back and
    with the host idle 1 ms between calls (`c1_gap`, `c1_resident_gap`) -- and the start() / process()
    callback path at batchFrames 1 and 64 (and resident). A report; never `value`."""
    import shutil
    import subprocess
    addon = os.path.join(ROOT, "meyda_amd", "addon", "meyda_napi.node")
    if not shutil.which("node"):
        return {"status": "skipped (node not found)"}
    if not os.path.exists(addon):
        return {"status": "skipped (meyda_amd/addon/meyda_napi.node not built)"}
    # the application-side setting INTEGRATION.md recommends for the real-time path (the facade itself
    # leaves the environment alone): kernel arguments in host memory
    env = dict(os.environ)
    env.setdefault("HIP_FORCE_DEV_KERNARG", "0")
    r = subprocess.run(["node", os.path.join(ROOT, "tools", "latency.js")], capture_output=True, text=True,
                       timeout=240, env=env)
    if r.returncode != 0:
        return {"status": "failed (rc %d): %s" % (r.returncode, r.stderr.strip()[-400:])}
    out = json.loads(r.stdout.strip().splitlines()[-1])
    out["status"] = "ok"
    out["env"] = {"HIP_FORCE_DEV_KERNARG": env["HIP_FORCE_DEV_KERNARG"]}
    out["note"] = ("c1: a launch per get() (the facade's default); c1_resident: options.resident -- one workgroup stays on "
                   "the device and takes each buffer from a pinned mailbox (MGX_FLAG_RESIDENT, DESIGN.md 9.1); *_gap: the "
                   "host idle 1 ms between calls, as between a real-time source's buffers; medians in us per call")
    return out


def capi_seed():
    import meyda_amd
    return meyda_amd.SEED


class Devices:
    """The devices this process drives (one under torchrun; N for a single-process --gpus N
    run), each with the two streams every pipelined loop of the run uses, created once: a
    stream's first launches carry a one-time cost of milliseconds (its hardware queue), which
    settle() absorbs."""

    def __init__(self, devs, single=False):
        self.devs = list(devs)
        self.single = single  # --single-stream: every step on stream 0 (launches never overlap)
        self.streams = {}
        for d in self.devs:
            with torch.cuda.device(d):
                self.streams[d] = [torch.cuda.current_stream(d), torch.cuda.Stream(device=d)]

    def stream(self, d, k):
        return self.streams[d][0 if self.single else k & 1]

    def sync(self):
        for d in self.devs:
            torch.cuda.synchronize(d)


class Workload:
    """One configuration's synthetic frames (each local device its own shard of one global
    stream, generated in HBM) and a plan per device."""

    def __init__(self, n, F, devs, first, precision):
        self.n, self.F = n, F
        self.frames, self.plans = {}, {}
        for i, d in enumerate(devs.devs):
            with torch.cuda.device(d):
                self.frames[d] = torch.empty(F, n, dtype=torch.float32, device="cuda:%d" % d)
                capi.synth_frames_device(self.frames[d], capi_seed(), first_frame=(first + i) * F)
                self.plans[d] = capi.Plan(buffer_size=n, precision=precision, device=d)

    def close(self):
        for p in self.plans.values():
            p.close()
        self.frames, self.plans = {}, {}


def pipelined(step, devs, first, count):
    """Steps first..first+count-1, consecutive steps alternating between each device's two
    streams and two output sets (step(k) launches step k on stream k & 1 of every local
    device): a stream of batches the way a streaming caller runs it, so step i+1's workgroups
    start on the CUs step i's last waves leave while it drains (one launch ends with ~45 us of
    SIMDs running out of waves). Forks from and joins back into stream 0."""
    for d in devs.devs:
        e = torch.cuda.Event()
        e.record(devs.stream(d, 0))
        devs.stream(d, 1).wait_event(e)
    for i in range(first, first + count):
        step(i)
    for d in devs.devs:
        e = torch.cuda.Event()
        e.record(devs.stream(d, 1))
        devs.stream(d, 0).wait_event(e)


def settle(step, devs, ms, dist=None):
    """Untimed steps for `ms` of wall time (clock ramp-up), before the warmup steps."""
    t0 = time.perf_counter()
    go = True
    while go:
        pipelined(step, devs, 0, 8)
        devs.sync()
        go = (time.perf_counter() - t0) * 1e3 < ms
        if dist:  # every rank runs the same number of (collective) steps
            t = torch.tensor([1 if go else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            go = bool(t.item())


def host_path(plan, frames, reps=3):
    """Secondary, never `value`: the PCIe-inclusive rate of mgx_extract_host, float32 frames in
    pageable host memory -> every feature in host memory (chunk i+1's copy beside chunk i's
    extraction), median of `reps` calls over the same F frames."""
    x = frames.cpu().numpy()
    plan.extract(x[:4096], FEATURES)  # staging allocation
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        plan.extract(x, FEATURES)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    return {"value": x.shape[0] / t, "unit": "frames/s", "ms_per_call": t * 1e3,
            "input_GBps": x.nbytes / t / 1e9,
            "note": "PCIe-inclusive: %d float32 frames from pageable host memory, features back to host" % x.shape[0]}


def _mfma_pass(c):
    # the DCT's v_mfma_f64_4x4x4_4b_f64: 4 blocks x 4x4x4 = 256 FMAs = 512 FLOP per wave instruction
    return {"instr_per_launch": c["SQ_INSTS_VALU_MFMA_F64"], "flop_per_launch": 512 * c["SQ_INSTS_VALU_MFMA_F64"],
            "busy_cycles_per_launch": c["SQ_VALU_MFMA_BUSY_CYCLES"], "gui_active_cycles": c["GRBM_GUI_ACTIVE"]}


def pmc_live(n, F, precision):
    """Counters of the same workload, measured in this run: rocprofv3 --pmc passes (one
    counter block each, kernel-trace only, MI355X_MICROARCH.md HBM section) over
    tools/pmc_probe.py in a child process. FETCH_SIZE is calibrated on the time-only feature
    set, which reads exactly the frames (gfx950 tallies streaming reads at about half their
    bytes); WRITE_SIZE is read as is. Returns (traffic bytes per launch, VALU mix, notes)."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None, None, "rocprofv3 not found"
    probe = os.path.join(ROOT, "tools", "pmc_probe.py")
    tmp = tempfile.mkdtemp(prefix="mgx_pmc_", dir="/tmp")
    mfma = "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
    passes = {"fetch_t": ("time_only", 26, "FETCH_SIZE"), "fetch": ("all", 26, "FETCH_SIZE"),
              "write": ("all", 26, "WRITE_SIZE"),
              "valu": ("all", 26, "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 "
                                  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS"),
              "mfma": ("all", 26, mfma),
              # VALU-busy (faithful mode is FP64-VALU bound): SQ_ACTIVE_INST_* count quad-cycles
              # of issue summed over the waves; GRBM_GUI_ACTIVE the kernel's cycles summed over the 8 XCDs
              "busy": ("all", 26, "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"),
              # config C4 exactly (40 mel bands, mfcc alone): north_star's MFMA utilisation of that line
              "mfma_c4": ("mfcc", 40, mfma)}
    got = {}
    reps = 3
    for key, (fset, bands, ctrs) in passes.items():
        d = os.path.join(tmp, key)
        env = dict(os.environ, PROBE_SET=fset, PROBE_N=str(n), PROBE_PREC=precision, PROBE_REPS=str(reps),
                   PROBE_BANDS=str(bands), TMPDIR="/tmp")
        cmd = ["timeout", "-s", "KILL", "90", prof, "--pmc", *ctrs.split(), "--kernel-trace", "--output-format", "csv",
               "-d", d, "-o", "run", "--", sys.executable, probe]
        r = subprocess.run(cmd, env=env, cwd="/tmp", capture_output=True, text=True)
        if r.returncode != 0:
            return None, None, "rocprofv3 pass %s failed (rc %d)" % (key, r.returncode)
        vals = {}
        for f in glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if "extract_kernel" in row.get("Kernel_Name", ""):
                    vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
        # per step: a large batch runs as several launches (mgx_extract_device's parts)
        got[key] = {k: float(np.sum(v)) / reps for k, v in vals.items()}
    shutil.rmtree(tmp, ignore_errors=True)
    frames_bytes = F * n * 4
    cal = frames_bytes / (got["fetch_t"]["FETCH_SIZE"] * 1024)  # true bytes per counted byte (KB counters)
    read = got["fetch"]["FETCH_SIZE"] * 1024 * cal
    write = got["write"]["WRITE_SIZE"] * 1024
    v = got["valu"]
    valu = {"instr_per_frame": v["SQ_INSTS_VALU"] / F, "cvt_per_frame": v["SQ_INSTS_VALU_CVT"] / F,
            "f64_per_frame": sum(v[k] for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_MUL_F64",
                                                "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")) / F,
            "lds_per_frame": v["SQ_INSTS_LDS"] / F}
    b = got["busy"]
    simds = 4 * torch.cuda.get_device_properties(0).multi_processor_count
    kcyc = b["GRBM_GUI_ACTIVE"] / 8.0  # the kernel's cycles (per XCD)
    valu["busy_counters"] = {k: b[k] for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES",
                                                  "SQ_WAVE_CYCLES", "GRBM_GUI_ACTIVE")}
    # issue quad-cycles x 4 over (kernel cycles x SIMDs): the fraction of SIMD cycles that issued VALU work
    valu["valu_busy_measured"] = 4.0 * b["SQ_ACTIVE_INST_VALU"] / (kcyc * simds)
    valu["any_busy_measured"] = 4.0 * b["SQ_ACTIVE_INST_ANY"] / (kcyc * simds)
    valu["busy_simds"] = simds
    valu["mfma_f64"] = _mfma_pass(got["mfma"])
    valu["mfma_f64_c4"] = dict(_mfma_pass(got["mfma_c4"]), config="C4: 40 mel bands x 13 MFCC, mfcc alone")
    note = ("live: rocprofv3 --pmc passes of this run over tools/pmc_probe.py (%d frames x N=%d, same features); "
            "FETCH_SIZE x %.4f (time-only calibration), reads %.4g B + writes %.4g B per launch" % (F, n, cal, read, write))
    return read + write, valu, note


def run_mode(step, devs, steps, warmup, dist):
    """W untimed steps, then exactly `steps` timed ones bracketed by a barrier and a device
    synchronisation on both sides, pipelined over two streams (pipelined()); HIP events on the
    launch stream around the whole timed region give the launch period (no events between the
    steps: an event pair per step cost 1-2 % of the step time, tools/step_overlap.py). Then an
    untimed single-stream pass with an event pair around each launch (the spread of single
    launches), and one more of 20 launches back to back on one stream with one event pair around
    them all: the mean launch duration (plus the small dispatch gap between serialised launches),
    which is what rocprofv3 reports per dispatch -- an event pair around every launch adds its own
    marker packets to each (~1 % of a 0.6 ms launch against the profiler's durations)."""
    d0 = devs.devs[0]
    s0 = devs.stream(d0, 0)
    pipelined(step, devs, 0, warmup)
    devs.sync()
    if dist:
        dist.barrier()
    devs.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s0)
    pipelined(step, devs, 0, steps)
    e1.record(s0)
    devs.sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    period = e0.elapsed_time(e1) / steps
    # the launch on its own (serialised on one stream), untimed by the step clock
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in ev:
        a.record(s0)
        step(0)  # every local device's stream 0: serialised behind the previous launch
        b.record(s0)
    devs.sync()
    iso = [a.elapsed_time(b) for a, b in ev]
    es0, es1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    es0.record(s0)
    for _ in range(20):
        step(0)
    es1.record(s0)
    devs.sync()
    serial = es0.elapsed_time(es1) / 20
    stats = {"period_ms": period, "launch_serial_ms": serial, "launch_alone_mean_ms": float(np.mean(iso)),
             "launch_alone_median_ms": float(np.median(iso)), "launch_alone_min_ms": float(np.min(iso)),
             "launch_alone_max_ms": float(np.max(iso))}
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # per-GPU step times reported separately (HIP events on each rank's stream)
        allr = [None] * dist.get_world_size()
        dist.all_gather_object(allr, stats)
        stats = {"rank0": stats, "per_rank_period_ms": [r["period_ms"] for r in allr],
                 "per_rank_launch_alone_ms": [r["launch_alone_mean_ms"] for r in allr],
                 "per_rank_launch_serial_ms": [r["launch_serial_ms"] for r in allr]}
    return elapsed, period, stats


def measure_shards(wl, devs, args, dist, feats=FEATURES):
    """The shards alone: every local device extracts its own shard (no data-path collective)."""
    sets = {d: [wl.plans[d].alloc_outputs(wl.F, feats, device="cuda:%d" % d) for _ in range(2)] for d in devs.devs}

    def step(k):
        for d in devs.devs:
            wl.plans[d].extract_device(wl.frames[d].data_ptr(), wl.F, sets[d][k & 1][1], devs.stream(d, k).cuda_stream)
    devs.sync()
    settle(step, devs, args.settle_ms, dist)
    return run_mode(step, devs, args.steps, args.warmup, dist)


def measure_gather(wl, devs, args, dist, mode, rank, world, gpus, out):
    """The same steps through the library's multi-device group: each rank's feature records
    gathered to rank 0 over RCCL inside every step (group.cpp). Updates `out` as it goes (the
    communicator's view, then the status and rates) so a deadline can report what it got."""
    d0 = devs.devs[0]
    n, F = wl.n, wl.F
    out["status"] = "creating the group"
    if mode == "torchrun":
        uid = [capi.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        group = capi.Group(buffer_size=n, rank=rank, nranks=world, unique_id=uid[0], precision=args.precision, device=d0)
    else:
        group = capi.Group(buffer_size=n, devices=devs.devs, precision=args.precision)
    comm = group.comm_info()
    out["rccl_comm"] = {"ranks": comm[0], "rank": comm[1], "device": comm[2], "group_ranks": group.nranks,
                        "local_ranks": group.num_local}
    out["transport"] = ("ipc rehearsal (MGX_GROUP_TRANSPORT=ipc: hipIpc-mapped transfer buffers + a shared-memory "
                        "mailbox in place of ncclSend/ncclRecv)" if os.environ.get("MGX_GROUP_TRANSPORT") == "ipc"
                        else "rccl")
    if group.nranks != gpus or comm[0] != gpus or comm[2] != d0 or comm[1] != group.first_local:
        raise RuntimeError("the RCCL communicator reports %s for a %d-GPU job on device %d" % (comm, gpus, d0))
    out["status"] = "running"
    # rank 0 holds the whole job's feature record; the other ranks only their transfer buffers
    # (two output sets: consecutive steps are in flight together, pipelined())
    root = group.first_local == 0
    plan = wl.plans[d0]
    with torch.cuda.device(d0):
        sets = [plan.alloc_outputs(F * gpus if root else 1, FEATURES, device="cuda:%d" % d0) for _ in range(2)]
    mask = capi.output_mask(sets[0][1])
    ptrs = [wl.frames[d].data_ptr() for d in devs.devs]

    def step_gather(k):
        group.extract_device(ptrs, [F] * gpus, sets[k & 1][1] if root else None, mask, args.chunks,
                             [devs.stream(d, k).cuda_stream for d in devs.devs])
    settle(step_gather, devs, args.settle_ms, dist)
    el_g, km_g, stats_g = run_mode(step_gather, devs, args.steps, args.warmup, dist)
    if root:  # spot check: the gathered record holds every rank's shard (last frame of each)
        chk = sets[0][0]["zcr"].view(gpus, F)[:, -1]
        out["finite_last_frames"] = bool(torch.all((chk >= 0) & (chk < n)).item())
    out.update({"status": "ok", "value": gpus * F * args.steps / el_g, "ms_per_step": el_g / args.steps * 1e3,
                "kernel_ms": km_g, "step_event_ms": stats_g})
    devs.sync()
    group.close()


def resolve_topology(gpus, env, ndev, allow_shared=False):
    """How this run maps onto GPUs; fails loudly (SystemExit) instead of measuring fewer GPUs
    than asked. Under torchrun (WORLD_SIZE set) --gpus must equal the world size and every
    local rank needs a GPU of its own (--allow-shared-gpu: a rehearsal only). Without torchrun
    --gpus N > 1 drives devices 0..N-1 from this one process. Returns (mode, gpus), mode one
    of "torchrun", "single" (one process, N devices) or "one"."""
    from meyda_amd import dist as mdist
    _, _, world = mdist.env_rank_world(env)
    if "WORLD_SIZE" in env:
        gpus = world if gpus is None else gpus
        if gpus != world:
            raise SystemExit("bench.py: --gpus %d but the launcher started %d ranks (WORLD_SIZE)" % (gpus, world))
        local_world = int(env.get("LOCAL_WORLD_SIZE", world))
        if ndev < local_world and not allow_shared:
            raise SystemExit("bench.py: %d ranks on this node but %d GPU(s) visible (one GPU per rank; "
                             "--allow-shared-gpu for a rehearsal)" % (local_world, ndev))
        return ("torchrun" if world > 1 else "one"), gpus
    gpus = 1 if gpus is None else gpus
    if gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if gpus > ndev:
        raise SystemExit("bench.py: --gpus %d but %d GPU(s) visible" % (gpus, ndev))
    return ("single" if gpus > 1 else "one"), gpus


class Watchdog:
    """Deadline of one gather phase of a multi-GPU run. The RCCL path cannot be interrupted
    once a peer is missing (a rank that failed, a message never posted), so when the deadline
    passes rank 0 prints the line it already has -- the shards measured without the gather,
    with the gather's status -- and every rank leaves with gather_exit_code() (3, or 0 under
    --allow-gather-failure); rank 0 prints before it leaves, so the line is never lost."""

    def __init__(self, seconds, emit, code):
        import threading
        self.emit = emit
        self.code = code
        self.t = threading.Timer(seconds, self._fire)
        self.t.daemon = True
        self.t.start()

    def _fire(self):
        try:
            self.emit("timed out")
        finally:
            sys.stdout.flush()
            sys.stderr.flush()
            os._exit(self.code)

    def cancel(self):
        self.t.cancel()


def gather_exit_code(args, statuses):
    """Exit status of a run from its gather phases' statuses: 0 when every gather that ran
    reports "ok" (or none ran: N = 1, --no-gather, shared GPUs), else 3 -- a failed or timed-out
    RCCL gather fails the run even though the shards' `value` was measured -- unless
    --allow-gather-failure asked for a shards-only run."""
    bad = [s for s in statuses if s is not None and s != "ok"]
    return 0 if not bad or getattr(args, "allow_gather_failure", False) else 3


def launch_ms(stats):
    """Rank 0's mean launch duration (run_mode: 20 launches serialised on one stream, one event pair)."""
    return (stats["rank0"] if "rank0" in stats else stats)["launch_serial_ms"]


def shard_fields(gpus, F, n, el, km, stats, steps, bytes_per_frame):
    """Rate and roofline of one config's shards (rank 0's launch duration)."""
    alone = launch_ms(stats)
    return {"value": gpus * F * steps / el, "unit": "frames/s", "ms_per_step": el / steps * 1e3,
            "kernel_ms": alone, "period_ms": km, "bytes_per_frame": bytes_per_frame,
            "roofline_frac": F * bytes_per_frame / (alone * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "frac_pipelined": F * bytes_per_frame / (km * 1e-3) / 1e9 / HBM_PEAK_GBS, "step_event_ms": stats}


def c5_field(gpus, F5, el, km, stats, steps, gather_on, chunks=0):
    """The `c5` field of the line (BASELINE.json configs[4]) from its shards' timing; its gather
    entry starts as "not run" at N > 1 (measure_gather fills it) and says why it is absent at
    N = 1."""
    c5 = dict(shard_fields(gpus, F5, C5_N, el, km, stats, steps, 4 * C5_N + 4 * OUT_FLOATS),
              buffer_size=C5_N, frames_per_gpu=F5, features=FEATURES, mel_bands=26, mfcc_coeffs=13,
              frames_total=gpus * F5,
              workload="C5: %d frames x bufferSize=%d per GPU (%d in all; BASELINE's 2,097,152 at 8 GPUs), every "
                       "feature incl. MFCC, frames sharded, records gathered to rank 0 over RCCL"
                       % (F5, C5_N, gpus * F5))
    if gather_on:
        c5["gather"] = {"status": "not run", "chunks": chunks or "auto"}
    elif gpus == 1:
        c5["gather"] = {"status": "skipped (1 GPU): nothing to gather; the RCCL path is timed at N > 1"}
    else:
        c5["gather"] = {"status": "off (--no-gather or shared GPUs)"}
    return c5


def c5_finish(c5, gpus):
    """C5's `value` as BASELINE.json configs[4] defines it ("frames sharded across GPUs with RCCL gather"):
    at N > 1 the gather-inclusive rate of the same steps (every rank's records to rank 0 inside each timed
    step), None when the gather did not complete; at N = 1 the one shard (nothing to gather). The shards'
    rate without the gather stays beside it as `shards_value`. Idempotent (a deadline may print the line
    before the gather phase ends)."""
    shards = c5.setdefault("shards_value", c5["value"])
    g = c5.get("gather") or {}
    if gpus == 1:
        c5["value"] = shards
        c5["value_source"] = "one GPU: its shard alone (nothing to gather)"
    elif g.get("status") == "ok":
        c5["value"] = g["value"]
        g["vs_shards"] = g["value"] / shards
        c5["value_source"] = ("gather-inclusive: every rank's feature records gathered to rank 0 over RCCL inside each "
                              "timed step (gather.*); shards_value: the shards alone, no data-path collective")
    else:
        c5["value"] = None
        c5["value_source"] = ("no gather-inclusive rate (gather: %s); shards_value: the shards alone"
                              % g.get("status", "not run"))
    return c5


def main():
    args = parse()
    from meyda_amd import dist as mdist
    mode, gpus = resolve_topology(args.gpus, os.environ, torch.cuda.device_count(), args.allow_shared_gpu)
    rank, local, world = mdist.env_rank_world()
    dist = None
    if mode == "torchrun":
        import torch.distributed as tdist
        mdist.init_control_plane()  # gloo: control plane only; the data path is the library's RCCL gather
        dist = tdist
        devs = Devices([local % torch.cuda.device_count()], args.single_stream)
    else:
        devs = Devices(range(gpus), args.single_stream)
    torch.cuda.set_device(devs.devs[0])
    # which GPU every rank / local device is (the driver's node: one each)
    me = [{"rank": rank + i, "device": d, "uuid": str(torch.cuda.get_device_properties(d).uuid),
           "pci_bus_id": torch.cuda.get_device_properties(d).pci_bus_id} for i, d in enumerate(devs.devs)]
    if dist:
        allr = [None] * world
        dist.all_gather_object(allr, me)
        placement = [x for r in allr for x in r]
    else:
        placement = me
    shared = len({p["uuid"] for p in placement}) != len(placement)
    if shared and not args.allow_shared_gpu:
        raise SystemExit("bench.py: ranks share a GPU: %s" % placement)
    n, F = args.n, args.frames
    first = rank if dist else 0  # each rank / device its own shard of one global synthetic stream
    # (MGX_GROUP_TRANSPORT=ipc: the cross-process rehearsal of the gather, whose ranks may share a GPU --
    # the chunks move through IPC-mapped buffers instead of RCCL, which refuses two ranks on one device)
    ipc_rehearsal = os.environ.get("MGX_GROUP_TRANSPORT") == "ipc"
    gather_on = gpus > 1 and not args.no_gather and (not shared or ipc_rehearsal)
    head = Workload(n, F, devs, first, args.precision)
    el_s, km_s, stats_s = measure_shards(head, devs, args, dist)
    value_s = gpus * F * args.steps / el_s
    gather = {"status": "not run", "chunks": args.chunks or "auto"} if gather_on else None
    line_box = {}
    failed = []

    # C5 (BASELINE configs[4]): the shards first (no collective), its gather after the headline's
    c5 = None
    if not args.no_c5:
        w5 = Workload(C5_N, args.c5_frames, devs, first, args.precision)
        el5, km5, st5 = measure_shards(w5, devs, args, dist)
        c5 = c5_field(gpus, args.c5_frames, el5, km5, st5, args.steps, gather_on, args.chunks)
        line_box["c5"] = c5
        if mode == "one" and not args.no_mfcc_exact and args.precision != "fast":
            d0 = devs.devs[0]
            c5["mfcc_exact"] = mfcc_exact_of(c5, timed_launches(
                args, devs, capi.Plan(buffer_size=C5_N, precision=args.precision, mfcc_reference=True, device=d0),
                FEATURES, 4 * C5_N + 4 * OUT_FLOATS, w5.frames[d0]))
    if mode == "one":
        line_box.update(secondary(args, head.plans[devs.devs[0]], head.frames[devs.devs[0]], devs, n, F))

    def emit_line(gather_status=None, target=None):
        """Rank 0's JSON line from what has been measured so far."""
        if rank != 0:
            return
        if target is not None and gather_status is not None:
            target["status"] = gather_status
        print(json.dumps(build_line(args, gpus, mode, placement, F, n, value_s, el_s, km_s, stats_s, gather,
                                    line_box)), flush=True)

    code = gather_exit_code(args, ["failed"])  # what a failed or timed-out gather phase exits with
    phases = []
    if gather_on:
        phases.append((head, gather))
        if c5 is not None:
            phases.append((w5, c5["gather"]))
    for wl, target in phases:
        wd = Watchdog(args.gather_timeout, lambda s, t=target: emit_line(s, t), code)
        try:
            measure_gather(wl, devs, args, dist, mode, rank, world, gpus, target)
            wd.cancel()
        except Exception as e:  # the line still reports the shards, with the gather's failure
            print("rank %d: gather failed: %r" % (rank, e), file=sys.stderr, flush=True)
            target["status"] = "failed on rank %d: %r" % (rank, e)
            failed.append(target)
            if rank == 0:
                emit_line()
                os._exit(code)
            wd.t.join()  # a failed peer waits for its deadline (rank 0 may be blocked on it)
    emit_line()
    if dist:
        dist.barrier()
        dist.destroy_process_group()
    rc = gather_exit_code(args, [t.get("status") for _, t in phases])
    if rc:
        print("bench.py: a gather did not complete (%s); exit %d (--allow-gather-failure: 0)"
              % ([t.get("status") for _, t in phases], rc), file=sys.stderr, flush=True)
        sys.exit(rc)


def timed_launches(args, devs, p, feats, bytes_per_frame, fr):
    """One plan's launches over the frames `fr` on devs' first device, timed as `value`'s are
    (settle, warmup, the pipelined timed steps, then the serialised launches for kernel_ms)."""
    dev = devs.devs[0]
    Fx = fr.shape[0]
    sets = [p.alloc_outputs(Fx, feats, device="cuda:%d" % dev) for _ in range(2)]

    def st(k):
        p.extract_device(fr.data_ptr(), Fx, sets[k & 1][1], devs.stream(dev, k).cuda_stream)
    settle(st, devs, args.settle_ms)
    el, km, stats = run_mode(st, devs, args.steps, args.warmup, None)
    alone = launch_ms(stats)
    return {"value": Fx * args.steps / el, "unit": "frames/s", "kernel_ms": alone, "period_ms": km,
            "bytes_per_frame": bytes_per_frame,
            "roofline_frac": Fx * bytes_per_frame / (alone * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "frac_pipelined": Fx * bytes_per_frame / (km * 1e-3) / 1e9 / HBM_PEAK_GBS}


def mfcc_exact_of(base, exact):
    """A config's reference-order MFCC timing (MGX_FLAG_MFCC_REFERENCE) beside its default one."""
    return dict(exact, flag="MGX_FLAG_MFCC_REFERENCE (mfcc.js:53-93 in the reference's own order)",
                cost_vs_config_kernel=exact["kernel_ms"] / base["kernel_ms"] - 1.0)


def secondary(args, plan, frames, devs, n, F):
    """Single-GPU secondary fields (never `value`): fast precision, configs C3 and C4 exactly,
    the reference-order MFCC, every output, the live PMC counters, the PCIe-inclusive host path,
    the facade's real-time latency and the CPU baselines."""
    out = {}
    dev = devs.devs[0]

    def timed(p, feats, bytes_per_frame, fr=frames):
        return timed_launches(args, devs, p, feats, bytes_per_frame, fr)
    if not args.no_fast and args.precision != "fast":
        # the fp32-butterfly mode beside the faithful one (same features and frames)
        out["fast_mode"] = dict(timed(capi.Plan(buffer_size=n, precision="fast", device=dev), FEATURES,
                                      4 * n + 4 * OUT_FLOATS), precision="fast (f32 butterflies; not bit-faithful)")
    if not args.no_mfcc_exact and args.precision != "fast":
        # north_star's "all features within 1e-5" per element for the MFCC too: the reference-order
        # mel sums, log and DCT (MGX_FLAG_MFCC_REFERENCE), same features and frames as `value`
        ex = timed(capi.Plan(buffer_size=n, precision=args.precision, mfcc_reference=True, device=dev), FEATURES,
                   4 * n + 4 * OUT_FLOATS)
        out["mfcc_exact"] = dict(ex, flag="MGX_FLAG_MFCC_REFERENCE (mfcc.js:53-93 in the reference's own order)")
    if not args.no_c4:
        # BASELINE config C4 exactly: 40-band mel + 13 MFCC, nothing else (4,148 B/frame)
        out["c4"] = dict(timed(capi.Plan(buffer_size=n, precision=args.precision, num_mel_bands=40, device=dev),
                               ["mfcc"], 4 * n + 4 * 13), features=["mfcc"], mel_bands=40, mfcc_coeffs=13)
        if not args.no_mfcc_exact and args.precision != "fast":
            out["c4"]["mfcc_exact"] = mfcc_exact_of(out["c4"], timed(
                capi.Plan(buffer_size=n, precision=args.precision, num_mel_bands=40, mfcc_reference=True, device=dev),
                ["mfcc"], 4 * n + 4 * 13))
    if not args.no_c3:
        # BASELINE config C3: spectral* + loudness + perceptual (4,232 B/frame)
        out["c3"] = dict(timed(plan, C3_FEATURES, 4 * n + 4 * (7 + 25 + 2)), features=C3_FEATURES)
    if not args.no_c2:
        # BASELINE config C2: 65,536 frames x N = 512, amplitudeSpectrum + spectralCentroid (3,076 B/frame)
        with torch.cuda.device(dev):
            f2 = torch.empty(65536, 512, dtype=torch.float32, device="cuda:%d" % dev)
            capi.synth_frames_device(f2, capi_seed())
        out["c2"] = dict(timed(capi.Plan(buffer_size=512, precision=args.precision, device=dev),
                               ["amplitudeSpectrum", "spectralCentroid"], 4 * 512 + 4 * 257, fr=f2),
                         features=["amplitudeSpectrum", "spectralCentroid"], buffer_size=512, frames=65536)
        del f2
    if not args.no_every_output:
        # EVERY output of the path -- the headline set plus the amplitude, power and complex
        # spectra -- with the 40-band mel of config C4, same frames
        feats_e = FEATURES + ["amplitudeSpectrum", "powerSpectrum", "complexSpectrum"]
        out["every_output"] = dict(timed(capi.Plan(buffer_size=n, precision=args.precision, num_mel_bands=40, device=dev),
                                         feats_e, 4 * n + 4 * (OUT_FLOATS + 2 * (n // 2) + 2 * n)),
                                   features=feats_e, mel_bands=40)
    if not args.no_pmc:
        try:
            out["pmc"] = pmc_live(n, F, args.precision)
        except Exception as e:  # the counters are a report, never the measurement itself
            out["pmc"] = (None, None, "rocprofv3 passes failed: %r" % (e,))
    if not args.no_host_path:
        out["host_path"] = host_path(plan, frames)
    if not args.no_latency:
        try:
            out["latency"] = latency_js()
        except Exception as e:
            out["latency"] = {"status": "failed: %r" % (e,)}
    if not args.no_cpu_baseline:
        cb = cpu_baseline(n, args.cpu_seconds)
        out["cpu_baseline"] = cb
        for key, c in cb.get("configs", {}).items():
            if key in out and isinstance(out[key], dict):
                out[key]["cpu_baseline"] = c
        if "latency" in out and "c1" in cb.get("configs", {}):
            out["latency"]["cpu_c1_us_per_call"] = cb["configs"]["c1"].get("value")
    return out


FP64_PEAK_TFLOPS = 78.6  # MI355X dense FP64 (vector and matrix share the pipe): 1,024 SIMDs x 32 FLOP/clk x 2.4 GHz


def roofline_fp64(n, F, kernel_ms, valu, precision):
    """The second roofline SURVEY §8(d) asks for beside the HBM one: the FFT's algorithmic flops
    (5 N log2 N per frame, the radix-2 count) over the kernel's launch duration against the FP64
    peak, and the SIMD cycles the kernel issued VALU work in (measured, rocprofv3 PMC), with the
    limit that binds named. Faithful mode computes every butterfly in f64 and converts every stage
    to f32 and back (jsfft's Float32Array stores), so its FP64-pipe issue, not HBM, is the bound."""
    flop = 5.0 * n * np.log2(n)
    tf = F * flop / (kernel_ms * 1e-3) / 1e12
    out = {"bound": "fp64" if precision == "faithful" else "valu", "unit": "TFLOP/s",
           "fft_flop_per_frame": flop, "achieved": tf, "peak": FP64_PEAK_TFLOPS, "frac": tf / FP64_PEAK_TFLOPS,
           "kernel_ms": kernel_ms,
           "note": "algorithmic FFT flops only (5 N log2 N per frame); the faithful butterflies also issue two f32<->f64 "
                   "conversions per value and stage, which occupy the same FP64 pipe and are not counted as flops"}
    if valu:
        for k in ("valu_busy_measured", "any_busy_measured", "est_valu_busy", "est_fp64_cvt_busy"):
            if k in valu:
                out[k] = valu[k]
        out["binding"] = ("FP64-pipe VALU issue: %.0f f64 + %.0f f32<->f64 conversion instructions of %.0f VALU per frame; "
                          "the kernel issues VALU work in %.0f %% of its SIMD cycles (measured), HBM at the roofline "
                          "fraction above" % (valu["f64_per_frame"], valu["cvt_per_frame"], valu["instr_per_frame"],
                                              100.0 * valu.get("valu_busy_measured", float("nan"))))
    return out


def build_line(args, gpus, mode, placement, F, n, value_s, el_s, km_s, stats_s, gather, extras):
    bytes_per_frame = 4 * n + 4 * OUT_FLOATS
    use_gather = gather is not None and gather.get("status") == "ok"
    # the path partitions (independent frames): `value` is the shards with no data-path collective;
    # the gather-inclusive rate of the same run is reported beside it (gather.value)
    value = value_s
    if use_gather:
        gather["vs_shards"] = gather["value"] / value_s
    elapsed = args.steps * 1e3 / (value / (gpus * F))  # ms for the K steps
    # the roofline of the extraction kernel: its average launch duration, 20 launches serialised on
    # one stream between one event pair (what rocprofv3 --stats reports per dispatch); the launch
    # period of the pipelined timed steps (value) is reported beside it
    alone_ms = launch_ms(stats_s)
    kernel_ms = alone_ms
    achieved = F * bytes_per_frame / (kernel_ms * 1e-3) / 1e9
    traffic, valu, traffic_note = extras.get("pmc") or (None, None, "not measured (--no-pmc or N > 1)")
    if valu is not None:
        # the faithful path is FP64-VALU bound. Issue costs per wave64
        # instruction measured by tools/ubench/op_rates.hip (profiles/r01_op_rates.log):
        # f64 ~5.0, f32<->f64 conversion 4.2 cycles; at the clock this run's kernel time implies
        cyc = km_s * 1e-3 * 2.4e9 * 1024 / F  # SIMD cycles per frame at the timed steps' rate (2.4 GHz, 1,024 SIMDs)
        valu["frame_simd_cycles"] = cyc
        valu["est_fp64_cvt_busy"] = (valu["f64_per_frame"] * 5.0 + valu["cvt_per_frame"] * 4.2) / cyc
        # FP64 pipe (vector and matrix share it): 78.6 TFLOP/s dense on MI355X (1,024 SIMDs x 32
        # FLOP/clk x 2.4 GHz; v_mfma_f64_4x4x4 issues every 16 cycles: tools/ubench/op_rates.hip)
        mf = valu["mfma_f64"]
        mf["tflops"] = mf["flop_per_launch"] / (km_s * 1e-3) / 1e12
        mf["peak_tflops"] = 78.6
        mf["frac"] = mf["tflops"] / mf["peak_tflops"]
        c4 = valu.get("mfma_f64_c4")
        c4_ms = (extras.get("c4") or {}).get("kernel_ms")
        if c4 and c4_ms:
            c4["tflops"] = c4["flop_per_launch"] / (c4_ms * 1e-3) / 1e12
            c4["peak_tflops"] = 78.6
            c4["frac"] = c4["tflops"] / c4["peak_tflops"]
    line = {
        "metric": "audio frames/sec (bufferSize=1024, all features) at 1/2/4/8 GPUs; % HBM roofline",
        "value": value,
        "unit": "frames/s",
        "n_gpus": gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64 butterflies / f32 storage" if args.precision == "faithful" else "f32",
        "data": "synthetic (seeded splitmix64 PCM generated in HBM)",
        "config": {"workload": "C3+C4 feature set: %d frames x bufferSize=%d per GPU; 13 scalars (rms, energy, zcr, "
                               "7 spectral*, loudness.total, perceptualSpread, perceptualSharpness) + "
                               "loudness.specific[24] + mfcc[13] of 26 mel bands, float32 outputs; no spectra" % (F, n),
                   "buffer_size": n, "frames_per_gpu": F, "features": FEATURES,
                   "mel_bands": 26, "mfcc_coeffs": 13, "precision": args.precision,
                   "parallelism": {"torchrun": "frame shards, one process per GPU (%d)" % gpus,
                                   "single": "frame shards, one process driving %d GPUs" % gpus,
                                   "one": "one GPU"}[mode],
                   "devices": placement,
                   "gather_to_rank0": use_gather,
                   "value_source": "the shards, no data-path collective" + (
                       "; the RCCL gather of every rank's records to rank 0 timed in the same run: gather.value"
                       if use_gather else "")},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_note,
                     "kernel": "extract_kernel<%d>" % n, "kernel_ms": kernel_ms,
                     "kernel_ms_source": "mean launch duration: 20 launches back to back on one stream after "
                                         "the timed steps, HIP events around them (step_event_ms.launch_serial_ms; "
                                         "launch_alone_* = an event pair around each launch, which adds ~1 %); "
                                         "rocprofv3 --stats of bench.py --single-stream: profiles/",
                     "period_ms": km_s,
                     "period_source": ("launch period of the timed steps: HIP events around the timed region / steps"
                                       + (" (one stream)" if args.single_stream else " (steps pipelined over two streams)")),
                     "frac_pipelined": F * bytes_per_frame / (km_s * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "step_event_ms": stats_s,
                     "bytes_per_frame": bytes_per_frame},
    }
    line["roofline_fp64"] = roofline_fp64(n, F, kernel_ms, valu, args.precision)
    if gpus > 1:
        line["gather"] = gather if gather is not None else {"status": "off (--no-gather or shared GPUs)"}
    if valu:
        line["valu"] = valu
    for k in ("c5", "fast_mode", "mfcc_exact", "c2", "c3", "c4", "every_output", "host_path", "latency",
              "cpu_baseline"):
        if k in extras:
            line[k] = extras[k]
    if line.get("c5"):
        c5_finish(line["c5"], gpus)
    if "mfcc_exact" in line and line["mfcc_exact"].get("kernel_ms"):
        line["mfcc_exact"]["cost_vs_value_kernel"] = line["mfcc_exact"]["kernel_ms"] / kernel_ms - 1.0
    return line


if __name__ == "__main__":
    main()
