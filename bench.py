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

Multi-GPU (torchrun, one process per GPU): each rank extracts its own 262,144-frame
shard of one global stream (weak scaling) through the library's multi-device group
(include/meyda_gpu.h, mgx_group_create_rank), which gathers every rank's per-frame
feature records to rank 0 over xGMI with RCCL point-to-point transfers, chunked so
that chunk i's transfer overlaps chunk i+1's extraction (the north star's gather is
inside the timed step; --no-gather times the shards alone). torch.distributed (gloo)
is only the control plane: the RCCL id broadcast, barriers and the max-over-ranks
elapsed time. Rank 0 prints the JSON line with the whole-job frames/s.
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


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=150.0,
                    help="untimed launches before the warmup steps, until the GPU clock has ramped "
                         "(3 warmup launches alone leave the first timed steps ~8%% slow)")
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--frames", type=int, default=262144, help="frames per GPU per step")
    ap.add_argument("--precision", default="faithful", choices=["faithful", "fast"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-buffer measurement")
    ap.add_argument("--cpu-seconds", type=float, default=6.0,
                    help="CPU baseline: seconds of the multi-thread run (1 thread and the C port: a third)")
    ap.add_argument("--also-fast", action="store_true", help="report the fp32 mode alongside")
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: time the shards alone, without the RCCL gather to rank 0")
    ap.add_argument("--chunks", type=int, default=0, help="N > 1: gather pipeline depth (0 = automatic)")
    ap.add_argument("--no-every-output", action="store_true",
                    help="N = 1: skip the secondary timing with every output (spectra too) and 40 mel bands")
    ap.add_argument("--no-pmc", action="store_true",
                    help="N = 1: skip the live rocprofv3 --pmc passes (HBM traffic, VALU instruction mix)")
    return ap.parse_args()


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


def cpu_baseline(n, seconds):
    """The reference's Node/jsfft CPU path as the build's JavaScript restatement
    (oracle/js/meyda_cpu.js, bit-exact to the reference's golden outputs), in the
    reference's per-buffer structure, timed on this host with 1 and CPU_THREADS
    worker_threads on the seeded stream; the C port beside it."""
    import shutil
    import subprocess
    threads = min(CPU_THREADS, os.cpu_count() or 1)
    js = os.path.join(ROOT, "oracle", "js", "bench_cpu.js")
    out = {"unit": "frames/s", "kind": "js-restatement"}
    if shutil.which("node"):
        def run(t, secs):
            r = subprocess.run(["node", js, str(n), str(secs), str(t), "reference"], capture_output=True, text=True,
                               timeout=120 + 4 * secs, check=True)
            return json.loads(r.stdout.strip().splitlines()[-1])
        one = run(1, max(1.0, seconds / 3))
        many = run(threads, seconds)
        out.update({"value": many["value"], "cores": threads, "cpu_model": many["cpu_model"],
                    "logical_cpus": many["logical_cpus"], "node": many["node"], "one_thread": one["value"],
                    "sample": "%d frames (N=%d, all features, seeded noise, the reference's per-buffer structure) "
                              "over %.1f s on %d worker_threads; 1 thread: %.0f frames/s"
                              % (many["frames"], n, many["seconds"], threads, one["value"])})
    else:  # no Node on this host: the C port stands in
        out.update({"kind": "port", "value": None, "note": "node not found"})
    out["port_c"] = cpu_port_c(n, max(1.0, seconds / 3), threads)
    if out.get("value") is None:
        out["value"] = out["port_c"]["value"]
        out["cores"] = threads
    return out


def capi_seed():
    import meyda_amd
    return meyda_amd.SEED


_STREAMS = []


def stream_pair():
    """The two streams every pipelined loop of the run uses, created once: a stream's first
    launches carry a one-time cost of milliseconds (its hardware queue), which settle() absorbs."""
    if not _STREAMS:
        _STREAMS.extend([torch.cuda.current_stream(), torch.cuda.Stream()])
    return _STREAMS


def settle(step, ms, dist=None):
    """Untimed steps for `ms` of wall time (clock ramp-up), before the warmup steps."""
    streams = stream_pair()
    t0 = time.perf_counter()
    go = True
    while go:
        pipelined(step, streams, 0, 8)
        torch.cuda.synchronize()
        go = (time.perf_counter() - t0) * 1e3 < ms
        if dist:  # every rank runs the same number of (collective) steps
            t = torch.tensor([1 if go else 0], dtype=torch.int32)
            dist.all_reduce(t, op=dist.ReduceOp.MIN)
            go = bool(t.item())


def pipelined(step, streams, first, count):
    """Steps first..first+count-1, consecutive steps alternating between the two streams and
    the two output sets (step(stream, k), k = i & 1): a stream of batches the way a streaming
    caller runs it, so step i+1's workgroups start on the CUs step i's last waves leave while it
    drains (one launch ends with ~45 us of SIMDs running out of waves). Forks
    from and joins back into streams[0]."""
    e = torch.cuda.Event()
    e.record(streams[0])
    streams[1].wait_event(e)
    for i in range(first, first + count):
        step(streams[i & 1].cuda_stream, i & 1)
    e = torch.cuda.Event()
    e.record(streams[1])
    streams[0].wait_event(e)


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
    passes = {"fetch_t": ("time_only", "FETCH_SIZE"), "fetch": ("all", "FETCH_SIZE"), "write": ("all", "WRITE_SIZE"),
              "valu": ("all", "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 "
                              "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS"),
              "mfma": ("all", "SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES "
                              "GRBM_GUI_ACTIVE")}
    got = {}
    reps = 3
    for key, (fset, ctrs) in passes.items():
        d = os.path.join(tmp, key)
        env = dict(os.environ, PROBE_SET=fset, PROBE_N=str(n), PROBE_PREC=precision, PROBE_REPS=str(reps), TMPDIR="/tmp")
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
    mm = got["mfma"]
    # the DCT's v_mfma_f64_4x4x4_4b_f64: 4 blocks x 4x4x4 = 256 FMAs = 512 FLOP per wave instruction
    valu["mfma_f64"] = {"instr_per_launch": mm["SQ_INSTS_VALU_MFMA_F64"], "flop_per_launch": 512 * mm["SQ_INSTS_VALU_MFMA_F64"],
                        "busy_cycles_per_launch": mm["SQ_VALU_MFMA_BUSY_CYCLES"], "gui_active_cycles": mm["GRBM_GUI_ACTIVE"]}
    note = ("live: rocprofv3 --pmc passes of this run over tools/pmc_probe.py (%d frames x N=%d, same features); "
            "FETCH_SIZE x %.4f (time-only calibration), reads %.4g B + writes %.4g B per launch" % (F, n, cal, read, write))
    return read + write, valu, note


def run_mode(step, steps, warmup, dist):
    """W untimed steps, then exactly `steps` timed ones bracketed by a barrier and a device
    synchronisation on both sides, pipelined over two streams (pipelined()); HIP events on the
    launch stream around the whole timed region give the launch period (no events between the
    steps: an event pair per step cost 1-2 % of the step time, tools/step_overlap.py). Then an
    untimed single-stream pass with an event pair around each launch: the launch duration on
    its own, which is what rocprofv3 reports per dispatch."""
    streams = stream_pair()
    pipelined(step, streams, 0, warmup)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(streams[0])
    pipelined(step, streams, 0, steps)
    e1.record(streams[0])
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    period = e0.elapsed_time(e1) / steps
    # the launch on its own (serialised on one stream), untimed by the step clock
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
    for a, b in ev:
        a.record(streams[0])
        step(streams[0].cuda_stream, 0)
        b.record(streams[0])
    torch.cuda.synchronize()
    iso = [a.elapsed_time(b) for a, b in ev]
    stats = {"period_ms": period, "launch_alone_mean_ms": float(np.mean(iso)),
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
                 "per_rank_launch_alone_ms": [r["launch_alone_mean_ms"] for r in allr]}
    return elapsed, period, stats


def main():
    args = parse()
    from meyda_amd import dist as mdist
    rank, local, world = mdist.env_rank_world()
    dist = None
    # one GPU per rank; (a box with fewer GPUs than ranks, a rehearsal only, shares them)
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    if world > 1:
        import torch.distributed as tdist
        mdist.init("gloo")  # control plane only; the data path is the library's RCCL gather
        dist = tdist
    n, F = args.n, args.frames
    frames = torch.empty(F, n, dtype=torch.float32, device="cuda")
    # each rank its own shard of one global synthetic stream
    capi.synth_frames_device(frames, capi_seed(), first_frame=rank * F)
    dev = torch.cuda.current_device()
    plan = capi.Plan(buffer_size=n, precision=args.precision, device=dev)
    gather = world > 1 and not args.no_gather
    if gather:
        uid = [capi.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        group = capi.Group(buffer_size=n, rank=rank, nranks=world, unique_id=uid[0], precision=args.precision,
                           device=dev)
        # rank 0 holds the whole job's feature record; the other ranks only their transfer buffers
        # (two output sets: consecutive steps are in flight together, pipelined())
        sets = [plan.alloc_outputs(F * world if rank == 0 else 1, FEATURES) for _ in range(2)]
        mask = capi.output_mask(sets[0][1])

        def step(s, k):
            group.extract_device([frames.data_ptr()], [F] * world, sets[k][1] if rank == 0 else None, mask,
                                 args.chunks, [s])
    else:
        sets = [plan.alloc_outputs(F, FEATURES) for _ in range(2)]

        def step(s, k):
            plan.extract_device(frames.data_ptr(), F, sets[k][1], s)
    torch.cuda.synchronize()
    settle(step, args.settle_ms, dist)
    elapsed, kernel_ms, step_stats = run_mode(step, args.steps, args.warmup, dist)
    fast = None
    if args.also_fast and args.precision != "fast" and world == 1:
        plan_f = capi.Plan(buffer_size=n, precision="fast", device=dev)

        def step_f(s, k):
            plan_f.extract_device(frames.data_ptr(), F, sets[k][1], s)
        settle(step_f, args.settle_ms)
        el_f, km_f, _ = run_mode(step_f, args.steps, args.warmup, dist)
        fast = {"value": world * F * args.steps / el_f, "kernel_ms": km_f,
                "roofline_frac": (F * (4 * n + 4 * OUT_FLOATS)) / (km_f * 1e-3) / 1e9 / HBM_PEAK_GBS}
    every = None
    if world == 1 and not args.no_every_output:
        # Secondary (never `value`): EVERY output of the path — the headline set plus the
        # amplitude, power and complex spectra — with the 40-band mel of config C4, same frames
        plan_e = capi.Plan(buffer_size=n, precision=args.precision, num_mel_bands=40, device=dev)
        feats_e = FEATURES + ["amplitudeSpectrum", "powerSpectrum", "complexSpectrum"]
        sets_e = [plan_e.alloc_outputs(F, feats_e) for _ in range(2)]

        def step_e(s, k):
            plan_e.extract_device(frames.data_ptr(), F, sets_e[k][1], s)
        settle(step_e, args.settle_ms)
        el_e, km_e, _ = run_mode(step_e, args.steps, args.warmup, dist)
        bpf_e = 4 * n + 4 * (OUT_FLOATS + 2 * (n // 2) + 2 * n)
        every = {"features": feats_e, "mel_bands": 40, "value": F * args.steps / el_e, "unit": "frames/s",
                 "kernel_ms": km_e, "bytes_per_frame": bpf_e,
                 "roofline_frac": F * bpf_e / (km_e * 1e-3) / 1e9 / HBM_PEAK_GBS}
        del sets_e
    if rank == 0:
        bytes_per_frame = 4 * n + 4 * OUT_FLOATS
        alone_ms = (step_stats["rank0"] if dist else step_stats)["launch_alone_median_ms"]
        achieved = F * bytes_per_frame / (kernel_ms * 1e-3) / 1e9
        traffic, valu, traffic_note = None, None, "not measured (--no-pmc or N > 1)"
        if world == 1 and not args.no_pmc:
            try:
                traffic, valu, traffic_note = pmc_live(n, F, args.precision)
            except Exception as e:  # the counters are a report, never the measurement itself
                traffic, valu, traffic_note = None, None, "rocprofv3 passes failed: %r" % (e,)
        if valu is not None:
            # the faithful path is FP64-VALU bound. Issue costs per wave64
            # instruction measured by tools/ubench/op_rates.hip (profiles/r01_op_rates.log):
            # f64 ~5.0, f32<->f64 conversion 4.2 cycles; at the clock this run's kernel time implies
            cyc = kernel_ms * 1e-3 * 2.4e9 * 1024 / F  # SIMD cycles per frame (2.4 GHz held, 1,024 SIMDs)
            valu["frame_simd_cycles"] = cyc
            valu["est_fp64_cvt_busy"] = (valu["f64_per_frame"] * 5.0 + valu["cvt_per_frame"] * 4.2) / cyc
            # FP64 pipe (vector and matrix share it): 78.6 TFLOP/s dense on MI355X (1,024 SIMDs x 32
            # FLOP/clk x 2.4 GHz; v_mfma_f64_4x4x4 issues every 16 cycles: tools/ubench/op_rates.hip)
            mf = valu["mfma_f64"]
            mf["tflops"] = mf["flop_per_launch"] / (kernel_ms * 1e-3) / 1e12
            mf["peak_tflops"] = 78.6
            mf["frac"] = mf["tflops"] / mf["peak_tflops"]
        line = {
            "metric": "audio frames/sec (bufferSize=1024, all features) at 1/2/4/8 GPUs; % HBM roofline",
            "value": world * F * args.steps / elapsed,
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64 butterflies / f32 storage" if args.precision == "faithful" else "f32",
            "data": "synthetic (seeded splitmix64 PCM generated in HBM)",
            "config": {"workload": "C3+C4 all features: %d frames x bufferSize=%d per GPU, float32 outputs" % (F, n),
                       "buffer_size": n, "frames_per_gpu": F, "features": FEATURES,
                       "mel_bands": 26, "mfcc_coeffs": 13,
                       "precision": args.precision, "parallelism": "frame shards, %d proc" % world,
                       "gather_to_rank0": bool(gather),
                       "gather": ("RCCL send/recv to rank 0 in the timed step, %s chunks" % (args.chunks or "auto"))
                       if gather else None},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_note,
                         "kernel": "extract_kernel<%d>" % n, "kernel_ms": kernel_ms,
                         "kernel_ms_source": "launch period: HIP events around the timed region / steps "
                                             "(steps pipelined over two streams); a launch on its own: step_event_ms",
                         "frac_launch_alone": F * bytes_per_frame / (alone_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "step_event_ms": step_stats,
                         "bytes_per_frame": bytes_per_frame},
        }
        if valu:
            line["valu"] = valu
        if fast:
            line["fast_mode"] = fast
        if every:
            line["every_output"] = every
        if world == 1 and not args.no_host_path:
            line["host_path"] = host_path(plan, frames)
        if not args.no_cpu_baseline and world == 1:
            line["cpu_baseline"] = cpu_baseline(n, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
