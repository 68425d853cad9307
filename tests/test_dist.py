"""Multi-process tests of the multi-GPU run's host side (CPU, gloo, world 2).

The GPU extraction and RCCL cannot run here. The world-2 test replays group.cpp's gather
protocol between two real processes: each rank extracts its shard of one global stream
(the CPU oracle stands in for the kernel), cuts it into the same chunks (mgx_shard_range),
packs each chunk into one transfer buffer (mgx_packed_layout) and sends it to rank 0 with
point-to-point messages (gloo send/recv in place of ncclSend/ncclRecv); rank 0 unpacks
every chunk into its record and checks it against one extraction of the whole batch. The
topology checks are bench.py's own (resolve_topology), which fail a run instead of
measuring fewer GPUs than asked.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_covers_exactly():
    from meyda_amd.dist import shard_range
    for total in (0, 1, 7, 64, 262144, 2097152 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
            assert sum(c for _, c in spans) == total
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_bench_topology_fails_loudly():
    sys.path.insert(0, ROOT)
    import bench
    rt = bench.resolve_topology
    assert rt(None, {}, 8) == ("one", 1)
    assert rt(4, {}, 8) == ("single", 4)
    assert rt(None, {"WORLD_SIZE": "8"}, 8) == ("torchrun", 8)
    assert rt(8, {"WORLD_SIZE": "8", "LOCAL_WORLD_SIZE": "8"}, 8) == ("torchrun", 8)
    assert rt(1, {"WORLD_SIZE": "1"}, 1) == ("one", 1)
    with pytest.raises(SystemExit, match="GPU"):
        rt(2, {}, 1)  # a 1-GPU box asked for 2: no silent n_gpus 1
    with pytest.raises(SystemExit, match="WORLD_SIZE"):
        rt(8, {"WORLD_SIZE": "4"}, 8)
    with pytest.raises(SystemExit, match="one GPU per rank"):
        rt(2, {"WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "2"}, 1)
    assert rt(2, {"WORLD_SIZE": "2", "LOCAL_WORLD_SIZE": "2"}, 1, allow_shared=True) == ("torchrun", 2)


def _pack(capi, d, mask, ref, sl, cn):
    """One chunk's transfer buffer, laid out by mgx_packed_layout (what the kernel writes)."""
    nbytes, off = capi.packed_layout(d, mask, cn)
    buf = np.zeros(nbytes, np.uint8)
    for j, k in enumerate(capi.SCALAR_NAMES):
        buf[off[k]:off[k] + 4 * cn] = ref["scalars"][sl, j].astype(np.float32).view(np.uint8)
    for k, src in (("loudness.specific", ref["loudness_specific"]), ("mfcc", ref["mfcc"])):
        b = np.ascontiguousarray(src[sl]).view(np.uint8).ravel()
        buf[off[k]:off[k] + b.size] = b
    return buf


def _worker(rank, world, port, total, n, nch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    sys.path.insert(0, ROOT)
    try:
        import torch.distributed as dist
        from meyda_amd import SEED, capi
        from meyda_amd.dist import init_control_plane
        from oracle import oracle
        r, _, w = init_control_plane()
        assert (r, w) == (rank, world)
        d = capi.make_desc(buffer_size=n)
        mask = (1 << 13) - 1 | capi.OUT_LOUDNESS_SPECIFIC | capi.OUT_MFCC
        counts = [capi.shard_range(total, world, i)[1] for i in range(world)]
        starts = [capi.shard_range(total, world, i)[0] for i in range(world)]
        x = oracle.synth_frames(SEED, starts[rank], counts[rank], n)  # this rank's shard of the global stream
        ref = oracle.extract(x)
        if rank == 0:
            rec = {"scalars": np.full((total, 13), np.nan, np.float32),
                   "loudness.specific": np.full((total, 24), np.nan, np.float32),
                   "mfcc": np.full((total, 13), np.nan, np.float32)}
            c0s = [capi.shard_range(counts[0], nch, c) for c in range(nch)]
            for c0, cn in c0s:  # the root's own shard in place
                rec["scalars"][c0:c0 + cn] = ref["scalars"][c0:c0 + cn]
                rec["loudness.specific"][c0:c0 + cn] = ref["loudness_specific"][c0:c0 + cn]
                rec["mfcc"][c0:c0 + cn] = ref["mfcc"][c0:c0 + cn]
            for c in range(nch):
                for p in range(1, world):
                    c0, cn = capi.shard_range(counts[p], nch, c)
                    if not cn:
                        continue
                    nbytes, off = capi.packed_layout(d, mask, cn)
                    t = torch.empty(nbytes, dtype=torch.uint8)
                    dist.recv(t, src=p)  # ncclRecv into the staging slot
                    buf = t.numpy()
                    dst = slice(starts[p] + c0, starts[p] + c0 + cn)
                    for j, k in enumerate(capi.SCALAR_NAMES):  # unpack_kernel's segments
                        rec["scalars"][dst, j] = buf[off[k]:off[k] + 4 * cn].view(np.float32)
                    for k in ("loudness.specific", "mfcc"):
                        wdt = rec[k].shape[1]
                        rec[k][dst] = buf[off[k]:off[k] + 4 * wdt * cn].view(np.float32).reshape(cn, wdt)
            whole = oracle.extract(oracle.synth_frames(SEED, 0, total, n))
            ok = (np.array_equal(rec["scalars"], whole["scalars"].astype(np.float32), equal_nan=True)
                  and np.array_equal(rec["mfcc"], whole["mfcc"], equal_nan=True)
                  and np.array_equal(rec["loudness.specific"], whole["loudness_specific"], equal_nan=True))
            q.put(("ok" if ok else "mismatch", rank))
        else:
            for c in range(nch):
                c0, cn = capi.shard_range(counts[rank], nch, c)
                if cn:  # ncclSend of the chunk's packed buffer
                    dist.send(torch.from_numpy(_pack(capi, d, mask, ref, slice(c0, c0 + cn), cn)), dst=0)
            q.put(("ok", rank))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent
        q.put(("error: %r" % (e,), rank))


# even and ragged shards, chunk counts; 4 ranks rehearse a wider gather (every peer into rank 0), and
# N = 2048 is C5's frame size
@pytest.mark.parametrize("world,n,total,nch", [(2, 512, 64, 1), (2, 512, 67, 3), (2, 512, 40, 8), (4, 512, 131, 3),
                                               (4, 2048, 37, 8)])
def test_gather_protocol_matches_single_process(world, n, total, nch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, n, nch, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(res, key=lambda t: t[1]) == [("ok", r) for r in range(world)], res


def test_bench_value_is_the_shards_rate():
    """The path partitions (independent frames): at N > 1 the line's value is the shards' rate;
    the RCCL gather-inclusive rate of the same run is reported beside it, never as value."""
    import types

    import bench
    args = types.SimpleNamespace(steps=10, warmup=2, precision="faithful", single_stream=False)
    st = {"launch_alone_mean_ms": 0.6, "launch_serial_ms": 0.6}
    line = bench.build_line(args, 8, "torchrun", [], 262144, 1024, 3.5e9, 10.0, 0.6, st,
                            {"status": "ok", "value": 2.8e9}, {})
    assert line["value"] == 3.5e9 and line["n_gpus"] == 8 and line["scaling"] == "weak"
    assert line["gather"]["value"] == 2.8e9 and abs(line["gather"]["vs_shards"] - 0.8) < 1e-12
    assert line["config"]["gather_to_rank0"] is True
    failed = bench.build_line(args, 8, "torchrun", [], 262144, 1024, 3.5e9, 10.0, 0.6, st,
                              {"status": "failed on rank 3"}, {})
    assert failed["value"] == 3.5e9 and failed["config"]["gather_to_rank0"] is False


def test_bench_c5_field_shape():
    """Config C5 (BASELINE.json configs[4]: N = 2048, all features incl. MFCC, 262,144 frames per
    GPU, RCCL gather) is a field of every line: at N = 1 its gather is reported as skipped, at
    N > 1 it starts as "not run" and, once measured, carries the gather-inclusive rate beside
    the shards' (vs_shards), never replacing `value`."""
    import types

    import bench
    st = {"launch_alone_mean_ms": 1.3, "launch_serial_ms": 1.3}
    one = bench.c5_field(1, 262144, 0.026, 1.3, st, 20, False)
    assert one["buffer_size"] == 2048 and one["frames_per_gpu"] == 262144 and one["frames_total"] == 262144
    assert one["bytes_per_frame"] == 4 * 2048 + 4 * 50 and one["features"] == bench.FEATURES
    assert one["gather"]["status"].startswith("skipped (1 GPU)")
    assert abs(one["value"] - 262144 * 20 / 0.026) < 1e-6 * one["value"]
    assert abs(one["roofline_frac"] - 262144 * 8392 / 1.3e-3 / 8e12) < 1e-12
    eight = bench.c5_field(8, 262144, 0.027, 1.35, {"rank0": st, "per_rank_period_ms": [1.35] * 8}, 20, True)
    assert eight["frames_total"] == 2097152 and eight["gather"]["status"] == "not run"
    assert eight["kernel_ms"] == 1.3
    shards = 8 * 262144 * 20 / 0.027
    args = types.SimpleNamespace(steps=20, warmup=5, precision="faithful", single_stream=False)
    st1 = {"launch_alone_mean_ms": 0.6, "launch_serial_ms": 0.6}
    # a gather that has not completed (a deadline printing the line mid-phase, or a failure): C5 has
    # no gather-inclusive value, the shards' rate beside it
    line = bench.build_line(args, 8, "torchrun", [], 262144, 1024, 3.5e9, 10.0, 0.6, st1,
                            {"status": "ok", "value": 2.8e9}, {"c5": eight})
    assert line["value"] == 3.5e9 and line["c5"]["frames_total"] == 2097152
    assert line["c5"]["value"] is None and abs(line["c5"]["shards_value"] - shards) < 1e-6 * shards
    assert "not run" in line["c5"]["value_source"]
    # BASELINE C5 is "frames sharded across GPUs with RCCL gather": once the gather ran, c5.value is the
    # gather-inclusive rate and the shards' rate stays beside it
    eight["gather"].update({"status": "ok", "value": 0.9 * shards})
    line = bench.build_line(args, 8, "torchrun", [], 262144, 1024, 3.5e9, 10.0, 0.6, st1,
                            {"status": "ok", "value": 2.8e9}, {"c5": eight})
    c5 = line["c5"]
    assert c5["value"] == 0.9 * shards and abs(c5["shards_value"] - shards) < 1e-6 * shards
    assert abs(c5["gather"]["vs_shards"] - 0.9) < 1e-12 and c5["value_source"].startswith("gather-inclusive")
    assert line["value"] == 3.5e9  # the headline keeps the shards (SURVEY §7 hard part 5), gather beside it
    # N = 1: nothing to gather, value = shards_value
    line1 = bench.build_line(args, 1, "one", [], 262144, 1024, 4.4e8, 10.0, 0.6, st1, None, {"c5": one})
    assert line1["c5"]["value"] == line1["c5"]["shards_value"] == one["shards_value"]
    assert line1["c5"]["value_source"].startswith("one GPU")
    p = bench.parse([])
    assert not p.no_c5 and p.c5_frames == 262144 and not p.strict_gather


def test_bench_line_carries_every_config():
    """The N = 1 line carries every BASELINE config beside `value` (C2, C3, C4, C5), the
    reference-order MFCC's rate with its cost against the headline kernel, the real-time latency
    and the C4 MFMA counters priced at C4's own launch time; none of them replaces `value`."""
    import types

    import bench
    args = types.SimpleNamespace(steps=20, warmup=5, precision="faithful", single_stream=False)
    st = {"launch_alone_mean_ms": 0.6, "launch_serial_ms": 0.6}
    mf = {"instr_per_launch": 655360.0, "flop_per_launch": 512 * 655360.0, "busy_cycles_per_launch": 1.0,
          "gui_active_cycles": 1.0}
    valu = {"instr_per_frame": 1200.0, "cvt_per_frame": 400.0, "f64_per_frame": 450.0, "lds_per_frame": 97.0,
            "mfma_f64": dict(mf, flop_per_launch=512 * 458752.0), "mfma_f64_c4": dict(mf)}
    extras = {"pmc": (1.13e9, valu, "note"), "c2": {"value": 1e9}, "c3": {"value": 5e8}, "c4": {"value": 5e8, "kernel_ms": 0.5},
              "c5": bench.c5_field(1, 262144, 0.026, 1.3, {"launch_alone_mean_ms": 1.3, "launch_serial_ms": 1.3}, 20, False),
              "mfcc_exact": {"value": 3.6e8, "kernel_ms": 0.75}, "latency": {"status": "ok", "c1": {"us_per_call": 25.0}}}
    line = bench.build_line(args, 1, "one", [], 262144, 1024, 4.5e8, 0.0116, 0.58, st, None, extras)
    assert line["value"] == 4.5e8 and "gather" not in line
    for k in ("c2", "c3", "c4", "c5", "mfcc_exact", "latency"):
        assert k in line, k
    assert abs(line["mfcc_exact"]["cost_vs_value_kernel"] - 0.25) < 1e-12
    c4 = line["valu"]["mfma_f64_c4"]
    assert abs(c4["tflops"] - 512 * 655360.0 / 0.5e-3 / 1e12) < 1e-9 and c4["peak_tflops"] == 78.6
    assert line["roofline"]["traffic"] == 1.13e9 and line["roofline"]["kernel_ms"] == 0.6


def test_failed_gather_fails_the_run():
    """At N > 1 a gather that failed or passed its deadline makes bench.py exit non-zero (status 3)
    after rank 0 has printed the line with the shards and the gather's status; a run whose gathers
    all completed, or a run with none (N = 1, --no-gather), exits 0; --allow-gather-failure keeps a
    shards-only run at 0."""
    import bench
    args = bench.parse([])
    assert not args.allow_gather_failure
    assert bench.gather_exit_code(args, []) == 0
    assert bench.gather_exit_code(args, [None]) == 0
    assert bench.gather_exit_code(args, ["ok", "ok"]) == 0
    assert bench.gather_exit_code(args, ["ok", "timed out"]) == 3
    assert bench.gather_exit_code(args, ["failed on rank 3: RuntimeError('ncclRecv')"]) == 3
    assert bench.gather_exit_code(args, ["not run"]) == 3  # a phase that never started is not a success
    lenient = bench.parse(["--allow-gather-failure"])
    assert bench.gather_exit_code(lenient, ["timed out"]) == 0


def test_bench_line_carries_fp64_roofline_and_all_core_cpu_baseline(monkeypatch):
    """the faithful path is FP64-bound, so the line reports the FP64 roofline (the FFT's
    algorithmic 5 N log2 N flops per frame against the 78.6 TFLOP/s FP64 peak, with the measured
    VALU-busy fraction and the binding limit named) beside the HBM one; and BASELINE.md's CPU baseline
    at os.cpus().length worker_threads beside the per-GPU share, with both counts stated."""
    import types

    import bench
    args = types.SimpleNamespace(steps=20, warmup=5, precision="faithful", single_stream=False)
    st = {"launch_alone_mean_ms": 0.6, "launch_serial_ms": 0.6}
    mf = {"instr_per_launch": 1.0, "flop_per_launch": 512.0, "busy_cycles_per_launch": 1.0, "gui_active_cycles": 1.0}
    valu = {"instr_per_frame": 1160.0, "cvt_per_frame": 394.0, "f64_per_frame": 438.0, "lds_per_frame": 92.0,
            "valu_busy_measured": 0.9, "any_busy_measured": 1.2, "mfma_f64": dict(mf), "mfma_f64_c4": dict(mf)}
    line = bench.build_line(args, 1, "one", [], 262144, 1024, 4.5e8, 0.0116, 0.58, st, None,
                            {"pmc": (1.13e9, valu, "note")})
    r = line["roofline_fp64"]
    assert r["fft_flop_per_frame"] == 5 * 1024 * 10 and r["peak"] == 78.6 and r["bound"] == "fp64"
    assert abs(r["achieved"] - 262144 * 51200 / 0.6e-3 / 1e12) < 1e-9
    assert abs(r["frac"] - r["achieved"] / 78.6) < 1e-12
    assert r["valu_busy_measured"] == 0.9 and "FP64-pipe" in r["binding"] and "est_fp64_cvt_busy" in r
    assert line["roofline"]["bound"] == "hbm"  # the contract's roofline stays the HBM one
    # without counters (N > 1, --no-pmc) the flop roofline is still there
    bare = bench.build_line(args, 8, "torchrun", [], 262144, 1024, 3.5e9, 10.0, 0.6, st, None, {})
    assert bare["roofline_fp64"]["frac"] > 0 and "binding" not in bare["roofline_fp64"]

    calls = []

    def fake_node(n, seconds, threads, fset="all", timeout_extra=120):
        calls.append((n, fset, threads))
        return {"value": 1000.0 * threads, "frames": 64 * threads, "seconds": seconds, "cpu_model": "cpu",
                "logical_cpus": 8, "node": "v12", "us_per_call": 11.0, "calls": 1000}
    monkeypatch.setattr(bench, "node_cpu", fake_node)
    monkeypatch.setattr(bench, "cpu_port_c", lambda n, s, t: {"value": 1.0, "cores": t, "kind": "port-c"})
    import shutil
    monkeypatch.setattr(shutil, "which", lambda _: "/usr/bin/node")
    cb = bench.cpu_baseline(1024, 0.1)
    allc = os.cpu_count()
    assert cb["cores"] == min(bench.CPU_THREADS, allc) and cb["all_cores"]["cores"] == allc
    assert cb["all_cores"]["value"] == 1000.0 * allc and "schedulable_cpus" in cb["all_cores"]
    assert (1024, "all", allc) in calls and cb["one_thread"] == 1000.0
