"""Measurement tooling stays in step with the product source: every timing ablation of
tools/ablate.py is anchored on text of meyda_amd/csrc/kernels.hip (a moved anchor would make the
ablation fail at build time, or measure nothing); the gather-trace reader splits a call into its waits."""
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_ablation_anchors_match_kernel_source():
    spec = importlib.util.spec_from_file_location("ablate", os.path.join(ROOT, "tools", "ablate.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    src = open(os.path.join(ROOT, "meyda_amd", "csrc", "kernels.hip")).read()
    stale = [name for name, pats in mod.PATCHES.items() if not all(a in src for a, _ in pats)]
    assert not stale, stale


def test_gather_trace_splits_a_call_into_its_waits(tmp_path, capsys):
    # tools/gather_trace.py on a synthetic two-rank trace (group.cpp's MGX_GROUP_TRACE lines: "ns rank tag chunk peer";
    # a call's first line carries its chunk count and bufferSize)
    spec = importlib.util.spec_from_file_location("gather_trace", os.path.join(ROOT, "tools", "gather_trace.py"))
    gt = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gt)
    us = 1000
    root = [(0, "call", 2, 1024), (10 * us, "take_wait", 0, 1), (40 * us, "taken", 0, 1), (50 * us, "fin_wait", 0, 1),
            (70 * us, "consumed", 0, 1), (100 * us, "call", 2, 1024)]
    peer = [(0, "call", 2, 1024), (5 * us, "post_wait", 0, 0), (35 * us, "posted", 0, 0), (100 * us, "call", 2, 1024)]
    for r, evs in ((0, root), (1, peer)):
        with open(tmp_path / ("t.%d" % r), "w") as f:
            for ns, tag, ch, p in evs:
                f.write("%d %d %s %d %d\n" % (ns, r, tag, ch, p))
    calls = gt.load(str(tmp_path / "t"))
    assert len(calls[0]) == 2 and len(calls[1]) == 2
    w, span = gt.waits(calls[0][0])
    assert abs(w["taken"] - 0.030) < 1e-9 and abs(w["consumed"] - 0.020) < 1e-9 and abs(span - 0.070) < 1e-9
    w, _ = gt.waits(calls[1][0])
    assert abs(w["posted"] - 0.030) < 1e-9
    gt.report({r: [c for c in cs if c[0][3] == 1024] for r, cs in calls.items()}, 20)
    out = capsys.readouterr().out
    assert "rank 0 (root)" in out and "rank 1 (peer)" in out and "post -> root's copy issued: median 5.0 us" in out


def test_reference_order_log_emulation_is_exact(tmp_path):
    # tools/emu/ref_ln_check.c: the reference-order MFCC's fast log (kernels.hip ref_ln: plan table, degree-6
    # polynomial, interval check, library fallback) against glibc's double log rounded to float32 on 23.5 M
    # floats -- the claim that lets the fast path replace the library log bit for bit
    import subprocess
    exe = str(tmp_path / "ref_ln_check")
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tools", "emu", "ref_ln_check.c"), "-lm",
                           "-o", exe])
    out = subprocess.run([exe], capture_output=True, text=True, timeout=120).stdout
    assert "checked 23538910 floats: 0 mismatches" in out, out[-2000:]
    assert "err " not in out, out[-2000:]  # the |y - ln x| bound held everywhere
