"""The JavaScript CPU restatement of the reference path (oracle/js/meyda_cpu.js) — the
cpu_baseline bench.py times on the GPU box — pinned bit for bit to the reference's own
golden outputs (tests/js/cpu_golden.js), and its timing harness's JSON contract."""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def node(*args, timeout=600):
    if not shutil.which("node"):
        pytest.skip("node is not installed")
    r = subprocess.run(["node", *args], capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_js_restatement_bit_exact_vs_reference_golden():
    out = node(os.path.join(ROOT, "tests", "js", "cpu_golden.js"))
    assert "cpu_golden: 13 checks passed" in out
    assert out.count("scalars worst rel 0\n") == 6


def test_js_cpu_bench_contract():
    out = node(os.path.join(ROOT, "oracle", "js", "bench_cpu.js"), "512", "0.3", "2")
    r = json.loads(out.strip().splitlines()[-1])
    assert r["threads"] == 2 and r["layout"] == "reference" and r["bufferSize"] == 512
    assert r["value"] > 0 and r["frames"] > 0 and len(r["per_thread"]) == 2
    assert r["node"].startswith("v") and r["cpu_model"]
