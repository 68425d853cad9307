"""Runs the JavaScript facade tests (tests/js/*.js) under Node through the N-API addon."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ADDON = os.path.join(ROOT, "meyda_amd", "addon", "meyda_napi.node")


def run_node(script):
    if not shutil.which("node"):
        pytest.skip("node is not installed")
    if not os.path.exists(ADDON):
        pytest.skip("N-API addon not built (make -C meyda_amd/addon)")
    r = subprocess.run(["node", "--expose-gc", os.path.join(ROOT, "tests", "js", script)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_facade_host_side():
    out = run_node("facade_cpu.js")
    assert "facade_cpu: 9 checks passed" in out


def test_facade_batched_delivery_host_side():
    """The batched callback path's JavaScript logic against a stand-in addon (no GPU)."""
    out = run_node("facade_batch.js")
    assert "facade_batch: 4 checks passed" in out


@pytest.mark.gpu
def test_facade_on_gpu():
    out = run_node("facade_gpu.js")
    assert "facade_gpu: 16 checks passed" in out
