"""Measurement tooling stays in step with the product source: every timing ablation of
tools/ablate.py is anchored on text of meyda_amd/csrc/kernels.hip (a moved anchor would make the
ablation fail at build time, or measure nothing)."""
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
