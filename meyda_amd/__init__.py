"""meyda_amd — MI355X-native engine for Meyda's per-buffer FFT + feature-extraction hot path.

Layout:
  csrc/        HIP kernels (kernels.hip) and the C-ABI host code (plan.cpp)
  libmeyda_gpu.so   built in-tree by `make` / __graft_entry__.build()
  addon/       N-API addon exposing the C ABI to Node
  js/          the Meyda-compatible JavaScript facade (get / start / stop / featureInfo)
  capi.py      ctypes binding used by the Python tests and bench.py
  dist.py      multi-GPU sharding (one process per GPU, torch.distributed)
"""
from .capi import (ALL_FEATURES, FEATURE_NAMES, SCALAR_NAMES, MgxError, Plan, device_count,  # noqa: F401
                   host_tables, lib, synth_frames_device)

SEED = 0x6D657964  # "meyd", SURVEY.md §8(d)
