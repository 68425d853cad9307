#!/usr/bin/env python3
"""Timing ablations, kept out of the product source: builds abl/libabl_<name>.so from a
patched copy of the kernel in which one part's work is skipped (results are WRONG: for
timing only, with MEYDA_AMD_LIB pointing at the variant). Each patch is anchored on text
of meyda_amd/csrc/kernels.hip and fails loudly if the anchor moved.
usage: ablate.py NAME [NAME ...]   (names: see PATCHES, or a+b+... for several at once; 'all' builds every one)"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "meyda_amd", "csrc")

# name -> list of (anchor, replacement); opaque(0) keeps the skipped code compiled but never run
PATCHES = {
    "no_phase2": [("    MGX_MARK(phase2_start);\n    prio_hi<4>();\n", "    MGX_MARK(phase2_start);\n    prio_hi<4>();\n    if (opaque(0)) {\n"),
                  ("    prio_lo<4>();\n    MGX_MARK(phase2_end);", "    }\n    prio_lo<4>();\n    MGX_MARK(phase2_end);")],
    "no_loud2": [("if (!LIGHT && q->need_spectrum && q->need_loudness) {", "if (opaque(0) && !LIGHT && q->need_spectrum && q->need_loudness) {")],
    "no_ln": [("        mfcc_log<CHAIN, SUB>(q, l2, recs, 0);", "        if (opaque(0)) mfcc_log<CHAIN, SUB>(q, l2, recs, 0);")],
    "no_dct": [("        mfcc_dct<CHAIN, SUB>(q, l2, recs, dct_lds, 0, f0);",
                "        if (opaque(0)) mfcc_dct<CHAIN, SUB>(q, l2, recs, dct_lds, 0, f0);")],
    # (the window copies in phase 2 and the scalar passes, kScalDefer)
    "no_scalars": [("      const bool defer = kScalDefer && q->scal_defer && !stolen;", "      const bool defer = opaque(0);"),
                   ("for (int i = l2; !defer && i <", "for (int i = l2; opaque(0) && i <"),
                   ("      if (q->scal_defer) {\n        prio_hi<4>();", "      if (opaque(0)) {\n        prio_hi<4>();"),
                   ("  if (kScalDefer && args_ptr()->scal_defer && (it & (kScalBatches - 1)) != 0) {\n    // the wave's last window",
                    "  if (opaque(0) && (it & (kScalBatches - 1)) != 0) {\n    // the wave's last window")],
    # the frame samples from the address instead of HBM (is the frame load's latency exposed?)
    "no_frame_load": [("  if (NT || nt) {\n    if constexpr (!NT) asm volatile(\"; nt frame\");\n#pragma unroll\n    for (int c = 0; c < CH; ++c) xv[c] = __builtin_nontemporal_load(p + (c * 64 + lane));",
                       "  if (true) {\n#pragma unroll\n    for (int c = 0; c < CH; ++c) { const uint32_t a = (uint32_t)(uintptr_t)(p + (c * 64 + lane)); "
                       "xv[c] = (float)((a >> 2) & 1023) * 0x1p-10f - 0.5f; }")],
    # the per-lane twiddle loads of passes >= 1 made lane-uniform scalar loads
    "twuni": [("""__device__ __forceinline__ double2 ld_tw(GTw p, int i) {
  const GD q = (GD)p;""", """__device__ __forceinline__ double2 ld_tw(GTw p, int i) {
  return ld_tw_u(p, __builtin_amdgcn_readfirstlane(i));
  const GD q = (GD)p;""")],
    # the window table loads (16 per frame at N = 1024) replaced by a constant
    "no_window_load": [("    for (int c = 0; c < CH; ++c) wv[c] = w[c * 64 + lane];",
                        "    for (int c = 0; c < CH; ++c) wv[c] = 0.5f + 0.25f * (c & 1);")],
    # (not an ablation: the DPP wave sums instead of the LDS transpose for the moments at N = 1024)
    "mom_dpp": [("  static constexpr bool MOM_LDS = true;", "  static constexpr bool MOM_LDS = N <= 512;")],
    # the amplitude as |re| + |im| (no f64 squares, no rsq/Heron step)
    "no_amp": [("        ar[r] = slot_amp_rsq(v[r].x, v[r].y, okr);\n        uint32_t b",
                "        ar[r] = fabsf(v[r].x) + fabsf(v[r].y); okr = true;\n        uint32_t b")],
    # the prefix row (stores, rolloff ballots) skipped: band sums read stale LDS
    "no_prefix": [("  const bool need_prefix = LIGHT ? false : SUB ? (bool)ap->need_prefix : true;",
                   "  const bool need_prefix = opaque(0);")],
    # MGX_FLAG_MFCC_REFERENCE (CHAIN kernels): the chains skipped (the occupancy / LDS-layout /
    # power-row cost alone)
    # (both branches: round 5's patch skipped only the paired form, so the unpaired chains ran in its place)
    "chain_none": [("        if (q->chain_pair) mel_chains<N, true>(q, opaque(lane), gbl(rows), recs, buf, true);\n"
                    "        else mel_chains<N, false>(q, opaque(lane), gbl(rows), recs, buf, true);",
                    "        if (opaque(0)) mel_chains<N, true>(q, opaque(lane), gbl(rows), recs, buf, true);")],
    # the power-row stores skipped (the chains read stale rows)
    "chain_norows": [("      for (int c = 0; c < R; ++c) {\n        const float a = amp[pa(c * 64 + lane)];",
                      "      for (int c = 0; opaque(0) && c < R; ++c) {\n        const float a = amp[pa(c * 64 + lane)];")],
    # the fence before the chains (a vmcnt(0) wait: the next frame's prefetch, the row stores) dropped
    "chain_nofence": [("""        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (q->chain_pair)""", """        if (q->chain_pair)""")],
    # the FFT passes after pass 0 skipped (the exchanges too): what the f64 butterflies cost
    "no_passes": [("      if (tame) run_passes<N, 1, FAITH, true, TWL>(v, lpf, buf, tw, twf, twm, twl);",
                   "      if (opaque(0)) run_passes<N, 1, FAITH, true, TWL>(v, lpf, buf, tw, twf, twm, twl);"),
                  ("      else run_passes<N, 1, FAITH, false, TWL>(v, lpf, buf, tw, twf, twm, twl);",
                   "      else if (opaque(0)) run_passes<N, 1, FAITH, false, TWL>(v, lpf, buf, tw, twf, twm, twl);")],
    # the whole FFT after stage 0 skipped
    "no_fft": [("      run_stages<N, 0, 0, FAITH, false, TWL>(v, lpf[0], tw, twf, twm, twl);",
                "      if (opaque(0)) run_stages<N, 0, 0, FAITH, false, TWL>(v, lpf[0], tw, twf, twm, twl);"),
               ("      if (tame) run_passes<N, 1, FAITH, true, TWL>(v, lpf, buf, tw, twf, twm, twl);",
                "      if (opaque(0)) run_passes<N, 1, FAITH, true, TWL>(v, lpf, buf, tw, twf, twm, twl);"),
               ("      else run_passes<N, 1, FAITH, false, TWL>(v, lpf, buf, tw, twf, twm, twl);",
                "      else if (opaque(0)) run_passes<N, 1, FAITH, false, TWL>(v, lpf, buf, tw, twf, twm, twl);"),
               # (the fast precision's f32 passes)
               ("      run_passes<N, 0, FAITH, false, TWL>(v, lpf, buf, tw, twf, twm, twl);",
                "      if (opaque(0)) run_passes<N, 0, FAITH, false, TWL>(v, lpf, buf, tw, twf, twm, twl);")],
    # two workgroup barriers per frame at the mel step (the cost of synchronising the workgroup's
    # four waves once per frame; timing only, the batch size must give every wave the same count)
    "bar2": [("  MGX_MARK(bands_done);\n", "  MGX_MARK(bands_done);\n  if (!CHAIN) { lds_barrier(); lds_barrier(); }\n")],
    # (CHAIN) the frames loaded like the default kernel's (plain loads instead of non-temporal ones)
    "chain_plainload": [("  if (NT || nt) {", "  if (nt) {")],
    # (CHAIN with paired batches) the pair's first batch's log and DCT skipped too (no_ln / no_dct skip the second's)
    "chain_nomfcc2": [("        if (CHAIN && q->chain_pair) mfcc_log<CHAIN, SUB>(q, l2, recs, 32);  // the pair's first batch",
                       "        if (opaque(0) && CHAIN && q->chain_pair) mfcc_log<CHAIN, SUB>(q, l2, recs, 32);"),
                      ("        if (CHAIN && q->chain_pair) mfcc_dct<CHAIN, SUB>(q, l2, recs, dct_lds, 32, f0 - wstride * FPW);",
                       "        if (opaque(0) && CHAIN && q->chain_pair) mfcc_dct<CHAIN, SUB>(q, l2, recs, dct_lds, 32, f0 - wstride * FPW);")],
    # (CHAIN) the chain weights as constants instead of loads (is the chains' cost the weights' load latency?)
    "chain_wconst": [("    for (int u = 0; u < 8; ++u) w[u] = wp[g * 8 + u];\n    const uint32_t cnn",
                      "    for (int u = 0; u < 8; ++u) w[u] = 0.125 * (u + 1 + (g & 1));\n    const uint32_t cnn")],
    # (CHAIN) ... and the power rows as constants too (the chains' arithmetic alone)
    "chain_rconst": [("    const f32x4 n0 = kAhead ? prn[0] : p0, n1 = kAhead ? prn[1] : p1;",
                      "    const f32x4 n0 = p0 * 0.5f + 1.0f, n1 = p1 * 0.5f + 1.0f;")],
    "no_mel": [("  } else if (!CHAIN && ap->need_mfcc) {\n    mel_energies", "  } else if (opaque(0) && !CHAIN && ap->need_mfcc) {\n    mel_energies")],
}


def build(name, flags=()):
    src = open(os.path.join(SRC, "kernels.hip")).read()
    # "a+b": the patches of a, then those of b (cumulative ablations)
    for old, new in [pt for part in name.split("+") for pt in PATCHES[part]]:
        if src.count(old) != 1:
            raise SystemExit("%s: anchor found %d times: %r" % (name, src.count(old), old[:60]))
        src = src.replace(old, new)
    os.makedirs(os.path.join(ROOT, "abl"), exist_ok=True)
    # the patched copy lives beside its library, outside the product source directory
    tmp = tempfile.NamedTemporaryFile("w", suffix=".hip", dir=os.path.join(ROOT, "abl"), prefix=".abl_", delete=False)
    tmp.write(src)
    tmp.close()
    out = os.path.join(ROOT, "abl", "libabl_%s.so" % name.replace("+", "_"))
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
           "-mllvm", "-disable-machine-licm", "-I", SRC, *flags, "-shared", "-o", out, "-x", "hip", tmp.name,
           os.path.join(SRC, "plan.cpp"), os.path.join(SRC, "group.cpp"), "-ldl"]
    return subprocess.Popen(cmd), tmp.name, out


def main():
    names = sys.argv[1:] or ["all"]
    if names == ["all"]:
        names = list(PATCHES)
    jobs = [build(n) for n in names]
    rc = 0
    try:
        for p, tmp, out in jobs:
            rc |= p.wait()
            print(("built " if p.returncode == 0 else "FAILED ") + out)
    finally:
        for p, tmp, _ in jobs:
            if p.poll() is None:
                p.kill()
                p.wait()
            if os.path.exists(tmp):
                os.unlink(tmp)
    sys.exit(rc)


if __name__ == "__main__":
    main()
