"""Host-side arithmetic of the multi-device groups (include/meyda_gpu.h "Multi-device
groups"; no GPU): the shard and chunk ranges (mgx_shard_range) and the packed transfer
layout (mgx_packed_layout), and a replay of the chunked gather built on them — every
rank's shard extracted by the CPU oracle, packed chunk by chunk, unpacked at the root
exactly as group.cpp does — against one extraction of the whole batch. Frame
independence (src/meyda.js:69-91) is what makes the sharding legal."""
import numpy as np
import pytest

SEED = 0x6D657964


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    capi.lib()
    return capi


def test_shard_range_matches_python_and_covers(capi):
    from meyda_amd.dist import shard_range
    for total in (0, 1, 5, 7, 64, 262144, 2097152 + 3):
        for n in (1, 2, 3, 7, 8):
            spans = [capi.shard_range(total, n, r) for r in range(n)]
            assert spans == [shard_range(total, n, r) for r in range(n)]
            assert spans[0][0] == 0 and sum(c for _, c in spans) == total
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
    with pytest.raises(capi.MgxError):
        capi.shard_range(10, 2, 2)


@pytest.mark.parametrize("n", [512, 1024, 2048])
def test_packed_layout(capi, n):
    d = capi.make_desc(buffer_size=n, num_mel_bands=40, num_mfcc_coeffs=20, scalar_f64=True)
    full = (1 << 18) - 1
    for frames in (1, 7, 32768):
        total, off = capi.packed_layout(d, full, frames)
        assert list(off) == capi.FIELDS
        width = {**{k: 8 for k in capi.SCALAR_NAMES}, "loudness.specific": 96, "mfcc": 80,
                 "amplitudeSpectrum": 2 * n, "powerSpectrum": 2 * n,
                 "complexSpectrum.real": 4 * n, "complexSpectrum.imag": 4 * n}
        at = 0
        for k in capi.FIELDS:
            assert off[k] == at and off[k] % 256 == 0
            at += -(-width[k] * frames // 256) * 256
        assert total == at
    # a mask selects fields; complex (bit 17) brings both arrays
    total, off = capi.packed_layout(d, (1 << 3) | capi.OUT_COMPLEX, 10)
    assert list(off) == ["spectralCentroid", "complexSpectrum.real", "complexSpectrum.imag"]
    assert capi.output_mask(capi.Outputs()) == 0


def replay_gather(capi, oracle, counts, nch, n):
    """group.cpp's chunk loop with the oracle as each rank's extractor: the root's own
    shard lands in place; every other rank's chunk crosses as one packed buffer."""
    d = capi.make_desc(buffer_size=n, scalar_f64=True)
    mask = (1 << 13) - 1 | capi.OUT_LOUDNESS_SPECIFIC | capi.OUT_MFCC | capi.OUT_AMPLITUDE
    total = sum(counts)
    start = np.concatenate([[0], np.cumsum(counts)[:-1]]).astype(int)
    root = {k: np.full((total,) + shp, np.nan, dt) for k, shp, dt in
            [("scalars", (13,), np.float64), ("loudness.specific", (24,), np.float32),
             ("mfcc", (13,), np.float32), ("amplitudeSpectrum", (n // 2,), np.float32)]}
    for r, cnt in enumerate(counts):
        x = oracle.synth_frames(SEED, int(start[r]), cnt, n) if cnt else np.zeros((0, n), np.float32)
        ref = oracle.extract(x) if cnt else None
        for c in range(nch):
            c0, cn = capi.shard_range(cnt, nch, c)
            if not cn:
                continue
            sl = slice(c0, c0 + cn)
            dst = slice(start[r] + c0, start[r] + c0 + cn)
            if r == 0:  # the root writes its own shard in place
                root["scalars"][dst] = ref["scalars"][sl]
                root["loudness.specific"][dst] = ref["loudness_specific"][sl]
                root["mfcc"][dst] = ref["mfcc"][sl]
                root["amplitudeSpectrum"][dst] = ref["amp"][sl]
                continue
            nbytes, off = capi.packed_layout(d, mask, cn)
            buf = np.zeros(nbytes, np.uint8)  # the transfer buffer of this chunk
            for j, k in enumerate(capi.SCALAR_NAMES):
                buf[off[k]:off[k] + 8 * cn] = ref["scalars"][sl, j].astype(np.float64).view(np.uint8)
            for k, src in (("loudness.specific", ref["loudness_specific"]), ("mfcc", ref["mfcc"]),
                           ("amplitudeSpectrum", ref["amp"])):
                b = np.ascontiguousarray(src[sl]).view(np.uint8).ravel()
                buf[off[k]:off[k] + b.size] = b
            # root: unpack (unpack_kernel's segments)
            for j, k in enumerate(capi.SCALAR_NAMES):
                root["scalars"][dst, j] = buf[off[k]:off[k] + 8 * cn].view(np.float64)
            for k in ("loudness.specific", "mfcc", "amplitudeSpectrum"):
                w = root[k].shape[1]
                root[k][dst] = buf[off[k]:off[k] + 4 * w * cn].view(np.float32).reshape(cn, w)
    return root


@pytest.mark.parametrize("counts,nch", [([40], 3), ([20, 20], 1), ([11, 10, 10], 4), ([3, 3, 2, 2, 2, 2, 2, 2], 8),
                                        ([5, 0, 4], 2)])
def test_chunked_gather_replay_equals_whole_batch(capi, oracle_mod, counts, nch):
    n = 512
    got = replay_gather(capi, oracle_mod, counts, nch, n)
    whole = oracle_mod.extract(oracle_mod.synth_frames(SEED, 0, sum(counts), n))
    assert np.array_equal(got["scalars"], whole["scalars"], equal_nan=True)
    assert np.array_equal(got["loudness.specific"], whole["loudness_specific"])
    assert np.array_equal(got["mfcc"], whole["mfcc"])
    assert np.array_equal(got["amplitudeSpectrum"], whole["amp"])
