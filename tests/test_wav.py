"""PCM/WAV ingest: header walk on the host (no GPU), device
decode and the PCM -> features path on the GPU, against decodeAudioData's scaling
and against the reference's own features for frames of audio/sound1.wav."""
import numpy as np
import pytest

import golden_io
import tolerance
import wavgen

FORMATS = ["u8", "s16", "s24", "s32", "f32"]


@pytest.fixture(scope="module")
def capi():
    from meyda_amd import capi
    capi.lib()
    return capi


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("variant", ["fmt16", "fmt18", "extensible", "extra_chunks"])
def test_parse_formats(capi, fmt, variant):
    rng = np.random.default_rng(1)
    codes = wavgen.random_codes(rng, 37, 2, fmt)
    kw = {"fmt16": {}, "fmt18": {"fmt_size": 18}, "extensible": {"extensible": True},
          "extra_chunks": {"extra_chunks": [(b"LIST", b"abc"), (b"junk", b"xy")]}}[variant]
    data = wavgen.wav_bytes(codes, fmt, rate=48000, **kw)
    info = capi.wav_parse(data)
    tag_bits = wavgen.TAGS[fmt][1]
    assert info["pcm_format"] == capi.PCM_FORMATS[fmt]
    assert (info["channels"], info["sample_rate"], info["bits_per_sample"]) == (2, 48000, tag_bits)
    assert info["block_align"] == 2 * tag_bits // 8
    assert info["sample_frames"] == 37
    assert data[info["data_offset"]:info["data_offset"] + info["data_bytes"]] == wavgen.encode(codes, fmt)


def test_parse_truncated_and_partial_frames(capi):
    codes = np.arange(20, dtype=np.int64).reshape(10, 2)
    data = wavgen.wav_bytes(codes, "s16", truncate=3)  # the last sample frame is cut
    info = capi.wav_parse(data)
    assert info["sample_frames"] == 9 and info["data_bytes"] == 36


@pytest.mark.parametrize("bad,match", [
    (b"RIFX\0\0\0\0WAVE", "not a RIFF"),
    (b"RIFF\4\0\0\0WAVE", "no fmt chunk"),
])
def test_parse_rejects(capi, bad, match):
    with pytest.raises(capi.MgxError, match=match):
        capi.wav_parse(bad)


def test_parse_rejects_encodings(capi):
    good = wavgen.wav_bytes(np.zeros((4, 1)), "s16")
    adpcm = bytearray(good)
    adpcm[20:22] = (2).to_bytes(2, "little")  # format tag 2 = MS ADPCM
    with pytest.raises(capi.MgxError, match="unsupported"):
        capi.wav_parse(bytes(adpcm))
    nodata = good[:good.index(b"data")]
    with pytest.raises(capi.MgxError, match="no data chunk"):
        capi.wav_parse(nodata)


def test_parse_matches_reference_wavs(capi):
    """The three reference recordings: the header values tools/gen_golden.js recorded."""
    import os
    m = golden_io.manifest()["wav"]
    base = "/root/reference/audio"
    if not os.path.isdir(base):
        pytest.skip("reference audio not present (GPU box)")
    for name, w in m.items():
        data = open(os.path.join(base, name + ".wav"), "rb").read()
        info = capi.wav_parse(data)
        assert info["sample_frames"] == w["samples"], name
        assert info["data_offset"] == w["dataOffset"], name
        assert (info["channels"], info["sample_rate"], info["bits_per_sample"]) == (
            w["fmt"]["channels"], w["fmt"]["rate"], w["fmt"]["bits"]), name


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", FORMATS)
def test_decode_device(capi, fmt):
    import torch
    rng = np.random.default_rng(7)
    codes = wavgen.random_codes(rng, 5000, 3, fmt)
    raw = np.frombuffer(wavgen.encode(codes, fmt), np.uint8)
    dev = torch.from_numpy(raw.copy()).cuda()
    for ch in range(3):
        out = torch.empty(5000, dtype=torch.float32, device="cuda")
        capi.pcm_decode_device(dev, 5000, fmt, 3, ch, out)
        want = wavgen.decode(codes[:, ch], fmt)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32)), (fmt, ch)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["s16", "f32", "s24"])
def test_extract_pcm_equals_extract_of_decoded(capi, fmt):
    rng = np.random.default_rng(3)
    n, channels = 512, 2
    codes = wavgen.random_codes(rng, n * 70 + 100, channels, fmt)  # 70 buffers + a partial one
    wav = wavgen.wav_bytes(codes, fmt)
    plan = capi.Plan(buffer_size=n, scalar_f64=True)
    feats = capi.ALL_FEATURES + ["amplitudeSpectrum"]
    got = plan.extract_wav(wav, feats, channel=1)
    frames = wavgen.decode(codes[:70 * n, 1], fmt).reshape(70, n)
    want = plan.extract(frames, feats)
    assert set(got) == set(want)
    for k in want:
        assert np.array_equal(np.asarray(got[k]), np.asarray(want[k]), equal_nan=True), k


@pytest.mark.gpu
def test_wav_of_reference_frames_matches_reference_features(capi):
    """Frames of sound1.wav (golden inputs are its int16 codes / 32768) re-encoded as a
    WAV file: WAV -> device decode -> features equals the reference's own features."""
    g = golden_io.load(512)
    idx = golden_io.idx(g["labels"], "sound1")
    codes = np.rint(g["input"][idx].astype(np.float64) * 32768).astype(np.int64)
    assert np.array_equal((codes / 32768).astype(np.float32), g["input"][idx])
    wav = wavgen.wav_bytes(codes.reshape(-1, 1), "s16")
    plan = capi.Plan(buffer_size=512, scalar_f64=True)
    out = plan.extract_wav(wav, capi.ALL_FEATURES + ["amplitudeSpectrum"])
    bad, _ = tolerance.check_spectra(out["amplitudeSpectrum"], g["amp"][idx])
    assert not bad
    assert not tolerance.check_vectors(out["mfcc"], g["mfcc"][idx])
    rms = out["rms"]
    assert np.allclose(rms, g["scalars"][idx, 0], rtol=1e-5, atol=0)


@pytest.mark.gpu
def test_extract_pcm_rejects_short_buffer_and_decodes_unaligned(capi):
    import torch
    n = 512
    rng = np.random.default_rng(5)
    codes = wavgen.random_codes(rng, 4 * n, 1, "s16")
    raw = wavgen.wav_bytes(codes, "s16")
    info = capi.wav_parse(raw)
    pcm = np.frombuffer(raw, np.uint8)[info["data_offset"]:info["data_offset"] + info["data_bytes"]]
    plan = capi.Plan(buffer_size=n)
    # claiming more sample frames than the buffer holds is refused before any copy
    with pytest.raises(capi.MgxError) as ei:
        plan.extract_pcm(pcm[:-2], 4 * n, "s16", 1, 0, ["rms"])
    assert ei.value.status == -1
    # device decode from an odd byte address (a caller's pointer need not be aligned)
    for fmt in ("s16", "s32", "f32"):
        c = wavgen.random_codes(rng, 777, 1, fmt)
        body = np.frombuffer(wavgen.wav_bytes(c, fmt), np.uint8)
        inf = capi.wav_parse(body.tobytes())
        data = body[inf["data_offset"]:inf["data_offset"] + inf["data_bytes"]]
        dev = torch.zeros(data.size + 1, dtype=torch.uint8, device="cuda")
        dev[1:] = torch.from_numpy(data.copy()).cuda()
        out = torch.empty(777, dtype=torch.float32, device="cuda")
        check = capi.lib().mgx_pcm_decode_device(dev.data_ptr() + 1, 777, capi.PCM_FORMATS[fmt], 1, 0,
                                                 out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        assert check == 0
        want = wavgen.decode(c[:, 0], fmt)
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32)), fmt
