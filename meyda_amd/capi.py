"""ctypes binding of the C ABI in include/meyda_gpu.h (libmeyda_gpu.so, built in-tree).

This is plumbing for the Python test suite and bench.py; the product host binding
for the reference's JavaScript API is the N-API addon (meyda_amd/addon/) used by
meyda_amd/js/meyda.js. There is no CPU fallback here: if the HIP library is
missing or no gfx950 device is present, every compute call raises.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MEYDA_AMD_LIB") or os.path.join(HERE, "libmeyda_gpu.so")

NUM_SCALARS = 13
NUM_BARK = 24
SCALAR_NAMES = ["rms", "energy", "zcr", "spectralCentroid", "spectralFlatness", "spectralSlope",
                "spectralRolloff", "spectralSpread", "spectralSkewness", "spectralKurtosis",
                "loudness.total", "perceptualSpread", "perceptualSharpness"]
FEATURE_NAMES = SCALAR_NAMES + ["loudness", "mfcc", "amplitudeSpectrum", "powerSpectrum",
                                "complexSpectrum", "buffer"]
WINDOWS = {"hanning": 0, "hamming": 1}
PRECISIONS = {"faithful": 0, "fast": 1}
MODES = {"per_buffer_fft": 0, "literal": 1}

STATUS = {0: "MGX_OK", -1: "MGX_E_INVALID_ARGUMENT", -2: "MGX_E_NOT_POWER_OF_TWO",
          -3: "MGX_E_UNSUPPORTED", -4: "MGX_E_DEVICE", -5: "MGX_E_OUT_OF_MEMORY",
          -6: "MGX_E_NO_DEVICE"}

# Every symbol include/meyda_gpu.h declares (checked by tests/test_capi_host.py).
EXPORTS = ["mgx_plan_desc_init", "mgx_plan_create", "mgx_plan_destroy", "mgx_plan_get_desc",
           "mgx_extract_device", "mgx_extract_host", "mgx_synth_frames_device",
           "mgx_get_host_tables", "mgx_is_power_of_two", "mgx_feature_index", "mgx_feature_name",
           "mgx_feature_info", "mgx_device_count", "mgx_abi_version", "mgx_last_error",
           "mgx_wav_parse", "mgx_pcm_decode_device", "mgx_extract_host_pcm",
           "mgx_shard_range", "mgx_packed_layout", "mgx_comm_unique_id", "mgx_group_create",
           "mgx_group_create_rank", "mgx_group_create_loopback", "mgx_group_create_loopback_rccl", "mgx_group_destroy",
           "mgx_group_info", "mgx_group_comm_info", "mgx_group_extract_device", "mgx_group_extract_host"]
COMM_ID_BYTES = 128
FLAG_DCT_SEQUENTIAL = 1  # mgx_plan_desc.flags
FLAG_MFCC_REFERENCE = 2  # mel sums, log and DCT in the reference's own order
FLAG_RESIDENT = 4  # one-frame host calls served by a workgroup that stays on the device (include/meyda_gpu.h)
# output selection bits of a group extraction (MGX_OUT_* in include/meyda_gpu.h)
OUT_LOUDNESS_SPECIFIC, OUT_MFCC, OUT_AMPLITUDE, OUT_POWER, OUT_COMPLEX = (1 << 13, 1 << 14, 1 << 15, 1 << 16,
                                                                          1 << 17)
# field order of mgx_packed_layout / mgx_outputs
FIELDS = SCALAR_NAMES + ["loudness.specific", "mfcc", "amplitudeSpectrum", "powerSpectrum",
                         "complexSpectrum.real", "complexSpectrum.imag"]
PCM_FORMATS = {"f32": 0, "s16": 1, "u8": 2, "s24": 3, "s32": 4}


class MgxError(RuntimeError):
    def __init__(self, status, message):
        super().__init__("%s (%d): %s" % (STATUS.get(status, "?"), status, message))
        self.status = status


class PlanDesc(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("buffer_size", ctypes.c_uint32),
                ("sample_rate", ctypes.c_double), ("window", ctypes.c_uint32),
                ("precision", ctypes.c_uint32), ("mode", ctypes.c_uint32),
                ("num_bark_bands", ctypes.c_uint32), ("num_mel_bands", ctypes.c_uint32),
                ("num_mfcc_coeffs", ctypes.c_uint32), ("scalar_f64", ctypes.c_uint32),
                ("device", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class Outputs(ctypes.Structure):
    _fields_ = [("scalars", ctypes.c_void_p * NUM_SCALARS),
                ("loudness_specific", ctypes.c_void_p), ("mfcc", ctypes.c_void_p),
                ("amplitude_spectrum", ctypes.c_void_p), ("power_spectrum", ctypes.c_void_p),
                ("complex_real", ctypes.c_void_p), ("complex_imag", ctypes.c_void_p)]


class HostTables(ctypes.Structure):
    _fields_ = [("window", ctypes.c_void_p), ("hanning", ctypes.c_void_p),
                ("hamming", ctypes.c_void_p), ("bark_scale", ctypes.c_void_p),
                ("bark_limits", ctypes.c_void_p), ("mel_bins", ctypes.c_void_p),
                ("dct", ctypes.c_void_p)]


class WavInfo(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("pcm_format", ctypes.c_uint32),
                ("channels", ctypes.c_uint32), ("sample_rate", ctypes.c_uint32),
                ("bits_per_sample", ctypes.c_uint32), ("block_align", ctypes.c_uint32),
                ("data_offset", ctypes.c_uint64), ("data_bytes", ctypes.c_uint64),
                ("sample_frames", ctypes.c_uint64)]


_lib = None


def lib():
    """Load libmeyda_gpu.so (fails loudly if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError("libmeyda_gpu.so not built (run `make` or __graft_entry__.build())")
        # torch ships its own libamdhip64 (SONAME libamdhip64.so.7). Load it first so
        # the loader resolves our DT_NEEDED libamdhip64.so.7 to that same runtime:
        # two HIP runtimes in one process leave the second without devices.
        try:
            import torch  # noqa: F401
            # multi-device groups load RCCL at run time: in a torch process use torch's own
            # librccl (built against the HIP runtime this process runs on)
            trccl = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
            if "MGX_RCCL_LIB" not in os.environ and os.path.exists(trccl):
                os.environ["MGX_RCCL_LIB"] = trccl
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.mgx_plan_desc_init.argtypes = [ctypes.POINTER(PlanDesc)]
        L.mgx_plan_desc_init.restype = None
        L.mgx_plan_create.argtypes = [ctypes.POINTER(PlanDesc), ctypes.POINTER(ctypes.c_void_p)]
        L.mgx_plan_destroy.argtypes = [ctypes.c_void_p]
        L.mgx_plan_get_desc.argtypes = [ctypes.c_void_p, ctypes.POINTER(PlanDesc)]
        L.mgx_extract_device.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.POINTER(Outputs), ctypes.c_void_p]
        L.mgx_extract_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                       ctypes.POINTER(Outputs)]
        L.mgx_synth_frames_device.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                              ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        L.mgx_get_host_tables.argtypes = [ctypes.POINTER(PlanDesc), ctypes.POINTER(HostTables)]
        L.mgx_is_power_of_two.argtypes = [ctypes.c_double]
        L.mgx_feature_index.argtypes = [ctypes.c_char_p]
        L.mgx_feature_name.argtypes = [ctypes.c_int]
        L.mgx_feature_name.restype = ctypes.c_char_p
        L.mgx_feature_info.argtypes = [ctypes.c_int]
        L.mgx_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
        L.mgx_last_error.restype = ctypes.c_char_p
        L.mgx_wav_parse.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.POINTER(WavInfo)]
        L.mgx_pcm_decode_device.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.mgx_extract_host_pcm.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(Outputs)]
        u64p = ctypes.POINTER(ctypes.c_uint64)
        L.mgx_shard_range.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, u64p, u64p]
        L.mgx_packed_layout.argtypes = [ctypes.POINTER(PlanDesc), ctypes.c_uint32, ctypes.c_uint64, u64p]
        L.mgx_packed_layout.restype = ctypes.c_uint64
        L.mgx_comm_unique_id.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.mgx_group_create.argtypes = [ctypes.POINTER(PlanDesc), ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32,
                                       ctypes.POINTER(ctypes.c_void_p)]
        L.mgx_group_create_rank.argtypes = [ctypes.POINTER(PlanDesc), ctypes.c_void_p, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]
        L.mgx_group_create_loopback.argtypes = [ctypes.POINTER(PlanDesc), ctypes.c_uint32,
                                                ctypes.POINTER(ctypes.c_void_p)]
        L.mgx_group_create_loopback_rccl.argtypes = [ctypes.POINTER(PlanDesc), ctypes.c_uint32,
                                                     ctypes.POINTER(ctypes.c_void_p)]
        L.mgx_group_destroy.argtypes = [ctypes.c_void_p]
        i32p = ctypes.POINTER(ctypes.c_int32)
        L.mgx_group_comm_info.argtypes = [ctypes.c_void_p, i32p, i32p, i32p]
        L.mgx_group_info.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32),
                                     ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
        L.mgx_group_extract_device.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), u64p,
                                               ctypes.POINTER(Outputs), ctypes.c_uint32, ctypes.c_uint32,
                                               ctypes.POINTER(ctypes.c_void_p)]
        L.mgx_group_extract_host.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                             ctypes.POINTER(Outputs)]
        _lib = L
    return _lib


def check(rc):
    if rc != 0:
        raise MgxError(rc, lib().mgx_last_error().decode())
    return rc


def make_desc(buffer_size=512, sample_rate=44100.0, window="hanning", precision="faithful",
              mode="per_buffer_fft", num_mel_bands=26, num_mfcc_coeffs=13, scalar_f64=False,
              device=0, dct_sequential=False, mfcc_reference=False, resident=False):
    d = PlanDesc()
    lib().mgx_plan_desc_init(ctypes.byref(d))
    d.buffer_size = buffer_size
    d.sample_rate = sample_rate
    d.window = WINDOWS[window]
    d.precision = PRECISIONS[precision]
    d.mode = MODES[mode]
    d.num_mel_bands = num_mel_bands
    d.num_mfcc_coeffs = num_mfcc_coeffs
    d.scalar_f64 = 1 if scalar_f64 else 0
    d.device = device
    d.flags = ((FLAG_DCT_SEQUENTIAL if dct_sequential else 0) | (FLAG_MFCC_REFERENCE if mfcc_reference else 0) |
               (FLAG_RESIDENT if resident else 0))
    return d


def host_tables(**kw):
    """Host tables (window, bark, limits, mel bins, dct) computed by the library: no GPU."""
    d = make_desc(**kw)
    n, nf, nc = d.buffer_size, d.num_mel_bands, d.num_mfcc_coeffs
    t = {"window": np.empty(n, np.float32), "hanning": np.empty(n, np.float32),
         "hamming": np.empty(n, np.float32), "bark_scale": np.empty(n, np.float32),
         "bark_limits": np.empty(NUM_BARK + 1, np.int32), "mel_bins": np.empty(nf + 2, np.int32),
         "dct": np.empty(nc * nf, np.float32)}
    ht = HostTables(*[t[k].ctypes.data for k in ("window", "hanning", "hamming", "bark_scale",
                                                  "bark_limits", "mel_bins", "dct")])
    check(lib().mgx_get_host_tables(ctypes.byref(d), ctypes.byref(ht)))
    return t


def device_count():
    c = ctypes.c_int(0)
    check(lib().mgx_device_count(ctypes.byref(c)))
    return c.value


class Plan:
    """One extraction plan (mirrors `new Meyda(ctx, src, bufferSize)`, src/meyda.js:17-97)."""

    def __init__(self, buffer_size=512, **kw):
        self.desc = make_desc(buffer_size=buffer_size, **kw)
        h = ctypes.c_void_p()
        check(lib().mgx_plan_create(ctypes.byref(self.desc), ctypes.byref(h)))
        self._h = h
        self.n = buffer_size
        self.scalar_dtype = np.float64 if kw.get("scalar_f64") else np.float32

    def close(self):
        if getattr(self, "_h", None):
            lib().mgx_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------- device (torch)
    def alloc_outputs(self, num_frames, features, device="cuda"):
        """Allocate torch device tensors for the requested features; returns (dict, Outputs)."""
        import torch
        st = torch.float64 if self.scalar_dtype == np.float64 else torch.float32
        L = self.n // 2
        out, o = {}, Outputs()
        for f in features:
            if f in SCALAR_NAMES:
                out[f] = torch.empty(num_frames, dtype=st, device=device)
                o.scalars[SCALAR_NAMES.index(f)] = out[f].data_ptr()
            elif f == "loudness":
                out["loudness.specific"] = torch.empty(num_frames, NUM_BARK, dtype=torch.float32, device=device)
                o.loudness_specific = out["loudness.specific"].data_ptr()
                out["loudness.total"] = torch.empty(num_frames, dtype=st, device=device)
                o.scalars[10] = out["loudness.total"].data_ptr()
            elif f == "mfcc":
                out[f] = torch.empty(num_frames, self.desc.num_mfcc_coeffs, dtype=torch.float32, device=device)
                o.mfcc = out[f].data_ptr()
            elif f == "amplitudeSpectrum":
                out[f] = torch.empty(num_frames, L, dtype=torch.float32, device=device)
                o.amplitude_spectrum = out[f].data_ptr()
            elif f == "powerSpectrum":
                out[f] = torch.empty(num_frames, L, dtype=torch.float32, device=device)
                o.power_spectrum = out[f].data_ptr()
            elif f == "complexSpectrum":
                out["complexSpectrum.real"] = torch.empty(num_frames, self.n, dtype=torch.float32, device=device)
                out["complexSpectrum.imag"] = torch.empty(num_frames, self.n, dtype=torch.float32, device=device)
                o.complex_real = out["complexSpectrum.real"].data_ptr()
                o.complex_imag = out["complexSpectrum.imag"].data_ptr()
            else:
                raise ValueError("unknown feature %r" % f)
        return out, o

    def extract_device(self, frames_ptr, num_frames, outputs, stream=None):
        """Launch on device pointers (async on `stream`, an int hipStream_t handle or None)."""
        check(lib().mgx_extract_device(self._h, ctypes.c_void_p(frames_ptr), num_frames,
                                       ctypes.byref(outputs), ctypes.c_void_p(stream or 0)))

    def extract_torch(self, frames, features, stream=None):
        """frames: a (F, N) float32 CUDA tensor. Returns a dict of device tensors."""
        import torch
        assert frames.is_cuda and frames.dtype == torch.float32 and frames.is_contiguous()
        assert frames.dim() == 2 and frames.shape[1] == self.n
        out, o = self.alloc_outputs(frames.shape[0], features, device=frames.device)
        if stream is None:
            stream = torch.cuda.current_stream(frames.device).cuda_stream
        self.extract_device(frames.data_ptr(), frames.shape[0], o, stream)
        return out

    # ------------------------------------------------------------------ host
    def extract(self, frames, features):
        """Host numpy in / numpy out (stages through the device)."""
        frames = np.ascontiguousarray(frames, dtype=np.float32)
        F, n = frames.shape
        assert n == self.n
        out, o = self._host_outputs(F, features)
        check(lib().mgx_extract_host(self._h, frames.ctypes.data, F, ctypes.byref(o)))
        return out

    def extract_pcm(self, pcm, sample_frames, fmt, channels, channel=0, features=()):
        """Raw interleaved PCM (bytes / numpy buffer) in host memory -> features of the
        floor(sample_frames / N) buffers of `channel` (decoded on the device)."""
        buf = np.frombuffer(pcm, dtype=np.uint8) if not isinstance(pcm, np.ndarray) else pcm.view(np.uint8)
        buf = np.ascontiguousarray(buf)
        fmt = PCM_FORMATS[fmt] if isinstance(fmt, str) else fmt
        F = sample_frames // self.n
        out, o = self._host_outputs(F, features)
        check(lib().mgx_extract_host_pcm(self._h, buf.ctypes.data, buf.size, sample_frames, fmt, channels, channel,
                                         ctypes.byref(o)))
        return out

    def extract_wav(self, wav_bytes, features, channel=0):
        """A whole .wav file (bytes) -> features of its full buffers (channel `channel`)."""
        info = wav_parse(wav_bytes)
        data = np.frombuffer(wav_bytes, dtype=np.uint8)[info["data_offset"]:info["data_offset"] + info["data_bytes"]]
        return self.extract_pcm(data, info["sample_frames"], info["pcm_format"], info["channels"], channel, features)

    def _host_outputs(self, F, features):
        n = self.n
        L = n // 2
        out, o = {}, Outputs()
        sd = self.scalar_dtype
        for f in features:
            if f in SCALAR_NAMES:
                out[f] = np.empty(F, sd)
                o.scalars[SCALAR_NAMES.index(f)] = out[f].ctypes.data
            elif f == "loudness":
                out["loudness.specific"] = np.empty((F, NUM_BARK), np.float32)
                out["loudness.total"] = np.empty(F, sd)
                o.loudness_specific = out["loudness.specific"].ctypes.data
                o.scalars[10] = out["loudness.total"].ctypes.data
            elif f == "mfcc":
                out[f] = np.empty((F, self.desc.num_mfcc_coeffs), np.float32)
                o.mfcc = out[f].ctypes.data
            elif f == "amplitudeSpectrum":
                out[f] = np.empty((F, L), np.float32)
                o.amplitude_spectrum = out[f].ctypes.data
            elif f == "powerSpectrum":
                out[f] = np.empty((F, L), np.float32)
                o.power_spectrum = out[f].ctypes.data
            elif f == "complexSpectrum":
                out["complexSpectrum.real"] = np.empty((F, n), np.float32)
                out["complexSpectrum.imag"] = np.empty((F, n), np.float32)
                o.complex_real = out["complexSpectrum.real"].ctypes.data
                o.complex_imag = out["complexSpectrum.imag"].ctypes.data
            else:
                raise ValueError("unknown feature %r" % f)
        return out, o


ALL_FEATURES = SCALAR_NAMES[:10] + ["loudness", "perceptualSpread", "perceptualSharpness", "mfcc"]


def shard_range(total, nranks, rank):
    """(start, count) of rank's contiguous shard (mgx_shard_range; host only)."""
    s, c = ctypes.c_uint64(), ctypes.c_uint64()
    check(lib().mgx_shard_range(total, nranks, rank, ctypes.byref(s), ctypes.byref(c)))
    return s.value, c.value


def output_mask(outputs):
    """MGX_OUT_* mask of the non-NULL fields of an Outputs structure."""
    m = 0
    for i in range(NUM_SCALARS):
        if outputs.scalars[i]:
            m |= 1 << i
    for bit, f in ((13, "loudness_specific"), (14, "mfcc"), (15, "amplitude_spectrum"),
                   (16, "power_spectrum"), (17, "complex_real")):
        if getattr(outputs, f):
            m |= 1 << bit
    return m


def packed_layout(desc, mask, num_frames):
    """(total_bytes, {field: offset}) of mgx_packed_layout (host only)."""
    off = (ctypes.c_uint64 * 19)()
    total = lib().mgx_packed_layout(ctypes.byref(desc), mask, num_frames, off)
    return total, {FIELDS[i]: off[i] for i in range(19) if off[i] != 2 ** 64 - 1}


def comm_unique_id():
    buf = ctypes.create_string_buffer(COMM_ID_BYTES)
    check(lib().mgx_comm_unique_id(buf, COMM_ID_BYTES))
    return buf.raw


class Group:
    """Frames sharded over several devices with an RCCL gather of the feature records to the
    root (rank 0) — include/meyda_gpu.h "Multi-device groups".

    Group(devices=[0, 1, ...], **plan_kw)                 one process, several devices
    Group(rank=r, nranks=n, unique_id=b, device=d, ...)   one process per device (torchrun)
    Group(loopback=n, device=d, ...)                      test transport: n ranks on one device,
                                                          chunks as device copies
    Group(loopback=n, transport="rccl", device=d, ...)    the same, chunks as RCCL send/recv to
                                                          self on a one-rank communicator
    """

    def __init__(self, buffer_size=512, devices=None, rank=None, nranks=None, unique_id=None, loopback=None,
                 transport="copy", **kw):
        h = ctypes.c_void_p()
        if loopback is not None:
            self.desc = make_desc(buffer_size=buffer_size, **kw)
            create = {"copy": lib().mgx_group_create_loopback, "rccl": lib().mgx_group_create_loopback_rccl}[transport]
            check(create(ctypes.byref(self.desc), loopback, ctypes.byref(h)))
        elif devices is not None:
            self.desc = make_desc(buffer_size=buffer_size, device=devices[0], **kw)
            arr = (ctypes.c_int32 * len(devices))(*devices)
            check(lib().mgx_group_create(ctypes.byref(self.desc), arr, len(devices), ctypes.byref(h)))
        else:
            self.desc = make_desc(buffer_size=buffer_size, **kw)
            check(lib().mgx_group_create_rank(ctypes.byref(self.desc), unique_id, nranks, rank, ctypes.byref(h)))
        self._h = h
        self.n = buffer_size
        self.scalar_dtype = np.float64 if kw.get("scalar_f64") else np.float32
        nr, first, nl = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        check(lib().mgx_group_info(h, ctypes.byref(nr), ctypes.byref(first), ctypes.byref(nl)))
        self.nranks, self.first_local, self.num_local = nr.value, first.value, nl.value

    def comm_info(self):
        """(ranks, rank, device) as this process's RCCL communicator reports them, or
        (-1, -1, -1) without one (mgx_group_comm_info)."""
        n, r, d = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        check(lib().mgx_group_comm_info(self._h, ctypes.byref(n), ctypes.byref(r), ctypes.byref(d)))
        return n.value, r.value, d.value

    def close(self):
        if getattr(self, "_h", None):
            lib().mgx_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def extract_device(self, frames_ptrs, counts, root_outputs, mask, num_chunks=0, streams=None):
        """frames_ptrs: device pointers of the local ranks' shards; counts: frames of every
        rank; root_outputs: an Outputs of device pointers on the root (None elsewhere)."""
        fp = (ctypes.c_void_p * len(frames_ptrs))(*frames_ptrs)
        cn = (ctypes.c_uint64 * len(counts))(*counts)
        st = None if streams is None else (ctypes.c_void_p * len(streams))(*streams)
        check(lib().mgx_group_extract_device(self._h, fp, cn, None if root_outputs is None else ctypes.byref(root_outputs),
                                             mask, num_chunks, st))

    def extract(self, frames, features):
        """Host numpy in / numpy out, sharded over the group's devices (single process)."""
        frames = np.ascontiguousarray(frames, dtype=np.float32)
        F, n = frames.shape
        assert n == self.n
        out, o = Plan._host_outputs(self, F, features)
        check(lib().mgx_group_extract_host(self._h, frames.ctypes.data, F, ctypes.byref(o)))
        return out


def synth_frames_device(tensor, seed, first_frame=0, stream=None):
    """Fill a (F, N) float32 CUDA tensor with the synthetic PCM of SURVEY.md §8(d)."""
    import torch
    F, n = tensor.shape
    if stream is None:
        stream = torch.cuda.current_stream(tensor.device).cuda_stream
    check(lib().mgx_synth_frames_device(ctypes.c_void_p(tensor.data_ptr()), F, n, seed, first_frame,
                                        ctypes.c_void_p(stream)))


def wav_parse(data):
    """RIFF/WAVE header of `data` (bytes): format, channels, rate, data offset/size (no GPU)."""
    buf = np.frombuffer(data, dtype=np.uint8)
    info = WavInfo()
    info.struct_size = ctypes.sizeof(WavInfo)
    check(lib().mgx_wav_parse(buf.ctypes.data, buf.size, ctypes.byref(info)))
    return {k: getattr(info, k) for k, _ in WavInfo._fields_ if k != "struct_size"}


def pcm_decode_device(pcm_u8, sample_frames, fmt, channels, channel, out, stream=None):
    """Decode interleaved PCM (a uint8 CUDA tensor) into `out` (float32 CUDA tensor)."""
    import torch
    fmt = PCM_FORMATS[fmt] if isinstance(fmt, str) else fmt
    if stream is None:
        stream = torch.cuda.current_stream(out.device).cuda_stream
    check(lib().mgx_pcm_decode_device(ctypes.c_void_p(pcm_u8.data_ptr()), sample_frames, fmt, channels, channel,
                                      ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream)))
