"""audio-network_amd — MI355X-native acoustic-FSK demodulator (host mirror).

Thin ctypes mirror of the C ABI in include/demod.h (libfskdemod.so built
in-tree from audio-network_amd/csrc). Names, argument meaning and error
behaviour follow the C entry points one-for-one, which in turn mirror the
Opus-decoder-shaped API at the reference's PCM insertion point
(hardware/src/playback.cpp:67-74,115-122).

Every compute call runs the HIP kernels on a gfx950 GPU. There is no CPU
fallback: if libfskdemod.so is missing, :func:`load_library` raises, and if no
MI355X is visible, :class:`Demodulator` raises DemodError(DEMOD_NO_DEVICE).
The frame/packing helpers are host byte work and need no GPU.

Load this package by path (the directory name has a hyphen), e.g.
``importlib.util.spec_from_file_location("audio_network_amd", ".../__init__.py")``.
"""
from __future__ import annotations

import ctypes
import os
import re
from typing import Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfskdemod.so")
# FSKD_LIB: another build of the same ABI (measurement A/B of two builds in
# one GPU call, scripts/gpu_run.sh); the product default is the in-tree build
_LIB_ENV = os.environ.get("FSKD_LIB")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "demod.h")

DEMOD_OK = 0
DEMOD_BAD_ARG = -1
DEMOD_BUFFER_TOO_SMALL = -2
DEMOD_INTERNAL_ERROR = -3
DEMOD_INVALID_PACKET = -4
DEMOD_UNIMPLEMENTED = -5
DEMOD_INVALID_STATE = -6
DEMOD_ALLOC_FAIL = -7
DEMOD_DEVICE_ERROR = -8
DEMOD_NO_DEVICE = -9
DEMOD_FRAME_TOO_LARGE = -10

DEMOD_MAX_TONES = 16
DEMOD_OPUS_LOOKAHEAD = 312  # Opus decoder delay at 48 kHz (OpusEncoder.kt:65-67)
DEMOD_MAX_FRAME_PAYLOAD = 4096

CH_LEFT, CH_RIGHT, CH_DOWNMIX = 0, 1, 2
METHOD_AUTO, METHOD_GOERTZEL, METHOD_FFT, METHOD_FOLDED, METHOD_RESIDUE = 0, 1, 2, 3, 4

FSK2_FREQS = (1500.0, 3000.0)                              # SURVEY §8 tone plan
FSK8_FREQS = tuple(1500.0 + 375.0 * i for i in range(8))
BENCH_SEED = 0x2C5DA044


class DemodCfg(ctypes.Structure):
    """Mirror of ``demod_cfg_t`` (include/demod.h)."""
    _fields_ = [
        ("fs", ctypes.c_double),
        ("n", ctypes.c_uint32),
        ("hop", ctypes.c_uint32),
        ("k", ctypes.c_uint32),
        ("channels", ctypes.c_uint32),
        ("channel_mode", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("method", ctypes.c_int32),
        ("lead_in", ctypes.c_uint32),
        ("freqs", ctypes.c_double * DEMOD_MAX_TONES),
    ]


DEMOD_PORT_AUDIO_RX = 58764
DEMOD_PORT_DISCOVERY = 58765
DEMOD_BROADCAST_MAGIC = 0x2C5DA044
DEMOD_INFO_STRING_CAP = 128
DEMOD_MAX_DECODED_FRAME = 11520
DEMOD_MSG_NONE = 0
DEMOD_MSG_DISCOVERY_REQUEST = 2
DEMOD_MSG_DISCOVERY_RESPONSE = 3
DEMOD_MSG_RECEIVER_INFORMATION = 1
DEMOD_MSG_RECEIVER_ERROR = 2


class DemodDiscovery(ctypes.Structure):
    """demod_discovery_t (include/demod.h) = DiscoveryResponse, ip.pb.h:17-24."""
    _fields_ = [
        ("protocol_version", ctypes.c_uint32),
        ("mac_address", ctypes.c_uint64),
        ("device_name", ctypes.c_char * DEMOD_INFO_STRING_CAP),
        ("currently_streaming", ctypes.c_int),
        ("opus_version", ctypes.c_char * DEMOD_INFO_STRING_CAP),
    ]


class DemodReceiverInfo(ctypes.Structure):
    """demod_receiver_info_t = ReceiverInformation, ip.pb.h:55-59."""
    _fields_ = [
        ("discovery_data", DemodDiscovery),
        ("max_encoded_frame_size", ctypes.c_uint32),
        ("max_decoded_frame_size", ctypes.c_uint32),
    ]


class DemodReceiverError(ctypes.Structure):
    """demod_receiver_error_t = ReceiverError, ip.pb.h:26-31."""
    _fields_ = [("audio_underflow", ctypes.c_int), ("audio_decode_error", ctypes.c_int)]


class DemodErrorModel(ctypes.Structure):
    """demod_error_model_t (include/demod.h): the decision rescue's derived bounds."""
    _fields_ = [("method", ctypes.c_int32), ("energy", ctypes.c_int32)] + [
        (f, ctypes.c_double) for f in ("rho_det", "rho_ref", "rho_first", "tau", "tau64", "t2e",
                                        "t2e64", "amb_d")]


class DemodPlanInfo(ctypes.Structure):
    """demod_plan_info_t (include/demod.h): a configuration's tone plan and constants."""
    _fields_ = [
        ("method", ctypes.c_int32), ("log2g", ctypes.c_int32), ("reinsch", ctypes.c_int32),
        ("f16", ctypes.c_int32), ("dcls", ctypes.c_int32), ("slide", ctypes.c_int32),
        ("perm", ctypes.c_uint64),
        ("slot_tone", ctypes.c_int32 * DEMOD_MAX_TONES),
        ("zcls", ctypes.c_int32 * DEMOD_MAX_TONES),
        ("fft_bins", ctypes.c_int32 * DEMOD_MAX_TONES),
        ("coef", ctypes.c_float * DEMOD_MAX_TONES),
        ("sgn", ctypes.c_float * DEMOD_MAX_TONES),
        ("rcoef", ctypes.c_double * DEMOD_MAX_TONES),
        ("rot_len", ctypes.c_uint32),
        ("rot64_len", ctypes.c_uint32),
        ("fold64", ctypes.c_int32),
        ("fft_pmask", ctypes.c_uint32),
    ]


ENERGY_RAW, ENERGY_FOLDED, ENERGY_PARSEVAL = 0, 1, 2


class DemodError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = strerror(code) if _lib is not None else str(code)
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


_lib: Optional[ctypes.CDLL] = None

_P = ctypes.c_void_p
_SZ = ctypes.c_size_t


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libfskdemod.so (raises FileNotFoundError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if _LIB_ENV and path == LIB_PATH:
        path = _LIB_ENV
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"{path} not built: run `make -C audio-network_amd/csrc` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    try:
        # Bind the HIP runtime once: torch ships its own libamdhip64.so.7; if it
        # is imported after this library, a second runtime would be loaded.
        import torch  # noqa: F401
    except ImportError:
        pass
    if path != LIB_PATH:
        import sys
        print(f"audio_network_amd: FSKD_LIB override active, loading {path} (measurement A/B "
              "only; entry points that build lacks stay unbound)", file=sys.stderr)
    lib = ctypes.CDLL(path)
    sig = {
        "demod_cfg_default": (None, [ctypes.POINTER(DemodCfg)]),
        "demod_create": (_P, [ctypes.POINTER(DemodCfg), ctypes.POINTER(ctypes.c_int)]),
        "demod_destroy": (None, [_P]),
        "demod_reset": (ctypes.c_int, [_P]),
        "demod_pending": (ctypes.c_int, [_P]),
        "demod_slide_windows": (ctypes.c_int, [_P]),
        "demod_method": (ctypes.c_int, [_P]),
        "demod_max_symbols": (ctypes.c_int, [_P, _SZ]),
        "demod_batch_launches": (ctypes.c_int, [_P, _SZ, ctypes.c_int]),
        "demod_rescue_tau": (ctypes.c_double, [_P]),
        "demod_rescue_tau64": (ctypes.c_double, [_P]),
        "demod_error_model": (ctypes.c_int, [ctypes.POINTER(DemodCfg), ctypes.POINTER(DemodErrorModel)]),
        "demod_plan_info": (ctypes.c_int, [ctypes.POINTER(DemodCfg), ctypes.POINTER(DemodPlanInfo),
                                           _P, _SZ, _P, _SZ]),
        "demodulate": (ctypes.c_int, [_P, _P, _SZ, _P, _SZ]),
        "demodulate_mags": (ctypes.c_int, [_P, _P, _SZ, _P, _P, _SZ]),
        "demod_batch": (ctypes.c_int, [_P, _P, _SZ, _P, _P]),
        "demod_batch_async": (ctypes.c_int, [_P, _P, _SZ, _P, _P, _P]),
        "demod_batch_spectrum_async": (ctypes.c_int, [_P, _P, _SZ, _P, _P, _P, _P]),
        "demod_frame_size": (_SZ, [_SZ]),
        "demod_frame_encode": (ctypes.c_int, [_P, _SZ, _P, _SZ]),
        "demod_frame_decode": (ctypes.c_int, [_P, _SZ, ctypes.POINTER(ctypes.c_void_p),
                                              ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
        "demod_bits_per_symbol": (ctypes.c_int, [ctypes.c_uint32]),
        "demod_pack_symbols": (ctypes.c_int, [_P, _SZ, ctypes.c_int, _P, _SZ]),
        "demod_unpack_symbols": (ctypes.c_int, [_P, _SZ, ctypes.c_int, _P, _SZ]),
        "demod_frame_symbols": (ctypes.c_longlong, [_P, _SZ, ctypes.c_int, _SZ, _P, _SZ]),
        "demod_frame_symbols_size": (ctypes.c_longlong, [_SZ, ctypes.c_int, _SZ]),
        "demod_frame_streams_async": (ctypes.c_longlong, [_P, _SZ, _SZ, ctypes.c_int, _SZ, _P,
                                                          _P]),
        "demod_broadcast_request_encode": (ctypes.c_int, [_P, _SZ]),
        "demod_broadcast_response_encode": (ctypes.c_int, [ctypes.POINTER(DemodDiscovery), _P,
                                                           _SZ]),
        "demod_broadcast_decode": (ctypes.c_int, [_P, _SZ, ctypes.POINTER(ctypes.c_uint32),
                                                  ctypes.POINTER(DemodDiscovery)]),
        "demod_hello_encode": (ctypes.c_int, [ctypes.POINTER(DemodReceiverInfo), _P, _SZ]),
        "demod_receiver_error_encode": (ctypes.c_int, [ctypes.POINTER(DemodReceiverError), _P,
                                                       _SZ]),
        "demod_to_transmitter_decode": (ctypes.c_int, [_P, _SZ, ctypes.POINTER(DemodReceiverInfo),
                                                       ctypes.POINTER(DemodReceiverError),
                                                       ctypes.POINTER(_SZ)]),
        "demod_streams_create": (_P, [ctypes.POINTER(DemodCfg), _SZ, ctypes.POINTER(ctypes.c_int)]),
        "demod_streams_destroy": (None, [_P]),
        "demod_streams_reset": (ctypes.c_int, [_P, _SZ]),
        "demod_streams_pending": (ctypes.c_int, [_P, _SZ]),
        "demod_streams_max_symbols": (ctypes.c_longlong, [_P, _P]),
        "demod_streams_push": (ctypes.c_int, [_P, _P, _P, _P, _P, _SZ, _P]),
        "demod_streams_push_packets": (ctypes.c_int, [_P, _P, _P, _P, _P, ctypes.c_int, _P, _P, _SZ,
                                                      _P]),
        "demod_synth_fsk": (ctypes.c_int, [ctypes.POINTER(DemodCfg), ctypes.c_uint64,
                                           ctypes.c_uint64, _SZ, ctypes.c_int, ctypes.c_int,
                                           _P, _P, _P]),
        "demod_read_ceiling_async": (ctypes.c_int, [_P, _SZ, _P]),
        "demod_group_unique_id": (ctypes.c_int, [_P]),
        "demod_group_shard": (ctypes.c_int, [_SZ, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_SZ),
                                             ctypes.POINTER(_SZ)]),
        "demod_group_block_bytes": (ctypes.c_longlong, [_SZ, ctypes.c_int, _SZ, _SZ, ctypes.c_int]),
        "demod_group_create": (_P, [ctypes.POINTER(DemodCfg), _SZ, ctypes.c_int, ctypes.c_int, _P,
                                    ctypes.POINTER(ctypes.c_int)]),
        "demod_group_create_local": (_P, [ctypes.POINTER(DemodCfg), _SZ, ctypes.c_int, _P,
                                          ctypes.POINTER(ctypes.c_int)]),
        "demod_group_destroy": (None, [_P]),
        "demod_group_world": (ctypes.c_int, [_P]),
        "demod_group_local_ranks": (ctypes.c_int, [_P]),
        "demod_group_rank_shard": (ctypes.c_int, [_P, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                                  ctypes.POINTER(_SZ), ctypes.POINTER(_SZ)]),
        "demod_group_rank_device": (ctypes.c_int, [_P, ctypes.c_int]),
        "demod_group_status": (ctypes.c_int, [_P]),
        "demod_group_wait": (ctypes.c_int, [_P, _P]),
        "demod_group_push": (ctypes.c_int, [_P, _P, _P, _P, _SZ, _P]),
        "demod_group_bucket_async": (ctypes.c_longlong, [_P, _P, _SZ, _SZ, _SZ, _P, _P]),
        "demod_strerror": (ctypes.c_char_p, [ctypes.c_int]),
        "demod_version_string": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        if _LIB_ENV and not hasattr(lib, name):
            continue  # an older build for an A/B: entry points it predates stay unbound
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def header_exports(path: str = HEADER_PATH) -> list:
    """Function names declared in include/demod.h."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", src)
    skip = {"defined", "sizeof"}
    decl = []
    for m in re.finditer(r"^[^#\n][^;{}]*?\b([a-z_][a-z0-9_]*)\s*\([^;{}]*\)\s*;", src, flags=re.M):
        if m.group(1) not in skip and not m.group(0).lstrip().startswith("typedef"):
            decl.append(m.group(1))
    return sorted(set(decl)) if decl else sorted(set(names) - skip)


def strerror(code: int) -> str:
    return load_library().demod_strerror(code).decode()


def version_string() -> str:
    return load_library().demod_version_string().decode()


def make_cfg(fs: float = 48000.0, n: int = 1024, hop: Optional[int] = None,
             freqs: Sequence[float] = FSK2_FREQS, channels: int = 1,
             channel_mode: int = CH_LEFT, device: int = 0,
             method: int = METHOD_AUTO, lead_in: int = 0) -> DemodCfg:
    cfg = DemodCfg()
    load_library().demod_cfg_default(ctypes.byref(cfg))
    cfg.fs = float(fs)
    cfg.n = int(n)
    cfg.hop = int(n if hop is None else hop)
    if len(freqs) > DEMOD_MAX_TONES:
        raise DemodError(DEMOD_BAD_ARG, "too many tones")
    cfg.k = len(freqs)
    cfg.channels = int(channels)
    cfg.channel_mode = int(channel_mode)
    cfg.device = int(device)
    cfg.method = int(method)
    cfg.lead_in = int(lead_in)
    for i in range(DEMOD_MAX_TONES):
        cfg.freqs[i] = float(freqs[i]) if i < len(freqs) else 0.0
    return cfg


def error_model(cfg: DemodCfg) -> dict:
    """demod_error_model: the decision rescue's bounds for cfg's tone plan (no GPU)."""
    m = DemodErrorModel()
    rc = load_library().demod_error_model(ctypes.byref(cfg), ctypes.byref(m))
    if rc != DEMOD_OK:
        raise DemodError(rc, "demod_error_model")
    return {f: getattr(m, f) for f, _ in DemodErrorModel._fields_}


def plan_info(cfg: DemodCfg) -> dict:
    """demod_plan_info: the plan cfg runs and its fp32 constants (no GPU); `rot`
    as float32 [rot_len][4], `rot64` as float64 (empty without a first pass)."""
    lib = load_library()
    info = DemodPlanInfo()
    rc = lib.demod_plan_info(ctypes.byref(cfg), ctypes.byref(info), None, 0, None, 0)
    if rc != DEMOD_OK:
        raise DemodError(rc, "demod_plan_info")
    rot = np.zeros((info.rot_len, 4), np.float32)
    rot64 = np.zeros(info.rot64_len, np.float64)
    rc = lib.demod_plan_info(ctypes.byref(cfg), ctypes.byref(info), _ptr(rot), rot.size,
                             _ptr(rot64), rot64.size)
    if rc != DEMOD_OK:
        raise DemodError(rc, "demod_plan_info")
    out = {f: getattr(info, f) for f, _ in DemodPlanInfo._fields_}
    for f in ("slot_tone", "zcls", "fft_bins", "coef", "sgn", "rcoef"):
        out[f] = np.array(out[f][:cfg.k])
    out["coef"] = out["coef"].astype(np.float32)
    out["sgn"] = out["sgn"].astype(np.float32)
    out["rot"] = rot
    out["rot64"] = rot64
    return out


def _ptr(a) -> int:
    """Address of a numpy array or a torch tensor (host or device)."""
    if a is None:
        return 0
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    return int(a.data_ptr())


_DTYPE_BYTES = {"int16": 2, "uint8": 1, "float32": 4}


def _check_dev(t, what: str, dtype: str, min_numel: int, device: Optional[int] = None,
               nullable: bool = False) -> None:
    """Validate a device tensor handed to the C ABI as a raw pointer: a short,
    strided, wrong-dtype or wrong-device tensor would otherwise become silent
    out-of-bounds device writes. Raises DemodError(DEMOD_BAD_ARG)."""
    if t is None:
        if nullable or min_numel == 0:
            return
        raise DemodError(DEMOD_BAD_ARG, f"{what}: required")
    if isinstance(t, int):
        raise DemodError(DEMOD_BAD_ARG, f"{what}: pass a device tensor, not a raw address")
    if not hasattr(t, "is_contiguous") or not hasattr(t, "device"):
        raise DemodError(DEMOD_BAD_ARG, f"{what}: expected a torch device tensor")
    if str(t.dtype) != "torch." + dtype:
        raise DemodError(DEMOD_BAD_ARG, f"{what}: dtype {t.dtype}, need torch.{dtype}")
    if not t.is_contiguous():
        raise DemodError(DEMOD_BAD_ARG, f"{what}: not contiguous")
    if t.device.type != "cuda" or (device is not None and t.device.index != device):
        raise DemodError(DEMOD_BAD_ARG, f"{what}: on {t.device}, need cuda:{device}")
    if t.numel() < min_numel:
        raise DemodError(DEMOD_BAD_ARG, f"{what}: {t.numel()} elements, need >= {min_numel}")


class Demodulator:
    """One demod_t handle (not thread-safe within a handle, like libopus)."""

    def __init__(self, cfg: Optional[DemodCfg] = None, **kw):
        self._lib = load_library()
        self.cfg = cfg if cfg is not None else make_cfg(**kw)
        err = ctypes.c_int(0)
        h = self._lib.demod_create(ctypes.byref(self.cfg), ctypes.byref(err))
        if not h:
            raise DemodError(err.value, "demod_create")
        self._h = h

    @property
    def k(self) -> int:
        return int(self.cfg.k)

    @property
    def n(self) -> int:
        return int(self.cfg.n)

    @property
    def hop(self) -> int:
        return int(self.cfg.hop)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.demod_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self) -> None:
        rc = self._lib.demod_reset(self._h)
        if rc < 0:
            raise DemodError(rc, "demod_reset")

    @property
    def method(self) -> int:
        """Detector in use: METHOD_GOERTZEL, METHOD_FOLDED, METHOD_RESIDUE or METHOD_FFT."""
        return int(self._lib.demod_method(self._h))

    def pending(self) -> int:
        return int(self._lib.demod_pending(self._h))

    @property
    def slide_windows(self) -> int:
        """Windows per tile of the segment-shared kernel (0: windows alone)."""
        return int(self._lib.demod_slide_windows(self._h))

    def max_symbols(self, n_frames: int) -> int:
        return int(self._lib.demod_max_symbols(self._h, n_frames))

    @property
    def rescue_tau(self) -> float:
        """The decision rescue's threshold factor tau (demod_rescue_tau; 0: off)."""
        return float(self._lib.demod_rescue_tau(self._h))

    @property
    def rescue_tau64(self) -> float:
        """The in-kernel rescue's double-stage threshold factor
        (demod_rescue_tau64; 0: flagged windows take the exact chain)."""
        return float(self._lib.demod_rescue_tau64(self._h))

    def batch_launches(self, n_windows: int, mags: bool = True) -> int:
        """Kernel launches one batch of n_windows makes (demod_batch_launches)."""
        return int(self._lib.demod_batch_launches(self._h, n_windows, 1 if mags else 0))

    def demodulate(self, pcm: np.ndarray, mags: bool = False, max_symbols: Optional[int] = None):
        """Streaming demodulate(pcm, n): pcm is int16, interleaved if stereo."""
        pcm = np.ascontiguousarray(pcm, dtype=np.int16)
        ch = int(self.cfg.channels)
        if pcm.size % ch:
            raise DemodError(DEMOD_BAD_ARG, "pcm length not a multiple of channels")
        n_frames = pcm.size // ch
        cap = self.max_symbols(n_frames) if max_symbols is None else int(max_symbols)
        sym = np.empty(max(cap, 1), dtype=np.uint8)
        mag = np.empty((max(cap, 1), self.k), dtype=np.float32) if mags else None
        rc = self._lib.demodulate_mags(self._h, _ptr(pcm), n_frames, _ptr(sym), _ptr(mag), cap)
        if rc < 0:
            raise DemodError(rc, "demodulate")
        return (sym[:rc], mag[:rc]) if mags else sym[:rc]

    def batch(self, pcm, n_windows: Optional[int] = None, mags: bool = False):
        """Batch hot path on host numpy windows [W][n] (or hop-strided)."""
        pcm = np.ascontiguousarray(pcm, dtype=np.int16)
        flat = pcm.reshape(-1)
        if n_windows is None:
            if pcm.ndim == 2 and self.hop == self.n:
                n_windows = pcm.shape[0]
            else:
                n_windows = 0 if flat.size < self.n else (flat.size - self.n) // self.hop + 1
        if n_windows and (n_windows - 1) * self.hop + self.n > flat.size:
            raise DemodError(DEMOD_BAD_ARG, "pcm shorter than n_windows")
        buf = flat
        if flat.ctypes.data % 16:
            buf = np.empty(flat.size + 8, dtype=np.int16)
            off = (-buf.ctypes.data % 16) // 2
            buf = buf[off:off + flat.size]
            buf[:] = flat
        sym = np.empty(max(n_windows, 1), dtype=np.uint8)
        mag = np.empty((max(n_windows, 1), self.k), dtype=np.float32) if mags else None
        rc = self._lib.demod_batch(self._h, _ptr(buf), n_windows, _ptr(sym), _ptr(mag))
        if rc < 0:
            raise DemodError(rc, "demod_batch")
        return (sym[:rc], mag[:rc]) if mags else sym[:rc]

    def _check_batch(self, d_pcm, n_windows: int, d_sym, d_mag, d_spec=None) -> None:
        n_windows = int(n_windows)
        if n_windows < 0:
            raise DemodError(DEMOD_BAD_ARG, "n_windows < 0")
        dev = int(self.cfg.device)
        need = (n_windows - 1) * self.hop + self.n if n_windows else 0
        _check_dev(d_pcm, "d_pcm", "int16", need, dev)
        _check_dev(d_sym, "d_sym", "uint8", n_windows, dev)
        _check_dev(d_mag, "d_mag", "float32", n_windows * self.k, dev, nullable=True)
        _check_dev(d_spec, "d_spec", "float32", n_windows * (self.n // 2 + 1), dev, nullable=True)

    def batch_device(self, d_pcm, n_windows: int, d_sym, d_mag=None) -> int:
        """Synchronous batch on device tensors (checked: dtype, contiguity,
        device, size)."""
        self._check_batch(d_pcm, n_windows, d_sym, d_mag)
        rc = self._lib.demod_batch(self._h, _ptr(d_pcm), n_windows, _ptr(d_sym), _ptr(d_mag))
        if rc < 0:
            raise DemodError(rc, "demod_batch")
        return rc

    def batch_async(self, d_pcm, n_windows: int, d_sym, d_mag=None, stream: int = 0) -> int:
        """Enqueue on a HIP stream (raw hipStream_t as int; 0 = default stream,
        e.g. torch.cuda.current_stream().cuda_stream)."""
        self._check_batch(d_pcm, n_windows, d_sym, d_mag)
        rc = self._lib.demod_batch_async(self._h, _ptr(d_pcm), n_windows, _ptr(d_sym),
                                         _ptr(d_mag), stream or None)
        if rc < 0:
            raise DemodError(rc, "demod_batch_async")
        return rc

    def batch_spectrum_async(self, d_pcm, n_windows: int, d_sym, d_mag=None, d_spec=None,
                             stream: int = 0) -> int:
        """FFT handles: symbols, tone-bin |X|^2 and the full |X[b]|^2 spectrum."""
        self._check_batch(d_pcm, n_windows, d_sym, d_mag, d_spec)
        rc = self._lib.demod_batch_spectrum_async(self._h, _ptr(d_pcm), n_windows, _ptr(d_sym),
                                                  _ptr(d_mag), _ptr(d_spec), stream or None)
        if rc < 0:
            raise DemodError(rc, "demod_batch_spectrum_async")
        return rc


class Streams:
    """demod_streams_t: n_streams independent streams behind one detector,
    one batch per push (include/demod.h, "many streams, one launch")."""

    def __init__(self, n_streams: int, cfg: Optional[DemodCfg] = None, **kw):
        self._lib = load_library()
        self.cfg = cfg if cfg is not None else make_cfg(**kw)
        self.n_streams = int(n_streams)
        err = ctypes.c_int(0)
        h = self._lib.demod_streams_create(ctypes.byref(self.cfg), self.n_streams, ctypes.byref(err))
        if not h:
            raise DemodError(err.value, "demod_streams_create")
        self._h = h

    @property
    def k(self) -> int:
        return int(self.cfg.k)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.demod_streams_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def reset(self, stream: int) -> None:
        rc = self._lib.demod_streams_reset(self._h, int(stream))
        if rc < 0:
            raise DemodError(rc, "demod_streams_reset")

    def pending(self, stream: int) -> int:
        rc = self._lib.demod_streams_pending(self._h, int(stream))
        if rc < 0:
            raise DemodError(rc, "demod_streams_pending")
        return rc

    def push(self, packets, mags: bool = False, cap: Optional[int] = None):
        """packets: one int16 array (interleaved if stereo) or None per stream,
        or one 2-D array whose rows are the streams' packets (equal lengths;
        its row addresses are computed, not read array by array).
        Returns the per-stream symbol arrays (and magnitude arrays)."""
        ch = int(self.cfg.channels)
        S = self.n_streams
        if isinstance(packets, np.ndarray) and packets.ndim == 2:
            if packets.shape[0] != S:
                raise DemodError(DEMOD_BAD_ARG, "one packet row per stream")
            rows_ok = (packets.dtype == np.int16 and packets.strides[0] >= 0
                       and (packets.shape[1] <= 1 or packets.strides[1] == 2))
            # rows need only be contiguous each (a column slice of a longer
            # recording is not copied)
            keep = packets if rows_ok else np.ascontiguousarray(packets, dtype=np.int16)
            if keep.shape[1] % ch:
                raise DemodError(DEMOD_BAD_ARG, "pcm length not a multiple of channels")
            frames = np.full(S, keep.shape[1] // ch, dtype=np.uintp)
            ptrs = np.zeros(S, dtype=np.uintp)
            if keep.shape[1]:
                ptrs += np.uintp(keep.ctypes.data)
                ptrs += np.arange(S, dtype=np.uintp) * np.uintp(keep.strides[0])
        else:
            if len(packets) != S:
                raise DemodError(DEMOD_BAD_ARG, "one packet (or None) per stream")
            keep = [np.ascontiguousarray(p, dtype=np.int16) if p is not None else None for p in packets]
            frames = np.array([0 if a is None else a.size // ch for a in keep], dtype=np.uintp)
            for a in keep:
                if a is not None and a.size % ch:
                    raise DemodError(DEMOD_BAD_ARG, "pcm length not a multiple of channels")
            ptrs = np.array([0 if a is None or a.size == 0 else a.ctypes.data for a in keep],
                            dtype=np.uintp)
        if cap is None:
            cap = int(self._lib.demod_streams_max_symbols(self._h, frames.ctypes.data))
        sym = np.empty(max(cap, 1), dtype=np.uint8)
        mag = np.empty((max(cap, 1), self.k), dtype=np.float32) if mags else None
        counts = np.zeros(S, dtype=np.uint32)
        rc = self._lib.demod_streams_push(self._h, ptrs.ctypes.data, frames.ctypes.data,
                                          _ptr(sym), _ptr(mag), cap, counts.ctypes.data)
        del keep
        if rc < 0:
            raise DemodError(rc, "demod_streams_push")
        e = [0] + np.cumsum(counts, dtype=np.int64).tolist()
        out_s = [sym[e[i]:e[i + 1]] for i in range(S)]
        if not mags:
            return out_s
        return out_s, [mag[e[i]:e[i + 1]] for i in range(S)]


# demod_decode_fn: opus_decode's signature (opus.h:462)
DECODE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                             ctypes.c_void_p, ctypes.c_int, ctypes.c_int)


def push_packets(streams: "Streams", decode, decoders: Sequence[int], packets: Sequence[Optional[bytes]],
                 frame_size: int, mags: bool = False, cap: Optional[int] = None):
    """demod_streams_push_packets: one encoded packet per stream (bytes, or
    None / b"" for none), decoded by `decode` (a DECODE_FN, or the address of
    a native demod_decode_fn such as opus_decode) with decoders[i] (a state
    pointer) into PCM, then pushed. Returns the per-stream symbol arrays (and
    magnitude arrays)."""
    lib = streams._lib
    S = streams.n_streams
    if len(packets) != S or len(decoders) != S:
        raise DemodError(DEMOD_BAD_ARG, "one packet and one decoder per stream")
    bufs = [ctypes.create_string_buffer(bytes(p), max(len(p), 1)) if p else None for p in packets]
    pk = (ctypes.c_void_p * S)(*[ctypes.addressof(b) if b is not None else None for b in bufs])
    lens = (ctypes.c_int32 * S)(*[len(p) if p else 0 for p in packets])
    decs = (ctypes.c_void_p * S)(*decoders)
    if cap is None:
        frames = np.full(S, frame_size, dtype=np.uintp)
        cap = int(lib.demod_streams_max_symbols(streams._h, frames.ctypes.data))
    sym = np.empty(max(cap, 1), dtype=np.uint8)
    mag = np.empty((max(cap, 1), streams.k), dtype=np.float32) if mags else None
    counts = np.zeros(S, dtype=np.uint32)
    fn = ctypes.cast(decode, ctypes.c_void_p) if not isinstance(decode, int) else ctypes.c_void_p(decode)
    rc = lib.demod_streams_push_packets(streams._h, fn, decs, pk, lens, int(frame_size), _ptr(sym),
                                        _ptr(mag), cap, counts.ctypes.data)
    del bufs
    if rc < 0:
        raise DemodError(rc, "demod_streams_push_packets")
    e = [0] + np.cumsum(counts, dtype=np.int64).tolist()
    out_s = [sym[e[i]:e[i + 1]] for i in range(S)]
    if not mags:
        return out_s
    return out_s, [mag[e[i]:e[i + 1]] for i in range(S)]


def synth_fsk(cfg: DemodCfg, seed: int, n_windows: int, amplitude: int, sigma: int,
              d_pcm, d_sym=None, stream: int = 0, w0: int = 0) -> None:
    """Device generator of the seeded FSK test signal into device buffers."""
    _check_dev(d_pcm, "d_pcm", "int16", int(n_windows) * int(cfg.n), int(cfg.device))
    _check_dev(d_sym, "d_sym", "uint8", int(n_windows), int(cfg.device), nullable=True)
    rc = load_library().demod_synth_fsk(ctypes.byref(cfg), ctypes.c_uint64(seed),
                                         ctypes.c_uint64(w0), n_windows,
                                         amplitude, sigma, _ptr(d_pcm), _ptr(d_sym),
                                         stream or None)
    if rc < 0:
        raise DemodError(rc, "demod_synth_fsk")


def read_ceiling_async(d_buf, n_bytes: int, stream: int = 0) -> None:
    """Read-only reference stream over a device buffer (demod_read_ceiling_async)."""
    if not hasattr(d_buf, "numel") or d_buf.numel() * d_buf.element_size() < n_bytes:
        raise DemodError(DEMOD_BAD_ARG, "read_ceiling_async: buffer smaller than n_bytes")
    rc = load_library().demod_read_ceiling_async(_ptr(d_buf), n_bytes, stream or None)
    if rc < 0:
        raise DemodError(rc, "demod_read_ceiling_async")


# ---- ip.proto framing (host) ---------------------------------------------

def frame_size(payload_len: int) -> int:
    return int(load_library().demod_frame_size(payload_len))


def frame_encode(payload: bytes) -> bytes:
    lib = load_library()
    src = (ctypes.c_uint8 * max(len(payload), 1)).from_buffer_copy(payload or b"\0")
    cap = lib.demod_frame_size(len(payload))
    out = (ctypes.c_uint8 * cap)()
    rc = lib.demod_frame_encode(src, len(payload), out, cap)
    if rc < 0:
        raise DemodError(rc, "demod_frame_encode")
    return bytes(out[:rc])


def frame_decode(buf: bytes) -> Tuple[bytes, int]:
    """Decode one delimited ToReceiver frame -> (payload, bytes consumed)."""
    lib = load_library()
    src = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
    pl = ctypes.c_void_p()
    pl_len = _SZ()
    used = _SZ()
    rc = lib.demod_frame_decode(src, len(buf), ctypes.byref(pl), ctypes.byref(pl_len),
                                ctypes.byref(used))
    if rc < 0:
        raise DemodError(rc, "demod_frame_decode")
    off = (pl.value or ctypes.addressof(src)) - ctypes.addressof(src)
    return bytes(buf[off:off + pl_len.value]), int(used.value)


# ---- ip.proto session messages (host; include/demod.h, demod_session.c) ----

def _discovery_struct(d: dict) -> DemodDiscovery:
    s = DemodDiscovery()
    s.protocol_version = int(d.get("protocol_version", 1))
    s.mac_address = int(d.get("mac_address", 0))
    s.device_name = bytes(d.get("device_name", b""))
    s.currently_streaming = int(bool(d.get("currently_streaming", False)))
    s.opus_version = bytes(d.get("opus_version", b""))
    return s


def _discovery_dict(s: DemodDiscovery) -> dict:
    return {"protocol_version": int(s.protocol_version), "mac_address": int(s.mac_address),
            "device_name": bytes(s.device_name), "currently_streaming": bool(s.currently_streaming),
            "opus_version": bytes(s.opus_version)}


def _session_call(fn, name, *args, cap=1024) -> bytes:
    out = (ctypes.c_uint8 * cap)()
    rc = fn(*args, out, cap)
    if rc < 0:
        raise DemodError(rc, name)
    return bytes(out[:rc])


def broadcast_request_encode() -> bytes:
    """BroadcastMessage{magic, discovery_request = true} (discovery.kt:44-48)."""
    return _session_call(load_library().demod_broadcast_request_encode,
                         "demod_broadcast_request_encode")


def broadcast_response_encode(d: dict) -> bytes:
    """BroadcastMessage{magic, discovery_response = d} (network.cpp:356-378)."""
    s = _discovery_struct(d)
    return _session_call(load_library().demod_broadcast_response_encode,
                         "demod_broadcast_response_encode", ctypes.byref(s))


def broadcast_decode(buf: bytes):
    """-> (which, magic, discovery dict or None); DemodError where nanopb fails."""
    lib = load_library()
    src = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
    magic = ctypes.c_uint32()
    d = DemodDiscovery()
    rc = lib.demod_broadcast_decode(src, len(buf), ctypes.byref(magic), ctypes.byref(d))
    if rc < 0:
        raise DemodError(rc, "demod_broadcast_decode")
    return rc, int(magic.value), (_discovery_dict(d) if rc == DEMOD_MSG_DISCOVERY_RESPONSE
                                  else None)


def hello_encode(info: dict) -> bytes:
    """Delimited ToTransmitter{receiver_information} (network.cpp:388-403)."""
    s = DemodReceiverInfo()
    s.discovery_data = _discovery_struct(info.get("discovery_data", {}))
    s.max_encoded_frame_size = int(info.get("max_encoded_frame_size", DEMOD_MAX_FRAME_PAYLOAD))
    s.max_decoded_frame_size = int(info.get("max_decoded_frame_size", DEMOD_MAX_DECODED_FRAME))
    return _session_call(load_library().demod_hello_encode, "demod_hello_encode",
                         ctypes.byref(s))


def receiver_error_encode(audio_underflow: bool, audio_decode_error: bool) -> bytes:
    """Delimited ToTransmitter{error}."""
    s = DemodReceiverError(int(bool(audio_underflow)), int(bool(audio_decode_error)))
    return _session_call(load_library().demod_receiver_error_encode,
                         "demod_receiver_error_encode", ctypes.byref(s))


def to_transmitter_decode(buf: bytes):
    """Delimited ToTransmitter -> (which, fields dict or None, bytes consumed)."""
    lib = load_library()
    src = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
    info = DemodReceiverInfo()
    err = DemodReceiverError()
    used = _SZ()
    rc = lib.demod_to_transmitter_decode(src, len(buf), ctypes.byref(info), ctypes.byref(err),
                                         ctypes.byref(used))
    if rc < 0:
        raise DemodError(rc, "demod_to_transmitter_decode")
    if rc == DEMOD_MSG_RECEIVER_INFORMATION:
        fields = {"discovery_data": _discovery_dict(info.discovery_data),
                  "max_encoded_frame_size": int(info.max_encoded_frame_size),
                  "max_decoded_frame_size": int(info.max_decoded_frame_size)}
    elif rc == DEMOD_MSG_RECEIVER_ERROR:
        fields = {"audio_underflow": bool(err.audio_underflow),
                  "audio_decode_error": bool(err.audio_decode_error)}
    else:
        fields = None
    return rc, fields, int(used.value)


def bits_per_symbol(k: int) -> int:
    return int(load_library().demod_bits_per_symbol(k))


def pack_symbols(symbols: np.ndarray, bits: int) -> bytes:
    sym = np.ascontiguousarray(symbols, dtype=np.uint8)
    cap = (sym.size * bits + 7) // 8
    out = np.empty(max(cap, 1), dtype=np.uint8)
    rc = load_library().demod_pack_symbols(_ptr(sym), sym.size, bits, _ptr(out), cap)
    if rc < 0:
        raise DemodError(rc, "demod_pack_symbols")
    return out[:rc].tobytes()


def unpack_symbols(data: bytes, n: int, bits: int) -> np.ndarray:
    src = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, np.uint8)
    if len(data) * 8 < n * bits:
        raise DemodError(DEMOD_BAD_ARG, "not enough packed bytes")
    out = np.empty(max(n, 1), dtype=np.uint8)
    rc = load_library().demod_unpack_symbols(_ptr(src), n, bits, _ptr(out), n)
    if rc < 0:
        raise DemodError(rc, "demod_unpack_symbols")
    return out[:n]


def frame_symbols(symbols: np.ndarray, bits: int,
                  max_payload: int = DEMOD_MAX_FRAME_PAYLOAD) -> bytes:
    """Symbols -> consecutive delimited ToReceiver frames (rank-0 framing)."""
    sym = np.ascontiguousarray(symbols, dtype=np.uint8)
    per = max_payload * 8 // bits
    nframes = (sym.size + per - 1) // per
    cap = nframes * frame_size(max_payload) + 16
    out = np.empty(cap, dtype=np.uint8)
    rc = load_library().demod_frame_symbols(_ptr(sym), sym.size, bits, max_payload,
                                            _ptr(out), cap)
    if rc < 0:
        raise DemodError(int(rc), "demod_frame_symbols")
    return out[:rc].tobytes()


def frame_symbols_size(n: int, bits: int, max_payload: int = DEMOD_MAX_FRAME_PAYLOAD) -> int:
    """Bytes frame_symbols produces for n symbols."""
    rc = int(load_library().demod_frame_symbols_size(n, bits, max_payload))
    if rc < 0:
        raise DemodError(rc, "demod_frame_symbols_size")
    return rc


def frame_streams_async(d_symbols, n_streams: int, n: int, bits: int, d_out,
                        max_payload: int = DEMOD_MAX_FRAME_PAYLOAD, stream: int = 0) -> int:
    """Device framing of [n_streams][n] symbols: stream s's frames (as
    frame_symbols would make them) at d_out[s * stride]; returns stride."""
    stride = frame_symbols_size(n, bits, max_payload)
    _check_dev(d_symbols, "d_symbols", "uint8", int(n_streams) * int(n))
    _check_dev(d_out, "d_out", "uint8", int(n_streams) * stride)
    if d_symbols is not None and d_out is not None and d_symbols.device != d_out.device:
        raise DemodError(DEMOD_BAD_ARG, "d_symbols and d_out on different devices")
    rc = int(load_library().demod_frame_streams_async(_ptr(d_symbols), n_streams, n, bits,
                                                      max_payload, _ptr(d_out), stream or None))
    if rc < 0:
        raise DemodError(rc, "demod_frame_streams_async")
    return rc


def iter_frames(stream: bytes):
    """Yield payloads of consecutive delimited frames (network.cpp:409-430 loop)."""
    pos = 0
    while pos < len(stream):
        payload, used = frame_decode(stream[pos:])
        yield payload
        pos += used


# ---- many streams over many GPUs (demod_group_*, RCCL) -----------------------

DEMOD_GROUP_ID_BYTES = 128


def group_unique_id() -> bytes:
    """demod_group_unique_id: a fresh RCCL group id (rank 0 shares it)."""
    buf = (ctypes.c_uint8 * DEMOD_GROUP_ID_BYTES)()
    rc = load_library().demod_group_unique_id(buf)
    if rc != DEMOD_OK:
        raise DemodError(rc, "demod_group_unique_id")
    return bytes(buf)


def group_shard(n_streams: int, rank: int, world: int) -> Tuple[int, int]:
    f, c = _SZ(), _SZ()
    rc = load_library().demod_group_shard(n_streams, rank, world, ctypes.byref(f), ctypes.byref(c))
    if rc != DEMOD_OK:
        raise DemodError(rc, "demod_group_shard")
    return f.value, c.value


def group_block_bytes(n_streams: int, world: int, steps: int, symbols_per_stream: int, bits: int) -> int:
    rc = load_library().demod_group_block_bytes(n_streams, world, steps, symbols_per_stream, bits)
    if rc < 0:
        raise DemodError(int(rc), "demod_group_block_bytes")
    return int(rc)


class Group:
    """demod_group_t: n_streams streams sharded over `world` GPUs, RCCL gathers.
    Group(cfg, n, rank=r, world=w, uid=...) is one rank of a multi-process
    group; Group(cfg, n, devices=[...]) drives every rank in this process."""

    def __init__(self, cfg: DemodCfg, n_streams: int, rank: int = 0, world: int = 1,
                 uid: Optional[bytes] = None, devices: Optional[Sequence[int]] = None):
        self._lib = load_library()
        err = ctypes.c_int(0)
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*devices)
            self._h = self._lib.demod_group_create_local(ctypes.byref(cfg), n_streams, len(devices), arr,
                                                         ctypes.byref(err))
        else:
            if uid is None:
                uid = group_unique_id()
            buf = (ctypes.c_uint8 * DEMOD_GROUP_ID_BYTES).from_buffer_copy(uid)
            self._h = self._lib.demod_group_create(ctypes.byref(cfg), n_streams, rank, world, buf,
                                                   ctypes.byref(err))
        if not self._h:
            raise DemodError(err.value, "demod_group_create")
        self.n_streams = n_streams
        self.k = cfg.k
        self.channels = int(cfg.channels)
        self.world = self._lib.demod_group_world(self._h)
        self.local_ranks = self._lib.demod_group_local_ranks(self._h)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.demod_group_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        self.close()

    def shard(self, local: int = 0) -> Tuple[int, int, int]:
        """(rank, first stream, count) of the local-th rank this process drives."""
        r, f, c = ctypes.c_int(), _SZ(), _SZ()
        rc = self._lib.demod_group_rank_shard(self._h, local, ctypes.byref(r), ctypes.byref(f),
                                              ctypes.byref(c))
        if rc != DEMOD_OK:
            raise DemodError(rc, "demod_group_rank_shard")
        return r.value, f.value, c.value

    def device(self, local: int = 0) -> int:
        """demod_group_rank_device: the GPU of the local-th rank this process drives."""
        rc = self._lib.demod_group_rank_device(self._h, local)
        if rc < 0:
            raise DemodError(rc, "demod_group_rank_device")
        return rc

    def status(self) -> int:
        """demod_group_status: DEMOD_OK while alive, else the code that killed it."""
        return self._lib.demod_group_status(self._h)

    def wait(self, streams: Optional[Sequence[int]] = None) -> None:
        """demod_group_wait: wait for the last bucket on `streams`; raises the
        lowest failing rank's code (the same on every rank)."""
        n = self.local_ranks
        ps = (ctypes.c_void_p * n)(*(streams or [0] * n))
        rc = self._lib.demod_group_wait(self._h, ps if streams else None)
        if rc != DEMOD_OK:
            raise DemodError(rc, "demod_group_wait")

    def push(self, packets: Sequence[np.ndarray], cap: Optional[int] = None):
        """One packet per stream this process owns -> (symbols of every stream,
        counts per stream)."""
        packets = [np.ascontiguousarray(p, dtype=np.int16) for p in packets]
        nf = (_SZ * len(packets))(*[p.size // self.channels for p in packets])
        ptrs = (ctypes.c_void_p * len(packets))(*[p.ctypes.data if p.size else None for p in packets])
        if cap is None:
            cap = sum(p.size for p in packets) * max(self.world, 1) + 64 * self.n_streams
        sym = np.zeros(max(cap, 1), np.uint8)
        counts = np.zeros(self.n_streams, np.uint32)
        rc = self._lib.demod_group_push(self._h, ptrs, nf, sym.ctypes.data, cap, counts.ctypes.data)
        if rc < 0:
            raise DemodError(rc, "demod_group_push")
        return sym[:rc], counts

    def bucket_async(self, d_pcm: Sequence, ring: int, wps: int, steps: int, d_all: Sequence,
                     streams: Optional[Sequence[int]] = None) -> int:
        """demod_group_bucket_async over the ranks this process drives."""
        n = len(d_all)
        pc = (ctypes.c_void_p * n)(*[_ptr(t) for t in d_pcm])
        pa = (ctypes.c_void_p * n)(*[_ptr(t) for t in d_all])
        ps = (ctypes.c_void_p * n)(*(streams or [0] * n))
        rc = self._lib.demod_group_bucket_async(self._h, pc, ring, wps, steps, pa, ps)
        if rc < 0:
            raise DemodError(int(rc), "demod_group_bucket_async")
        return int(rc)
