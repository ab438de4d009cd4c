"""oracle.py — TEST INFRASTRUCTURE ONLY: ctypes wrapper of liboracle.so.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / CPU baseline; nothing on the
product path (audio-network_amd/) uses it.

Parity status: the reference contains no demodulator, so
the Goertzel restatement in fsk_oracle.c has no reference counterpart to be
compared with directly. Its spectral values are pinned to the reference's own
FFT code instead: opus_fft_c (libopus celt/kiss_fft.c:569-589, fixed point, the
four static sizes 480/240/120/60) agrees with oracle Goertzel powers at every
bin to the reference's Q15 precision (tests/test_oracle.py, golden fixture
tests/golden/ref_kissfft.npz); and to independent known answers (numpy.fft,
direct DFT, closed forms) at 1e-9. Frame bytes are pinned to the reference's
own nanopb (oracle/_ref).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_NANOPB = os.path.join(HERE, "_ref", "libnanopb_ref.so")
REF_KISSFFT = os.path.join(HERE, "_ref", "libkissfft_ref.so")
REF_KISSFFT_CUSTOM = os.path.join(HERE, "_ref", "libkissfft_custom.so")  # CUSTOM_MODES build
KISSFFT_PRESHIFT = 14  # int16 samples << 14: the Q31 range opus_fft_c is built for

_lib = None
_P = ctypes.c_void_p
_SZ = ctypes.c_size_t


def build() -> None:
    subprocess.run(["make", "-C", HERE], check=True, capture_output=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = ctypes.CDLL(LIB)
        D = ctypes.POINTER(ctypes.c_double)
        L.oracle_sine_lut.argtypes = [_P]
        L.oracle_synth_fsk.argtypes = [ctypes.c_double, ctypes.c_uint32, ctypes.c_uint32, D,
                                       ctypes.c_uint64, _SZ, _SZ, ctypes.c_int, ctypes.c_int, _P, _P]
        for nm in ("oracle_goertzel", "oracle_goertzel_f32"):
            getattr(L, nm).argtypes = [_P, _SZ, _SZ, ctypes.c_uint32, ctypes.c_uint32, D,
                                       ctypes.c_double, _P, _P]
        L.oracle_goertzel_omp.argtypes = [_P, _SZ, _SZ, ctypes.c_uint32, ctypes.c_uint32, D,
                                          ctypes.c_double, _P, _P, ctypes.c_int]
        L.oracle_dft_power.argtypes = [_P, ctypes.c_uint32, ctypes.c_uint32, D, ctypes.c_double, _P]
        L.oracle_fft_power.argtypes = [_P, ctypes.c_uint32, _P]
        L.oracle_fft_power.restype = ctypes.c_int
        L.oracle_fft_demod.argtypes = [_P, _SZ, _SZ, ctypes.c_uint32, ctypes.c_uint32, D,
                                       ctypes.c_double, _P, _P]
        L.oracle_fft_demod.restype = ctypes.c_int
        L.oracle_fft_demod_omp.argtypes = [_P, _SZ, _SZ, ctypes.c_uint32, ctypes.c_uint32, D,
                                           ctypes.c_double, _P, _P, ctypes.c_int]
        L.oracle_fft_demod_omp.restype = ctypes.c_int
        L.oracle_stream_create.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_int, ctypes.c_uint32, D, ctypes.c_double]
        L.oracle_stream_create.restype = _P
        L.oracle_stream_destroy.argtypes = [_P]
        L.oracle_stream_push.argtypes = [_P, _P, _SZ, _P, _P, _SZ]
        L.oracle_stream_push.restype = ctypes.c_long
        L.oracle_stream_pending.argtypes = [_P]
        L.oracle_stream_pending.restype = ctypes.c_int
        L.oracle_stream_set_lead_in.argtypes = [_P, ctypes.c_uint32]
        _lib = L
    return _lib


MAX_TONES = 64  # fixed coefficient arrays in fsk_oracle.c


def _freqs(freqs: Sequence[float]):
    if len(freqs) > MAX_TONES:
        raise ValueError(f"oracle takes at most {MAX_TONES} tones per call, got {len(freqs)}")
    arr = (ctypes.c_double * len(freqs))(*[float(f) for f in freqs])
    return arr


def sine_lut() -> np.ndarray:
    out = np.empty(16384, np.int16)
    lib().oracle_sine_lut(out.ctypes.data)
    return out


def synth_fsk(freqs: Sequence[float], n: int, n_windows: int, seed: int, amplitude: int = 8000,
              sigma: int = 400, fs: float = 48000.0, w0: int = 0):
    pcm = np.empty((n_windows, n), np.int16)
    sym = np.empty(n_windows, np.uint8)
    lib().oracle_synth_fsk(fs, n, len(freqs), _freqs(freqs), seed, w0, n_windows, amplitude,
                           sigma, pcm.ctypes.data, sym.ctypes.data)
    return pcm, sym


def goertzel(x: np.ndarray, freqs: Sequence[float], n: int, hop: Optional[int] = None,
             n_windows: Optional[int] = None, fs: float = 48000.0, threads: int = 0):
    """Double Goertzel over windows x[w*hop : w*hop+n]; returns (sym, P)."""
    x = np.ascontiguousarray(x, np.int16).reshape(-1)
    hop = n if hop is None else hop
    if n_windows is None:
        n_windows = 0 if x.size < n else (x.size - n) // hop + 1
    k = len(freqs)
    sym = np.empty(n_windows, np.uint8)
    P = np.empty((n_windows, k), np.float64)
    if threads:
        lib().oracle_goertzel_omp(x.ctypes.data, n_windows, hop, n, k, _freqs(freqs), fs,
                                  sym.ctypes.data, P.ctypes.data, threads)
    else:
        lib().oracle_goertzel(x.ctypes.data, n_windows, hop, n, k, _freqs(freqs), fs,
                              sym.ctypes.data, P.ctypes.data)
    return sym, P


def goertzel_f32(x: np.ndarray, freqs: Sequence[float], n: int, fs: float = 48000.0):
    x = np.ascontiguousarray(x, np.int16).reshape(-1)
    W = x.size // n
    k = len(freqs)
    sym = np.empty(W, np.uint8)
    P = np.empty((W, k), np.float32)
    lib().oracle_goertzel_f32(x.ctypes.data, W, n, n, k, _freqs(freqs), fs, sym.ctypes.data,
                              P.ctypes.data)
    return sym, P


def dft_power(x: np.ndarray, freqs: Sequence[float], fs: float = 48000.0) -> np.ndarray:
    x = np.ascontiguousarray(x, np.int16).reshape(-1)
    P = np.empty(len(freqs), np.float64)
    lib().oracle_dft_power(x.ctypes.data, x.size, len(freqs), _freqs(freqs), fs, P.ctypes.data)
    return P


def fft_power(x: np.ndarray) -> np.ndarray:
    x = np.ascontiguousarray(x, np.int16).reshape(-1)
    P = np.empty(x.size // 2 + 1, np.float64)
    rc = lib().oracle_fft_power(x.ctypes.data, x.size, P.ctypes.data)
    if rc:
        raise ValueError(f"oracle_fft_power: {rc}")
    return P


def fft_demod(x: np.ndarray, freqs: Sequence[float], n: int, hop: Optional[int] = None,
              fs: float = 48000.0, threads: int = 0):
    x = np.ascontiguousarray(x, np.int16).reshape(-1)
    hop = n if hop is None else hop
    W = 0 if x.size < n else (x.size - n) // hop + 1
    sym = np.empty(W, np.uint8)
    P = np.empty((W, len(freqs)), np.float64)
    if threads:
        rc = lib().oracle_fft_demod_omp(x.ctypes.data, W, hop, n, len(freqs), _freqs(freqs), fs,
                                        sym.ctypes.data, P.ctypes.data, threads)
    else:
        rc = lib().oracle_fft_demod(x.ctypes.data, W, hop, n, len(freqs), _freqs(freqs), fs,
                                    sym.ctypes.data, P.ctypes.data)
    if rc:
        raise ValueError(f"oracle_fft_demod: {rc}")
    return sym, P


class Stream:
    """Streaming restatement of demodulate(pcm, n)."""

    def __init__(self, freqs, n=1024, hop=None, channels=1, channel_mode=0, fs=48000.0,
                 lead_in=0):
        self.k = len(freqs)
        self._h = lib().oracle_stream_create(n, n if hop is None else hop, channels,
                                             channel_mode, self.k, _freqs(freqs), fs)
        if lead_in:
            lib().oracle_stream_set_lead_in(self._h, lead_in)
        self.channels = channels
        self.n = n

    def push(self, pcm: np.ndarray):
        pcm = np.ascontiguousarray(pcm, np.int16).reshape(-1)
        frames = pcm.size // self.channels
        cap = frames // 8 + 2
        sym = np.empty(cap, np.uint8)
        P = np.empty((cap, self.k), np.float64)
        rc = lib().oracle_stream_push(self._h, pcm.ctypes.data, frames, sym.ctypes.data,
                                      P.ctypes.data, cap)
        if rc < 0:
            raise ValueError(rc)
        return sym[:rc], P[:rc]

    def pending(self) -> int:
        return lib().oracle_stream_pending(self._h)

    def __del__(self):
        try:
            lib().oracle_stream_destroy(self._h)
        except Exception:
            pass


# ---- reference nanopb (oracle/_ref, built from /root/reference by ref.mk) ----
_ref = None


def ref_nanopb() -> Optional[ctypes.CDLL]:
    """The reference's own nanopb + ip.pb.c, or None if oracle/_ref is absent."""
    global _ref
    if _ref is None and os.path.exists(REF_NANOPB):
        R = ctypes.CDLL(REF_NANOPB)
        R.ref_encode_to_receiver.argtypes = [_P, _SZ, _P, _SZ]
        R.ref_encode_to_receiver.restype = ctypes.c_int
        R.ref_decode_to_receiver.argtypes = [_P, _SZ, _P, _SZ, ctypes.POINTER(_SZ),
                                             ctypes.POINTER(_SZ)]
        R.ref_decode_to_receiver.restype = ctypes.c_int
        _ref = R
    return _ref


def ref_encode(payload: bytes) -> bytes:
    R = ref_nanopb()
    src = (ctypes.c_uint8 * max(len(payload), 1)).from_buffer_copy(payload or b"\0")
    out = (ctypes.c_uint8 * (len(payload) + 32))()
    n = R.ref_encode_to_receiver(src, len(payload), out, len(payload) + 32)
    if n < 0:
        raise ValueError("nanopb encode failed")
    return bytes(out[:n])


def ref_decode(buf: bytes):
    """-> (rc, payload, consumed) with rc 0 ok, -1 error, -10 too large."""
    R = ref_nanopb()
    src = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
    out = (ctypes.c_uint8 * 8192)()
    pl = _SZ()
    used = _SZ()
    rc = R.ref_decode_to_receiver(src, len(buf), out, 8192, ctypes.byref(pl), ctypes.byref(used))
    return rc, bytes(out[:pl.value]), int(used.value)


class RefDisc(ctypes.Structure):
    """ref_disc of nanopb_ref_harness.c: a flat DiscoveryResponse (ip.pb.h:17-24)."""
    _fields_ = [("protocol_version", ctypes.c_uint32), ("mac_address", ctypes.c_uint64),
                ("device_name", ctypes.c_char * 128), ("currently_streaming", ctypes.c_int32),
                ("opus_version", ctypes.c_char * 128)]


def _ref_session():
    R = ref_nanopb()
    if R is not None and not getattr(R, "_session_bound", False):
        R.ref_encode_broadcast.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_int,
                                           ctypes.POINTER(RefDisc), _P, _SZ]
        R.ref_encode_broadcast.restype = ctypes.c_int
        R.ref_decode_broadcast.argtypes = [_P, _SZ, ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(RefDisc)]
        R.ref_decode_broadcast.restype = ctypes.c_int
        R.ref_encode_to_transmitter.argtypes = [ctypes.c_int, ctypes.POINTER(RefDisc),
                                                ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                                ctypes.c_int, _P, _SZ]
        R.ref_encode_to_transmitter.restype = ctypes.c_int
        u32p, i32p = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32)
        R.ref_decode_to_transmitter.argtypes = [_P, _SZ, i32p, ctypes.POINTER(RefDisc), u32p, u32p,
                                                i32p, i32p, ctypes.POINTER(_SZ)]
        R.ref_decode_to_transmitter.restype = ctypes.c_int
        R._session_bound = True
    return R


def _ref_disc(d: dict) -> RefDisc:
    r = RefDisc()
    r.protocol_version = d.get("protocol_version", 0)
    r.mac_address = d.get("mac_address", 0)
    r.device_name = d.get("device_name", b"")
    r.currently_streaming = int(bool(d.get("currently_streaming", False)))
    r.opus_version = d.get("opus_version", b"")
    return r


def _disc_dict(r: RefDisc) -> dict:
    return {"protocol_version": int(r.protocol_version), "mac_address": int(r.mac_address),
            "device_name": bytes(r.device_name), "currently_streaming": bool(r.currently_streaming),
            "opus_version": bytes(r.opus_version)}


def ref_broadcast_encode(which: int, magic: int, req: bool = True, d: Optional[dict] = None):
    """Reference nanopb pb_encode of a BroadcastMessage (network.cpp:486-492)."""
    R = _ref_session()
    out = (ctypes.c_uint8 * 1024)()
    rd = _ref_disc(d or {})
    n = R.ref_encode_broadcast(which, magic, int(req), ctypes.byref(rd), out, 1024)
    if n < 0:
        raise ValueError("nanopb encode failed")
    return bytes(out[:n])


def ref_broadcast_decode(buf: bytes):
    """Reference pb_decode of one datagram -> (rc, which, magic, discovery dict or None)."""
    R = _ref_session()
    src = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
    magic, which, rd = ctypes.c_uint32(), ctypes.c_int32(), RefDisc()
    rc = R.ref_decode_broadcast(src, len(buf), ctypes.byref(magic), ctypes.byref(which),
                                ctypes.byref(rd))
    if rc:
        return rc, None, None, None
    return 0, int(which.value), int(magic.value), (_disc_dict(rd) if which.value == 3 else None)


def ref_to_transmitter_encode(which: int, info: Optional[dict] = None, underflow=False,
                              decode_error=False) -> bytes:
    """Reference pb_encode_delimited of a ToTransmitter (network.cpp:388-403)."""
    R = _ref_session()
    info = info or {}
    rd = _ref_disc(info.get("discovery_data", {}))
    out = (ctypes.c_uint8 * 1024)()
    n = R.ref_encode_to_transmitter(which, ctypes.byref(rd), info.get("max_encoded_frame_size", 0),
                                    info.get("max_decoded_frame_size", 0), int(underflow),
                                    int(decode_error), out, 1024)
    if n < 0:
        raise ValueError("nanopb encode failed")
    return bytes(out[:n])


def ref_to_transmitter_decode(buf: bytes):
    """Reference pb_decode_delimited -> (rc, which, fields dict or None, consumed)."""
    R = _ref_session()
    src = (ctypes.c_uint8 * max(len(buf), 1)).from_buffer_copy(buf or b"\0")
    which, rd = ctypes.c_int32(), RefDisc()
    me, md = ctypes.c_uint32(), ctypes.c_uint32()
    uf, de = ctypes.c_int32(), ctypes.c_int32()
    used = _SZ()
    rc = R.ref_decode_to_transmitter(src, len(buf), ctypes.byref(which), ctypes.byref(rd),
                                     ctypes.byref(me), ctypes.byref(md), ctypes.byref(uf),
                                     ctypes.byref(de), ctypes.byref(used))
    if rc:
        return rc, None, None, int(used.value)
    if which.value == 1:
        f = {"discovery_data": _disc_dict(rd), "max_encoded_frame_size": int(me.value),
             "max_decoded_frame_size": int(md.value)}
    elif which.value == 2:
        f = {"audio_underflow": bool(uf.value), "audio_decode_error": bool(de.value)}
    else:
        f = None
    return 0, int(which.value), f, int(used.value)


# ---- reference FFT (libopus opus_fft_c, oracle/_ref, built by ref.mk) --------
_ref_kf = None


def ref_kissfft() -> Optional[ctypes.CDLL]:
    """The reference's own fixed-point opus_fft_c (static states), or None."""
    global _ref_kf
    if _ref_kf is None and os.path.exists(REF_KISSFFT):
        R = ctypes.CDLL(REF_KISSFFT)
        R.ref_fft_static_size.argtypes = [ctypes.c_int]
        R.ref_fft_static_size.restype = ctypes.c_int
        R.ref_fft_static32.argtypes = [ctypes.c_int, _P, ctypes.c_int, _P, _P]
        R.ref_fft_static32.restype = ctypes.c_int
        _ref_kf = R
    return _ref_kf


def ref_fft_static(which: int, x: np.ndarray):
    """opus_fft_c of int16 frame x with static state kfft[which]; returns the
    reference's raw complex output (X / nfft, scaled by 2^KISSFFT_PRESHIFT)."""
    R = ref_kissfft()
    n = R.ref_fft_static_size(which)
    x32 = (np.ascontiguousarray(x, np.int16).astype(np.int32) << KISSFFT_PRESHIFT)
    if x32.size != n:
        raise ValueError(f"kfft[{which}] is {n}-point, got {x32.size} samples")
    re = np.empty(n)
    im = np.empty(n)
    rc = R.ref_fft_static32(which, x32.ctypes.data, n, re.ctypes.data, im.ctypes.data)
    if rc != n:
        raise ValueError(f"ref_fft_static32: {rc}")
    return re + 1j * im


_ref_kfc = None


def ref_kissfft_custom() -> Optional[ctypes.CDLL]:
    """The same opus_fft_c compiled with CUSTOM_MODES (any nfft it can
    factor, e.g. the north-star N = 1024), or None."""
    global _ref_kfc
    if _ref_kfc is None and os.path.exists(REF_KISSFFT_CUSTOM):
        R = ctypes.CDLL(REF_KISSFFT_CUSTOM)
        R.ref_fft_custom32.argtypes = [ctypes.c_int, _P, _P, _P]
        R.ref_fft_custom32.restype = ctypes.c_int
        _ref_kfc = R
    return _ref_kfc


def ref_fft_custom(x: np.ndarray):
    """opus_fft_c of int16 frame x with a state opus_fft_alloc'd for len(x)
    (kissfft_custom_harness.c); the reference's raw complex output (X / nfft,
    scaled by 2^KISSFFT_PRESHIFT)."""
    R = ref_kissfft_custom()
    x32 = (np.ascontiguousarray(x, np.int16).astype(np.int32) << KISSFFT_PRESHIFT)
    n = x32.size
    re = np.empty(n)
    im = np.empty(n)
    rc = R.ref_fft_custom32(n, x32.ctypes.data, re.ctypes.data, im.ctypes.data)
    if rc != n:
        raise ValueError(f"ref_fft_custom32({n}): {rc}")
    return re + 1j * im
