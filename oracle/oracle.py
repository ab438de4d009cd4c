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

    def __init__(self, freqs, n=1024, hop=None, channels=1, channel_mode=0, fs=48000.0):
        self.k = len(freqs)
        self._h = lib().oracle_stream_create(n, n if hop is None else hop, channels,
                                             channel_mode, self.k, _freqs(freqs), fs)
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
