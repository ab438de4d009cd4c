"""Dump the detectors' raw fp32 tone powers (rescue off) and spectra for the
emulation check (tests/fp32emu.py): gpurun_out/<dir>/<case>.npz."""
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
os.environ["FSKD_NO_RESCUE"] = "1"
spec = importlib.util.spec_from_file_location("audio_network_amd", os.path.join(ROOT, "audio-network_amd", "__init__.py"))
A = importlib.util.module_from_spec(spec)
sys.modules["audio_network_amd"] = A
spec.loader.exec_module(A)
import error_model as EM  # noqa: E402

out = os.path.join(ROOT, "gpurun_out", sys.argv[1] if len(sys.argv) > 1 else "emu")
os.makedirs(out, exist_ok=True)
cases = [c for c in EM.CASES if c[2] == c[3] and c[4] != 2] + [
    ("plain_k3_ws", (1500.0, 2250.0, 3000.0), 1024, 1024, 1)]
W = 256
for name, freqs, n, hop, method in cases:
    x = EM.family("fsk_s400", freqs, n, W, 300)[:W * n]
    with A.Demodulator(A.make_cfg(n=n, hop=hop, freqs=freqs, method=method)) as d:
        _, mag = d.batch(x, n_windows=W, mags=True)
    np.savez(os.path.join(out, name + ".npz"), x=x, mag=mag, freqs=np.asarray(freqs), n=n, method=method)
    print(name, "ok", flush=True)
