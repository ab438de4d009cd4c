#!/usr/bin/env python3
"""Cost of the decision rescue by detector and signal.

Per (detector, signal): the batch time with the rescue on, off
(FSKD_NO_RESCUE=1) and the number of windows the detector flags
(FSKD_NO_RESCUE=flags leaves bit 7 on them), interleaved medians; the
rescued symbols are checked against the oracle on a sample.

Signals: the bench level (A 8000, sigma 400), a quiet signal (A 20,
sigma 10), pure noise (sigma 2000), two tones of equal amplitude in every
window (every window a near tie), digital silence.

    python scripts/rescue_cost.py [--windows 262144] [--reps 20] [--only fft]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def handle(A, cfg, mode):
    old = os.environ.pop("FSKD_NO_RESCUE", None)
    if mode:
        os.environ["FSKD_NO_RESCUE"] = mode
    try:
        return A.Demodulator(cfg)
    finally:
        os.environ.pop("FSKD_NO_RESCUE", None)
        if old is not None:
            os.environ["FSKD_NO_RESCUE"] = old


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=1 << 18)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="", help="run the detectors whose name contains this")
    args = ap.parse_args()
    import torch
    import bench
    A, _ = bench.load_pkg()
    from oracle import oracle as O
    W, n = args.windows, 1024
    rng = np.random.default_rng(5)
    t = np.arange(W * n, dtype=np.float64)
    f8 = A.FSK8_FREQS
    odd8 = tuple(46.875 * (32 + 9 * i) for i in range(8))
    dets = [("goertzel K=2", A.FSK2_FREQS, A.METHOD_GOERTZEL, n),
            ("fold F16 K=8", f8, A.METHOD_FOLDED, n),
            ("residue K=8", odd8, A.METHOD_RESIDUE, n),
            ("fft hop 256", A.FSK2_FREQS, A.METHOD_FFT, 256)]
    dets = [d for d in dets if args.only in d[0]]
    for name, freqs, method, hop in dets:
        cfg = A.make_cfg(freqs=freqs, method=method, hop=hop)
        sigs = {}
        d_pcm = torch.empty((W, n), dtype=torch.int16, device="cuda")
        A.synth_fsk(cfg, 17, W, 8000, 400, d_pcm)
        sigs["bench A8000 s400"] = d_pcm.clone()
        A.synth_fsk(cfg, 18, W, 20, 10, d_pcm)
        sigs["quiet A20 s10"] = d_pcm.clone()
        A.synth_fsk(cfg, 19, W, 0, 2000, d_pcm)
        sigs["noise s2000"] = d_pcm.clone()
        x = 6000 * (np.sin(2 * np.pi * freqs[0] * t / 48000.0 + 0.3)
                     + np.sin(2 * np.pi * freqs[1] * t / 48000.0 + 1.1))
        x += rng.normal(0, 5, x.size)
        sigs["two equal tones"] = torch.from_numpy(np.clip(np.round(x), -32768, 32767)
                                                   .astype(np.int16).reshape(W, n)).cuda()
        sigs["silence"] = torch.zeros((W, n), dtype=torch.int16, device="cuda")
        del d_pcm
        n_eval = (W * n - n) // hop + 1
        sym = torch.empty(n_eval, dtype=torch.uint8, device="cuda")
        mag = torch.empty((n_eval, len(freqs)), dtype=torch.float32, device="cuda")
        hs = {m: handle(A, cfg, m) for m in ("", "1", "flags")}
        for sname, pcm in sigs.items():
            def run(h):
                h.batch_async(pcm, n_eval, sym, mag)
            times = {"": [], "1": []}
            for _ in range(3):
                run(hs[""]), run(hs["1"])
            torch.cuda.synchronize()
            for r in range(args.reps):
                for m in (("", "1") if r % 2 == 0 else ("1", "")):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    run(hs[m])
                    torch.cuda.synchronize()
                    times[m].append(time.perf_counter() - t0)
            run(hs["flags"])
            torch.cuda.synchronize()
            flagged = int((sym >= 128).sum().item())
            run(hs[""])
            torch.cuda.synchronize()
            # oracle check on the first 2048 windows
            k = min(2048, n_eval)
            flat = pcm.reshape(-1)[:(k - 1) * hop + n].cpu().numpy()
            ref = (O.fft_demod(flat, freqs, n, hop, threads=8)[0] if method == A.METHOD_FFT
                   else O.goertzel(flat, freqs, n, hop, threads=8)[0])
            mism = int((sym[:k].cpu().numpy() != ref).sum())
            on, off = float(np.median(times[""])), float(np.median(times["1"]))
            print(json.dumps({"detector": name, "signal": sname, "windows": n_eval,
                              "flagged": flagged, "flagged_frac": round(flagged / n_eval, 6),
                              "ms_rescue_on": round(on * 1e3, 4), "ms_rescue_off": round(off * 1e3, 4),
                              "cost_frac": round((on - off) / off, 4),
                              "oracle_mismatches_first_2048": mism}), flush=True)
        for h in hs.values():
            h.close()
        del sigs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
