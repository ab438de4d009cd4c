#!/usr/bin/env python3
"""bench.py — Goertzel FSK demodulation throughput on MI355X.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`; for N > 1
launched by torch.distributed.run, one rank per GPU. Rank 0 prints ONE JSON
line.

Workload (BASELINE.json configs[1]): 2-FSK Goertzel on 2^20 windows x 1024
int16 samples (2 GiB) per GPU, resident in HBM before timing. One step = one
demod_batch_async launch over the whole batch (symbols + |X_k|^2 written to
HBM) and, for N > 1, the RCCL all-gather of every rank's decoded symbols
(the only collective of the path). Weak scaling: every rank
demodulates its own 2^20 windows (disjoint slices of one seeded stream).

value = samples demodulated by all ranks / wall time per step (Msamples/s).
roofline = algorithmic bytes per launch (2048 B in + 1 B symbol + 4K B
magnitudes per window) / mean kernel duration from HIP events
recorded on the launch stream, vs the 8 TB/s HBM peak. traffic = HBM bytes per
launch from the committed rocprofv3 PMC summary (profiles/), or null.
cpu_baseline = the oracle's C restatement (OpenMP over the host cores) on a
bounded sample of the same windows (rank 0, N = 1 only), which also re-checks
parity of the timed GPU output on that sample.
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
VALU_PEAK_TFLOPS = 157.3  # MI355X fp32 vector peak (MI355X_MICROARCH.md)
METRIC = "PCM Msamples/s demodulated + symbol-error-rate vs reference, 1/2/4/8 MI355X"
MIN_WARMUP = 64


def load_pkg():
    spec = importlib.util.spec_from_file_location(
        "audio_network_amd", os.path.join(ROOT, "audio-network_amd", "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["audio_network_amd"] = mod
    spec.loader.exec_module(mod)
    spec = importlib.util.spec_from_file_location(
        "audio_network_amd.dist", os.path.join(ROOT, "audio-network_amd", "dist.py"))
    dmod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(dmod)
    return mod, dmod


def pmc_traffic(config: str, windows: int):
    """HBM bytes per launch from profiles/pmc_<config>.json (rocprofv3 PMC)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        if int(d.get("windows", -1)) != windows:
            return None
        return float(d["hbm_bytes_per_launch"])
    except Exception:
        return None


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(A, d_pcm, d_sym, d_mag, freqs, seconds: float, threads: int, fft: bool,
                 hop: int):
    """Oracle (C, OpenMP) on a bounded sample of the timed windows: the first
    S stream windows (Goertzel) or the FFT windows over the first S*n samples."""
    sys.path.insert(0, ROOT)
    from oracle import oracle as O

    n = 1024
    S = min(d_pcm.shape[0], 4096 if fft else 65536)
    flat = d_pcm[:S].cpu().numpy().reshape(-1)
    n_win = (S * n - n) // hop + 1
    gsym = d_sym[:n_win].cpu().numpy()
    gmag = d_mag[:n_win].cpu().numpy().astype(np.float64) if d_mag is not None else None

    def run():
        if fft:
            return O.fft_demod(flat, freqs, n, hop, threads=threads)
        return O.goertzel(flat, freqs, n, hop, threads=threads)

    def timed(fn, budget):
        passes, t0 = 0, time.perf_counter()
        while True:
            fn()
            passes += 1
            el = time.perf_counter() - t0
            if el >= budget:
                return passes, el

    sym, P = run()  # warm + parity reference
    passes, el = timed(run, seconds)
    msps = passes * S * n / el / 1e6
    # single-thread rate on a slice of the same sample (SURVEY §8d asks for both)
    S1 = max(1, S // 16)
    flat1 = flat[:S1 * n]
    fn1 = ((lambda: O.fft_demod(flat1, freqs, n, hop, threads=1)) if fft else
           (lambda: O.goertzel(flat1, freqs, n, hop, threads=1)))
    p1, el1 = timed(fn1, max(1.0, seconds / 5))
    msps1 = p1 * S1 * n / el1 / 1e6
    # ... and the fp32 variant of the scalar recurrence, hop = n only
    msps1_f32 = None
    if not fft and hop == n:
        pf, elf = timed(lambda: O.goertzel_f32(flat1, freqs, n), max(1.0, seconds / 5))
        msps1_f32 = round(pf * S1 * n / elf / 1e6, 3)
    parity = {"windows_checked": int(n_win), "symbol_mismatches": int((sym != gsym).sum())}
    if gmag is not None:
        parity["max_rel_mag_err"] = float((np.abs(gmag - P).max(1) / P.max(1)).max())
    what = ("double radix-2 FFT, argmax over tone bins" if fft else "double Goertzel")
    base = {"value": round(msps, 3), "unit": "Msamples/s", "cores": int(threads),
            "kind": "port", "single_thread_value": round(msps1, 3),
            "single_thread_fp32_value": msps1_f32,
            "host_cpu": cpu_model(), "host_cpus_visible": os.cpu_count(),
            "sample": f"first {S * n} samples ({n_win} windows, hop {hop}) of the timed batch, "
                      f"{passes} passes in {el:.1f} s, oracle/fsk_oracle.c {what}, OpenMP"}
    return base, parity


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=["fsk2", "fsk8", "fft", "streams"], default="fsk2",
                    help="fsk2 = configs[1] (default), fsk8 = configs[2], fft = configs[3]: "
                         "sliding 1024-pt full-spectrum FFT (hop --hop) over the same stream, "
                         "streams = configs[4]: 1024 streams x 2048 windows sharded over ranks "
                         "(strong scaling)")
    ap.add_argument("--hop", type=int, default=256, help="window advance for --config fft")
    ap.add_argument("--windows", type=int, default=1 << 20, help="windows per GPU (fsk2/fsk8)")
    ap.add_argument("--no-mags", action="store_true", help="symbols only")
    ap.add_argument("--method", choices=["auto", "goertzel", "folded", "residue"], default="auto")
    ap.add_argument("--plan", choices=["survey", "odd"], default="survey",
                    help="fsk8 tone plan: survey = SURVEY §8 (1500 + 375 i Hz, multiples of 8 "
                         "bins), odd = integer bins 32 + 9 i (every residue class mod 8: the "
                         "generic integer-bin path, DESIGN.md §4.3)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (= RCCL over xGMI) on the real node; gloo only to rehearse the "
                         "multi-rank path with several ranks sharing one GPU")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    if args.dist_backend == "gloo":
        local = local % torch.cuda.device_count()  # rehearsal: ranks may share a GPU
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    A, D = load_pkg()
    freqs = A.FSK8_FREQS if args.config == "fsk8" else A.FSK2_FREQS
    if args.config == "fsk8" and args.plan == "odd":
        freqs = tuple(46.875 * (32 + 9 * i) for i in range(8))
    K = len(freqs)
    n = 1024
    method = {"auto": A.METHOD_AUTO, "goertzel": A.METHOD_GOERTZEL,
              "folded": A.METHOD_FOLDED, "residue": A.METHOD_RESIDUE}[args.method]
    hop = n
    if args.config == "fft":
        method, hop = A.METHOD_FFT, int(args.hop)
    if args.config == "streams":
        # config 5: 1024 independent streams x 2^21 samples (2048 windows each);
        # rank r demodulates the contiguous stream shard D.shard_range(1024, r, N)
        n_streams, wps = 1024, 2048
        s_first, s_count = D.shard_range(n_streams, rank, world)
        W, w0, total_windows = s_count * wps, s_first * wps, n_streams * wps
    else:
        W = int(args.windows)
        w0, total_windows = rank * W, world * W
    # windows the detector evaluates over the rank's W x n-sample stream slice
    n_eval = (W * n - n) // hop + 1
    cfg = A.make_cfg(freqs=freqs, n=n, hop=hop, device=local, method=method)
    dev = torch.device("cuda", local)
    d_pcm = torch.empty((W, n), dtype=torch.int16, device=dev)
    d_true = torch.empty(W, dtype=torch.uint8, device=dev)
    d_sym = torch.empty(n_eval, dtype=torch.uint8, device=dev)
    d_mag = None if args.no_mags else torch.empty((n_eval, K), dtype=torch.float32, device=dev)
    A.synth_fsk(cfg, A.BENCH_SEED, W, 8000, 400, d_pcm, d_true, w0=w0)
    torch.cuda.synchronize()
    demod = A.Demodulator(cfg)
    main = torch.cuda.current_stream()
    gunits, gunit = (n_streams, wps) if args.config == "streams" else (world, W)
    # N > 1: kernels run on a compute stream into double-buffered symbol slots;
    # the RCCL gather of step t-1's symbols is issued on the default stream
    # (waiting only for step t-1's kernel) and so overlaps step t's kernel.
    comp = torch.cuda.Stream(device=dev) if world > 1 else main
    slots = [d_sym, torch.empty_like(d_sym)] if world > 1 else [d_sym]
    # config 5: every rank frames its own streams on the device (one
    # ToReceiver run per stream, demod_frame_streams_async) and RCCL gathers
    # the frames; the other configs gather symbols and rank 0 frames them.
    dev_framing = args.config == "streams"
    if dev_framing:
        bits = A.bits_per_symbol(K)
        fstride = A.frame_symbols_size(wps, bits)
        fslots = [torch.empty(max(s_count * fstride, 1), dtype=torch.uint8, device=dev)
                  for _ in slots]
    kdone = [torch.cuda.Event() for _ in slots]   # kernel wrote the slot
    gdone = [torch.cuda.Event() for _ in slots]   # gather finished reading the slot
    st = {"i": 0, "prev": None, "used": [False] * len(slots)}

    def gather(slot):
        main.wait_event(kdone[slot])
        if dev_framing:
            out = D.gather_symbols(fslots[slot][:s_count * fstride], gunits, world, unit=fstride)
        else:
            out = D.gather_symbols(slots[slot], gunits, world, unit=gunit)
        gdone[slot].record(main)
        return out

    def step(ev=None):
        slot = st["i"] % len(slots)
        st["i"] += 1
        if st["used"][slot]:
            comp.wait_event(gdone[slot])
        if ev is not None:
            ev[0].record(comp)
        demod.batch_async(d_pcm, n_eval, slots[slot], d_mag, stream=comp.cuda_stream)
        if ev is not None:
            ev[1].record(comp)
        if dev_framing:
            A.frame_streams_async(slots[slot], s_count, wps, bits, fslots[slot],
                                  stream=comp.cuda_stream)
        out = None
        if world > 1:
            kdone[slot].record(comp)
            if st["prev"] is not None:
                out = gather(st["prev"])
            st["prev"] = slot
            st["used"][slot] = True
        return out

    def flush():
        out = None
        if world > 1 and st["prev"] is not None:
            out = gather(st["prev"])
            st["prev"] = None
        return out

    # Sustained HBM streaming shows a power-management transient: launch
    # times rise ~25 % after ~10 launches and settle back by ~60 (dispatch
    # series in profiles/round1/). Warm up for at least
    # MIN_WARMUP launches so the K timed steps see the steady state.
    warmup = max(args.warmup, MIN_WARMUP)
    for _ in range(warmup):
        step()
    flush()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(evs[i])
    all_sym = flush()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kts = np.array([a.elapsed_time(b) for a, b in evs])
    kernel_ms = float(kts.mean())
    ms_per_step = elapsed / args.steps * 1e3

    # Practical read ceiling of this box for the same access pattern: the
    # read-only reference stream (8 KiB per wave, 16 B/lane nt loads, no
    # compute; demod_read_ceiling_async) over the same input buffer, after the
    # timed region, median of 20 launches (HIP events on the launch stream).
    ceil_gbps = None
    if args.config != "fft":
        nb = (d_pcm.numel() * 2) // 8192 * 8192
        cev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
               for _ in range(20)]
        for _ in range(8):
            A.read_ceiling_async(d_pcm, nb, stream=comp.cuda_stream)
        for a, b in cev:
            a.record(comp)
            A.read_ceiling_async(d_pcm, nb, stream=comp.cuda_stream)
            b.record(comp)
        torch.cuda.synchronize()
        ceil_gbps = nb / (float(np.median([a.elapsed_time(b) for a, b in cev])) / 1e3) / 1e9

    # correctness of the timed output: every symbol vs the transmitted one
    # (sliding windows straddle two symbols: compare the aligned ones only)
    d_sym = slots[(st["i"] - 1) % len(slots)]
    if hop == n:
        sym_err = int((d_sym != d_true).sum().item())
    else:
        step_w = n // hop
        sym_err = int((d_sym[::step_w][:W] != d_true).sum().item())
    framed = None
    if dev_framing:
        # frames of the last step: gathered (N > 1) or this rank's own (N = 1)
        frames = all_sym if world > 1 else fslots[(st["i"] - 1) % len(slots)][:s_count * fstride]
        all_true = D.gather_symbols(d_true, gunits, world, unit=gunit) if world > 1 else d_true
        if rank == 0:
            fb = frames.cpu().numpy()
            back = np.concatenate([D.unframe_symbols(A, fb[i * fstride:(i + 1) * fstride].tobytes(),
                                                     wps, K) for i in range(gunits)])
            sym_err = int((back != all_true.cpu().numpy()).sum())
            framed = {"frames_bytes": int(fb.size), "frame_bytes_per_stream": fstride,
                      "bits_per_symbol": bits, "framing": "device (demod_frame_streams_async)",
                      "gathered": "frames" if world > 1 else "n/a (1 rank)",
                      "roundtrip_ok": sym_err == 0}
    elif world > 1:
        all_true = D.gather_symbols(d_true, gunits, world, unit=gunit)
        sym_err = int((all_sym != all_true).sum().item())
        if rank == 0:
            # rank 0 frames the gathered symbols as ip.proto ToReceiver messages
            stream_bytes = D.frame_symbols(A, all_sym.cpu().numpy(), K)
            back = D.unframe_symbols(A, stream_bytes, all_sym.numel(), K)
            framed = {"frames_bytes": len(stream_bytes), "bits_per_symbol": A.bits_per_symbol(K),
                      "roundtrip_ok": bool((back == all_sym.cpu().numpy()).all())}

    if rank == 0:
        samples = total_windows * n  # stream samples demodulated (each counted once)
        value = samples / (ms_per_step / 1e3) / 1e6
        alg_bytes = W * 2 * n + n_eval * (1 + (0 if args.no_mags else 4 * K))
        achieved = alg_bytes / (kernel_ms / 1e3) / 1e9
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_effective": warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.config == "streams" else "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (seeded splitmix64 FSK, A=8000, Irwin-Hall noise sigma=400)",
            "config": {
                "workload": ("configs[4]: 1024 streams x 2048 windows (2^21 samples each), "
                             f"sharded by stream over {world} GPU(s), 2-FSK"
                             if args.config == "streams" else
                             f"configs[3]: sliding 1024-pt full-spectrum FFT, hop {hop}, "
                             f"{n_eval} windows over a {W * n}-sample int16 stream per GPU"
                             if args.config == "fft" else
                             ("configs[1]: 2-FSK" if K == 2 else
                              "configs[2]: 8-FSK" + (" (integer bins 32 + 9 i)" if args.plan == "odd"
                                                     else ""))
                             + f" Goertzel, {W} x {n}-sample int16 windows per GPU, HBM-resident"),
                "tones_hz": list(freqs),
                "windows_per_gpu": n_eval,
                "hop": hop,
                "n": n,
                "outputs": "symbols" + ("" if args.no_mags else " + |X_k|^2"),
                "parallelism": (f"dp{world} (stream shards; per-rank device framing, RCCL "
                                "all-gather of ToReceiver frames)" if dev_framing else
                                f"dp{world} (independent window shards, RCCL symbol all-gather)"),
            },
            "detector": {A.METHOD_GOERTZEL: "goertzel", A.METHOD_FOLDED: "folded",
                         A.METHOD_RESIDUE: "residue",
                         A.METHOD_FFT: "fft1024"}.get(demod.method, str(demod.method)),
            "kernel_ms_p10_p50_p90": [round(float(np.percentile(kts, q)), 4) for q in (10, 50, 90)],
            "symbol_errors": sym_err,
            "symbol_error_rate": sym_err / float(total_windows),
            "kernel_ms": round(kernel_ms, 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": pmc_traffic(args.config if args.plan == "survey" else "fsk8odd", W),
                "alg_bytes_per_launch": alg_bytes,
                # this box's read-only ceiling for the same access pattern
                # (see above) and the kernel's achieved rate as a fraction of it
                "read_ceiling": round(ceil_gbps, 1) if ceil_gbps else None,
                "frac_of_read_ceiling": round(achieved / ceil_gbps, 4) if ceil_gbps else None,
                "kernel": ("fft1024_quad_kernel<4>" if demod.method == A.METHOD_FFT else
                           ("fold_tile_kernel<%d,4>" if demod.method == A.METHOD_FOLDED
                            else "residue_tile_kernel<%d,4>" if demod.method == A.METHOD_RESIDUE
                            else "goertzel_tile_kernel<%d,4>") % K),
            },
        }
        if args.config == "fft":
            # the FFT is reported against the VALU roof too.
            # Algorithmic flops per window: 2.5 N log2 N for the real N-point
            # FFT + 3 per |X[b]|^2 over the N/2+1 bins.
            fpw = 2.5 * n * 10 + 3 * (n // 2 + 1)
            tf = fpw * n_eval / (kernel_ms / 1e3) / 1e12
            out["roofline_valu"] = {"bound": "valu", "achieved": round(tf, 2),
                                    "peak": VALU_PEAK_TFLOPS, "unit": "TFLOP/s",
                                    "frac": round(tf / VALU_PEAK_TFLOPS, 4),
                                    "flop_per_window": fpw}
        if framed:
            out["framing"] = framed
        if world == 1 and not args.no_cpu_baseline:
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            base, parity = cpu_baseline(A, d_pcm, d_sym, d_mag, freqs, args.cpu_seconds, threads,
                                        args.config == "fft", hop)
            out["cpu_baseline"] = base
            out["parity_sample"] = parity
        print(json.dumps(out), flush=True)
    demod.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
