import importlib.util, os, sys, numpy as np, torch
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
spec = importlib.util.spec_from_file_location("audio_network_amd", os.path.join(ROOT, "audio-network_amd", "__init__.py"),
    submodule_search_locations=[os.path.join(ROOT, "audio-network_amd")])
A = importlib.util.module_from_spec(spec); sys.modules["audio_network_amd"] = A; spec.loader.exec_module(A)
W, n = 1 << 20, 1024
f8 = A.FSK8_FREQS
d_pcm = torch.empty((W, n), dtype=torch.int16, device="cuda")
A.synth_fsk(A.make_cfg(freqs=f8), 7, W, 8000, 400, d_pcm)
dem = A.Demodulator(freqs=f8)
sym = torch.empty(W, dtype=torch.uint8, device="cuda")
big = torch.empty(W * 8 + (64 << 20), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream()
def run(mag, label, reps=80):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s); dem.batch_async(d_pcm, W, sym, mag, stream=s.cuda_stream); b.record(s)
    torch.cuda.synchronize()
    t = np.array([a.elapsed_time(b) for a, b in ev[20:]]) * 1e3
    print(f"{label:40s} median {np.median(t):6.1f} us", flush=True)
run(None, "no mags")
for off_mb in (0, 1, 3, 16, 37):
    off = (off_mb << 20) // 4
    run(big[off:off + W * 8], f"mags at +{off_mb} MiB")
run(None, "no mags")
sep = torch.empty((W, 8), dtype=torch.float32, device="cuda")
run(sep, "mags separate alloc")
run(d_mag_first := sep, "mags separate alloc (again)")
for rep in range(3):
    other = torch.empty((W, 8), dtype=torch.float32, device="cuda")
    run(other, f"mags fresh alloc {rep}")
