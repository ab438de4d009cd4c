"""configs[4] on the GPU with a real RCCL collective.

The full config-5 workload — 1024 independent streams x 2048 windows
(2^21 windows, 4 GiB of int16 PCM) — through the path every rank of the
8-GPU run takes: demod_batch_async -> demod_frame_streams_async (device
framing of one ToReceiver run per stream) -> dist.gather_symbols
(all_gather_into_tensor under the "nccl" backend, i.e. RCCL) of the frames,
overlapped with the next step's kernel. It runs as bench.py --config streams
--force-dist in a child process, so torch.distributed is initialised (nccl,
world_size 1, tcp://127.0.0.1) before any other GPU work of that process.
Checks: every gathered frame decodes to the transmitted symbols of all 1024
streams, a 65536-window sample equals the oracle bit-for-bit, and the per-step
overhead above the detector kernel (frame kernel, gather, launch) is reported.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config5_streams_rccl_gather_world1():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU visible")
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("MASTER_PORT", None)
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--config", "streams",
                        "--force-dist", "--dist-backend", "nccl", "--steps", "20", "--warmup", "5",
                        "--cpu-seconds", "2"],
                       capture_output=True, timeout=400, cwd=ROOT, env=env)
    out = r.stdout.decode()
    assert r.returncode == 0, (out[-2000:], r.stderr.decode()[-4000:])
    line = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
    print("\n" + json.dumps({k: line.get(k) for k in ("ms_per_step", "kernel_ms", "overhead",
                                                      "framing", "symbol_errors")}))
    assert line["config"]["windows_per_gpu"] == 1024 * 2048
    assert line["symbol_errors"] == 0
    fr = line["framing"]
    assert fr["roundtrip_ok"] and "RCCL" in fr["gathered"]
    assert fr["frames_bytes"] == 1024 * fr["frame_bytes_per_stream"]
    ov = line["overhead"]
    assert ov["frame_kernel_ms"] is not None and ov["gather_ms"] is not None
    ps = line["parity_sample"]
    assert ps["symbol_mismatches"] == 0 and ps["max_rel_mag_err"] <= 1e-5
