"""CPU checks of bench.py's reporting helpers and of the decision checker the
GPU parity tests rely on (tests/decision.py): no GPU, no compute calls."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from decision import BAND, check_decisions

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_margin_stats_histogram():
    P = np.array([[1.0, 0.0], [1.0, 1.0 - 1e-7], [1.0, 0.5], [2.0, 2.0 - 4e-5], [3.0, 2.9]])
    m = bench.margin_stats(P)
    assert m["windows"] == 5 and sum(m["hist_counts"]) == 5
    assert m["min_margin"] == pytest.approx(1e-7, rel=1e-6)
    assert m["below_4e-5"] == 2
    # bins [0,1e-6) [1e-6,1e-5) [1e-5,1e-4) [1e-4,1e-3) [1e-3,1e-2) [1e-2,1e-1) [1e-1,1]
    assert m["hist_counts"] == [1, 0, 1, 0, 0, 1, 2]
    assert bench.margin_stats(np.ones((4, 1))) == {}


def test_cpu_share_is_sane():
    visible, affinity, quota, threads, why = bench.cpu_share()
    assert 1 <= threads <= affinity <= visible
    assert quota is None or threads >= 1
    assert isinstance(why, str) and why


def test_pmc_traffic_matches_config_and_hop():
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_fsk2.json")))
    W = int(d["windows"])
    assert bench.pmc_traffic("fsk2", W) == pytest.approx(d["hbm_bytes_per_launch"])
    assert bench.pmc_traffic("fsk2", W + 1) is None          # other workload size
    assert bench.pmc_traffic("fsk2", W, hop=256) is None     # other hop
    assert bench.pmc_traffic("no_such_config", W) is None
    f = json.load(open(os.path.join(ROOT, "profiles", "pmc_fft.json")))
    assert f["hop"] == 256
    assert bench.pmc_traffic("fft", int(f["windows"]), hop=256) == pytest.approx(f["hbm_bytes_per_launch"])
    # every traffic file is within a few % of its algorithmic bytes
    for name in ("fsk2", "fsk8", "fsk8odd", "fft", "fft1024"):
        t = json.load(open(os.path.join(ROOT, "profiles", f"pmc_{name}.json")))
        assert 0.99 < t["traffic_over_alg"] < 1.1, name


def test_bench_help_lists_the_contract_flags():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, timeout=120, cwd=ROOT)
    out = r.stdout.decode()
    assert r.returncode == 0
    for flag in ("--gpus", "--steps", "--warmup", "--config", "--dist-backend", "--no-extras"):
        assert flag in out


def test_decision_checker_requires_the_oracle_symbol_everywhere():
    ref_P = np.array([[10.0, 1.0], [1.0, 10.0], [5.0, 5.0 * (1 - BAND / 2)], [0.0, 0.0]])
    ref_sym = ref_P.argmax(axis=1)
    mag = ref_P.astype(np.float32).copy()
    sym = mag.argmax(axis=1)
    assert check_decisions(sym, mag, ref_sym, ref_P) == 2      # the near tie and the zero window
    # a near tie the fp32 powers resolve the other way is a mismatch: the
    # rescue must have decided it in double
    mag2 = mag.copy()
    mag2[2] = [4.9999, 5.0]
    with pytest.raises(AssertionError):
        check_decisions(mag2.argmax(axis=1), mag2, ref_sym, ref_P)
    # a rescued window: double decision, fp32-rounded powers tied
    ref3 = np.array([[1.0 + 2e-9, 1.0]])
    assert check_decisions(np.array([0]), ref3.astype(np.float32), np.array([0]), ref3) == 1
    # ... but never a leftover ambiguous flag
    with pytest.raises(AssertionError):
        check_decisions(np.array([0x80]), None, np.array([0]), ref3)


def test_decision_checker_silence_exemption_needs_the_energy_scale():
    ref_P = np.array([[1e-16, 3e-16]])                         # rounding noise of a zero tone content
    mag = np.zeros((1, 2), np.float32)
    with pytest.raises(AssertionError):
        check_decisions(np.array([0]), mag, np.array([1]), ref_P)
    assert check_decisions(np.array([0]), mag, np.array([1]), ref_P, denom=np.array([1e9])) == 1


def test_decision_checker_rejects_wrong_decisions():
    ref_P = np.array([[10.0, 1.0], [1.0, 10.0]])
    ref_sym = ref_P.argmax(axis=1)
    mag = ref_P.astype(np.float32)
    with pytest.raises(AssertionError):                        # not the argmax of its own powers
        check_decisions(np.array([1, 1]), mag, ref_sym, ref_P)
    bad = mag[:, ::-1].copy()
    with pytest.raises(AssertionError):                        # differs from the oracle
        check_decisions(bad.argmax(axis=1), bad, ref_sym, ref_P)


def test_world_size_must_match_gpus():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"],
                       capture_output=True, timeout=120, cwd=ROOT, env=env)
    assert r.returncode == 2 and b"WORLD_SIZE=2" in r.stderr


def test_gpus_n_self_launches_torchrun(monkeypatch):
    """--gpus N > 1 without WORLD_SIZE starts torch.distributed.run as a child
    (before any GPU call) with N ranks on 127.0.0.1 and the same arguments."""
    calls = []
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd, env=None: calls.append(cmd) or 0)
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0 and len(calls) == 1
    cmd = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"]


def test_parity_all_counts_against_the_oracle():
    """bench.parity_all (CPU tensors standing in for device ones): the oracle's
    own output checks clean, a changed symbol, a leftover flag bit and a
    perturbed power are each counted; the strided sample reads the right
    windows."""
    import torch
    from oracle import oracle as O
    f = (1500.0, 3000.0)
    pcm, _ = O.synth_fsk(f, 1024, 96, 11, 8000, 400)
    sym, P = O.goertzel(pcm, f, 1024)
    d_pcm = torch.from_numpy(pcm.copy())
    mag = torch.from_numpy(P.astype(np.float32))
    out = bench.parity_all(d_pcm, torch.from_numpy(sym.copy()), mag, f, 1024, 1024, False, chunk=40)
    assert out["windows_checked"] == 96 and out["symbol_mismatches"] == 0
    assert out["flag_bits_left"] == 0 and out["windows_above_1e-5_of_max_P"] == 0
    bad = sym.copy()
    bad[5] ^= 1
    bad[70] |= 0x80
    mag[33, int(np.argmax(P[33]))] *= 1.001
    out = bench.parity_all(d_pcm, torch.from_numpy(bad), mag, f, 1024, 1024, False, chunk=40)
    assert out["symbol_mismatches"] == 2 and out["flag_bits_left"] == 1
    assert out["windows_above_1e-5_of_max_P"] == 1
    flat = pcm.reshape(-1)
    s2, P2 = O.fft_demod(flat, f, 1024, 256)
    out = bench.parity_all(torch.from_numpy(flat.copy()), torch.from_numpy(s2.copy()),
                           torch.from_numpy(P2.astype(np.float32)), f, 1024, 256, True, every=9, chunk=7)
    assert out["windows_checked"] == len(range(0, s2.size, 9)) and out["symbol_mismatches"] == 0


def _watchdog_run(code):
    return subprocess.run([sys.executable, "-c", f"import sys; sys.path.insert(0, {ROOT!r}); "
                           "import bench, time; " + code],
                          capture_output=True, text=True, timeout=60)


def test_extras_watchdog_prints_headline_and_exits_nonzero():
    """N > 1: a hung extra measurement ends at the watchdog's deadline with rank
    0's headline line printed (the extra marked) and the process exiting
    non-zero (VERDICT r3 weak 5 iii: a hung collective must not look like
    success)."""
    r = _watchdog_run("bench.extras_watchdog(lambda: {'value': 1.5, 'streams': {'error': 't'}}, 0, 0.3); "
                      "time.sleep(30)")
    assert r.returncode == 3 and "watchdog" in r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["value"] == 1.5 and line["extra_keys"] == ["streams"]
    # other ranks exit without printing
    r = _watchdog_run("bench.extras_watchdog(lambda: {'value': 1.5}, 1, 0.3); time.sleep(30)")
    assert r.returncode == 3 and r.stdout.strip() == ""


def test_extras_watchdog_disarmed_stays_silent():
    r = _watchdog_run("e = bench.extras_watchdog(lambda: {'value': 1.5}, 0, 0.5); e.set(); "
                      "time.sleep(1.0); print('main done')")
    assert r.returncode == 0 and r.stdout.strip() == "main done"


def test_extras_watchdog_after_the_line_only_exits():
    """A teardown that hangs after rank 0 printed its line: the watchdog ends
    the process without a second line, non-zero."""
    r = _watchdog_run("e = bench.extras_watchdog(lambda: {'value': 1.5}, 0, 0.5); e.printed = True; "
                      "print('{\"value\": 2.0}', flush=True); time.sleep(30)")
    assert r.returncode == 3 and r.stdout.strip().splitlines() == ['{"value": 2.0}']


def test_implied_magnitude_bounds_per_shipped_config():
    """the magnitude bound the derived error model implies
    on an aligned window, per shipped configuration. configs[2] (fold F16) and
    configs[3] (the FFT) are proven within north_star's 1e-5; configs[1] under
    AUTO (the plain bank) is not (~7e-5: its bar is measured, parity_all), and
    DEMOD_METHOD_FOLDED proves it on the same plan."""
    A = bench.load_pkg()[0]
    b = bench.implied_mag_bounds(A)
    for key in ("configs[2]", "configs[3]_fsk2_hop256", "configs[3]_fsk8_hop256",
                "configs[1]_method_folded"):
        assert b[key]["within_1e-5"] and b[key]["bound"] <= 1e-5, (key, b[key])
    assert b["configs[1]"]["detector"] == "goertzel" and not b["configs[1]"]["within_1e-5"]
    assert 5e-5 < b["configs[1]"]["bound"] < 1e-4
    assert b["configs[1]_method_folded"]["detector"] == "folded"
    assert "MEASURED" in b["note"]


def test_settle_warmup_waits_out_a_transient(monkeypatch):
    """bench.settle_warmup (round 6): untimed chunks until two consecutive
    chunks agree within 1 % and the last is within 3 % of the fastest; a
    transient (slow chunks after fast ones) is waited out, a steady device
    stops after two chunks, and the cap bounds a device that never settles.
    A fake clock advances by each step's scheduled time (deterministic)."""
    clock = [0.0]

    class FakeCuda:
        @staticmethod
        def synchronize():
            pass

    class FakeTorch:
        cuda = FakeCuda

    class FakeTime:
        @staticmethod
        def perf_counter():
            return clock[0]

    monkeypatch.setattr(bench, "time", FakeTime)

    def make(schedule):
        it = iter(schedule)

        def fn():
            clock[0] += next(it, schedule[-1]) * 1e-3
        return fn
    chunk = 4
    n, times = bench.settle_warmup(FakeTorch, make([2.0] * 400), chunk=chunk)
    assert n == 2 * chunk and times == [2.0, 2.0]
    # fast, then a transient 30 % slower for 5 chunks, then back
    sched = [2.0] * chunk + [2.6] * (5 * chunk) + [2.0] * 400
    n, times = bench.settle_warmup(FakeTorch, make(sched), chunk=chunk)
    assert n == 8 * chunk and times[-2:] == [2.0, 2.0], times
    # a ramp down from a high start settles once it flattens at the floor
    sched = [3.0] * chunk + [2.5] * chunk + [2.05] * chunk + [2.0] * 400
    n, times = bench.settle_warmup(FakeTorch, make(sched), chunk=chunk)
    assert times[-1] == 2.0 and n == 5 * chunk, times
    # never settles: alternating chunks, capped
    alt = ([2.0] * chunk + [3.0] * chunk) * 50
    n, times = bench.settle_warmup(FakeTorch, make(alt), chunk=chunk, max_chunks=6)
    assert n == 6 * chunk and len(times) == 6
