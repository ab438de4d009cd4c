"""configs[0]: the native host C test (tests/native/config1.c) — one 1024-sample
2-FSK buffer through the oracle, the C ABI and the frame codec."""
import fcntl
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
NATIVE = os.path.join(HERE, "native")


def _make(*targets):
    """make under an exclusive lock: xdist workers share tests/native/."""
    with open(os.path.join(NATIVE, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", NATIVE, "-s", *targets], check=True, capture_output=True)


def _build_and_run():
    _make()
    return subprocess.run([os.path.join(NATIVE, "config1")], capture_output=True, text=True,
                          timeout=120)


def test_config1_native_host_build():
    r = _build_and_run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "config1 OK" in r.stdout


@pytest.mark.gpu
def test_config1_native_gpu_branch():
    r = _build_and_run()
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu demodulate: symbol" in r.stdout
    assert "gpu demod_streams_push: 3 streams OK" in r.stdout


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_wire_codecs_under_sanitizers(seed):
    """The ABI's byte codecs (csrc/demod_frame.c, csrc/demod_session.c: what
    fskrx parses off the network) built with AddressSanitizer + UBSan and
    fuzzed on exact-size buffers (tests/native/fuzz_wire.c): round trips at
    every payload size, truncations, mutations, random bytes; any read past
    an input or undefined behaviour aborts the run."""
    _make("fuzz_wire")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(NATIVE, "fuzz_wire"), "200000", str(seed)],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fuzz_wire OK" in r.stdout


def test_group_shard_and_padding_arithmetic():
    """The multi-GPU group's shard and padding arithmetic through the C ABI
    (tests/native/group_arith.c): shards contiguous,
    balanced and covering every stream once; a bucket's gathered block holds
    every rank's frames; bad arguments refused. No device needed."""
    _make("group_arith")
    r = subprocess.run([os.path.join(NATIVE, "group_arith")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "group arithmetic OK" in r.stdout


@pytest.mark.gpu
def test_group_world1_push_equals_streams_push_native():
    """The same C program on the GPU: a world-1 RCCL group's pushes equal
    demod_streams_push byte for byte (stereo-free mono, lead-in, ragged
    packets, a too-small buffer refused before anything is consumed)."""
    _make("group_arith")
    r = subprocess.run([os.path.join(NATIVE, "group_arith")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "gpu demod_group_push: world 1 equals demod_streams_push" in r.stdout


def test_group_agreement_protocol_over_threads():
    """demod_group_push's agreement protocol (csrc/group_flow.h, VERDICT r5
    item 1) run over threads with injected failures (tests/native/
    group_flow_test.cpp, ASan + UBSan): a refusal on any rank (arguments, cap,
    NULL symbols, total > INT_MAX) returns the lowest failing rank's code on
    every rank with no push anywhere; a failed push returns its code on every
    rank and kills the group; a dead peer ends every other rank at the deadline
    (DEMOD_DEVICE_ERROR), never a hang; 300 random fault plans agree."""
    _make("group_flow_test")
    r = subprocess.run([os.path.join(NATIVE, "group_flow_test")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "group flow OK" in r.stdout


def test_rescue_bounds_checking_build_compiles(tmp_path):
    """the bounds-checking build of the rescue launch
    (FSKD_BOUNDS_DEBUG: RS_CHECK reports and clamps an out-of-range index,
    the instrument that found round 5's dense-run fault) stays buildable for
    gfx950."""
    import shutil
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    csrc = os.path.join(os.path.dirname(HERE), "audio-network_amd", "csrc")
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-mcode-object-version=5", "-I" + os.path.join(os.path.dirname(HERE), "include"),
                        "-DFSKD_BOUNDS_DEBUG", "-c", os.path.join(csrc, "rescue.hip"),
                        "-o", str(tmp_path / "rescue_dbg.o")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
