"""The C-ABI library loads and exports what include/demod.h declares.

No compute calls here (CPU container): argument validation happens before any
device work, and without a GPU demod_create must fail loudly with
DEMOD_NO_DEVICE — there is no CPU fallback.
"""
import ctypes
import subprocess

import pytest


def test_library_exports_every_header_symbol(A):
    lib = A.load_library()
    declared = A.header_exports()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", A.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    assert set(declared) <= exported


def test_library_targets_gfx950_only(A):
    """The embedded code objects are gfx950 and nothing else."""
    import re
    blob = open(A.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa-+(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets


def test_cfg_struct_layout(A):
    assert ctypes.sizeof(A.DemodCfg) == 8 + 4 * 8 + 8 * 16
    cfg = A.make_cfg()
    assert cfg.n == 1024 and cfg.hop == 1024 and cfg.k == 2 and cfg.fs == 48000.0
    assert tuple(cfg.freqs[:2]) == (1500.0, 3000.0)


@pytest.mark.parametrize("bad", [
    dict(n=1000), dict(n=32), dict(n=8192), dict(hop=0), dict(hop=12), dict(hop=2048),
    dict(channels=3), dict(freqs=()), dict(freqs=(30000.0,)), dict(freqs=(-1.0,)),
    dict(fs=0.0), dict(channels=2, channel_mode=5),
    dict(method=3, freqs=(1500.0, 1546.875)),        # FOLDED needs multiples of 8 bins
    dict(method=3, freqs=(1000.0,)),                  # non-integer bin
])
def test_create_rejects_bad_config(A, bad):
    kw = dict(bad)
    with pytest.raises(A.DemodError) as e:
        A.Demodulator(**kw)
    assert e.value.code == A.DEMOD_BAD_ARG


def test_fft_detector_needs_n1024(A):
    with pytest.raises(A.DemodError) as e:
        A.Demodulator(n=512, method=A.METHOD_FFT)
    assert e.value.code == A.DEMOD_UNIMPLEMENTED


def test_create_without_gpu_fails_loudly(A):
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(A.DemodError) as e:
        A.Demodulator()
    assert e.value.code == A.DEMOD_NO_DEVICE


def test_strerror_and_version(A):
    assert A.strerror(A.DEMOD_NO_DEVICE).startswith("no gfx950")
    assert A.strerror(12345) == "unknown error"
    assert "gfx950" in A.version_string()


def test_integration_doc_maps_every_export(A):
    """INTEGRATION.md §1 names every entry point include/demod.h declares
    (mapped to the reference interface it replaces, or marked as having none)."""
    import os
    doc = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "INTEGRATION.md")).read()
    missing = [n for n in A.header_exports() if n not in doc]
    assert not missing, missing


def test_lead_in_field_and_validation(A):
    """demod_cfg_t.lead_in replaced round 1's `reserved` (same offset): the
    Opus decoder delay the streaming entry drops; values >= 2^31 are rejected
    before any device work."""
    assert A.DemodCfg.lead_in.offset == 8 + 7 * 4 and A.DEMOD_OPUS_LOOKAHEAD == 312
    cfg = A.make_cfg(lead_in=A.DEMOD_OPUS_LOOKAHEAD)
    assert cfg.lead_in == 312
    bad = A.make_cfg()
    bad.lead_in = 0x80000000
    with pytest.raises(A.DemodError) as e:
        A.Demodulator(bad)
    assert e.value.code == A.DEMOD_BAD_ARG


def test_device_tensor_checks(A):
    """The Python mirror validates tensors before handing raw pointers to the
    C ABI (a short / strided / wrong-dtype / host tensor would otherwise be an
    out-of-bounds device access): DemodError(DEMOD_BAD_ARG), no GPU needed."""
    torch = pytest.importorskip("torch")
    chk = A._check_dev
    ok_shape = torch.zeros(4, dtype=torch.int16)
    for t, dtype, need in [
        (torch.zeros(4, dtype=torch.int32), "int16", 4),          # dtype
        (torch.zeros(3, dtype=torch.int16), "int16", 4),          # too short
        (torch.zeros(8, dtype=torch.int16)[::2], "int16", 4),     # strided
        (ok_shape, "int16", 4),                                   # host tensor
        (12345, "int16", 4),                                      # raw address
        (None, "uint8", 4),                                       # missing
    ]:
        with pytest.raises(A.DemodError) as e:
            chk(t, "x", dtype, need, 0)
        assert e.value.code == A.DEMOD_BAD_ARG
    chk(None, "mags", "float32", 10, 0, nullable=True)
    with pytest.raises(A.DemodError):
        A.frame_streams_async(torch.zeros(10, dtype=torch.uint8), 2, 5, 1,
                              torch.zeros(1, dtype=torch.uint8))


def test_batch_launches_matches_the_split_rule(A):
    """demod_batch_launches without a GPU is only reachable through a handle,
    which needs a device; the rule itself is checked on the GPU
    (test_gpu_parity.py::test_batch_launch_slices) - here: the export exists
    and rejects a NULL handle."""
    lib = A.load_library()
    assert lib.demod_batch_launches(None, 10, 1) == A.DEMOD_BAD_ARG


def test_plan_info_fft_pmask_and_pass0_forms(A):
    """demod_plan_info without a device: the FFT's tones-only post-pass blocks
    (fft_pmask, against the kernel's bin layout restated in
    tests/test_gpu_fft_pmask.py) and the rescue first pass's form (fold64: 1
    the fold, 2 the residue fold, 0 segments)."""
    import numpy as np
    from test_gpu_fft_pmask import pmask
    rng = np.random.default_rng(5)
    for _ in range(40):
        k = int(rng.integers(2, 17))
        bins = sorted(int(b) for b in rng.choice(np.arange(1, 512), size=k, replace=False))
        if min(np.diff(bins)) < 2:
            continue
        cfg = A.make_cfg(freqs=tuple(46.875 * b for b in bins), method=A.METHOD_FFT)
        assert A.plan_info(cfg)["fft_pmask"] == pmask(bins)
    bin_ = 46.875
    cases = [((1500.0, 3000.0), A.METHOD_AUTO, 1),                              # plain K = 2, fold form
             (tuple(1500.0 + 375.0 * i for i in range(8)), A.METHOD_AUTO, 1),   # fold detector
             (tuple(bin_ * (32 + 9 * i) for i in range(8)), A.METHOD_AUTO, 2),  # residue detector
             (tuple(1234.5 + 1111.1 * i for i in range(8)), A.METHOD_GOERTZEL, 0)]
    for freqs, method, form in cases:
        info = A.plan_info(A.make_cfg(freqs=freqs, method=method))
        assert info["fold64"] == form, (freqs, info["method"], info["fold64"])
        assert info["fft_pmask"] == 0
