# Fold detector's segment-shared form (fold_slide_kernel): GPU tests, then
# the sliding probe with and without it (FSKD_NO_SLIDE=1: direct kernels).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fold_slide
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_fold_slide.py tests/test_gpu_slide.py "tests/test_gpu_parity.py::test_fft_detector_spectrum_vs_reference_kissfft" "tests/test_gpu_parity.py::test_tone_bank_vs_reference_kissfft" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_fold_slide.log 2>&1 && \
timeout -k 10 200 python -u scripts/sliding_probe.py --hops 1024,512,256,128,64 > $O/sliding_probe.log 2>&1 && \
FSKD_NO_SLIDE=1 timeout -k 10 200 python -u scripts/sliding_probe.py --hops 512,256,128,64 > $O/sliding_probe_direct.log 2>&1
