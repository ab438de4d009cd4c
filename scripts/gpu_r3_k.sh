# Round 3: ballot-based ambiguity test (window_sum.h ws_ambiguous) and the
# trivial-twiddle skip in the FFT rescue: the GPU suite, the rescue probe A/B,
# the default bench line (with the sustained phase).
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3k}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 scripts/bin/fft_probe 256 8 10 rsc > $O/probe_rsc_256.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
