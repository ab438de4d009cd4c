# FFT detector variants (probe, interleaved) + SQ counters for default vs TWLDS, then GPU FFT tests.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
PROBE_FILTER=fft timeout -k 10 300 $R/scripts/bin/probe 1048576 8 10 > $O/probe_fft.log 2>&1 || exit 1
cd /tmp
PROBE_FILTER="hop=256" timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d $O/pmc_fftvar -o run -- $R/scripts/bin/probe 1048576 1 3 > $O/pmc_fftvar.log 2>&1 || exit 1
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -x -q -k "fft or FFT" > $O/pytest_fft.log 2>&1
