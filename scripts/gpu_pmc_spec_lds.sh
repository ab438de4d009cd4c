# LDS counters of the spectrum store (and the fold segment-shared form) in
# scripts/slide_spec_runs.py: bank conflicts vs LDS issue.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_lds
mkdir -p $O
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- python3 $R/scripts/slide_spec_runs.py > $O/p1.log 2>&1
