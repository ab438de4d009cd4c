# SQ counters for the quad-layout FFT detector (hop 256), two passes
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp
PROBE_FILTER="hop=256 swz=1 QUAD" timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU --output-format csv -d $O/pmc_fftq1 -o run -- $R/scripts/bin/probe 1048576 1 3 > $O/pmc_fftq1.log 2>&1 || exit 1
PROBE_FILTER="hop=256 swz=1 QUAD" timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM --output-format csv -d $O/pmc_fftq2 -o run -- $R/scripts/bin/probe 1048576 1 3 > $O/pmc_fftq2.log 2>&1 || exit 1
PROBE_FILTER="hop=256 swz=1 QUAD" timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_LEVEL_LDS --output-format csv -d $O/pmc_fftq3 -o run -- $R/scripts/bin/probe 1048576 1 3 > $O/pmc_fftq3.log 2>&1
exit 0
