# Counter passes over scripts/bin/fft_probe (shipped FFT kernel + one variant):
# issue/wait shares, TA / TCP (L1) stalls, LDS activity.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_fftp
mkdir -p $O
cd /tmp
F="${FFT_FILTER:-PF0 MINW4 REG}"
P="$R/scripts/bin/fft_probe 256 1 3"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU --output-format csv -d $O/p1 -o run -- $P "$F" > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_READ_TAGCONFLICT_STALL_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_LDS --output-format csv -d $O/p2 -o run -- $P "$F" > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY TA_DATA_STALLED_BY_TC_CYCLES SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_LDS_DATA_FIFO_FULL --output-format csv -d $O/p3 -o run -- $P "$F" > $O/p3.log 2>&1
exit 0
