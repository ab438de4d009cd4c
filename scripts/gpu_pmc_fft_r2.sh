# SQ/GRBM counters of the SHIPPED fft1024_quad_kernel (bench.py --config fft,
# hop 256), one pass per counter group.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_fft_r2
mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
B="python3 $R/bench.py --config fft --no-cpu-baseline --no-extras --steps 5 --warmup 2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o run -- $B > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- $B > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_INST_LEVEL_LDS SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA --output-format csv -d $O/p3 -o run -- $B > $O/p3.log 2>&1
exit 0
