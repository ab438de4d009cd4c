# SQ counters of the shipped 2-FSK (plain bank) and 8-FSK (fold F16) kernels
# inside bench.py: VALU / LDS issue, wave cycles, effective clock.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_gz_r2
mkdir -p $O
cd /tmp
for cfg in fsk2 fsk8; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/$cfg -o run -- python3 $R/bench.py --config $cfg --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $O/$cfg.log 2>&1 || exit 1
done
