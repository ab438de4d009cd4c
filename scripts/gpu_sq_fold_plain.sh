#!/bin/bash
# SQ counters of the 2-FSK survey plan through the plain bank (AUTO) and the
# fold detector (--method folded), configs[1] at full size: where the fold's
# extra ~2 % goes. One rocprofv3 --pmc pass each.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:-r6sq}
mkdir -p "$O"
for m in auto folded; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d "$O/sq_$m" -o run -- python3 "$R/bench.py" --method $m --no-cpu-baseline --no-rescue-ab --no-extras --sustain 0 --warmup 2 --steps 5) > "$O/sq_$m.log" 2>&1 || exit $?
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d "$O/sq2_$m" -o run -- python3 "$R/bench.py" --method $m --no-cpu-baseline --no-rescue-ab --no-extras --sustain 0 --warmup 2 --steps 5) > "$O/sq2_$m.log" 2>&1 || exit $?
done
