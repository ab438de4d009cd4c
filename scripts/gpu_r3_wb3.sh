# Round 3, late: the 2-FSK headline batch with its default 4 write-back
# bursts against FSKD_WB_BURSTS=0 (one write-back at the kernel's end),
# bench.py interleaved, three rounds; then the closing check (gpu_r3_z.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3wb3}
mkdir -p $O
cd $R
B="python3 bench.py --no-cpu-baseline --no-rescue-ab --no-extras --sustain 0 --steps 40 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 120 $B > $O/fsk2_bursts_$i.log 2>&1 || exit $?
  FSKD_WB_BURSTS=0 timeout -k 10 120 $B > $O/fsk2_off_$i.log 2>&1 || exit $?
done
bash scripts/gpu_r3_z.sh ${2:-r3z3}
