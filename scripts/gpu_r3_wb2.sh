# Round 3, late: forced write-back bursts on the 2-FSK headline batch (9 MiB
# of output, no bursts by default) and burst counts around the 8-FSK default
# (7), bench.py interleaved, three rounds (FSKD_WB_BURSTS=<n>: n bursts).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r3wb2}
mkdir -p $O
cd $R
B="python3 bench.py --no-cpu-baseline --no-rescue-ab --no-extras --sustain 0 --steps 40 --warmup 5"
for i in 1 2 3; do
  for nb in def 1 2 4; do
    if [ $nb = def ]; then timeout -k 10 120 $B > $O/fsk2_${nb}_$i.log 2>&1 || exit $?
    else FSKD_WB_BURSTS=$nb timeout -k 10 120 $B > $O/fsk2_${nb}_$i.log 2>&1 || exit $?; fi
  done
  for nb in def 4 10; do
    if [ $nb = def ]; then timeout -k 10 120 $B --config fsk8 > $O/fsk8_${nb}_$i.log 2>&1 || exit $?
    else FSKD_WB_BURSTS=$nb timeout -k 10 120 $B --config fsk8 > $O/fsk8_${nb}_$i.log 2>&1 || exit $?; fi
  done
done
