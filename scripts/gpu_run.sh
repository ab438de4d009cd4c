# GPU-box launcher (replaces the round-3 one-off gpu_r3_*.sh scripts):
#   gpurun -- bash scripts/gpu_run.sh <outdir> <step> [<step> ...]
# Writes under gpurun_out/<outdir>/. Steps run in order, each under its own
# time limit; the first failing step ends the call (no retries).
#   tests            pytest -m gpu (whole suite)
#   tests:<expr>     pytest -m gpu -k <expr>
#   smoke            __graft_entry__.smoke()
#   bench            the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   benchq[:<args>]  headline only (no CPU baseline / extras / rescue A/B), extra bench args
#   benchcfg:<args>  bench.py --no-cpu-baseline <args> (e.g. "--config fsk8")
#   ab:<N>:<envA>:<envB>:<args>  N interleaved rounds of bench.py <args> with env A, env B
#   kt               rocprofv3 --kernel-trace --stats of the driver's command
#   pmc              HBM PMC passes (FETCH_SIZE, WRITE_SIZE separately): fsk2, fsk8, fft, fft+spectrum
#   sq[:<args>]      one SQ pass (issue counts) of the tones-only FFT kernel
#   sqw[:<ENV=V|-> <args>]  one SQ pass of its wait states (SQ_WAIT_ANY / _INST_ANY / _INST_LDS)
#   testsall[:<args>] pytest -m gpu without -x (all failures in one call)
#   testsk:<expr>    pytest -m gpu -k <expr> without -x
#   ktr:<case>       rocprofv3 --kernel-trace --stats of scripts/rescue_probe.py <case>
#   sqr:<case>       one SQ pass of scripts/rescue_probe.py <case> (rescue worst case)
#   precision        scripts/precision_probe.py
#   py:<script args> python3 <script args> (probes under scripts/)
#   pyt:<secs>:<args> the same under a time limit of its own
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/${1:?outdir}
shift
mkdir -p "$O"
cd "$R"
i=0
for st in "$@"; do
  i=$((i + 1))
  name=${st%%:*}
  arg=${st#*:}
  [ "$arg" = "$st" ] && arg=""
  log="$O/$(printf %02d $i)_${name}.log"
  echo "[$(date +%T)] step $i: $st" | tee -a "$O/steps.log"
  case "$name" in
    tests)
      if [ -n "$arg" ]; then k=(-k "$arg"); else k=(); fi
      timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests "${k[@]}" > "$log" 2>&1 || exit $? ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$log" 2>&1 || exit $? ;;
    bench)
      timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$log" 2>&1 || exit $? ;;
    benchq)
      timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-rescue-ab --no-extras --sustain 0 --steps 100 --warmup 10 $arg > "$log" 2>&1 || exit $? ;;
    benchcfg)
      timeout -k 10 400 python3 bench.py --no-cpu-baseline $arg > "$log" 2>&1 || exit $? ;;
    ab)
      IFS=: read -r n ea eb rest <<< "$arg"
      for r in $(seq 1 "$n"); do
        env $ea timeout -k 10 200 python3 bench.py --no-cpu-baseline $rest > "$O/$(printf %02d $i)_ab_A_$r.log" 2>&1 || exit $?
        env $eb timeout -k 10 200 python3 bench.py --no-cpu-baseline $rest > "$O/$(printf %02d $i)_ab_B_$r.log" 2>&1 || exit $?
      done ;;
    kt)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 "$R/bench.py" --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --sustain 0) > "$log" 2>&1 || exit $? ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        for cfg in fsk2 fsk8; do
          (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_${cfg}_$c" -o run -- python3 "$R/bench.py" --config $cfg --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5) > "$O/pmc_${cfg}_$c.log" 2>&1 || exit $?
        done
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_fft_$c" -o run -- python3 "$R/bench.py" --config fft --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5) > "$O/pmc_fft_$c.log" 2>&1 || exit $?
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_fftspec_$c" -o run -- python3 "$R/bench.py" --config fft --spectrum --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5) > "$O/pmc_fftspec_$c.log" 2>&1 || exit $?
      done ;;
    sq)
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d "$O/sq_fft" -o run -- python3 "$R/bench.py" --config fft --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5 $arg) > "$log" 2>&1 || exit $? ;;
    sqw)
      # where the FFT kernel's waves wait: parked at s_waitcnt / barrier
      # (SQ_WAIT_ANY) vs issue-stalled (SQ_WAIT_INST_ANY, its LDS part)
      # sqw:<ENV=VAL|-> [bench args]: the environment of the profiled run (e.g.
      # FSKD_FFT_SWP=3), "-" for none; output under sqw_<i>/
      ev=${arg%% *}; rest=${arg#* }; [ "$rest" = "$arg" ] && rest=""
      [ -z "$ev" ] || [ "$ev" = "-" ] && ev="X=1"
      (cd /tmp && export $ev && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d "$O/sqw_$i" -o run -- python3 "$R/bench.py" --config fft --no-cpu-baseline --no-rescue-ab --warmup 2 --steps 5 $rest) > "$log" 2>&1 || exit $? ;;
    testsk)
      # pytest -m gpu -k <expr> without -x (the expression stays one argument)
      timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests -k "$arg" > "$log" 2>&1 || exit $? ;;
    testsall)
      # the GPU suite without -x (every failure of a change set in one call)
      timeout -k 10 1100 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests $arg > "$log" 2>&1 || exit $? ;;
    ktr)
      # kernel trace of one rescue worst case (scripts/rescue_probe.py <case>)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktr_$i" -o run -- python3 "$R/scripts/rescue_probe.py" $arg) > "$log" 2>&1 || exit $? ;;
    sqr)
      # one SQ pass (issue / wait counts) of a rescue worst case
      (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$O/sqr_$i" -o run -- python3 "$R/scripts/rescue_probe.py" $arg 3) > "$log" 2>&1 || exit $? ;;
    precision)
      timeout -k 10 600 python3 -u scripts/precision_probe.py $arg > "$log" 2>&1 || exit $? ;;
    py)
      timeout -k 10 600 python3 -u $arg > "$log" 2>&1 || exit $? ;;
    pyt)
      # pyt:<seconds>:<script args>: python3 under its own shorter time limit
      secs=${arg%%:*}; rest=${arg#*:}
      timeout -k 10 "$secs" python3 -u $rest > "$log" 2>&1 || exit $? ;;
    *)
      echo "unknown step $st" >&2; exit 2 ;;
  esac
done
echo "[$(date +%T)] done" | tee -a "$O/steps.log"
