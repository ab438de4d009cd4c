# (rerun on the spill-free spectrum kernel, into prof_ss2)
# rocprofv3 kernel-trace stats and HBM PMC passes (FETCH_SIZE, WRITE_SIZE in
# separate runs) of scripts/slide_spec_runs.py.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_ss2
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/scripts/slide_spec_runs.py > $O/kt.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o run -- python3 $R/scripts/slide_spec_runs.py > $O/pmc_$c.log 2>&1 || exit 1
done
