# PMC passes (one counter set per pass) for kernel regex $1 over tools/level_profile.py 200 (2 folds).
# usage: gpu_pmc_sets.sh KERNEL "SET1" "SET2" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K=$1; shift
D=gpurun_out/pmcs_$K
mkdir -p $D
n=0
for set in "$@"; do
  n=$((n+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex $K --pmc $set -d $D/p$n -o p$n -- python3 tools/level_profile.py 200 > $D/p$n.log 2>&1 || { echo "pass $n ($set) failed"; tail -5 $D/p$n.log; }
done
python3 tools/pmc_summary.py 2 $D/*/*_counter_collection.csv $K
