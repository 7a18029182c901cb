# Bounds-checked debug build over small folds, then the given GPU test files, then an A/B bench.
mkdir -p gpurun_out
echo "== dbg" && timeout -k 10 300 python tools/dbg_check.py > gpurun_out/dbg.log 2>&1 && tail -2 gpurun_out/dbg.log && \
echo "== pytest $*" && { timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_new.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_new.log; [ $rc -eq 0 ]; }
