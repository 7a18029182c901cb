# Split-point sharing check: bounds-checked debug folds, the sharing parity tests, the full GPU
# suite, per-level profile and a short bench.  Each GPU step has its own limit; any failure ends it.
mkdir -p gpurun_out
timeout -k 10 300 python tools/dbg_check.py > gpurun_out/dbg.log 2>&1; rc=$?; tail -4 gpurun_out/dbg.log; [ $rc -eq 0 ] && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_share.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_share.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_share.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python tools/level_profile.py 200 > gpurun_out/levels.txt 2>&1 && cat gpurun_out/levels.txt && \
CCJ_SHARE_SPLITS=-1 timeout -k 10 300 python tools/level_profile.py 200 > gpurun_out/levels_noshare.txt 2>&1 && head -1 gpurun_out/levels_noshare.txt
