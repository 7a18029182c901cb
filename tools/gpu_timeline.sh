# Kernel trace of a few n=200 folds for tools/trace_timeline.py (args: extra env assignments via caller).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tl
env ${TL_ENV} CCJ_PROFILE_REPS=2 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o tl -- python3 tools/level_profile.py 200 > gpurun_out/tl/run.log 2>&1
rc=$?
f=$(find gpurun_out/tl -name '*kernel_trace.csv' | head -1)
[ -n "$f" ] && python3 tools/${TL_TOOL:-trace_timeline.py} "$f" -2
exit $rc
