# Kernel-time summary of one n=200 profile run (rocprofv3 kernel trace + stats only).
# usage: tools/gpu_kstats.sh [env assignments for the profiled run are taken from the caller]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ks
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ks -o ks --output-format csv -- python3 tools/level_profile.py 200 > gpurun_out/ks/run.log 2>&1
rc=$?
cat gpurun_out/ks/ks_kernel_stats.csv 2>/dev/null | cut -c1-150
exit $rc
