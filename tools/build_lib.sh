# Rebuild ccj_amd/lib/libccj_hip.so and the bounds-checked libccj_hip_dbg.so (what
# __graft_entry__.build() does first), for quick iteration.  Extra args go to both hipcc lines.
cd "$(dirname "$0")/.." || exit 1
SRC="ccj_amd/csrc/ccj_host.cc ccj_amd/csrc/ccj_params_io.cc ccj_amd/csrc/ccj_kernels.hip ccj_amd/csrc/ccj_backtrack.hip ccj_amd/csrc/ccj_wfinal.cc ccj_amd/csrc/ccj_pf.cc ccj_amd/csrc/ccj_pf.hip"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value -Iinclude -Iccj_amd/csrc -shared"
[ -n "$NODBG" ] || /opt/rocm/bin/hipcc $FLAGS -DCCJ_DEBUG_BOUNDS $SRC -o ccj_amd/lib/libccj_hip_dbg.so -lrccl -lpthread "$@" &
/opt/rocm/bin/hipcc $FLAGS $SRC -o ccj_amd/lib/libccj_hip.so -lrccl -lpthread "$@"
rc=$?
wait $! || rc=1
exit $rc
