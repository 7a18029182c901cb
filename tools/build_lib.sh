# Rebuild ccj_amd/lib/libccj_hip.so and the bounds-checked libccj_hip_dbg.so (what
# __graft_entry__.build() does first), incrementally (one object per source under build/).
# NODBG=1 skips the debug library.  Extra arguments go to make (e.g. EXTRA=-DCCJ_ABLATE_ILOOP,
# ARCH=gfx950); a changed compile line rebuilds every object (ccj_amd/csrc/Makefile stamps).
cd "$(dirname "$0")/.." || exit 1
if [ -n "$NODBG" ]; then make -s -C ccj_amd/csrc -j8 "$@" all; else make -s -C ccj_amd/csrc -j8 "$@" all dbg; fi
