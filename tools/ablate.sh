#!/bin/bash
# Timing-only variant builds of the fill.  CCJ_ABLATE_* variants give WRONG results by construction
# (never used by tests); the others are tuning candidates.  usage: tools/ablate.sh name:flags ...
cd "$(dirname "$0")/.."
SRC="ccj_amd/csrc/ccj_host.cc ccj_amd/csrc/ccj_params_io.cc ccj_amd/csrc/ccj_kernels.hip ccj_amd/csrc/ccj_backtrack.hip ccj_amd/csrc/ccj_wfinal.cc ccj_amd/csrc/ccj_pf.cc ccj_amd/csrc/ccj_pf.hip"
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  mkdir -p build/abl_$name
  objs=""
  for f in $SRC; do
    o=build/abl_$name/$(basename $f).o
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-value -Wno-unused-result $flags \
      -Iinclude -Iccj_amd/csrc -c $f -o $o &
    objs="$objs $o"
  done
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $objs -o ccj_amd/lib/libccj_hip_$name.so -lrccl -lpthread || exit 1
done
