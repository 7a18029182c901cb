#!/bin/bash
# Timing-only variant builds of the fill.  CCJ_ABLATE_* variants give WRONG results by construction
# (never used by tests); the others are tuning candidates.  usage: tools/ablate.sh name:flags ...
cd "$(dirname "$0")/.."
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value -Wno-unused-result $flags \
    -Iinclude -Iccj_amd/csrc ccj_amd/csrc/ccj_host.cc ccj_amd/csrc/ccj_params_io.cc ccj_amd/csrc/ccj_kernels.hip ccj_amd/csrc/ccj_backtrack.hip -o ccj_amd/lib/libccj_hip_$name.so -lrccl || exit 1
done
