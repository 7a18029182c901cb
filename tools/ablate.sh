#!/bin/bash
# Timing-only ablation builds of the fill (results are WRONG by construction; never used by tests).
cd "$(dirname "$0")/.."
for v in iloop:-DCCJ_ABLATE_ILOOP linear:-DCCJ_ABLATE_LINEAR pterm:-DCCJ_ABLATE_PTERM; do
  name=${v%%:*}; flag=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-value -Wno-unused-result $flag \
    -Iinclude -Iccj_amd/csrc ccj_amd/csrc/ccj_host.cc ccj_amd/csrc/ccj_kernels.hip -o ccj_amd/lib/libccj_hip_abl_$name.so || exit 1
done
