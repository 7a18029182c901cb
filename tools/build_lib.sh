# Rebuild only ccj_amd/lib/libccj_hip.so (what __graft_entry__.build() does first), for quick iteration.
cd "$(dirname "$0")/.." && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value \
  -Iinclude -Iccj_amd/csrc -shared ccj_amd/csrc/ccj_host.cc ccj_amd/csrc/ccj_params_io.cc ccj_amd/csrc/ccj_kernels.hip \
  ccj_amd/csrc/ccj_backtrack.hip ccj_amd/csrc/ccj_wfinal.cc -o ccj_amd/lib/libccj_hip.so -lrccl "$@"
