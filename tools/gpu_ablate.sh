# Per-variant level timings on the GPU for every ccj_amd/lib/libccj_hip_<v>.so given on the command line.
mkdir -p gpurun_out
for v in "" "$@"; do
  echo "== variant '$v'"
  CCJ_LIB_VARIANT=$v timeout -k 10 300 python tools/level_profile.py 200 > gpurun_out/abl_$v.txt 2>&1 || { cat gpurun_out/abl_$v.txt; exit 1; }
  head -1 gpurun_out/abl_$v.txt
done
