mkdir -p gpurun_out
for v in "" abl_iloop abl_linear abl_pterm; do
  echo "== variant '$v'"
  CCJ_LIB_VARIANT=$v timeout -k 10 300 python tools/level_profile.py 200 2>&1 | head -1 || exit 1
done
