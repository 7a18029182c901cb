# FETCH_SIZE / WRITE_SIZE per launch of the opt-in LDS-tile interior-loop kernel (CCJ_ILOOP_TILES=1)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tiletr
for c in FETCH_SIZE WRITE_SIZE; do
  CCJ_ILOOP_TILES=1 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "k_iltile|k_level4d" --pmc $c -d gpurun_out/tiletr/$c -o p -- python3 tools/fold_once.py 200 2 > gpurun_out/tiletr/$c.log 2>&1 || exit 1
done
echo "tile traffic ok"
