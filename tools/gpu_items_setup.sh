# work-item setup kernels (k_items split, k_build_il): parity in items mode, then setup/step A/B
mkdir -p gpurun_out
echo "== items parity" && { CCJ_ILOOP_TILES=0 timeout -k 10 600 python -u -m pytest tests/test_gpu_items.py tests/test_gpu_large.py tests/test_gpu_shard.py -x -q --timeout 300 --timeout-method thread > gpurun_out/items_parity.log 2>&1; rc=$?; tail -2 gpurun_out/items_parity.log; [ $rc -eq 0 ]; } && \
bash tools/gpu_ab.sh "CCJ_ILOOP_TILES=0|" "CCJ_ILOOP_TILES=1|"
