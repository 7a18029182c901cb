# k_ppush XCD-aware block order vs linear (libccj_hip_pplin.so): parity, per-launch traffic, fill A/B
mkdir -p gpurun_out
echo "== parity" && { timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pp_parity.log 2>&1; rc=$?; tail -2 gpurun_out/pp_parity.log; [ $rc -eq 0 ]; } && \
echo "== traffic" && bash tools/gpu_pmc_ab.sh "k_ppush" "CCJ_X=0" "CCJ_LIB_VARIANT=pplin" > gpurun_out/pp_pmc.txt 2>&1 && cat gpurun_out/pp_pmc.txt && \
echo "== timing" && bash tools/gpu_ab.sh "CCJ_X=0|" "CCJ_LIB_VARIANT=pplin|"
