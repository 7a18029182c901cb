# push-form P terms: parity subset, bench A/B against the pull kernel (CCJ_PTERM_PULL=1), spans
# per wave (CCJ_PP_S) and inner-loop slice lengths (CCJ_PP_HS), then serialised (--pmc) kernel
# times and HBM traffic of both forms
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
echo "== pytest" && { timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ]; } || exit 1
CCJ_PP_S=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread -k "t04_200 or 220" > gpurun_out/pytest_gpu4.log 2>&1 || { tail gpurun_out/pytest_gpu4.log; exit 1; }
tail -1 gpurun_out/pytest_gpu4.log
b() { timeout -k 10 200 python bench.py --steps 10 --no-cpu-baseline > gpurun_out/b.json 2>/dev/null || exit 1
      python -c "import json;a=json.load(open('gpurun_out/b.json'));print('$1',round(a['ms_per_step'],2),round(a['breakdown_ms']['fill_device'],2),a['mfe'])"; }
for r in 1 2; do
  CCJ_PTERM_PULL=1 b pull
  CCJ_PP_HS=32 b s8hs32
  CCJ_PP_HS=16 b s8hs16
  CCJ_PP_HS=64 b s8hs64
  CCJ_PP_S=4 CCJ_PP_HS=32 b s4hs32
done
for v in push pull; do
  D=gpurun_out/pmc_$v; mkdir -p $D
  [ $v = pull ] && export CCJ_PTERM_PULL=1
  P="--kernel-trace --output-format csv --kernel-include-regex k_p"
  timeout -k 10 300 rocprofv3 $P --pmc FETCH_SIZE -d $D/fetch -o f -- python3 tools/level_profile.py 200 > $D/fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 $P --pmc WRITE_SIZE -d $D/write -o w -- python3 tools/level_profile.py 200 > $D/write.log 2>&1 || exit 1
done
