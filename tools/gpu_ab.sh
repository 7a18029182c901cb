# Alternating A/B timings of variants on one box.  Each variant is "ENV assignments|extra arguments"
# (either part may be empty; CCJ_LIB_VARIANT=x selects ccj_amd/lib/libccj_hip_x.so, e.g. the
# timing-only builds of tools/ablate.sh).
#   MODE=bench (default): bench.py lines (step, fill, level chain, setup);  extra args go to bench.py
#                         (e.g. "|--n 400 --seed 6", "CCJ_X=1|--pf")
#   MODE=level          : tools/level_profile.py N (fill median of 5 folds)
#   REPS (default 3) rounds over all variants;  N (default 200) for MODE=level
#   bash tools/gpu_ab.sh "|" "CCJ_SHARE_SPLITS=-1|"
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.txt
for rep in $(seq 1 "${REPS:-3}"); do
  for v in "$@"; do
    envp="${v%%|*}"; args=""; [ "$v" != "$envp" ] && args="${v#*|}"
    if [ "${MODE:-bench}" = level ]; then
      env $envp timeout -k 10 200 python3 tools/level_profile.py "${N:-200}" > gpurun_out/ab/out.txt 2>&1 || { echo "FAIL $v"; tail -5 gpurun_out/ab/out.txt; exit 1; }
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab/out.txt').readline()); print('%-34s fill %.2f min %.2f level %.2f' % (sys.argv[1], d['fill_ms_median'], d['fill_ms_min'], d['level4d_ms_uninstrumented']))" "$v" | tee -a gpurun_out/ab/ab.txt
    else
      env $envp timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline $args > gpurun_out/ab/out.json 2> gpurun_out/ab/err.txt || { echo "FAIL $v"; tail -5 gpurun_out/ab/err.txt; exit 1; }
      python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab/out.json')); b=d.get('breakdown_ms', {})
print('%-34s step %.2f fill %.2f level %s setup %s mfe %s' % (sys.argv[1], d['ms_per_step'], b.get('fill_device', d.get('fill_ms', 0)), b.get('level4d_levels', '-'), d.get('setup_ms', '-'), d.get('mfe', d.get('energy'))))" "$v" | tee -a gpurun_out/ab/ab.txt
    fi
  done
done
