# Alternating A/B timing of variants (n=200 bench lines): tools/gpu_ab.sh "ENV=a|--bench-args" ...
# Each variant is "env assignments|extra bench.py arguments" (either part may be empty).
mkdir -p gpurun_out/ab
: > gpurun_out/ab/ab.txt
for rep in 1 2 3; do
  for v in "$@"; do
    envp="${v%%|*}"; args=""; [ "$v" != "$envp" ] && args="${v#*|}"
    env $envp timeout -k 10 120 python bench.py --steps 8 --warmup 2 --no-cpu-baseline $args > gpurun_out/ab/out.json 2> gpurun_out/ab/err.txt || { echo "FAIL $v"; tail -5 gpurun_out/ab/err.txt; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/out.json')); print('%-34s step %.2f fill %.2f level %.2f setup %.2f mfe %s' % (sys.argv[1], d['ms_per_step'], d['breakdown_ms']['fill_device'], d['breakdown_ms']['level4d_levels'], d['setup_ms'], d['mfe']))" "$v" | tee -a gpurun_out/ab/ab.txt
  done
done
