# Secondary BASELINE configs on 1 GPU (the headline line is bench.py's default): n=100 Turner04 (seed 3, config 2),
# n=200 DirksPierce09, n=400 Turner04 (config-5 per-GPU size). One JSON line each.
mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
timeout -k 10 300 python bench.py --n 100 --seed 3 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/configs.jsonl 2> gpurun_out/cfg.err && \
timeout -k 10 300 python bench.py --n 200 --params DirksPierce09 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/configs.jsonl 2>> gpurun_out/cfg.err && \
timeout -k 10 600 python bench.py --n 400 --seed 6 --steps 2 --warmup 1 --no-cpu-baseline >> gpurun_out/configs.jsonl 2>> gpurun_out/cfg.err
rc=$?
cut -c1-400 gpurun_out/configs.jsonl
[ $rc -ne 0 ] && tail -5 gpurun_out/cfg.err
exit $rc
