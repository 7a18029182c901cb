# interior-loop path by sequence length: alternating bench runs, tiles (default) vs work items
# (CCJ_ILOOP_TILES=0), n = 100 .. 400 (Turner04, seed 5; n=400 seed 6)
mkdir -p gpurun_out
for rep in 1 2; do
  for n in 100 150 200 300 400; do
    st=6; [ $n -ge 300 ] && st=3; seed=5; [ $n -eq 400 ] && seed=6
    for v in 1 0; do
      CCJ_ILOOP_TILES=$v timeout -k 10 300 python bench.py --n $n --seed $seed --steps $st --warmup 1 --no-cpu-baseline > gpurun_out/ils.json 2> gpurun_out/ils.err || { echo "FAIL n=$n tiles=$v"; tail -3 gpurun_out/ils.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/ils.json')); print('n=%s tiles=%s step %.2f fill %.2f setup %.2f' % (sys.argv[1], sys.argv[2], d['ms_per_step'], d['breakdown_ms']['fill_device'], d['setup_ms']))" $n $v
    done
  done
done
