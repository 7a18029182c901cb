# Level-profile timings for several values of one environment variable: VAR v1 v2 ...
mkdir -p gpurun_out
VAR=$1; shift
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python tools/level_profile.py 200 > gpurun_out/sweep_$v.txt 2>&1 || { cat gpurun_out/sweep_$v.txt; exit 1; }
  echo "$VAR=$v $(head -1 gpurun_out/sweep_$v.txt)"
done
