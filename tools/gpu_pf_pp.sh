# PF parity + PF bench line, MFE parity at BASELINE sizes, and k_ppush FETCH/WRITE per launch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pp
echo "== pytest" && { timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pf or large or configs" > gpurun_out/pytest_pp.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pp.log; [ $rc -eq 0 ]; } && \
echo "== pf bench" && timeout -k 10 400 python bench.py --pf --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pp/pf_bench.json 2> gpurun_out/pp/pf_bench.err && \
python3 -c "import json;d=json.load(open('gpurun_out/pp/pf_bench.json'));print('pf ms/step',d['ms_per_step'],{k:round(v,2) for k,v in d.get('kernel_ms',{}).items()} if isinstance(d.get('kernel_ms'),dict) else '')" && \
echo "== mfe bench" && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/pp/bench.json 2>/dev/null && \
python3 -c "import json;d=json.load(open('gpurun_out/pp/bench.json'));print('mfe ms/step',d['ms_per_step'],'fill',d['breakdown_ms']['fill_device'])" && \
for c in FETCH_SIZE WRITE_SIZE; do timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --output-format csv --kernel-include-regex "k_ppush|k_level4d|k_iloop" --pmc $c -d gpurun_out/pp/$c -o p -- python3 tools/fold_once.py 200 2 > gpurun_out/pp/$c.log 2>&1 || exit 1; done && \
python3 - <<'PY'
import glob, sys
sys.path.insert(0, "tools")
from make_profiles import pmc, FETCH_FACTOR, WRITE_FACTOR
for c, fac in (("FETCH_SIZE", FETCH_FACTOR), ("WRITE_SIZE", WRITE_FACTOR)):
    f = glob.glob(f"gpurun_out/pp/{c}/**/*counter_collection.csv", recursive=True)[0]
    for k, (b, nl) in sorted(pmc(f, c).items()):
        print(c, k, "%.1f MB/launch" % (fac * b / max(nl, 1) / 1e6), nl)
PY
