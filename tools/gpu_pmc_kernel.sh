# PMC passes for one kernel (regex $1) over tools/level_profile.py 200 (2 folds).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
K=${1:-k_level4d}
D=gpurun_out/pmc_$K
mkdir -p $D
P="--kernel-trace --output-format csv --kernel-include-regex $K"
timeout -k 10 300 rocprofv3 $P --pmc FETCH_SIZE -d $D/fetch -o f -- python3 tools/level_profile.py 200 > $D/fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 $P --pmc TCC_HIT_sum TCC_MISS_sum -d $D/tcc -o tcc -- python3 tools/level_profile.py 200 > $D/tcc.log 2>&1 && \
timeout -k 10 300 rocprofv3 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $D/sq -o sq -- python3 tools/level_profile.py 200 > $D/sq.log 2>&1 && \
timeout -k 10 300 rocprofv3 $P --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS -d $D/sq2 -o sq2 -- python3 tools/level_profile.py 200 > $D/sq2.log 2>&1
rc=$?
python3 tools/pmc_summary.py 2 $D/*/*_counter_collection.csv $K
exit $rc
