# SQ counters of the level chain's two kernels, standalone (PMC passes serialise dispatches), over
# tools/fold_once.py 200 (1 fold): instruction mix, wave cycles, busy and wait shares.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/leadpmc
mkdir -p $D
P="--kernel-trace --output-format csv --kernel-include-regex k_level4d"
timeout -k 10 -s KILL 200 rocprofv3 $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY -d $D/sq -o sq -- python3 tools/fold_once.py 200 > $D/sq.log 2>&1 && \
timeout -k 10 -s KILL 200 rocprofv3 $P --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $D/sq2 -o sq2 -- python3 tools/fold_once.py 200 > $D/sq2.log 2>&1
rc=$?
for k in k_level4d_lead k_level4d\(; do echo "== $k"; python3 tools/pmc_summary.py 1 $D/*/*_counter_collection.csv "$k"; done
exit $rc
