cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tlb
export CCJ_PROFILE_REPS=1
timeout -s KILL 120 rocprofv3 --list-avail > gpurun_out/tlb/avail.txt 2>&1
grep -i -E "UTCL|TLB|TRANSLATION" gpurun_out/tlb/avail.txt | head -30
