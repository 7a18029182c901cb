#!/bin/bash
# Fill-time A/B of MFE library variants on one box (tools/level_profile.py 200, 5 reps each).
# usage (GPU box): tools/mfe_ab.sh variant ...   ("-" = the default libccj_hip.so)
cd "$(dirname "$0")/.."
for v in "$@"; do
  [ "$v" = "-" ] && v=""
  echo "== ${v:-default}"
  CCJ_LIB_VARIANT=$v timeout -k 10 120 python3 tools/level_profile.py 200 | head -1 || exit 1
done
