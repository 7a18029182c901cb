# tile parity + counters (tools/gpu_tile_iter.sh), then alternating fills of extra variants
bash tools/gpu_tile_iter.sh || exit 1
[ $# -gt 0 ] && bash tools/gpu_tile_var.sh "$@"
