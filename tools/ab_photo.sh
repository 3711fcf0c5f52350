#!/bin/bash
# A/B of photometric-kernel builds on one box: tools/ab_photo.sh <out dir> <lib>...
# (each lib an alternative libdro_amd.so; "default" = the in-tree one), interleaved twice.
set -u
OUT=$1; shift
mkdir -p "$OUT"
for round in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = default ]; then env_lib=""; else env_lib="DRO_LIB_PATH=$lib"; fi
    env $env_lib timeout -k 10 120 python tools/bench_photo.py --iters 50 > "$OUT/photo_$(basename $lib)_$round.log" 2>&1 || exit $?
    echo "$(basename $lib) $round: $(grep photometric "$OUT/photo_$(basename $lib)_$round.log")"
  done
done
