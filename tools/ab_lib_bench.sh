#!/bin/bash
# Interleaved bench A/B of the in-tree library against alternative builds:
# tools/ab_lib_bench.sh <out dir> <rounds> <lib.so>...   (each run with DRO_LIB_PATH set)
set -u
OUT=$1; ROUNDS=$2; shift 2
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for lib in default "$@"; do
    if [ "$lib" = default ]; then envs=""; else envs="DRO_LIB_PATH=$lib"; fi
    tag=$(basename "$lib" .so)
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline \
      > "$OUT/bench_${tag}_$r.log" 2>&1 || { echo "$lib failed"; exit 1; }
    echo "$tag $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_${tag}_$r.log")"
  done
done
