#!/bin/bash
# Interleaved bench A/B on one box: tools/ab_bench.sh <out dir> <rounds> "<NAME=env ...>" ...
# each variant a quoted env assignment list ("base" = none); prints ms/step per run.
set -u
OUT=$1; ROUNDS=$2; shift 2
mkdir -p "$OUT"
for r in $(seq 1 "$ROUNDS"); do
  for v in "$@"; do
    tag=$(echo "$v" | tr -c 'A-Za-z0-9=_\n' '_' | tr '=' '-')
    if [ "$v" = base ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline \
      > "$OUT/bench_${tag}_$r.log" 2>&1 || { echo "variant $v failed"; exit 1; }
    echo "$v $r: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/bench_${tag}_$r.log")"
  done
done
