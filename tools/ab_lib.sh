#!/bin/bash
# A/B of two builds of libdro_amd.so on one box: bench.py alternately with each
# (copied over the in-tree library between runs), ABAB order.
# usage: tools/ab_lib.sh <tag> <a.so> <b.so> [bench args...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; A=$2; B=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
LIB=dro-sfm_amd/libdro_amd.so
cp "$LIB" "$OUT/orig.so"
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then cp "$A" "$LIB"; else cp "$B" "$LIB"; fi
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline "$@" > "$OUT/bench_${v}$r.log" 2>&1
    st=$?
    echo "$v$r exit $st: $(tail -n 1 "$OUT/bench_${v}$r.log" | cut -c1-160)"
    if [ $st -ne 0 ]; then cp "$OUT/orig.so" "$LIB"; exit $st; fi
  done
done
cp "$OUT/orig.so" "$LIB"; rm -f "$OUT/orig.so"
