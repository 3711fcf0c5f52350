#!/bin/bash
# Extra PMC passes over the roofline kernel (one counter group per run):
# instruction-cache and address-translation behaviour of the conv engine.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-pmcprobe}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
pass() {  # name counters...
  local name=$1; shift
  echo "== $name: $*"
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- python bench.py --roofline-only > "$OUT/$name.log" 2>&1
  local st=$?
  echo "   exit $st"
  case $st in 0|1) ;; *) echo "!! stopping"; exit $st;; esac
}
case "${PROBE:-all}" in
  insts) pass ifetch SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS; echo "== done"; exit 0 ;;
esac
pass icache SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
pass ifetch SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS
pass utcl1 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum
echo "== done"
