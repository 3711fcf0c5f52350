# plane-sweep A/B over the tuning overrides of dro_plane_sweep_forward (one box)
set -e
OUT=gpurun_out/${1:-sweep}
mkdir -p "$OUT"
run() { echo "== $*"; env "$@" timeout -k 10 120 python tools/bench_sweep.py; }
: > "$OUT/sweep.log"
for cfg in "DRO_X=0" "DRO_SWEEP_THREADS=1024" "DRO_SWEEP_THREADS=1024 DRO_SWEEP_BLOCKS=256" "DRO_SWEEP_THREADS=256" "DRO_X=1" \
           "DRO_SWEEP_BLOCKS=256" "DRO_SWEEP_WIDE=1"; do
  run $cfg >> "$OUT/sweep.log" 2>&1
done
grep -v amdgpu.ids "$OUT/sweep.log"
