#!/bin/bash
# One GPU session on the MI355X box: each GPU step under its own time limit;
# stop at the first crash-class exit (fault/abort/segv/timeout), continue past
# ordinary test failures (exit 1) so later measurements still run.
# usage: tools/gpu_session.sh <tag> <steps...>   steps: smoke tests bench prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
crash() { case $1 in 0|1|2|5) return 1;; *) return 0;; esac; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local st=$?
  echo "   exit $st"; tail -n 5 "$OUT/$name.log"
  if crash $st; then echo "!! crash-class exit $st in $name: stopping"; exit $st; fi
  if grep -qE "illegal memory access|Memory access fault|hipErrorIllegalAddress|HSA_STATUS_ERROR|AcceleratorError" "$OUT/$name.log"; then
    echo "!! GPU fault reported in $name: stopping"; exit 99
  fi
  return 0
}
for step in "$@"; do
  case $step in
    smoke) run smoke 600 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) run pytest_gpu 1100 python -u -m pytest tests -m gpu -x -v --timeout=300 --timeout-method=thread -p no:cacheprovider ;;
    testsall) run pytest_gpu 1100 python -u -m pytest tests -m gpu -v --timeout=300 --timeout-method=thread -p no:cacheprovider ;;
    testsm) rm -f "$OUT/parity_margins.jsonl"; run pytest_gpu 1100 env DRO_PARITY_LOG="$OUT/parity_margins.jsonl" python -u -m pytest tests -m gpu -v --durations=15 --timeout=300 --timeout-method=thread -p no:cacheprovider ;;
    bench) run bench 900 python bench.py --steps 20 --warmup 5 ;;
    benchq) run bench 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ;;
    benchab) run bench_a 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline ;;
    benche) run bench_eager 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --eager ;;
    benchms) run bench_miopen_strided 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --miopen-strided-convs ;;
    benchpipe) run bench_pipeline 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --pipeline gpu ;;
    dp2) run bench_dp2_gloo_onegpu 600 env DRO_DIST_BACKEND=gloo DRO_BENCH_DEVICE=0 python bench.py --gpus 2 --steps 10 --warmup 3 --no-roofline ;;
    prof) run rocprof 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline ;;
    profms) run rocprof_ms 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profms" -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --miopen-strided-convs ;;
    roof) run roofline_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/roof" -o run -- python bench.py --roofline-only ;;
    roofonly) run roofonly 300 python bench.py --roofline-only ;;
    pmc) run pmc_fetch 600 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python bench.py --roofline-only &&
         run pmc_write 600 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python bench.py --roofline-only &&
         run pmc_traffic 60 python tools/pmc_traffic.py "$OUT" ;;
    pmcsq) run pmc_sq 120 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$OUT/pmc_sq" -o run -- python bench.py --roofline-only ;;
    croof) run croof_stats 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/croof" -o run -- python tools/conv_roofline.py run "$OUT/croof" &&
         run croof_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/croof_fetch" -o run -- python tools/conv_roofline.py run "$OUT/croof_fetch" &&
         run croof_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/croof_write" -o run -- python tools/conv_roofline.py run "$OUT/croof_write" &&
         run croof_mfma 300 timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$OUT/croof_mfma" -o run -- python tools/conv_roofline.py run "$OUT/croof_mfma" &&
         run croof_table 60 python tools/conv_roofline.py table "$OUT/croof" --pmc-dirs "$OUT/croof_fetch" "$OUT/croof_write" "$OUT/croof_mfma" ;;
    tl) run step_timeline 300 python tools/step_timeline.py ;;
    photo) run photo_stats 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/photo" -o run -- python tools/bench_photo.py --iters 20 ;;
    w:*) wl=${step#w:}; run "bench_$wl" 900 python bench.py --workload "$wl" --steps 10 --warmup 3 ;;
    envr:*) kv=${step#envr:}; run "roof_${kv%%=*}_${kv#*=}" 300 env "$kv" python bench.py --roofline-only ;;
    envb:*) kv=${step#envb:}; run "bench_${kv%%=*}" 600 env "$kv" python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline ;;
    k:*) kk=${step#k:}; run "pytest_k_${kk//[^a-zA-Z0-9]/_}" 900 python -u -m pytest tests -m gpu -v --timeout=300 --timeout-method=thread -p no:cacheprovider -k "$kk" ;;
    ms:*) kk=${step#ms:}; run "pytest_ms_${kk//[^a-zA-Z0-9]/_}" 900 env DRO_NATIVE_STRIDED=0 python -u -m pytest tests -m gpu -v --timeout=300 --timeout-method=thread -p no:cacheprovider -k "$kk" ;;
    t:*) f=${step#t:}; run "pytest_$(basename "$f" .py)" 900 python -u -m pytest "$f" -m gpu -v --timeout=300 --timeout-method=thread -p no:cacheprovider ;;
    py:*) f=${step#py:}; run "py_$(basename "$f" .py)" 600 python "$f" ;;
    *) echo "unknown step $step" ;;
  esac
done
echo "== done"
