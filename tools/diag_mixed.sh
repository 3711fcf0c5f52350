# native stride-2 parity diagnosis: sensitivity of the step to the stem output's rounding
set -e
mkdir -p gpurun_out/r4aa
for cfg in "DIAG_NOISE=1e-7 DIAG_SEED=0" "DIAG_NOISE=1e-7 DIAG_SEED=1" "DIAG_NOISE=1e-6 DIAG_SEED=0"; do
  env $cfg DIAG_FWD=exact DIAG_FWD_EXACT_K=7 DIAG_SERIAL=1 timeout -k 10 300 python tools/diag_strided_ab.py oracle > "gpurun_out/r4aa/${cfg// /_}.log" 2>&1
  echo "exact stem x (1 + noise) $cfg:"; grep "HIP native vs fp64 on own" "gpurun_out/r4aa/${cfg// /_}.log"
done
