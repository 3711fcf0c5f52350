#!/bin/bash
# A/B of the channels-last cost kernels' pixel tile: TPS="8 4" (the in-tree build is TP_DEFAULT,
# others dro-sfm_amd/libab_tp<N>.so built with -DDRO_WARP_CL_TP=<N>): warp-cost tests + probe per build
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abtp
for v in ${TPS:-8 4}; do
  if [ $v = ${TP_DEFAULT:-8} ]; then L=""; else L="DRO_LIB_PATH=$GRAFT_REPO_ROOT/dro-sfm_amd/libab_tp$v.so"; fi
  env $L timeout -k 10 120 python3 -u -m pytest tests/test_hip_parity.py -x -q --timeout 120 -m gpu -k "warp_cost" > gpurun_out/abtp/t_$v.log 2>&1 || { echo "tests $v failed"; exit 1; }
  env $L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/abtp/p$v -o p -- python3 -u tools/warp_state_probe.py 8 10 > gpurun_out/abtp/probe_$v.txt 2>&1 || exit 1
  echo "tp $v: $(tail -1 gpurun_out/abtp/t_$v.log)"
done
