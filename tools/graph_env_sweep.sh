#!/bin/bash
# hipGraph dispatch settings vs the per-node floor (tools/graph_launch_floor.py):
# tools/graph_env_sweep.sh <out dir>
set -u
OUT=$1
mkdir -p "$OUT"
for v in base DEBUG_HIP_FORCE_GRAPH_QUEUES=1 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 \
         DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 DEBUG_HIP_GRAPH_BATCH_SIZE=1 \
         DEBUG_HIP_GRAPH_BATCH_SIZE=64; do
  if [ "$v" = base ]; then envs=""; else envs="$v"; fi
  for e in 1 262144; do
    env $envs timeout -k 10 60 python3 tools/graph_launch_floor.py 512 $e > "$OUT/floor_${v}_$e.log" 2>&1 || { echo "$v failed"; exit 1; }
    echo "$v E=$e: $(grep -h nodes "$OUT/floor_${v}_$e.log" | tr '\n' ' ')"
  done
done
