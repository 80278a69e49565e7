#!/bin/bash
# host-side probe under several HIP graph-submission settings (development; see tools/host_probe.py)
set -e
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 150 python -u tools/host_probe.py > $O/default.json 2> $O/default.err
for v in "DEBUG_HIP_GRAPH_BATCH_SIZE=1" "DEBUG_HIP_GRAPH_BATCH_SIZE=8" "DEBUG_HIP_GRAPH_BATCH_SIZE=64" \
         "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1"; do
  env $v timeout -k 10 150 python -u tools/host_probe.py > $O/$v.json 2> $O/$v.err
done
