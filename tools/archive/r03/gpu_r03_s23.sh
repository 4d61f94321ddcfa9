#!/bin/bash
# r03 session 23: latencies of the stream memory operations vs events (device hand-off design)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03_s23
mkdir -p $O
timeout -k 10 120 ./tools/_probe_streamops > $O/probe.log 2>&1; echo "probe rc $?"; cat $O/probe.log
