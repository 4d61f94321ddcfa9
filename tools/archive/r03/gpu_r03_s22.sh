#!/bin/bash
# r03 session 22: stream memory operation probe + device hand-off diagnostic
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s22
mkdir -p $O
timeout -k 10 60 ./tools/_probe_streamops > $O/probe.log 2>&1; echo "probe rc $?"; cat $O/probe.log
timeout -k 10 120 python -u tools/diag_handoff.py 2 > $O/diag2.log 2>&1; echo "diag rc $?"; tail -12 $O/diag2.log
echo ALLDONE
