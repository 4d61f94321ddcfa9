#!/bin/bash
# r04 session 20: phase timeline of the dense step's chain kernels alone on
# the chip (stepwise launches, one stream) vs beside the dose stream
# (pipelined) -- is the policy kernel's 40 us staging phase contention?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s20
mkdir -p $O
timeout -k 10 300 python3 tools/trace_env.py --mode dense --steps 24 > $O/trace_alone.json 2> $O/trace_alone.err || { tail -30 $O/trace_alone.err; exit 1; }
timeout -k 10 300 python3 tools/trace_env.py --mode dense --pipelined --steps 24 > $O/trace_piped.json 2> $O/trace_piped.err || { tail -30 $O/trace_piped.err; exit 1; }
python3 - <<'PY'
import json
for n in ("alone", "piped"):
    d = json.load(open(f"gpurun_out/r04_s20/trace_{n}.json"))
    print(n, " ".join(f"{k}={v['median']:.1f}/{v['p90']:.1f}" for k, v in d["phases_us"].items()))
    for k, v in d["kernel_span_us"].items():
        print("   ", k, {a: round(b, 1) for a, b in v.items()})
PY
echo ALLDONE
