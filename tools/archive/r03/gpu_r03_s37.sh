#!/bin/bash
# r03 session 37: kernel census of the configs[3] vision iteration with bf16x3 conv products
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r03_s37
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --vision --no-cpu --no-steady --no-c3d --steps 4 --warmup 2 --conv-precision bf16x3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
find $O/prof -name "*.db" -delete
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r03_s37/kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total ms", tot / 1e6)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:28]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:100]}')
PY
