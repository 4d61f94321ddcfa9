#!/bin/bash
# r04 session 36: the PPO update's kernel timeline (rocprofv3 kernel trace of
# the bench's update phase): gaps between k_ppo_grad_mfma and
# k_ppo_reduce_adam per minibatch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s36
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 4 --warmup 2 --no-cpu --no-c3d --no-steady > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY' > $O/update_gaps.txt
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"][:60], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
idx = [i for i, k in enumerate(ks) if "k_ppo_grad_mfma<0>" in k[0]]
# the timed f32 update: the second run of 80 consecutive grad launches
runs, cur = [], []
for i in idx:
    if cur and i - cur[-1] > 2: runs.append(cur); cur = []
    cur.append(i)
runs.append(cur)
print("runs of f32 grad launches:", [len(r) for r in runs])
r = runs[1] if len(runs) > 1 else runs[0]
g1, g2, dg, dr = [], [], [], []
for a in r:
    g, red = ks[a], ks[a + 1]
    dg.append((g[2] - g[1]) / 1e3); dr.append((red[2] - red[1]) / 1e3)
    g1.append((red[1] - g[2]) / 1e3)
    if a + 2 < len(ks): g2.append((ks[a + 2][1] - red[2]) / 1e3)
import statistics as st
print("grad us", round(st.median(dg), 2), "reduce_adam us", round(st.median(dr), 2),
      "gap grad->reduce", round(st.median(g1), 2), "gap reduce->next", round(st.median(g2[:-1]), 2))
first = ks[r[0] - 6: r[0]]
for k in first: print("before:", k[0], round((k[2] - k[1]) / 1e3, 2))
span = (ks[r[-1] + 1][2] - ks[r[0]][1]) / 1e3
print("span of", len(r), "minibatches us", round(span, 1), "per mb", round(span / len(r), 2))
PY
cat $O/update_gaps.txt
rm -rf $O/prof
echo ALLDONE
