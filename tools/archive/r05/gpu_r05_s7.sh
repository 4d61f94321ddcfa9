#!/bin/bash
# r05 session 7: dataflow rollout sweep (variant builds): dose-load cache bits,
# loads in flight, chain / dose wave split, claim chunk; timing-only
# diagnostics d1 (dose waves do not wait), d2 (chain waves do not wait), d3 (neither)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r05_s7
mkdir -p $O
B="--no-cpu --no-c3d --no-update --no-steady --steps 20 --warmup 4 --rollout-groups 16"
timeout -k 10 200 python3 bench.py $B > $O/base.json 2> $O/base.err || { tail -20 $O/base.err; exit 1; }
for v in fnt fsc1nt fu12 fcw6 fcw4 fch4 fch1 fd1 fd2 fd3; do
  RT_LIB_PATH=_variants/librtenv_$v.so timeout -k 10 200 python3 bench.py $B > $O/$v.json 2> $O/$v.err || { tail -20 $O/$v.err; exit 1; }
done
python3 - <<'PY'
import json
O = "gpurun_out/r05_s7"
for v in ["base", "fnt", "fsc1nt", "fu12", "fcw6", "fcw4", "fch4", "fch1", "fd1", "fd2", "fd3"]:
    d = json.load(open(f"{O}/{v}.json"))
    print(f"{v:7s} value {d['value']/1e6:7.3f} M  {d['ms_per_step']:.4f} ms  timed {d['roofline']['timed_pass_ms_per_step']:.4f}")
PY
echo ALLDONE
