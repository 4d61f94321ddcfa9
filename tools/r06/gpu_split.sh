#!/bin/bash
# round 6: CU-split pipelined rollout (chain kernels on RT_PIPE_CHAIN_CUS CUs,
# k_dense on the rest): probe the CU-mask mapping and the masked read
# bandwidth, check the split rollout bitwise, sweep the split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r06_split; mkdir -p $O
hipcc --offload-arch=gfx950 -O3 tools/r06/cumask_probe.hip -o /tmp/cumask_probe || exit 1
timeout -k 10 120 /tmp/cumask_probe > $O/probe.txt 2>&1 || { cat $O/probe.txt; exit 1; }
cat $O/probe.txt
RT_PIPE_CHAIN_CUS=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rollout.py tests/test_gpu_headline.py > $O/pytest64.log 2>&1 || { tail -30 $O/pytest64.log; exit 1; }
tail -2 $O/pytest64.log
for K in ${SPLITS:-0 32 64 96}; do
  RT_PIPE_CHAIN_CUS=$K timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d --no-update > $O/b$K.json 2> $O/b$K.err || { tail -20 $O/b$K.err; exit 1; }
  python3 - $O/b$K.json $K <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
s = d["steady_state"]; r = d["roofline"]
print("chain_cus", sys.argv[2], "value %.3f M" % (d["value"] / 1e6), "ms %.4f" % d["ms_per_step"], "steady %.4f" % s["ms_per_step"],
      "kms", {k: round(v, 4) for k, v in r["kernel_ms_all"].items()}, "steady kms", {k: round(v, 4) for k, v in s["kernel_ms_per_step"].items()})
PY
done
echo ALLDONE
