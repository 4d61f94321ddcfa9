#!/bin/bash
# r04 session 7: dose-stream shape sweep of the pipelined dense rollout
# (k_dense_persist blocks per CU x float4 loads in flight per thread; variant
# builds through RT_LIB_PATH, two runs each, staggered phases), plus the raw
# phase stamps of the pipelined rollout (staggered) for per-block analysis
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04_s7
mkdir -p $O
timeout -k 10 300 python3 tools/trace_env.py --mode dense --pipelined --stagger --steps 24 --dump $O/stamps.npy > $O/trace_stagger.json 2> $O/trace_stagger.err || { tail -30 $O/trace_stagger.err; exit 1; }
for rep in 1 2; do
for v in b6u8 b4u8 b4u12 b3u16 b5u8; do
  RT_LIB_PATH=tools/_variants/$v.so timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-c3d > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { tail -30 $O/bench_${v}_$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_${v}_$rep.json')); r=d['roofline']; s=d['steady_state']; print('$v', $rep, 'value', round(d['value']/1e6,3), 'ms', round(d['ms_per_step'],4), 'steady', round(s['ms_per_step'],4), 'kms', {k: round(x,4) for k,x in r['kernel_ms_all'].items()}, 'steady kms', {k: round(x,4) for k,x in s['kernel_ms_per_step'].items()}, 'iso', round(r['isolated']['kernel_ms'],4))"
done
done
echo ALLDONE
