# C3D kernels: parity tests (stages, extractor, configs[3]/[4]) then the vision bench with a kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-c3d}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_c3d.py tests/test_gpu_configs.py tests/test_gpu_vision.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/c3dprof -o run -- python3 bench.py --vision --no-cpu --steps 16 --warmup 4 > $OUT/bench.json 2> $OUT/bench.err || exit 1
python tools/rocpd_stats.py /tmp/c3dprof/run_results.db $OUT/kernel_stats.csv | head -14
timeout -k 10 300 python -u bench.py --vision --no-cpu > $OUT/bench_plain.json 2> $OUT/bench_plain.err || exit 1
python -c "import json; d=json.loads(open('$OUT/bench_plain.json').read().strip().splitlines()[-1]); print('vision env steps/s', round(d['value']), 'update_ms', round(d['ppo_update_ms'],1), 'train', round(d['train_env_steps_per_s']), 'c3d fwd TF/s', round(d['roofline']['c3d_mfma']['achieved'],1))"
