# conv1 weight gradient: 2 column groups x 4 tiles at 4 waves/SIMD (tree) vs 1 x 7 at 2 waves (_variants kt7): parity, stage timings at 64^3, vision benches 64^3 / 128^3
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${OUT:-kt}
mkdir -p $OUT
NOBENCH=1 OUT=${OUT#gpurun_out/} VARS=kt7 bash tools/archive/gpu_c3d_var_ab.sh || exit 1
for v in tree kt7; do
  if [ $v = tree ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/_variants/librtenv_$v.so; fi
  for gr in 64 128; do
    timeout -k 10 480 python -u bench.py --vision --grid $gr --no-cpu > $OUT/v${gr}_$v.json 2> $OUT/v${gr}_$v.err || exit 1
    python -c "import json; d=json.loads(open('$OUT/v${gr}_$v.json').read().strip().splitlines()[-1]); s=d['c3d_mfma']['stages']['conv1']; print('$v grid $gr', 'upd_ms', round(d['ppo_update_ms'],1), 'conv1 wgrad ms', round(s['wgrad_ms'],3), 'train TF/s', round(d['c3d_mfma']['train_pass']['achieved'],1))"
  done
done
