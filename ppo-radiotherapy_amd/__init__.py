"""MI355X-native vectorised radiotherapy environment + PPO trainer.

Drop-in for rmaguado/ppo-radiotherapy's hot path: the environment step
(environment.py / draw_line.py / transforms.py) runs as hand-written HIP
kernels for gfx950 behind the C-ABI in include/rtenv.h (librtenv.so); the
rollout storage, GAE and the PPO update run in PyTorch-ROCm.

Import as `import _rtpkg; import ppo_radiotherapy_amd` (the directory name is
hyphenated)."""

__version__ = "0.1.0"

PACKAGE_DIR = __path__[0]
