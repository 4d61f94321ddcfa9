"""Drop-in for the reference's environment.py: `from environment import RadiotherapyEnv`.

The env runs on the MI355X (HIP kernels behind include/rtenv.h); see
ppo-radiotherapy_amd/env.py for the single-env facade and vec_env.py for the
vectorised env used by train.py."""
import _rtpkg  # noqa: F401
from ppo_radiotherapy_amd.env import RadiotherapyEnv  # noqa: F401
from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv  # noqa: F401
