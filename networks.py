"""Drop-in for the reference's networks.py (same classes and state-dict keys)."""
import _rtpkg  # noqa: F401
from ppo_radiotherapy_amd.networks import FeaturesExtractor3D, PPO, PPO_3DCNN, layer_init  # noqa: F401
