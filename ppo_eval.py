"""Drop-in for the reference's ppo_eval.py."""
import _rtpkg  # noqa: F401
from ppo_radiotherapy_amd.evaluate import evaluate  # noqa: F401
