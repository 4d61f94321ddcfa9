"""Episode-end census of the headline rollout (tests/test_gpu_headline.py)
for candidate tumour libraries / policies: how many envs end episodes by
irradiation vs the t = 100 truncation inside 128 steps."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")]
import _rtpkg  # noqa
import numpy as np
from ppo_radiotherapy_amd import assets
import test_gpu_headline as H


def golden(name):
    return dict(np.load(os.path.join(REPO, "tests", "golden", name)))


syn = assets.synthetic_library((64, 64, 64), 1000, 0)
for kind, lib, still in (("synthetic64", syn, False), ("rods+syn trained", H.beam_line_library(syn), False),
                         ("rods+syn still", H.beam_line_library(syn), True)):
    rec, env, _ = H.run_headline_rollout(golden, "dense", lib, still=still)
    I = rec["infos"]
    done = I[..., 17] > 0.5
    ln = np.where(done, I[..., 19], 0)
    irr = ((ln > 0) & (ln < 100))
    print(kind, "envs with irradiation end", int(irr.any(0).sum()), "irr episodes", int(irr.sum()),
          "trunc episodes", int((ln == 100).sum()), "median irr len", float(np.median(ln[irr])) if irr.any() else -1,
          "mean reward", float(rec["rewards"].mean()), flush=True)
    if kind != "synthetic64":
        s = H.pick_sample(rec)
        print("sample", len(s), flush=True)
    env.close()
