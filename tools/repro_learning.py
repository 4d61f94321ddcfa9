"""Reproduce the reference's published learning outcome (README.md:44,
notebooks/figures/reward_curves.png: visionless, configs/default.yaml,
final-step episodic total reward plateauing near 4.6 from ~1.5e7 to 2.5e7 env
steps).

Runs train.py's `train()` on configs/default.yaml with only total_timesteps
raised to 2.5e7 (the figure's x range), writing the reference's TensorBoard
tags as scalars.jsonl under a scratch directory, and summarises the
charts/episodic_* series into 250 bins of 1e5 env steps plus the plateau
window means -> the JSON committed under profiles/.

    python tools/repro_learning.py --out gpurun_out/learning [--total 25000000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: E402,F401
import torch  # noqa: E402

from ppo_radiotherapy_amd import config as config_mod, logger  # noqa: E402
from ppo_radiotherapy_amd import train as train_mod  # noqa: E402

TAGS = {"charts/episodic_total_reward": "total", "charts/episodic_tumour_reward": "tumour",
        "charts/episodic_lung_reward": "lung", "charts/episodic_distance_reward": "distance",
        "charts/episodic_return": "return", "charts/episodic_length": "length"}


class ProgressWriter(logger.JsonlWriter):
    """scalars.jsonl plus one progress line per 25 iterations (gpurun's
    liveness check) and in-memory episodic series for the summary."""

    def __init__(self, logdir, n_iter):
        super().__init__(logdir)
        self.n_iter, self.it, self.t0 = n_iter, 0, time.time()
        self.series = {k: ([], []) for k in TAGS.values()}

    def add_scalar(self, tag, value, global_step=None):
        super().add_scalar(tag, value, global_step)
        if tag in TAGS:
            s, v = self.series[TAGS[tag]]
            s.append(int(global_step))
            v.append(float(value))
        if tag == "perf/env_steps_per_s":
            self.it += 1
            if self.it % 25 == 0 or self.it == self.n_iter:
                tot = self.series["total"][1][-2000:]
                print(f"iter {self.it}/{self.n_iter} step {global_step} {value:.0f} env steps/s "
                      f"recent final-step total reward {np.mean(tot) if tot else float('nan'):.3f} "
                      f"({time.time() - self.t0:.0f} s)", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="configs/default.yaml")
    ap.add_argument("--out", default="gpurun_out/learning")
    ap.add_argument("--total", type=int, default=25_000_000)
    ap.add_argument("--scratch", default="/tmp/repro_learning")
    ap.add_argument("--step-mode", default=None)
    ap.add_argument("--seed", type=int, default=None, help="override the config's seed (seed spread)")
    ap.add_argument("--fused-update", type=int, default=None,
                    help="0: the torch autograd update (train.py's own arithmetic path) instead of rt_ppo_update")
    a = ap.parse_args()
    cfg = config_mod.load(a.config)
    cfg.total_timesteps = a.total
    if a.seed is not None:
        cfg.seed = a.seed
    if a.step_mode:
        cfg.step_mode = a.step_mode
    if a.fused_update is not None:
        cfg.fused_update = bool(a.fused_update)
    cfg = config_mod.derive(cfg)
    torch.manual_seed(cfg.seed)
    np.random.seed(cfg.seed)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    w = ProgressWriter(os.path.join(a.scratch, "tensorboard"), int(cfg.num_iterations))
    t0 = time.time()
    train_mod.train(cfg, w, dev, output_dir=a.scratch, run_name="repro")
    wall = time.time() - t0
    w.close()
    os.makedirs(a.out, exist_ok=True)
    bin_w = 100_000
    nb = (a.total + bin_w - 1) // bin_w
    bins = {}
    for k, (s, v) in w.series.items():
        s, v = np.asarray(s), np.asarray(v)
        b = np.minimum(s // bin_w, nb - 1)
        cnt = np.bincount(b, minlength=nb)
        bins[k] = [round(float(x), 6) if c else None
                   for x, c in zip(np.bincount(b, weights=v, minlength=nb) / np.maximum(cnt, 1), cnt)]
    s_tot, v_tot = (np.asarray(x) for x in w.series["total"])
    plateau = {}
    for lo, hi in ((15e6, 25e6), (20e6, 25e6)):
        m = (s_tot >= lo) & (s_tot < hi)
        plateau[f"{lo / 1e6:.0f}M-{hi / 1e6:.0f}M"] = {
            k: float(np.mean(np.asarray(w.series[k][1])[m])) for k in TAGS.values()} if m.any() else None
    out = {"config": {k: cfg[k] for k in ("exp_name", "seed", "num_envs", "num_steps", "num_minibatches",
                                          "update_epochs", "learning_rate", "anneal_lr", "total_timesteps",
                                          "num_iterations", "visionless", "grid", "tumour_library", "step_mode")},
           "fused_update": bool(cfg.get("fused_update", True)),
           "wall_s": wall, "env_steps": int(cfg.num_iterations * cfg.batch_size),
           "logged_rows": len(s_tot), "bin_env_steps": bin_w,
           "reference": "README.md:44 / notebooks/figures/reward_curves.png: episodic total reward plateau ~4.6 "
                        "(1.5e7-2.5e7 env steps), tumour ~4.6, lung ~-8e-4, distance ~-0.005",
           "plateau_means": plateau, "bins": bins}
    with open(os.path.join(a.out, "learning_summary.json"), "w") as f:
        json.dump(out, f)
    print(json.dumps({"wall_s": wall, "plateau_means": plateau}))


if __name__ == "__main__":
    main()
