"""Scalar logging with the reference's TensorBoard tags (train.py:42-88,304-309).

Uses torch.utils.tensorboard when the tensorboard package is importable;
otherwise writes the same (tag, value, step) records as JSON lines to
`<logdir>/scalars.jsonl`, so runs stay comparable without the dependency."""
from __future__ import annotations

import json
import os
import time


class JsonlWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, "scalars.jsonl")
        self._f = open(self.path, "a", buffering=1)

    def add_scalar(self, tag, value, global_step=None):
        self._f.write(json.dumps({"tag": tag, "value": float(value), "step": int(global_step or 0),
                                  "wall_time": time.time()}) + "\n")

    def add_text(self, tag, text, global_step=None):
        self._f.write(json.dumps({"tag": tag, "text": str(text), "step": int(global_step or 0)}) + "\n")

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def make_writer(logdir: str):
    try:
        from torch.utils.tensorboard import SummaryWriter  # needs the tensorboard package

        return SummaryWriter(logdir)
    except Exception:  # noqa: BLE001
        return JsonlWriter(logdir)


EPISODE_TAGS = ("charts/episodic_return", "charts/episodic_length", "charts/episodic_tumour_reward",
                "charts/episodic_lung_reward", "charts/episodic_distance_reward", "charts/episodic_total_reward")


def log_episode_steps(writer, rows):
    """log_episode_statistics (train.py:42-66) at every rollout step where
    episodes finished (train.py:159-161), at that step's own global_step:
    rows = IterStats.episode_steps (global_step, n, mean r, mean l, mean
    tumour / lung / distance / total reward of the finishing step)."""
    for gs, _, r, l, tum, lung, dist, tot in rows:
        for tag, v in zip(EPISODE_TAGS, (r, l, tum, lung, dist, tot)):
            writer.add_scalar(tag, v, gs)


def log_iteration(writer, global_step: int, st):
    """The reference's tag set: episode statistics per rollout step (as
    train.py logs them), losses once per iteration (train.py:252-268)."""
    if st.episode_steps is not None:
        log_episode_steps(writer, st.episode_steps)
    elif st.episodes:  # iteration aggregate (a trainer without per-step rows)
        for tag, v in zip(EPISODE_TAGS, (st.episodic_return, st.episodic_length, st.tumour_reward,
                                         st.lung_reward, st.distance_reward, st.total_reward)):
            writer.add_scalar(tag, v, global_step)
    writer.add_scalar("charts/learning_rate", st.learning_rate, global_step)
    writer.add_scalar("losses/value_loss", st.value_loss, global_step)
    writer.add_scalar("losses/policy_loss", st.policy_loss, global_step)
    writer.add_scalar("losses/entropy", st.entropy, global_step)
    writer.add_scalar("losses/old_approx_kl", st.old_approx_kl, global_step)
    writer.add_scalar("losses/approx_kl", st.approx_kl, global_step)
    writer.add_scalar("losses/clipfrac", st.clipfrac, global_step)
    writer.add_scalar("losses/explained_variance", st.explained_variance, global_step)
    writer.add_scalar("perf/rollout_s", st.rollout_s, global_step)
    writer.add_scalar("perf/update_s", st.update_s, global_step)
