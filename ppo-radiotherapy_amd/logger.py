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


def log_iteration(writer, global_step: int, st):
    """The reference's tag set; episode means cover the episodes that finished
    during the iteration (the reference writes them per rollout step)."""
    if st.episodes:
        writer.add_scalar("charts/episodic_return", st.episodic_return, global_step)
        writer.add_scalar("charts/episodic_length", st.episodic_length, global_step)
        writer.add_scalar("charts/episodic_tumour_reward", st.tumour_reward, global_step)
        writer.add_scalar("charts/episodic_lung_reward", st.lung_reward, global_step)
        writer.add_scalar("charts/episodic_distance_reward", st.distance_reward, global_step)
        writer.add_scalar("charts/episodic_total_reward", st.total_reward, global_step)
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
