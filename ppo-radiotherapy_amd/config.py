"""YAML configs with the reference's keys (configs/*.yaml.template) and its
runtime-derived fields (train.py:291-297).

OmegaConf is used when importable (the reference's loader); otherwise a small
attribute dict over yaml.safe_load with the same `cfg.key` access and
`save()` round trip."""
from __future__ import annotations

import yaml

try:  # pragma: no cover - omegaconf is not in this image
    import omegaconf  # type: ignore
except Exception:  # noqa: BLE001
    omegaconf = None

# keys of configs/default.yaml.template with their reference values
DEFAULTS = {
    "exp_name": "default", "seed": 1, "torch_deterministic": True, "cuda": True, "save_model": True,
    "use_tqdm": False, "total_timesteps": 10000000, "num_saves": 5, "learning_rate": 3e-4, "num_envs": 16,
    "num_steps": 2048, "anneal_lr": False, "num_minibatches": 32, "update_epochs": 10, "gamma": 0.99,
    "gae_lambda": 0.95, "norm_adv": True, "clip_coef": 0.1, "clip_vloss": True, "ent_coef": 0.0, "vf_coef": 0.5,
    "max_grad_norm": 0.5, "feature_dim": 64, "visionless": True, "batch_size": 0, "minibatch_size": 0,
    "num_iterations": 0, "save_frequency_iterations": 0,
    # additions of this framework (optional in user configs)
    "grid": None,              # None: the reference grid and assets (67x43x70); else [D,H,W] synthetic
    "tumour_library": "auto",  # auto | reference | synthetic | reference_style
    "n_synthetic_tumours": 1000,
    # env step formulation: dense = the reference's full-volume
    # lung reductions every step; incremental = maintained on the touched
    # voxels (visionless only; same rewards and termination bit for bit)
    "step_mode": "dense",
    # checkpoint / resume: with every saved .model, a full trainer
    # checkpoint {output_dir}/checkpoints/{run_name}/{exp_name}_{iteration}.ckpt;
    # resume_from: such a file -> the run continues at its iteration + 1
    "save_checkpoint": True,
    "resume_from": None,
    # arithmetic (include/rtenv.h, passed per call): the fused visionless
    # update's 64x64 layer products and the C3D forward products, "f32" (the
    # reference's) or "bf16x3"
    "update_precision": "f32",
    "conv_precision": "f32",
}


class _Loader(yaml.SafeLoader):
    """YAML 1.1 loader that also reads `3e-4` as a float (as OmegaConf does;
    plain PyYAML would return the string)."""


_Loader.add_implicit_resolver(
    "tag:yaml.org,2002:float",
    __import__("re").compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
        |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
        |\.[0-9_]+(?:[eE][-+][0-9]+)?
        |[-+]?\.(?:inf|Inf|INF)
        |\.(?:nan|NaN|NAN))$""", __import__("re").X),
    list("-+0123456789."))


class Config(dict):
    """dict with attribute access (the subset of DictConfig train.py uses)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as exc:
            raise AttributeError(k) from exc

    def __setattr__(self, k, v):
        self[k] = v


def load(path: str) -> Config:
    with open(path) as f:
        raw = yaml.load(f, Loader=_Loader) or {}
    cfg = Config(DEFAULTS)
    cfg.update(raw)
    return cfg


def derive(cfg: Config, world: int = 1) -> Config:
    """train.py:292-297.  num_envs is the global env count (split across ranks)."""
    cfg.batch_size = int(cfg.num_envs * cfg.num_steps)
    cfg.minibatch_size = int(cfg.batch_size // cfg.num_minibatches)
    cfg.num_iterations = cfg.total_timesteps // cfg.batch_size
    cfg.save_frequency_iterations = cfg.num_iterations // cfg.num_saves if cfg.num_saves > 0 else 0
    if cfg.num_envs % world:
        raise ValueError(f"num_envs={cfg.num_envs} must be divisible by the world size {world}")
    return cfg


def save(cfg: Config, path: str):
    with open(path, "w") as f:
        yaml.safe_dump(dict(cfg), f, sort_keys=False)
