"""`python train.py --config-file X --output-dir Y` (reference: train.py:20-29,91-324).

Same CLI, same config keys, same output layout:
  {output_dir}/{run_name}/config.yaml
  {output_dir}/tensorboard/{run_name}/          (TensorBoard or scalars.jsonl)
  {output_dir}/models/{run_name}/{exp_name}_{iteration}.model   (agent.state_dict())
plus, with `save_checkpoint` (default), a full trainer checkpoint beside each
model in {output_dir}/checkpoints/{run_name}/{exp_name}_{iteration}.ckpt that
`resume_from` continues (PPOTrainer.state_dict: agent, Adam state, counters).

Multi-GPU: launch with `python -m torch.distributed.run --nproc-per-node N
train.py ...`; `num_envs` is the global env count, sharded evenly over the
ranks (one process per GPU, RCCL gradient all-reduce per optimizer step).
"""
from __future__ import annotations

import argparse
import os
import random
import time

import numpy as np
import torch
import torch.distributed as dist

from . import assets, config as config_mod, logger
from .networks import PPO, PPO_3DCNN
from .ppo import PPOTrainer, broadcast_parameters
from .vec_env import RadiotherapyVecEnv


def get_argparser():
    parser = argparse.ArgumentParser(description="PPO radiotherapy (MI355X)", add_help=True)
    parser.add_argument("--config-file", type=str, default="config.yaml", help="path to the config file")
    parser.add_argument("--output-dir", type=str, help="path to the output directory")
    return parser


def _library(cfg):
    grid = tuple(cfg.grid) if cfg.get("grid") else None
    kind = cfg.get("tumour_library", "auto")
    if kind == "reference" or (kind == "auto" and grid is None):
        lib = assets.reference_library()
        if grid is not None and tuple(grid) != lib.shape:
            raise ValueError("the reference tumour library exists only at 67x43x70")
        return lib
    n = int(cfg.get("n_synthetic_tumours", 1000))
    if kind == "reference_style":  # graphics.py's generator (assets.reference_style_library)
        return assets.reference_style_library(n, int(cfg.seed), grid)
    return assets.synthetic_library(grid or (64, 64, 64), n, int(cfg.seed))


def env_seed(seed: int, rank: int, start_iteration: int) -> int:
    """Key of a rank's tumour-sampling stream (RadiotherapyVecEnv.reset(seed)).
    A fresh run keys it seed + rank; a run resumed at iteration k > 1 folds k
    in, so it does not replay the tumours of iteration 1."""
    s = seed + rank
    if start_iteration > 1:
        s ^= (start_iteration * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    return s & 0xFFFFFFFFFFFFFFFF


def train(cfg, writer, device, output_dir=None, run_name=None, rank=0, world=1):
    """train.py:91-282 on the device-resident env."""
    lib = _library(cfg)
    n_local = int(cfg.num_envs) // world
    envs = RadiotherapyVecEnv(n_local, visionless=bool(cfg.visionless), library=lib, device=device,
                              seed=int(cfg.seed) + rank, env_id_base=rank * n_local,
                              step_mode=str(cfg.get("step_mode", "dense")))
    obs_shape = envs.single_observation_space.shape
    act_shape = envs.single_action_space.shape
    Model = PPO if cfg.visionless else PPO_3DCNN
    agent = Model(obs_shape, act_shape, int(cfg.feature_dim)).to(device)
    if not cfg.visionless:
        agent.summary()
    broadcast_parameters(agent)
    gen = torch.Generator(device=device)
    gen.manual_seed(int(cfg.seed) * 7919 + rank)
    tr = PPOTrainer(cfg, envs, agent, device, rank, world, gen)
    start = 1
    if cfg.get("resume_from"):
        ck = torch.load(cfg.resume_from, map_location=device, weights_only=True)
        tr.load_state_dict(ck)
        start = tr.iteration + 1
        if rank == 0:
            print(f"resumed from {cfg.resume_from} at iteration {start}")
    tr.reset(seed=env_seed(int(cfg.seed), rank, start))
    iterator = range(start, int(cfg.num_iterations) + 1)
    if cfg.use_tqdm and rank == 0:
        try:
            from tqdm import tqdm

            iterator = tqdm(iterator)
        except Exception:  # noqa: BLE001
            pass
    t_start = time.perf_counter()
    for iteration in iterator:
        st = tr.train_iteration(iteration, int(cfg.num_iterations))
        if rank == 0 and writer is not None:
            logger.log_iteration(writer, tr.global_step, st)
            sps = tr.global_step / max(time.perf_counter() - t_start, 1e-9)
            writer.add_scalar("perf/env_steps_per_s", sps, tr.global_step)
            writer.add_scalar("perf/updates_per_s",
                              int(cfg.update_epochs) * int(cfg.num_minibatches) / max(st.update_s, 1e-9),
                              tr.global_step)
        if (cfg.save_model and output_dir is not None and
                ((cfg.save_frequency_iterations and iteration % cfg.save_frequency_iterations == 0)
                 or iteration == cfg.num_iterations)):
            # the fused update's state is whole (no lost grid arrival) before it is saved
            tr.check_device_status()
            # every rank takes part (the checkpoint gathers all ranks' generator states)
            ckpt = tr.state_dict() if cfg.get("save_checkpoint", True) else None
            if rank == 0:
                os.makedirs(f"{output_dir}/models/{run_name}", exist_ok=True)
                model_path = f"{output_dir}/models/{run_name}/{cfg.exp_name}_{iteration}.model"
                torch.save(agent.state_dict(), model_path)
                print(f"model saved to {model_path}")
                if ckpt is not None:
                    os.makedirs(f"{output_dir}/checkpoints/{run_name}", exist_ok=True)
                    torch.save(ckpt, f"{output_dir}/checkpoints/{run_name}/{cfg.exp_name}_{iteration}.ckpt")
    envs.close()
    return agent


def main(argv=None):
    args = get_argparser().parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    cfg = config_mod.derive(config_mod.load(args.config_file), world)
    output_dir = args.output_dir or "runs"
    run_name = f"{cfg.exp_name}_{int(time.time())}"

    if cfg.cuda:
        assert torch.cuda.is_available(), "CUDA is not available"
        torch.cuda.set_device(local)
    device = torch.device("cuda", local) if cfg.cuda else torch.device("cpu")
    if world > 1:
        dist.init_process_group("nccl" if cfg.cuda else "gloo",
                                device_id=device if cfg.cuda else None)
        # one run name for all ranks
        t = torch.tensor([int(time.time())], dtype=torch.int64, device=device)
        dist.broadcast(t, 0)
        run_name = f"{cfg.exp_name}_{int(t.item())}"

    writer = None
    if rank == 0:
        os.makedirs(f"{output_dir}/{run_name}", exist_ok=True)
        config_mod.save(cfg, f"{output_dir}/{run_name}/config.yaml")
        writer = logger.make_writer(f"{output_dir}/tensorboard/{run_name}")
        writer.add_text("hyperparameters",
                        "|param|value|\n|-|-|\n%s" % ("\n".join(f"|{k}|{v}|" for k, v in cfg.items())))

    # seeding (train.py:311-315); per-rank offsets for the env and sampling streams
    random.seed(cfg.seed)
    np.random.seed(cfg.seed)
    torch.manual_seed(cfg.seed)
    torch.backends.cudnn.deterministic = bool(cfg.torch_deterministic)
    if rank == 0:
        print("Using", device, f"x{world}" if world > 1 else "")
    agent = train(cfg, writer, device, output_dir, run_name, rank, world)
    if writer is not None:
        writer.close()
    if world > 1:
        dist.destroy_process_group()
    return agent
