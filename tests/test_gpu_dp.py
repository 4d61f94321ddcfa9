"""Data-parallel path of the fused update on the GPU: two ranks (gloo,
sharing the one GPU of the test box) run rollout + update on the HIP env;
replicas stay identical and equal the average-gradient step.

(The 8-GPU RCCL run is the driver's; this covers rt_ppo_grad -> all-reduce ->
rt_adam_step with real kernels.)"""
import os
import queue
import socket
import sys
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import _rtpkg  # noqa: F401
    import torch.distributed as dist
    from types import SimpleNamespace

    from ppo_radiotherapy_amd import assets
    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer, broadcast_parameters
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        lib = assets.synthetic_library((32, 32, 32), 50, 0)
        env = RadiotherapyVecEnv(64, library=lib, seed=11 + rank, env_id_base=64 * rank)
        torch.manual_seed(100 + rank)  # different inits: broadcast must align them
        agent = PPO((9,), (6,), 64).cuda()
        broadcast_parameters(agent)
        cfg = SimpleNamespace(num_steps=16, num_minibatches=4, update_epochs=2, learning_rate=3e-4, anneal_lr=False,
                              gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True,
                              ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5, seed=rank)
        tr = PPOTrainer(cfg, env, agent, "cuda", rank=rank, world=world,
                        generator=torch.Generator(device="cuda").manual_seed(rank))
        assert tr.fused_update and tr.fused_policy
        tr.reset()
        for it in (1, 2):
            tr.train_iteration(it, 2)
        torch.cuda.synchronize()
        flat = torch.cat([p.detach().reshape(-1) for p in tr.params]).cpu().numpy()
        q.put((rank, flat, int(tr._adam_step)))
        env.close()
        dist.destroy_process_group()
    except Exception as exc:  # surfaced by the parent
        q.put((rank, repr(exc), -1))


def test_fused_update_data_parallel_two_ranks():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    deadline = time.time() + 300
    while len(res) < world and time.time() < deadline:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert len(res) == world, res
    res.sort(key=lambda r: r[0])
    for r in res:
        assert not isinstance(r[1], str), r[1]
    assert res[0][2] == res[1][2] == 2 * 2 * 4
    np.testing.assert_array_equal(res[0][1], res[1][1])  # replicas identical after 16 optimizer steps
