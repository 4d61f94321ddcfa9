"""Data-parallel path of the fused update on the GPU: two ranks (gloo,
sharing the one GPU of the test box) run rollout + update on the HIP env.

Checked: the replicas stay bitwise identical, AND they equal a single-process
float64 update on the concatenated batch -- train.py:183-248 with the
minibatch i of an epoch = the union of the ranks' minibatches i, advantages
normalised with the union's statistics (rt_ppo_adv_sums -> all-reduce ->
rt_ppo_adv_finalize), torch autograd + clip_grad_norm_ + Adam in f64.  A
wrong all-reduce scale (sum instead of mean) or rank-local advantage
statistics keep replicas identical but fail the f64 comparison.

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

N_ENVS, T, N_MB, EPOCHS = 64, 16, 4, 2
HP = dict(clip_coef=0.1, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5, lr=3e-4)


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
        env = RadiotherapyVecEnv(N_ENVS, library=lib, seed=11 + rank, env_id_base=N_ENVS * rank)
        torch.manual_seed(100 + rank)  # different inits: broadcast must align them
        agent = PPO((9,), (6,), 64).cuda()
        broadcast_parameters(agent)
        cfg = SimpleNamespace(num_steps=T, num_minibatches=N_MB, update_epochs=EPOCHS, learning_rate=HP["lr"],
                              anneal_lr=False, gamma=0.99, gae_lambda=0.95, norm_adv=True,
                              clip_coef=HP["clip_coef"], clip_vloss=True, ent_coef=HP["ent_coef"],
                              vf_coef=HP["vf_coef"], max_grad_norm=HP["max_grad_norm"], seed=rank)
        tr = PPOTrainer(cfg, env, agent, "cuda", rank=rank, world=world,
                        generator=torch.Generator(device="cuda").manual_seed(rank))
        assert tr.fused_update and tr.fused_policy
        tr.reset()
        tr.train_iteration(1, 2)  # a first iteration moves the Adam state off zero
        tr.rollout()
        tr.compute_gae()
        tr._bind_batch()
        # numpy only through the queue (torch CPU tensors travel as shared-memory fds)
        sd0 = {k: v.detach().cpu().numpy().copy() for k, v in agent.state_dict().items()}
        adam0 = (tr._exp_avg.cpu().numpy().copy(), tr._exp_avg_sq.cpu().numpy().copy(), tr._adam_step)
        batch = {k: getattr(tr, "_b_" + k).cpu().numpy().copy()
                 for k in ("obs", "actions", "logprobs", "adv", "ret", "val")}
        tr.record_perms = []
        n = tr.update()
        torch.cuda.synchronize()
        flat = torch.cat([p.detach().reshape(-1) for p in tr.params]).cpu().numpy()
        perms = [p.cpu().numpy() for p in tr.record_perms]
        q.put((rank, flat, int(tr._adam_step), sd0, adam0, batch, perms, n))
        env.close()
        dist.destroy_process_group()
    except Exception as exc:  # surfaced by the parent
        import traceback

        q.put((rank, traceback.format_exc() + repr(exc), -1, None, None, None, None, None))


def _reference_update(sd0, adam0, batches, perms, names):
    """Single-process float64 update on the concatenated batch (train.py:183-248)."""
    from ppo_radiotherapy_amd.networks import PPO

    agent = PPO((9,), (6,), 64).double()
    agent.load_state_dict({k: torch.from_numpy(v).double() for k, v in sd0.items()})
    params = [dict(agent.named_parameters())[k] for k in names]
    opt = torch.optim.Adam(params, lr=HP["lr"], eps=1e-5)
    # the fused Adam state after the first iteration (flat, in `names` order)
    m, v, step = torch.from_numpy(adam0[0]), torch.from_numpy(adam0[1]), adam0[2]
    off = 0
    for p in params:
        k = p.numel()
        opt.state[p] = {"step": torch.tensor(float(step), dtype=torch.float64),
                        "exp_avg": m[off:off + k].double().view_as(p).clone(),
                        "exp_avg_sq": v[off:off + k].double().view_as(p).clone()}
        off += k
    cat = {k: torch.cat([torch.from_numpy(b[k]) for b in batches]).double() for k in batches[0]}
    B = batches[0]["adv"].size
    mbs = B // N_MB
    clip = HP["clip_coef"]
    for e in range(EPOCHS):
        for i in range(N_MB):
            rows = torch.cat([torch.as_tensor(perms[r][e][i * mbs:(i + 1) * mbs]) + r * B
                              for r in range(len(batches))])
            adv = cat["adv"][rows]
            adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            _, newlogp, entropy, newv = agent.get_action_and_value(cat["obs"][rows], cat["actions"][rows])
            ratio = (newlogp - cat["logprobs"][rows]).exp()
            pg = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
            nv = newv.view(-1)
            ret, val = cat["ret"][rows], cat["val"][rows]
            vl = 0.5 * torch.max((nv - ret) ** 2, (val + torch.clamp(nv - val, -clip, clip) - ret) ** 2).mean()
            loss = pg - HP["ent_coef"] * entropy.mean() + HP["vf_coef"] * vl
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(params, HP["max_grad_norm"])
            opt.step()
    return torch.cat([p.detach().reshape(-1) for p in params]).numpy()


def test_fused_update_data_parallel_two_ranks():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp

    from ppo_radiotherapy_amd.networks import PPO

    names = [n for n, _ in PPO((9,), (6,), 64).named_parameters()]  # trainer flat-buffer order
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
    assert res[0][2] == res[1][2] == 2 * EPOCHS * N_MB
    assert res[0][7] == EPOCHS * N_MB
    np.testing.assert_array_equal(res[0][1], res[1][1])  # replicas identical
    for k in res[0][3]:
        np.testing.assert_array_equal(res[0][3][k], res[1][3][k])  # same start on both ranks
    want = _reference_update(res[0][3], res[0][4], [r[5] for r in res], [r[6] for r in res],
                             names)
    p0 = np.concatenate([res[0][3][k].reshape(-1) for k in names]).astype(np.float64)
    got = res[0][1].astype(np.float64)
    moved = np.linalg.norm(want - p0)
    err = np.linalg.norm(got - want)
    assert moved > 1e-3, moved
    assert err <= 2e-3 * moved, (err, moved)
    assert np.abs(got - want).max() <= 2e-5, np.abs(got - want).max()


# --- vision agent (configs[4]'s split): C3D kernels + micro-batched autograd update
VIS_GRID, VIS_ENVS, VIS_T, VIS_MB, VIS_MICRO = (32, 32, 32), 8, 8, 2, 12
VIS_HP = dict(clip_coef=0.1, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5, lr=3e-4)


def _vision_worker(rank, world, port, q):
    import _rtpkg  # noqa: F401
    import torch.distributed as dist
    from types import SimpleNamespace

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import dp_ref
    from ppo_radiotherapy_amd import assets
    from ppo_radiotherapy_amd.networks import PPO_3DCNN
    from ppo_radiotherapy_amd.ppo import PPOTrainer, broadcast_parameters
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        lib = assets.synthetic_library(VIS_GRID, 50, 0)
        env = RadiotherapyVecEnv(VIS_ENVS, visionless=False, library=lib, seed=21 + rank,
                                 env_id_base=VIS_ENVS * rank)
        torch.manual_seed(200 + rank)
        agent = PPO_3DCNN((4, *VIS_GRID), (6,), 64).cuda()
        broadcast_parameters(agent)
        cfg = SimpleNamespace(num_steps=VIS_T, num_minibatches=VIS_MB, update_epochs=2, learning_rate=VIS_HP["lr"],
                              anneal_lr=False, gamma=0.99, gae_lambda=0.95, norm_adv=True,
                              clip_coef=VIS_HP["clip_coef"], clip_vloss=True, ent_coef=VIS_HP["ent_coef"],
                              vf_coef=VIS_HP["vf_coef"], max_grad_norm=VIS_HP["max_grad_norm"], seed=rank,
                              micro_batch=VIS_MICRO)
        tr = PPOTrainer(cfg, env, agent, "cuda", rank=rank, world=world,
                        generator=torch.Generator(device="cuda").manual_seed(rank))
        assert not tr.fused_update and tr.compact_obs and tr.collective
        tr.reset()
        tr.train_iteration(1, 2)  # Adam state off zero
        tr.rollout()
        tr.compute_gae()
        tr._bind_batch()
        sd0 = {k: v.detach().cpu().numpy().copy() for k, v in agent.state_dict().items()}
        opt0 = dp_ref.optimizer_state_numpy(tr.optimizer)
        batch = dp_ref.trainer_batch(tr)
        tr.record_perms = []
        tr.update()
        torch.cuda.synchronize()
        flat = torch.cat([p.detach().reshape(-1) for p in tr.params]).cpu().numpy()
        q.put((rank, flat, sd0, opt0, batch, [p.cpu().numpy() for p in tr.record_perms]))
        env.close()
        dist.destroy_process_group()
    except Exception as exc:  # surfaced by the parent
        import traceback

        q.put((rank, traceback.format_exc() + repr(exc), None, None, None, None))


def test_vision_micro_batched_update_data_parallel_two_ranks():
    """PPO_3DCNN on the HIP env and the C3D kernels, two gloo ranks on the one
    GPU, micro_batch < minibatch (train.py:215-218 across ranks): replicas
    identical AND equal to a single-process f64 update of the union batch
    (tests/dp_ref.py); rank-local advantage statistics would fail it."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import dp_ref
    from ppo_radiotherapy_amd.networks import PPO_3DCNN

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_vision_worker, args=(r, world, port, q)) for r in range(world)]
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
    np.testing.assert_array_equal(res[0][1], res[1][1])  # replicas identical
    args = (res[0][2], res[0][3], [r[4] for r in res], [r[5] for r in res], VIS_MB, VIS_HP)
    want = dp_ref.union_update_f64(PPO_3DCNN((4, *VIS_GRID), (6,), 64), *args)
    local = dp_ref.union_update_f64(PPO_3DCNN((4, *VIS_GRID), (6,), 64), *args, local_norm=True)
    p0 = np.concatenate([v.reshape(-1) for v in res[0][2].values()]).astype(np.float64)
    got = res[0][1].astype(np.float64)
    moved = np.linalg.norm(want - p0)
    err = np.linalg.norm(got - want)
    assert moved > 1e-3, moved
    assert err <= 5e-3 * moved, (err, moved)
    assert np.linalg.norm(local - want) > 10 * err, (np.linalg.norm(local - want), err)
