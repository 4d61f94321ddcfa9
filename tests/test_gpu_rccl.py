"""The trainer's collective code path over RCCL (the `nccl` backend) on the
one GPU of the test box.

RCCL does not run two ranks on one device, so this is a world-1 process
group: the all-reduces are identities, but every call the 8-GPU run makes
goes through RCCL here with the trainer's own buffers and dtypes — the f64
advantage-sum all-reduce (rt_ppo_adv_sums -> all-reduce ->
rt_ppo_adv_finalize), the f32 flat-gradient all-reduce between the grad and
Adam kernels per minibatch, both as the library's own RCCL communicator
(rt_ppo_update_dp, the whole update in one call) and as the Python loop
around torch.distributed.all_reduce (bitwise the same), the
bench's MAX all-reduce of an f64 scalar and a barrier.  The collective update
must agree with the single-call rt_ppo_update from the same state (same
generator draws, same batch): train.py:183-248 either way, the only
difference being where the per-minibatch advantage statistics and ‖g‖² are
formed.  (The 2-rank data-parallel maths is tests/test_gpu_dp.py, over gloo.)"""
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


def _worker(port, q):
    import copy
    from types import SimpleNamespace

    import _rtpkg  # noqa: F401
    import torch.distributed as dist

    from ppo_radiotherapy_amd import assets
    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dev = torch.device("cuda", 0)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
        backend = dist.get_backend()
        lib = assets.synthetic_library((32, 32, 32), 50, 0)
        env = RadiotherapyVecEnv(256, library=lib, seed=5)
        torch.manual_seed(7)
        agent = PPO((9,), (6,), 64).cuda()
        cfg = SimpleNamespace(num_steps=16, num_minibatches=4, update_epochs=2, learning_rate=3e-4,
                              anneal_lr=False, gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.2,
                              clip_vloss=True, ent_coef=0.01, vf_coef=0.5, max_grad_norm=0.5, seed=0)
        tr = PPOTrainer(cfg, env, agent, "cuda", rank=0, world=1,
                        generator=torch.Generator(device="cuda").manual_seed(0))
        assert tr.fused_update and not tr.collective
        tr.reset()
        tr.train_iteration(1, 2)  # Adam state off zero
        tr.rollout()
        tr.compute_gae()
        start = copy.deepcopy(tr.state_dict())
        out = {}
        # collective paths: the library's own RCCL communicator (rt_ppo_update_dp,
        # one call per update), the per-minibatch Python loop around
        # torch.distributed.all_reduce (cfg.native_dp = False); then the single
        # call rt_ppo_update
        for mode in ("native", "loop", "single"):
            tr.load_state_dict(copy.deepcopy(start))
            tr.collective = mode != "single"
            tr.cfg.native_dp = mode == "native"
            tr._dp_comm = None if mode == "native" else False
            n = tr.update()
            torch.cuda.synchronize()
            if mode == "native":
                assert tr._dp_comm, "the native RCCL path did not run"
            out[mode] = (n, tr.flat_param.detach().cpu().numpy().copy(), tr._exp_avg.cpu().numpy().copy(),
                         tr._exp_avg_sq.cpu().numpy().copy(), int(tr._adam_step))
        # the native update runs the loop's kernels around RCCL's all-reduce: bitwise
        for a, b in zip(out["native"][1:4], out["loop"][1:4]):
            assert np.array_equal(a, b)
        out[True], out[False] = out["native"], out["single"]
        t = torch.tensor([1.5], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py max_over_ranks
        dist.barrier()
        torch.cuda.synchronize()
        q.put((backend, out[True], out[False], float(t.item())))
        env.close()
        dist.destroy_process_group()
    except Exception as exc:  # surfaced by the parent
        import traceback

        q.put((traceback.format_exc() + repr(exc), None, None, None))


def test_collective_update_over_rccl_matches_single_call():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    res = None
    deadline = time.time() + 240
    while res is None and time.time() < deadline:
        try:
            res = q.get(timeout=2)
        except queue.Empty:
            if p.exitcode not in (None, 0):
                break
    p.join(timeout=30)
    if p.is_alive():
        p.kill()
    assert res is not None, f"worker exit code {p.exitcode}"
    backend, coll, single, mx = res
    assert coll is not None, backend  # the traceback
    assert backend == "nccl"
    assert mx == 1.5
    assert coll[0] == single[0] == 8 and coll[4] == single[4]
    # same kernels either side of the identity all-reduce; the statistics and
    # the clip norm are formed by different reductions (f64 sums vs the fused
    # kernel's), so the agreement is to f32 rounding, not bitwise
    for a, b in zip(coll[1:4], single[1:4]):
        np.testing.assert_allclose(a, b, rtol=2e-5, atol=2e-7)
    assert np.abs(coll[1] - single[1]).max() < 1e-5
