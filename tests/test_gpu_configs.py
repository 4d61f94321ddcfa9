"""BASELINE configs[3] and configs[4] at their real per-GPU sizes.

* configs[4] (C3D, 128^3, 4096 envs over 8 GPUs = 512 per GPU): the 512-env
  vision env at 128^3 for 101 steps (every env crosses the t = 100 truncation
  and its Philox tumour redraw), sampled envs replayed on the oracle with
  their full 4-channel observations rebuilt from the oracle's state
  (environment.py:245-257); the C3D stage kernels at the 128^3 stage dims
  (126^3 conv -> 63^3 pool, 61^3 -> 30^3, 28^3 -> 14^3) and at a grid of the
  other pool-padding parity (networks.py:18-20), vs torch f32 and f64
  autograd; the whole extractor at 128^3 vs its torch modules in f64.
* configs[3] (vision.yaml C3D, 512 envs, 64^3): the T = 16 C3D rollout with
  compact storage (dose/pose/tumour snapshots) replayed on the
  oracle, rendered observation rows vs the oracle's, and one 4096-sample
  compact-storage PPO minibatch: its gradient is micro-batch invariant
  (128 vs 1024 rows per kernel call) and a sample subset's gradient matches
  float64 autograd of the reference loss (train.py:200-238).
"""
import os
import sys
from types import SimpleNamespace

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import rt_rng  # noqa: E402
import test_gpu_c3d as C  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def oracle_vision_obs(lib, tid, oe):
    """environment.py:245-257 from the oracle's state: clip(stack[lungs,
    tumour, dose, beam(pos, dir) + beam(pos, [1, 0, 0])], 0, 1)."""
    pos, d, _ = oe.pose()
    view = O.beam_dense(lib.shape, pos, d) + O.beam_dense(lib.shape, pos, np.array([1.0, 0.0, 0.0]))
    obs = np.stack([lib.lungs.astype(np.float32), lib.tumour_dense(tid), oe.dose, view])
    return np.clip(obs, np.float32(0), np.float32(1))


# ---------------------------------------------------------------- configs[4]
def test_config4_vision_env_128_vs_oracle():
    """512 vision envs at 128^3, 101 steps (truncation autoreset at step 100
    with a Philox redraw); 4 sampled envs: rewards, components, done every
    step, full observations at 5 steps, dose volumes at the end."""
    from ppo_radiotherapy_amd import assets
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    lib = assets.synthetic_library((128, 128, 128), 1000, 0)
    N, T, seed = 512, 101, 4242
    env = RadiotherapyVecEnv(N, visionless=False, library=lib, seed=seed)
    obs, _ = env.reset()
    g = torch.Generator(device="cuda").manual_seed(3)
    sample = [0, 177, 300, 511]
    check_at = {0, 1, 57, 99, 100}
    K = lib.n_tumours
    oes, tids = {}, {}
    for e in sample:
        tids[e] = rt_rng.tumour_draw(seed, e, 0, K)
        oes[e] = O.OracleEnv(lib.lungs.astype(np.float32), lib.tumour_dense(tids[e]))
        oes[e].reset()
    draws = {e: 1 for e in sample}
    pending = {e: False for e in sample}
    for t in range(T + 1):
        if t in check_at or t == T:
            for e in sample:
                want = oracle_vision_obs(lib, tids[e], oes[e])
                got = obs[e].cpu().numpy()
                np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg=f"env {e} t {t}")
        if t == T:
            break
        a = torch.rand((N, 6), device="cuda", generator=g) * 2.4 - 1.2
        obs, rew, term, _, infos = env.step(a)
        a_h, r_h, term_h = a.cpu().numpy(), rew.cpu().numpy(), term.cpu().numpy()
        rc = {k: infos["reward_components"][k].cpu().numpy() for k in ("tumour", "lung", "distance_to_tumour")}
        dz = {k: infos["doses"][k].cpu().numpy() for k in ("tumour", "lung")}
        stepped = infos["_reward_components"].cpu().numpy()
        for e in sample:
            if pending[e]:
                tids[e] = rt_rng.tumour_draw(seed, e, draws[e], K)
                draws[e] += 1
                oes[e].reset(lib.tumour_dense(tids[e]))
                assert not stepped[e] and r_h[e] == 0.0 and not term_h[e]
                pending[e] = False
                continue
            _, oi, done = oes[e].step(a_h[e])
            assert abs(r_h[e] - oi[0]) <= 1e-5, (e, t, r_h[e], oi[0])
            assert abs(rc["tumour"][e] - oi[1]) <= 1e-5 and abs(rc["lung"][e] - oi[2]) <= 1e-5
            assert abs(rc["distance_to_tumour"][e] - oi[3]) <= 1e-5
            # doses (environment.py:233-236): bit-exact -- doses.lung through the
            # lung sum plan gathered from the C-order rows (k_dense<true>)
            assert dz["tumour"][e] == np.float32(oi[4]) and dz["lung"][e] == np.float32(oi[5]), (e, t)
            assert bool(term_h[e]) == done, (e, t)
            pending[e] = done
    assert all(draws[e] >= 2 for e in sample)  # every sampled env crossed an autoreset
    dose = env.dose()
    for e in sample:
        np.testing.assert_array_equal(dose[e].cpu().numpy().view(np.uint32), oes[e].dose.view(np.uint32))
    env.close()


# stage shapes of the 128^3 extractor and of a grid with the other first-pool parity
STAGES_128 = [  # cin, groups, dims, pool_pad, batch
    (4, 1, (128, 128, 128), (0, 0, 0), 1),
    (4, 1, (127, 129, 128), (1, 1, 0), 1),
    (16, 2, (63, 63, 63), (0, 0, 0), 2),
    (16, 4, (30, 30, 30), (0, 0, 0), 2),
    (16, 2, (64, 63, 64), (0, 0, 0), 1),
]
IDS_128 = ["conv1-128", "conv1-127x129x128-pad", "conv2-63", "conv3-30", "conv2-64x63x64"]


@pytest.mark.parametrize("cin,groups,dims,pad,B", STAGES_128, ids=IDS_128)
def test_config4_c3d_stage_forward(cin, groups, dims, pad, B):
    C.test_conv_relu_pool_forward(cin, groups, dims, pad, B)


@pytest.mark.parametrize("cin,groups,dims,pad,B", STAGES_128, ids=IDS_128)
def test_config4_c3d_stage_backward(cin, groups, dims, pad, B):
    C.test_conv_relu_pool_backward(cin, groups, dims, pad, B)


def test_config4_features_extractor_128():
    """FeaturesExtractor3D((4, 128, 128, 128)) on the fused kernels vs its
    torch modules in float64: features and every parameter gradient."""
    from ppo_radiotherapy_amd.networks import FeaturesExtractor3D

    torch.manual_seed(1)
    shape = (4, 128, 128, 128)
    fe = FeaturesExtractor3D(shape, 64)
    assert fe.n_flatten == 16 * 14 ** 3
    ref = FeaturesExtractor3D(shape, 64).double()
    ref.load_state_dict({k: v.double() for k, v in fe.state_dict().items()})
    fe = fe.cuda()
    x = torch.rand((2, *shape))
    x[:, 3] = (x[:, 3] > 0.97).float()  # sparse beam-view-like channel
    f = fe(x.cuda())
    fr = ref(x.double())
    torch.testing.assert_close(f.cpu().double(), fr, rtol=1e-4, atol=1e-5)
    gf = torch.randn_like(fr)
    f.backward(gf.float().cuda())
    fr.backward(gf)
    for (n, p), q in zip(fe.named_parameters(), ref.parameters()):
        err = float((p.grad.cpu().double() - q.grad).abs().max()) / (float(q.grad.abs().max()) + 1e-12)
        assert err < 2e-3, (n, err)


# ---------------------------------------------------------------- configs[3]
def _ppo_loss_f64(agent, obs, actions, logprobs, adv, ret, val, adv_mean, adv_std, cfg):
    """train.py:200-238 (the reference loss) in float64 on the CPU."""
    _, newlogprob, entropy, newvalue = agent.get_action_and_value(obs, actions)
    ratio = (newlogprob - logprobs).exp()
    a = (adv - adv_mean) / (adv_std + 1e-8)
    pg = torch.max(-a * ratio, -a * torch.clamp(ratio, 1 - cfg.clip_coef, 1 + cfg.clip_coef)).mean()
    nv = newvalue.view(-1)
    vu = (nv - ret) ** 2
    vc = val + torch.clamp(nv - val, -cfg.clip_coef, cfg.clip_coef)
    v_loss = 0.5 * torch.max(vu, (vc - ret) ** 2).mean()
    return pg - cfg.ent_coef * entropy.mean() + cfg.vf_coef * v_loss


def test_config3_vision_rollout_and_minibatch():
    from ppo_radiotherapy_amd import assets
    from ppo_radiotherapy_amd.networks import PPO_3DCNN
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    lib = assets.synthetic_library((64, 64, 64), 1000, 0)
    N, seed = 512, 77
    env = RadiotherapyVecEnv(N, visionless=False, library=lib, seed=seed)
    torch.manual_seed(5)
    agent = PPO_3DCNN((4, 64, 64, 64), (6,), 64).cuda()
    with torch.no_grad():
        agent.actor_logstd.fill_(0.2)
    cfg = SimpleNamespace(num_steps=16, num_minibatches=2, update_epochs=1, learning_rate=3e-4, anneal_lr=False,
                          gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.0,
                          vf_coef=0.5, max_grad_norm=0.5, micro_batch=128, seed=1)
    tr = PPOTrainer(cfg, env, agent, "cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    assert tr.compact_obs and not tr.fused_policy
    tr.reset()
    tr.rollout()
    tr.compute_gae()
    torch.cuda.synchronize()
    T = tr.T
    # ---- rollout: sampled envs on the oracle
    acts = tr.actions.cpu().numpy()
    rews = tr.rewards.cpu().numpy()
    pose_s = tr.pose_snap.cpu().numpy()
    tum_s = tr.tumour_snap.cpu().numpy()
    sample = [3, 200, 511]
    render_rows = []
    for e in sample:
        tid = rt_rng.tumour_draw(seed, e, 0, lib.n_tumours)
        oe = O.OracleEnv(lib.lungs.astype(np.float32), lib.tumour_dense(tid))
        oe.reset()
        for t in range(T):
            pos, d, _ = oe.pose()
            assert tum_s[t, e] == tid
            np.testing.assert_allclose(pose_s[t, e], np.concatenate([pos, d]), rtol=0, atol=1e-13)
            dose_t = tr.dose_snap[t, e].cpu().numpy().reshape(lib.shape)
            np.testing.assert_array_equal(dose_t.view(np.uint32), oe.dose.view(np.uint32), err_msg=f"{e} {t}")
            if t in (0, 9, T - 1):
                render_rows.append((t * N + e, oracle_vision_obs(lib, tid, oe)))
            _, oi, done = oe.step(acts[t, e])
            assert abs(rews[t, e] - oi[0]) <= 1e-5, (e, t)
            assert not done
    tr._bind_batch()
    rows = torch.tensor([r for r, _ in render_rows], device="cuda")
    got = tr._obs_rows(rows).cpu().numpy()
    for k, (_, want) in enumerate(render_rows):
        np.testing.assert_array_equal(got[k].view(np.uint32), want.view(np.uint32))
    # ---- one compact-storage minibatch (4096 samples) of the update
    M = tr.minibatch_size
    assert M == 4096
    mb = torch.randperm(tr.batch_size, device="cuda", generator=torch.Generator(device="cuda").manual_seed(9))[:M]
    a = tr._b_adv[mb]
    am, asd = a.mean(), a.std()
    grads = {}
    for micro in (128, 1024):
        tr.cfg.micro_batch = micro
        st = tr._minibatch_loss_backward(mb, am, asd)
        grads[micro] = tr.flat_grad.clone()
        assert torch.isfinite(st).all()
    g128, g1024 = grads[128], grads[1024]
    assert float((g128 - g1024).abs().max()) <= 1e-4 * float(g1024.abs().max())
    # a 12-sample subset's share of the minibatch gradient vs float64 autograd
    sub = mb[:12]
    tr._loss_backward(sub, am, asd, weight=sub.numel() / M)
    mine = tr.flat_grad.clone().cpu().double()
    ref = PPO_3DCNN((4, 64, 64, 64), (6,), 64).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in agent.state_dict().items()})
    obs_sub = tr._obs_rows(sub).cpu().double()
    loss = _ppo_loss_f64(ref, obs_sub, tr._b_actions[sub].cpu().double(), tr._b_logprobs[sub].cpu().double(),
                         tr._b_adv[sub].cpu().double(), tr._b_ret[sub].cpu().double(), tr._b_val[sub].cpu().double(),
                         am.double().cpu(), asd.double().cpu(), cfg) * (sub.numel() / M)
    loss.backward()
    want = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    names = [n for n, _ in ref.named_parameters()]
    off = 0
    for n, p in zip(names, ref.parameters()):
        k = p.numel()
        err = float((mine[off:off + k] - want[off:off + k]).abs().max())
        scale = float(want[off:off + k].abs().max()) + 1e-12
        assert err <= 2e-3 * scale + 1e-9, (n, err, scale)
        off += k
    env.close()
