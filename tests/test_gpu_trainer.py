"""PPO update paths on the GPU: fused HIP update (rt_ppo_grad / rt_adam_step)
vs autograd and a float64 reference; fused policy."""
import os
import sys
from types import SimpleNamespace

import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
sys.path.insert(0, os.path.dirname(__file__))


def _cfg(**kw):
    c = dict(num_steps=32, num_minibatches=4, update_epochs=3, learning_rate=3e-4, anneal_lr=True, gamma=0.99,
             gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.01, vf_coef=0.5,
             max_grad_norm=0.5)
    c.update(kw)
    return SimpleNamespace(**c)


def _make(fused=False, prec="f32"):
    from fake_env import FakeVecEnv, torch_gae

    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = torch.device("cuda")
    torch.manual_seed(0)
    agent = PPO((9,), (6,), 64).to(dev)
    gen = torch.Generator(device=dev).manual_seed(5)
    tr = PPOTrainer(_cfg(fused_update=fused, update_precision=prec), FakeVecEnv(256), agent, dev, generator=gen,
                    gae_fn=torch_gae)
    g = torch.Generator(device="cpu").manual_seed(1)
    for t in (tr.obs, tr.actions, tr.logprobs, tr.advantages, tr.returns, tr.values):
        t.copy_(torch.randn(t.shape, generator=g))
    return tr


@pytest.mark.parametrize("fused,prec", [(False, "f32"), (True, "f32"), (True, "bf16x3")],
                         ids=["torch", "fused", "fused-bf16x3"])
def test_update_matches_float64_reference(fused, prec):
    """The eager torch update and the fused HIP update (f32 and bf16x3 layer
    products, same tolerances) vs a CPU float64 run of the same minibatches
    (2 iterations x 3 epochs x 4 minibatches)."""
    from fake_env import FakeVecEnv, torch_gae

    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer

    e = _make(fused, prec)
    assert e.fused_update == fused
    rec = []
    orig = torch.randperm

    def rp(*a, **k):
        out = orig(*a, **k)
        rec.append(out.cpu())
        return out

    torch.randperm = rp
    if fused:  # the fused update shuffles with rt_ppo_shuffle_epochs: record those permutations
        e.record_perms = []
    try:
        e.update()
        e.update()
    finally:
        torch.randperm = orig
    if fused:
        rec.extend(p.cpu() for p in e.record_perms)
    torch.manual_seed(0)
    c = PPOTrainer(_cfg(), FakeVecEnv(256), PPO((9,), (6,), 64).double(), "cpu", gae_fn=torch_gae)
    for tc, te in zip((c.obs, c.actions, c.logprobs, c.advantages, c.returns, c.values),
                      (e.obs, e.actions, e.logprobs, e.advantages, e.returns, e.values)):
        tc.data = te.detach().cpu().double()
    c.optimizer = torch.optim.Adam(c.params, lr=3e-4, eps=1e-5)
    it = iter(rec)
    torch.randperm = lambda *a, **k: next(it)
    try:
        c.update()
        c.update()
    finally:
        torch.randperm = orig
    for p, q in zip(e.params, c.params):
        torch.testing.assert_close(p.detach().cpu().double(), q.detach(), rtol=1e-4, atol=2e-6)
    torch.testing.assert_close(e._last_stats.cpu().double(), c._last_stats.detach().double(), rtol=1e-3, atol=1e-6)


def _policy_ptrs(agent, grads=False):
    import ctypes

    from ppo_radiotherapy_amd.ppo import PPOTrainer

    named = dict(agent.named_parameters())
    ts = [named[k].grad if grads else named[k] for k in PPOTrainer.POLICY_ORDER]
    return (ctypes.c_void_p * 13)(*[t.data_ptr() for t in ts]), ts


@pytest.mark.parametrize("prec", ["f32", "bf16x3"])
@pytest.mark.parametrize("mb,clip_vloss,norm_adv,ent", [(4096, 1, 1, 0.0), (3001, 1, 0, 0.01), (77, 0, 1, 0.0)])
def test_fused_grad_matches_autograd(mb, clip_vloss, norm_adv, ent, prec):
    """rt_ppo_grad vs float64 autograd of train.py:200-238 on one minibatch
    (ragged sizes: partial last tile; ratios spread across both clip edges),
    with the 64x64 layer products in f32 and in bf16x3 (same 2e-4 gate)."""
    import ctypes

    from ppo_radiotherapy_amd import _lib
    from ppo_radiotherapy_amd.networks import PPO

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = torch.device("cuda")
    torch.manual_seed(11)
    agent = PPO((9,), (6,), 64).to(dev)
    with torch.no_grad():
        agent.actor_logstd.copy_(torch.linspace(-0.7, 0.2, 6).view(1, 6))
        agent.actor_mean[4].weight.mul_(30.0)
    B = 8192
    g = torch.Generator(device="cpu").manual_seed(2)
    obs = (torch.rand(B, 9, generator=g) * 2 - 1).to(dev)
    with torch.no_grad():
        act, logp, _, val = agent.get_action_and_value(obs)
    logp = (logp + 0.3 * torch.randn(B, generator=g).to(dev)).contiguous()   # ratios around [0.5, 2]
    adv = (torch.randn(B, generator=g) * 3 + 0.5).to(dev)
    val = (val.view(-1) + 0.2 * torch.randn(B, generator=g).to(dev)).contiguous()
    ret = (val + torch.randn(B, generator=g).to(dev)).contiguous()
    idx = torch.randperm(B, generator=g)[:mb].to(dev)
    a = adv[idx]
    stats2 = torch.stack([a.mean(), a.std()]).contiguous()
    for p in agent.parameters():
        p.grad = torch.full_like(p, float("nan"))   # written, not accumulated
    pp, _ = _policy_ptrs(agent)
    gp, grads = _policy_ptrs(agent, grads=True)
    hp = _lib.RtPpoHparams(clip_coef=0.1, clip_vloss=clip_vloss, norm_adv=norm_adv, ent_coef=ent, vf_coef=0.5,
                           max_grad_norm=0.5, adam_beta1=0.9, adam_beta2=0.999, adam_eps=1e-5,
                           precision=_lib.PPO_PREC[prec])
    batch = _lib.RtPpoBatch(obs.data_ptr(), act.data_ptr(), logp.data_ptr(), adv.data_ptr(), ret.data_ptr(),
                            val.data_ptr(), B)
    L = _lib.load()
    ws = torch.empty(int(L.rt_ppo_workspace_floats(mb)), device=dev)
    st = torch.zeros(6, device=dev)
    acc = torch.ones(6, device=dev)
    _lib.check(L.rt_ppo_grad(pp, gp, ctypes.byref(batch), idx.data_ptr(), mb, stats2.data_ptr(),
                             ctypes.byref(hp), ws.data_ptr(), ws.numel(), st.data_ptr(), acc.data_ptr(), None),
               "rt_ppo_grad")
    torch.cuda.synchronize()
    # float64 autograd reference (ppo.PPOTrainer._loss_backward, the reference's formulas)
    ref = PPO((9,), (6,), 64).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in agent.state_dict().items()})
    i = idx.cpu()
    d = lambda t: t.detach().cpu().double()[i]
    _, nlp, ent_t, nv = ref.get_action_and_value(d(obs), d(act))
    lr_ = nlp - d(logp)
    ratio = lr_.exp()
    A = d(adv)
    if norm_adv:
        A = (A - A.mean()) / (A.std() + 1e-8)
    pg = torch.max(-A * ratio, -A * torch.clamp(ratio, 0.9, 1.1)).mean()
    nv = nv.view(-1)
    R, V = d(ret), d(val)
    if clip_vloss:
        vc = V + torch.clamp(nv - V, -0.1, 0.1)
        vl = 0.5 * torch.max((nv - R) ** 2, (vc - R) ** 2).mean()
    else:
        vl = 0.5 * ((nv - R) ** 2).mean()
    loss = pg - ent * ent_t.mean() + 0.5 * vl
    loss.backward()
    named = dict(ref.named_parameters())
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    for k, gk in zip(PPOTrainer.POLICY_ORDER, grads):
        r = named[k].grad
        scale = float(r.abs().max()) + 1e-12
        err = float((gk.detach().cpu().double() - r).abs().max()) / scale
        assert err < 2e-4, (k, err)
    want = torch.stack([pg, vl, ent_t.mean(), (-lr_).mean(), ((ratio - 1) - lr_).mean(),
                        ((ratio - 1).abs() > 0.1).double().mean()]).detach()
    torch.testing.assert_close(st.cpu().double(), want, rtol=2e-4, atol=2e-6)
    torch.testing.assert_close(acc.cpu().double(), want + 1.0, rtol=2e-4, atol=2e-6)
    frac = float(want[5])
    assert 0.2 < frac < 0.95  # both clip branches exercised


@pytest.mark.parametrize("max_norm,div", [(0.5, 1), (0.0, 1), (0.5, 3), (0.5, 8)])
def test_fused_adam_matches_torch(max_norm, div):
    """rt_adam_step == clip_grad_norm_ + torch.optim.Adam(eps=1e-5) step by
    step; grad_div = the data-parallel average of a SUM all-reduce (torch's
    grad.div_(world) before the clip), bitwise the same division."""
    from ppo_radiotherapy_amd import _lib

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(4)
    n = 10061
    p0 = torch.randn(n, generator=g).to(dev)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=3e-4, eps=1e-5, foreach=True)
    mine, m, v = p0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    ws = torch.empty(256, device=dev)
    hp = _lib.RtPpoHparams(clip_coef=0.1, clip_vloss=1, norm_adv=1, ent_coef=0.0, vf_coef=0.5,
                           max_grad_norm=max_norm, adam_beta1=0.9, adam_beta2=0.999, adam_eps=1e-5)
    import ctypes
    L = _lib.load()
    for step in range(1, 6):
        grad = (torch.randn(n, generator=g) * 0.05 * step).to(dev)
        lr = 3e-4 * (1 - 0.1 * step)
        opt.param_groups[0]["lr"] = lr
        ref.grad = grad.clone().div_(div)
        if max_norm > 0:
            torch.nn.utils.clip_grad_norm_([ref], max_norm)
        opt.step()
        gm = grad.clone()
        _lib.check(L.rt_adam_step(n, mine.data_ptr(), gm.data_ptr(), m.data_ptr(), v.data_ptr(), step, lr,
                                  ctypes.byref(hp), div, ws.data_ptr(), None), "rt_adam_step")
        torch.cuda.synchronize()
        torch.testing.assert_close(gm, ref.grad, rtol=1e-6, atol=1e-9)
        torch.testing.assert_close(mine, ref.detach(), rtol=1e-6, atol=1e-7)


def test_fused_policy_matches_torch_agent():
    """rt_policy_sample: mean/value as the torch agent, log_prob consistent
    with the sampled action, unit-normal noise."""
    import ctypes

    import numpy as np

    from ppo_radiotherapy_amd import _lib
    from ppo_radiotherapy_amd.networks import PPO

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = torch.device("cuda")
    torch.manual_seed(3)
    agent = PPO((9,), (6,), 64).to(dev)
    with torch.no_grad():
        agent.actor_logstd.fill_(-0.5)
        agent.actor_mean[4].weight.mul_(50.0)  # non-trivial means
    N = 20000
    obs = torch.rand(N, 9, device=dev) * 2 - 1
    done = (torch.rand(N, device=dev) < 0.3).to(torch.uint8)
    out = {k: torch.zeros(s, device=dev) for k, s in
           dict(obs=(N, 9), done=(N,), act=(N, 6), logp=(N,), val=(N,)).items()}
    named = dict(agent.named_parameters())
    order = ["actor_mean.0.weight", "actor_mean.0.bias", "actor_mean.2.weight", "actor_mean.2.bias",
             "actor_mean.4.weight", "actor_mean.4.bias", "actor_logstd", "critic.0.weight", "critic.0.bias",
             "critic.2.weight", "critic.2.bias", "critic.4.weight", "critic.4.bias"]
    ptrs = (ctypes.c_void_p * 13)(*[named[k].data_ptr() for k in order])
    L = _lib.load()
    _lib.check(L.rt_policy_sample(ptrs, 13, N, obs.data_ptr(), done.data_ptr(), out["obs"].data_ptr(),
                                  out["done"].data_ptr(), out["act"].data_ptr(), out["logp"].data_ptr(),
                                  out["val"].data_ptr(), 123, 0, 0, None), "rt_policy_sample")
    torch.cuda.synchronize()
    assert torch.equal(out["obs"], obs) and torch.equal(out["done"], done.float())
    with torch.no_grad():
        mean = agent.actor_mean(obs)
        _, logp_t, _, val_t = agent.get_action_and_value(obs, out["act"])
    torch.testing.assert_close(out["val"], val_t.view(-1), rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(out["logp"], logp_t, rtol=1e-4, atol=1e-4)
    z = ((out["act"] - mean) / np.exp(-0.5)).cpu().numpy()
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01
    assert abs(np.corrcoef(z[:, 0], z[:, 1])[0, 1]) < 0.03


@pytest.mark.parametrize("n", [1, 1000, 3001, 32768, 262144])
def test_shuffle_is_a_permutation_and_adv_stats(n):
    """rt_ppo_shuffle: a bijection of [0, n) that depends on the key;
    rt_ppo_adv_stats: minibatch mean / unbiased std as torch computes them."""
    from ppo_radiotherapy_amd import _lib

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = torch.device("cuda")
    L = _lib.load()
    p1 = torch.empty(n, dtype=torch.int64, device=dev)
    p2 = torch.empty(n, dtype=torch.int64, device=dev)
    _lib.check(L.rt_ppo_shuffle(n, 12345, p1.data_ptr(), None), "shuffle")
    _lib.check(L.rt_ppo_shuffle(n, 67890, p2.data_ptr(), None), "shuffle")
    torch.cuda.synchronize()
    assert torch.equal(torch.sort(p1).values, torch.arange(n, device=dev))
    if n >= 1000:
        assert float((p1 != p2).double().mean()) > 0.99
        # no residual order: rank correlation with the identity is small
        r = torch.corrcoef(torch.stack([p1.double(), torch.arange(n, device=dev, dtype=torch.float64)]))[0, 1]
        assert abs(float(r)) < 0.1
    if n % 8 == 0:
        mb = n // 8
        adv = torch.randn(n, device=dev) * 3 + 1
        st = torch.empty((8, 2), device=dev)
        ws = torch.empty(8 * 32 * 4, device=dev)
        _lib.check(L.rt_ppo_adv_stats(adv.data_ptr(), p1.data_ptr(), mb, 8, st.data_ptr(), ws.data_ptr(),
                                      ws.numel(), None), "adv_stats")
        a = adv[p1].view(8, mb)
        torch.testing.assert_close(st, torch.stack([a.mean(1), a.std(1)], 1), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n,epochs", [(1000, 3), (262144, 10), (77, 40)])
def test_shuffle_epochs_equals_per_epoch_shuffles(n, epochs):
    """rt_ppo_shuffle_epochs (every epoch of an update in one launch; more than
    32 keys take several) = rt_ppo_shuffle per epoch with the same keys."""
    import ctypes

    from ppo_radiotherapy_amd import _lib

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = torch.device("cuda")
    L = _lib.load()
    keys = [(0x9E3779B97F4A7C15 * (e + 1)) & (2 ** 62 - 1) for e in range(epochs)]
    got = torch.empty((epochs, n), dtype=torch.int64, device=dev)
    _lib.check(L.rt_ppo_shuffle_epochs(n, epochs, (ctypes.c_uint64 * epochs)(*keys), got.data_ptr(), None), "epochs")
    for e, k in enumerate(keys):
        one = torch.empty(n, dtype=torch.int64, device=dev)
        _lib.check(L.rt_ppo_shuffle(n, k, one.data_ptr(), None), "shuffle")
        assert torch.equal(got[e], one), e


def test_fused_checkpoint_resume_is_bitwise():
    """load_state_dict restores the parameters, the Adam moments and
    step and the epoch-shuffle stream bitwise (through torch.save /
    weights_only load), so the resumed trainer's next update equals the
    continuous run's bit for bit."""
    import io

    a = _make(True)
    a.update()
    buf = io.BytesIO()
    torch.save(a.state_dict(), buf)
    buf.seek(0)
    ck = torch.load(buf, map_location="cuda", weights_only=True)
    b = _make(True)
    with torch.no_grad():
        b.flat_param.add_(1.0)
        b._exp_avg.fill_(3.0)
    b.load_state_dict(ck)
    assert torch.equal(a.flat_param, b.flat_param)
    assert torch.equal(a._exp_avg, b._exp_avg) and torch.equal(a._exp_avg_sq, b._exp_avg_sq)
    assert a._adam_step == b._adam_step > 0
    assert torch.equal(a._host_gen.get_state(), b._host_gen.get_state())
    a.update()
    b.update()
    torch.cuda.synchronize()
    assert torch.equal(a.flat_param, b.flat_param)
    assert torch.equal(a._exp_avg_sq, b._exp_avg_sq)


@pytest.mark.parametrize("max_norm", [0.0, 0.5])
def test_update_call_equals_grad_plus_adam(max_norm):
    """rt_ppo_update (k_ppo_grad_mfma -> k_ppo_reduce_adam per minibatch, the
    reduce + clip + Adam in one launch behind a grid arrival) vs the same
    minibatches through the separate entry points rt_ppo_grad + rt_adam_step
    (grad_div 1), from the same state, permutation and advantage statistics
    (ADVICE r4).  Without clipping the two are bitwise equal (params, Adam
    moments, the last gradient, the loss statistics); with clipping
    rt_adam_step takes ||g|| from its own partial sums (k_gnorm, another
    summation order), so the clip coefficient agrees to f32 rounding."""
    import ctypes

    from ppo_radiotherapy_amd import _lib

    tr = _make(fused=True)
    dev = tr.device
    tr._bind_batch()
    batch = tr._batch_struct()
    L = _lib.load()
    mbs, n_mb = tr.minibatch_size, tr.batch_size // tr.minibatch_size
    perm = torch.randperm(tr.batch_size, generator=torch.Generator().manual_seed(9)).to(dev)
    adv = torch.empty((n_mb, 2), device=dev)
    _lib.check(L.rt_ppo_adv_stats(tr._b_adv.data_ptr(), perm.data_ptr(), mbs, n_mb, adv.data_ptr(),
                                  tr._ws.data_ptr(), tr._ws.numel(), None), "rt_ppo_adv_stats")
    hp = _lib.RtPpoHparams(clip_coef=0.1, clip_vloss=1, norm_adv=1, ent_coef=0.01, vf_coef=0.5,
                           max_grad_norm=max_norm, adam_beta1=0.9, adam_beta2=0.999, adam_eps=1e-5)
    state = [tr.flat_param, tr._exp_avg, tr._exp_avg_sq]
    with torch.no_grad():
        tr._exp_avg.normal_(0, 1e-3)
        tr._exp_avg_sq.uniform_(0, 1e-5)
    start = [t.clone() for t in state]
    n, lr, step0 = tr.flat_param.numel(), 2.5e-4, 7
    stats_a, acc_a = torch.zeros(6, device=dev), torch.zeros(6, device=dev)
    _lib.check(L.rt_ppo_update(tr._policy_ptrs, tr._grad_ptrs, ctypes.byref(batch), perm.data_ptr(), mbs, n_mb,
                               adv.data_ptr(), ctypes.byref(hp), tr.flat_param.data_ptr(), tr.flat_grad.data_ptr(),
                               tr._exp_avg.data_ptr(), tr._exp_avg_sq.data_ptr(), n, step0, lr, tr._ws.data_ptr(),
                               tr._ws.numel(), stats_a.data_ptr(), acc_a.data_ptr(), None), "rt_ppo_update")
    torch.cuda.synchronize()
    got = [t.clone() for t in state] + [tr.flat_grad.clone()]
    with torch.no_grad():
        for t, s in zip(state, start):
            t.copy_(s)
    stats_b, acc_b = torch.zeros(6, device=dev), torch.zeros(6, device=dev)
    for i in range(n_mb):
        _lib.check(L.rt_ppo_grad(tr._policy_ptrs, tr._grad_ptrs, ctypes.byref(batch), perm.data_ptr() + 8 * i * mbs,
                                 mbs, adv.data_ptr() + 8 * i, ctypes.byref(hp), tr._ws.data_ptr(), tr._ws.numel(),
                                 stats_b.data_ptr(), acc_b.data_ptr(), None), "rt_ppo_grad")
        _lib.check(L.rt_adam_step(n, tr.flat_param.data_ptr(), tr.flat_grad.data_ptr(), tr._exp_avg.data_ptr(),
                                  tr._exp_avg_sq.data_ptr(), step0 + i, lr, ctypes.byref(hp), 1,
                                  tr._norm_ws.data_ptr(), None), "rt_adam_step")
    torch.cuda.synchronize()
    ref = [t.clone() for t in state] + [tr.flat_grad.clone()]
    assert torch.equal(stats_a, stats_b) and torch.equal(acc_a, acc_b)
    for name, a, b in zip(("param", "exp_avg", "exp_avg_sq", "grad"), got, ref):
        if max_norm == 0.0:
            assert torch.equal(a, b), name
        else:
            torch.testing.assert_close(a, b, rtol=2e-6, atol=1e-9, msg=name)
    assert not torch.equal(got[0], start[0])  # the update moved the parameters


@pytest.mark.parametrize("max_norm", [0.5, 0.0])
def test_update_split_form_equals_fused(max_norm, monkeypatch):
    """rt_ppo_update's two-kernel form (k_ppo_grad + k_ppo_reduce, then k_adam
    with the reduce's norm partials) -- what a failed co-residency check or a
    missing host-mapped fault flag selects, forced here by the debug knob
    RT_PPO_UPDATE_SPLIT -- is bitwise the fused reduce + Adam form
    (k_adam sums the same partials in the same order), and neither raises the
    lost-arrival flag (rt_ppo_status)."""
    import ctypes

    from ppo_radiotherapy_amd import _lib

    tr = _make(fused=True)
    dev = tr.device
    tr._bind_batch()
    batch = tr._batch_struct()
    L = _lib.load()
    mbs, n_mb = tr.minibatch_size, tr.batch_size // tr.minibatch_size
    perm = torch.randperm(tr.batch_size, generator=torch.Generator().manual_seed(5)).to(dev)
    adv = torch.empty((n_mb, 2), device=dev)
    _lib.check(L.rt_ppo_adv_stats(tr._b_adv.data_ptr(), perm.data_ptr(), mbs, n_mb, adv.data_ptr(),
                                  tr._ws.data_ptr(), tr._ws.numel(), None), "rt_ppo_adv_stats")
    hp = _lib.RtPpoHparams(clip_coef=0.1, clip_vloss=1, norm_adv=1, ent_coef=0.01, vf_coef=0.5,
                           max_grad_norm=max_norm, adam_beta1=0.9, adam_beta2=0.999, adam_eps=1e-5)
    state = [tr.flat_param, tr._exp_avg, tr._exp_avg_sq]
    start = [t.clone() for t in state]
    n = tr.flat_param.numel()
    outs = []
    for split in (False, True):
        with torch.no_grad():
            for t, s0 in zip(state, start):
                t.copy_(s0)
        if split:
            monkeypatch.setenv("RT_PPO_UPDATE_SPLIT", "1")
        stats, acc = torch.zeros(6, device=dev), torch.zeros(6, device=dev)
        _lib.check(L.rt_ppo_update(tr._policy_ptrs, tr._grad_ptrs, ctypes.byref(batch), perm.data_ptr(), mbs, n_mb,
                                   adv.data_ptr(), ctypes.byref(hp), tr.flat_param.data_ptr(),
                                   tr.flat_grad.data_ptr(), tr._exp_avg.data_ptr(), tr._exp_avg_sq.data_ptr(), n, 3,
                                   3e-4, tr._ws.data_ptr(), tr._ws.numel(), stats.data_ptr(), acc.data_ptr(), None),
                   "rt_ppo_update")
        torch.cuda.synchronize()
        monkeypatch.delenv("RT_PPO_UPDATE_SPLIT", raising=False)
        outs.append([t.clone() for t in state] + [tr.flat_grad.clone(), stats, acc])
        assert L.rt_ppo_status() == 0
    for name, a, b in zip(("param", "exp_avg", "exp_avg_sq", "grad", "stats", "accum"), *outs):
        assert torch.equal(a, b), name
    assert not torch.equal(outs[0][0], start[0])


@pytest.mark.parametrize("n,mb,epochs", [(262144, 32768, 10), (8192, 2048, 3), (3000, 1000, 33)])
def test_shuffle_adv_equals_separate_calls(n, mb, epochs):
    """rt_ppo_shuffle_adv (the epochs' permutations and the minibatch
    advantage statistics in one pass) is bitwise rt_ppo_shuffle_epochs +
    rt_ppo_adv_stats, and its sums form is bitwise rt_ppo_adv_sums (33
    epochs: two key batches)."""
    import ctypes

    from ppo_radiotherapy_amd import _lib

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = torch.device("cuda")
    L = _lib.load()
    adv = (torch.randn(n, generator=torch.Generator().manual_seed(3)) * 2 + 0.3).to(dev)
    keys = (ctypes.c_uint64 * epochs)(*[(0x9E3779B97F4A7C15 * (e + 1)) & (2 ** 62 - 1) for e in range(epochs)])
    k = epochs * (n // mb)
    ws = torch.empty(128 * k, device=dev)
    p1, p2 = torch.empty((epochs, n), dtype=torch.int64, device=dev), torch.empty((epochs, n), dtype=torch.int64, device=dev)
    s1, s2 = torch.empty((k, 2), device=dev), torch.empty((k, 2), device=dev)
    q1, q2 = torch.empty((k, 2), dtype=torch.float64, device=dev), torch.empty((k, 2), dtype=torch.float64, device=dev)
    _lib.check(L.rt_ppo_shuffle_epochs(n, epochs, keys, p1.data_ptr(), None), "shuffle_epochs")
    _lib.check(L.rt_ppo_adv_stats(adv.data_ptr(), p1.data_ptr(), mb, k, s1.data_ptr(), ws.data_ptr(), ws.numel(),
                                  None), "adv_stats")
    _lib.check(L.rt_ppo_adv_sums(adv.data_ptr(), p1.data_ptr(), mb, k, q1.data_ptr(), ws.data_ptr(), ws.numel(),
                                 None), "adv_sums")
    _lib.check(L.rt_ppo_shuffle_adv(n, epochs, keys, p2.data_ptr(), adv.data_ptr(), mb, None, s2.data_ptr(),
                                    ws.data_ptr(), ws.numel(), None), "shuffle_adv stats")
    torch.cuda.synchronize()
    assert torch.equal(p1, p2) and torch.equal(s1, s2)
    p2.zero_()
    _lib.check(L.rt_ppo_shuffle_adv(n, epochs, keys, p2.data_ptr(), adv.data_ptr(), mb, q2.data_ptr(), None,
                                    ws.data_ptr(), ws.numel(), None), "shuffle_adv sums")
    torch.cuda.synchronize()
    assert torch.equal(p1, p2) and torch.equal(q1, q2)
    assert torch.equal(p1[0].sort().values, torch.arange(n, device=dev))  # a permutation
    assert L.rt_ppo_shuffle_adv(n, epochs, keys, p2.data_ptr(), adv.data_ptr(), mb, q2.data_ptr(), s2.data_ptr(),
                                ws.data_ptr(), ws.numel(), None) == -1  # exactly one output form


def test_lost_arrival_writes_nothing_and_reports():
    """The fused reduce + Adam's lost-arrival path, forced
    by the debug knob RT_PPO_FORCE_LOST_ARRIVAL (an arrival count that never
    comes, a 16-poll budget): the update leaves parameters and Adam moments
    bitwise untouched, rt_ppo_status and the trainer's check_device_status
    report RT_EDEVICE after the sync, and the next update call refuses.  The
    fault flag is sticky per process, so the case runs in a child process."""
    import subprocess
    import sys

    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    here = os.path.dirname(os.path.abspath(__file__))
    code = f"""
import os, sys
sys.path[:0] = [{os.path.dirname(here)!r}, {here!r}]
import _rtpkg
import torch
import test_gpu_trainer as T
from ppo_radiotherapy_amd import _lib
tr = T._make(fused=True)
p0, m0, v0 = tr.flat_param.clone(), tr._exp_avg.clone(), tr._exp_avg_sq.clone()
os.environ["RT_PPO_FORCE_LOST_ARRIVAL"] = "1"
tr.update()
torch.cuda.synchronize()
assert _lib.load().rt_ppo_status() == -3, "rt_ppo_status"
assert torch.equal(tr.flat_param, p0) and torch.equal(tr._exp_avg, m0) and torch.equal(tr._exp_avg_sq, v0)
try:
    tr.check_device_status()
    raise SystemExit("check_device_status did not raise")
except _lib.RtError as e:
    assert "RT_EDEVICE" in str(e), e
del os.environ["RT_PPO_FORCE_LOST_ARRIVAL"]
try:
    tr.update()
    raise SystemExit("the next update ran")
except _lib.RtError as e:
    assert "RT_EDEVICE" in str(e), e
print("lost-arrival ok")
"""
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "lost-arrival ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
