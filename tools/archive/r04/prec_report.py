"""Error of rt_ppo_grad against float64 autograd for each precision of the
64x64 layer products (RT_PPO_PREC_F32 / _BF16X3): per parameter tensor, max
|g - g64| / max |g64| (the gate of tests/test_gpu_trainer.py, 2e-4), on the
test's minibatch (4096 of 8192 samples, ratios across both clip edges).

    python tools/prec_report.py [OUT.json]
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import _rtpkg  # noqa: F401,E402
import torch  # noqa: E402

from ppo_radiotherapy_amd import _lib  # noqa: E402
from ppo_radiotherapy_amd.networks import PPO  # noqa: E402
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(11)
    agent = PPO((9,), (6,), 64).to(dev)
    with torch.no_grad():
        agent.actor_logstd.copy_(torch.linspace(-0.7, 0.2, 6).view(1, 6))
        agent.actor_mean[4].weight.mul_(30.0)
    B, mb = 8192, 4096
    g = torch.Generator(device="cpu").manual_seed(2)
    obs = (torch.rand(B, 9, generator=g) * 2 - 1).to(dev)
    with torch.no_grad():
        act, logp, _, val = agent.get_action_and_value(obs)
    logp = (logp + 0.3 * torch.randn(B, generator=g).to(dev)).contiguous()
    adv = (torch.randn(B, generator=g) * 3 + 0.5).to(dev)
    val = (val.view(-1) + 0.2 * torch.randn(B, generator=g).to(dev)).contiguous()
    ret = (val + torch.randn(B, generator=g).to(dev)).contiguous()
    idx = torch.randperm(B, generator=g)[:mb].to(dev)
    a = adv[idx]
    stats2 = torch.stack([a.mean(), a.std()]).contiguous()
    named = dict(agent.named_parameters())
    for p in agent.parameters():
        p.grad = torch.zeros_like(p)
    pp = (ctypes.c_void_p * 13)(*[named[k].data_ptr() for k in PPOTrainer.POLICY_ORDER])
    gp = (ctypes.c_void_p * 13)(*[named[k].grad.data_ptr() for k in PPOTrainer.POLICY_ORDER])
    hp = _lib.RtPpoHparams(clip_coef=0.1, clip_vloss=1, norm_adv=1, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
                           adam_beta1=0.9, adam_beta2=0.999, adam_eps=1e-5)
    batch = _lib.RtPpoBatch(obs.data_ptr(), act.data_ptr(), logp.data_ptr(), adv.data_ptr(), ret.data_ptr(),
                            val.data_ptr(), B)
    L = _lib.load()
    ws = torch.empty(int(L.rt_ppo_workspace_floats(mb)), device=dev)
    st = torch.zeros(6, device=dev)
    # float64 autograd of the same minibatch
    ref = PPO((9,), (6,), 64).double()
    ref.load_state_dict({k: v.double().cpu() for k, v in agent.state_dict().items()})
    i = idx.cpu()
    d = lambda t: t.detach().cpu().double()[i]
    _, nlp, _, nv = ref.get_action_and_value(d(obs), d(act))
    ratio = (nlp - d(logp)).exp()
    A = d(adv)
    A = (A - A.mean()) / (A.std() + 1e-8)
    pg = torch.max(-A * ratio, -A * torch.clamp(ratio, 0.9, 1.1)).mean()
    nv = nv.view(-1)
    R, V = d(ret), d(val)
    vc = V + torch.clamp(nv - V, -0.1, 0.1)
    vl = 0.5 * torch.max((nv - R) ** 2, (vc - R) ** 2).mean()
    (pg + 0.5 * vl).backward()
    rn = dict(ref.named_parameters())
    out = {"minibatch": mb, "gate": 2e-4, "rel_err": {}}
    for prec, code in _lib.PPO_PREC.items():
        _lib.check(L.rt_ppo_set_precision(code), "rt_ppo_set_precision")
        _lib.check(L.rt_ppo_grad(pp, gp, ctypes.byref(batch), idx.data_ptr(), mb, stats2.data_ptr(),
                                 ctypes.byref(hp), ws.data_ptr(), ws.numel(), st.data_ptr(), None, None),
                   "rt_ppo_grad")
        torch.cuda.synchronize()
        errs = {}
        for k in PPOTrainer.POLICY_ORDER:
            r = rn[k].grad
            errs[k] = float((named[k].grad.detach().cpu().double() - r).abs().max() / (r.abs().max() + 1e-12))
        out["rel_err"][prec] = {"max": max(errs.values()), "per_tensor": errs}
    _lib.check(L.rt_ppo_set_precision(0), "rt_ppo_set_precision")
    print(json.dumps({p: v["max"] for p, v in out["rel_err"].items()}))
    if len(sys.argv) > 1:
        json.dump(out, open(sys.argv[1], "w"), indent=1)


if __name__ == "__main__":
    main()
