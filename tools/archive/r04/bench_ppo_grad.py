"""Micro-benchmark of rt_ppo_grad (fused PPO minibatch gradient) and
rt_adam_step on synthetic data: average kernel-chain time per call at several
minibatch sizes.  RT_PPO_GRAD_BLOCKS / RT_PPO_GRAD_KERNEL select the grid cap
and the kernel variant (MFMA default, 'valu')."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import _rtpkg  # noqa: F401,E402
import torch  # noqa: E402

from ppo_radiotherapy_amd import _lib  # noqa: E402
from ppo_radiotherapy_amd.networks import PPO  # noqa: E402
from ppo_radiotherapy_amd.ppo import PPOTrainer  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    agent = PPO((9,), (6,), 64).to(dev)
    B = 262144
    obs = torch.rand(B, 9, device=dev) * 2 - 1
    with torch.no_grad():
        act, logp, _, val = agent.get_action_and_value(obs)
    logp = logp.contiguous()
    val = val.view(-1).contiguous()
    adv = torch.randn(B, device=dev)
    ret = val + torch.randn(B, device=dev)
    for p in agent.parameters():
        p.grad = torch.zeros_like(p)
    named = dict(agent.named_parameters())
    pp = (ctypes.c_void_p * 13)(*[named[k].data_ptr() for k in PPOTrainer.POLICY_ORDER])
    gp = (ctypes.c_void_p * 13)(*[named[k].grad.data_ptr() for k in PPOTrainer.POLICY_ORDER])
    hp = _lib.RtPpoHparams(clip_coef=0.1, clip_vloss=1, norm_adv=1, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
                           adam_beta1=0.9, adam_beta2=0.999, adam_eps=1e-5)
    batch = _lib.RtPpoBatch(obs.data_ptr(), act.data_ptr(), logp.data_ptr(), adv.data_ptr(), ret.data_ptr(),
                            val.data_ptr(), B)
    L = _lib.load()
    res = {}
    for mb in [int(x) for x in os.environ.get("MBS", "4096,16384,32768,65536").split(",")]:
        idx = torch.randperm(B, device=dev)[:mb]
        stats2 = torch.tensor([0.0, 1.0], device=dev)
        ws = torch.empty(int(L.rt_ppo_workspace_floats(mb)), device=dev)
        st = torch.zeros(6, device=dev)
        call = lambda: _lib.check(L.rt_ppo_grad(pp, gp, ctypes.byref(batch), idx.data_ptr(), mb, stats2.data_ptr(),
                                                ctypes.byref(hp), ws.data_ptr(), ws.numel(), st.data_ptr(), None,
                                                _lib.stream_handle()), "rt_ppo_grad")
        for _ in range(5):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            call()
        e1.record()
        torch.cuda.synchronize()
        res[mb] = e0.elapsed_time(e1) / n * 1000.0
    print(json.dumps({"kernel": os.environ.get("RT_PPO_GRAD_KERNEL", "mfma"),
                      "blocks_cap": os.environ.get("RT_PPO_GRAD_BLOCKS", "256"), "us_per_call": res}))


if __name__ == "__main__":
    main()
