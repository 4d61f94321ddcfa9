"""Phase timeline of k_ppo_grad_mfma (one minibatch step of 32768 samples):
per wave, s_memrealtime stamps (csrc/rt_trace.h, traced library built by
tools/trace_env.py --build-only) at kernel entry (0), after the parameter
staging (1), after its first tile (6), after its tile loop (2), after the
16-lane partial sums (3), after the W2 reduction phase (4) and at exit (5).

    python tools/trace_update.py [--mb 32768]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "tools", "_trace", "librtenv_trace.so")
PHASES = {"stage": (0, 1), "first_tile": (1, 6), "tiles": (1, 2), "sum16": (2, 3), "w2_reduce": (3, 4),
          "rest_reduce": (4, 5), "wave": (0, 5)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=32768)
    a = ap.parse_args()
    import torch
    import _rtpkg  # noqa: F401
    from ppo_radiotherapy_amd import _lib
    _lib.LIB_PATH = OUT
    L = _lib.load(build_if_missing=False)
    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    dev = torch.device("cuda")
    torch.manual_seed(0)
    agent = PPO((9,), (6,), 64).to(dev)
    B = 262144
    obs = torch.rand(B, 9, device=dev) * 2 - 1
    with torch.no_grad():
        act, logp, _, val = agent.get_action_and_value(obs)
    logp, val = logp.contiguous(), val.view(-1).contiguous()
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
    idx = torch.randperm(B, device=dev)[:a.mb]
    stats2 = torch.tensor([0.0, 1.0], device=dev)
    ws = torch.empty(int(L.rt_ppo_workspace_floats(a.mb)), device=dev)
    st = torch.zeros(6, device=dev)
    for _ in range(4):
        _lib.check(L.rt_ppo_grad(pp, gp, ctypes.byref(batch), idx.data_ptr(), a.mb, stats2.data_ptr(),
                                 ctypes.byref(hp), ws.data_ptr(), ws.numel(), st.data_ptr(), None,
                                 _lib.stream_handle()), "rt_ppo_grad")
    torch.cuda.synchronize()
    buf = np.zeros(8192 * 16, np.uint64)
    L.rt_trace_read_update.argtypes = [ctypes.c_void_p]
    assert L.rt_trace_read_update(buf.ctypes.data) == 0
    nw = 256 * 8
    t = buf.reshape(8192, 16)[:nw].astype(np.int64)
    t0 = t[:, 0].min()
    us = (t - t0) * 0.01
    out = {"mb": a.mb, "phases_us": {}}
    for name, (s0, s1) in PHASES.items():
        d = us[:, s1] - us[:, s0]
        out["phases_us"][name] = {"median": float(np.median(d)), "p90": float(np.percentile(d, 90)),
                                  "max": float(d.max())}
    out["entry_us"] = [float(np.percentile(us[:, 0], q)) for q in (0, 50, 100)]
    out["exit_us"] = [float(np.percentile(us[:, 5], q)) for q in (0, 50, 100)]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
