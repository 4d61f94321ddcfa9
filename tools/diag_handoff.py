"""Which envs / steps of the device hand-off rollout differ from the stepwise launches (debug aid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch  # noqa: E402
import _rtpkg  # noqa: E402,F401
from test_gpu_rollout import _trainer  # noqa: E402
from ppo_radiotherapy_amd import assets  # noqa: E402

lib = assets.synthetic_library((40, 36, 44), 60, 2)
n = 1000
G = int(sys.argv[1]) if len(sys.argv) > 1 else 2
a = _trainer(True, lib, n, "dense")
b = _trainer(False, lib, n, "dense")
a.env.set_rollout_groups(G)
a.env.set_dense_handoff(1)
for first, count in [(0, 8), (8, 8)]:
    a.rollout_steps(first, count)
    b.rollout_steps(first, count)
    torch.cuda.synchronize()
    bad = (a.rewards.view(torch.int32) != b.rewards.view(torch.int32))[first:first + count]
    steps, envs = torch.nonzero(bad, as_tuple=True)
    print(f"run {first}: {int(bad.sum())} wrong rewards; steps {sorted(set(steps.tolist()))[:10]}; "
          f"env range {envs.min().item() if len(envs) else None}..{envs.max().item() if len(envs) else None}; "
          f"n envs {len(set(envs.tolist()))}")
    bi = (a.infos.view(torch.int32) != b.infos.view(torch.int32))[first:first + count]
    print("  infos cols differing:", torch.nonzero(bi.any(0).any(0)).flatten().tolist(),
          "dose equal:", torch.equal(a.env.dose(), b.env.dose()))
    if len(envs):
        ue = sorted(set(envs.tolist()))
        print("  bad envs head", ue[:20], "per-step counts", bad.sum(1).tolist())
        e = envs[0].item()
        print("  first bad env", e, "a", a.rewards[first:first + count, e].tolist()[:4], "b",
              b.rewards[first:first + count, e].tolist()[:4])
