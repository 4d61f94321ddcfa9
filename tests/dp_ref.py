"""Single-process float64 reference of the data-parallel PPO update
(train.py:183-248) for the autograd (vision / micro-batched) path.

The DP update stands for ONE process training on the union of the ranks'
batches: minibatch i of epoch e is the union of every rank's minibatch i,
its advantages are normalised with the union's mean and unbiased std
(train.py:215-218), the gradient is the mean loss over the union, then
clip_grad_norm_ and Adam.  `local_norm=True` gives the rank-local
normalisation bug instead (each rank's rows normalised with its own rows'
statistics), so a test can show it is sensitive to that difference."""
import numpy as np
import torch

BATCH_KEYS = ("obs", "actions", "logprobs", "adv", "ret", "val")


def trainer_batch(tr) -> dict:
    """The trainer's bound batch as numpy (after _bind_batch); compact vision
    storage renders its observations (tr._obs_rows)."""
    out = {}
    for k in BATCH_KEYS:
        t = getattr(tr, "_b_" + k)
        if k == "obs" and t is None:
            t = tr._obs_rows(torch.arange(tr.batch_size, device=tr.device))
        out[k] = t.detach().cpu().numpy().copy()
    return out


def optimizer_state_numpy(opt) -> dict:
    sd = opt.state_dict()
    return {"state": {i: {k: (v.detach().cpu().numpy().copy() if torch.is_tensor(v) else v) for k, v in s.items()}
                      for i, s in sd["state"].items()},
            "param_groups": sd["param_groups"]}


def union_update_f64(agent, sd0, opt_state, batches, perms, n_mb, hp, local_norm=False):
    """agent: a fresh module of the trainer's architecture (converted to f64
    on the CPU here); sd0: its start state dict (numpy); opt_state: the
    trainer's torch Adam state before the update (optimizer_state_numpy) or
    None; batches[r], perms[r][e]: rank r's batch and epoch permutations.
    Returns the flat parameters (agent.parameters() order) after the update."""
    agent = agent.double().cpu()
    agent.load_state_dict({k: torch.from_numpy(np.asarray(v)).double() for k, v in sd0.items()})
    params = list(agent.parameters())
    opt = torch.optim.Adam(params, lr=hp["lr"], eps=1e-5)
    if opt_state is not None:
        opt.load_state_dict({"state": {i: {k: (torch.from_numpy(v) if isinstance(v, np.ndarray) else v)
                                           for k, v in s.items()} for i, s in opt_state["state"].items()},
                             "param_groups": opt_state["param_groups"]})
    cat = {k: torch.cat([torch.from_numpy(b[k]) for b in batches]).double() for k in BATCH_KEYS}
    B = batches[0]["adv"].size
    mbs = B // n_mb
    clip = hp["clip_coef"]
    for e in range(len(perms[0])):
        for i in range(n_mb):
            parts = [torch.as_tensor(perms[r][e][i * mbs:(i + 1) * mbs]) + r * B for r in range(len(batches))]
            rows = torch.cat(parts)
            adv = cat["adv"][rows]
            if local_norm:
                adv = torch.cat([(a - a.mean()) / (a.std() + 1e-8) for a in adv.split(mbs)])
            else:
                adv = (adv - adv.mean()) / (adv.std() + 1e-8)
            _, newlogp, entropy, newv = agent.get_action_and_value(cat["obs"][rows], cat["actions"][rows])
            ratio = (newlogp - cat["logprobs"][rows]).exp()
            pg = torch.max(-adv * ratio, -adv * torch.clamp(ratio, 1 - clip, 1 + clip)).mean()
            nv = newv.view(-1)
            ret, val = cat["ret"][rows], cat["val"][rows]
            vl = 0.5 * torch.max((nv - ret) ** 2, (val + torch.clamp(nv - val, -clip, clip) - ret) ** 2).mean()
            loss = pg - hp["ent_coef"] * entropy.mean() + hp["vf_coef"] * vl
            opt.zero_grad()
            loss.backward()
            torch.nn.utils.clip_grad_norm_(params, hp["max_grad_norm"])
            opt.step()
    return torch.cat([p.detach().reshape(-1) for p in params]).numpy()
