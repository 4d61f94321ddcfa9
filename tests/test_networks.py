"""Policy networks vs the reference (networks.py) on saves/20M.model."""
import numpy as np
import pytest
import torch

from ppo_radiotherapy_amd.networks import PPO, PPO_3DCNN, FeaturesExtractor3D


def test_ppo_matches_reference_checkpoint(golden):
    z = golden("policy_ref.npz")
    sd = {k[4:]: torch.tensor(v) for k, v in z.items() if k.startswith("sd::")}
    agent = PPO((9,), (6,), 64)
    agent.load_state_dict(sd)  # same module names/shapes as the reference
    x = torch.tensor(z["obs"])
    a = torch.tensor(z["actions"])
    with torch.no_grad():
        mean = agent.actor_mean(x)
        _, logp, ent, val = agent.get_action_and_value(x, a)
    torch.testing.assert_close(mean, torch.tensor(z["mean"]), rtol=0, atol=1e-6)
    torch.testing.assert_close(val, torch.tensor(z["value"]), rtol=0, atol=1e-5)
    torch.testing.assert_close(logp, torch.tensor(z["logprob"]), rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(ent, torch.tensor(z["entropy"]), rtol=1e-6, atol=1e-6)


def test_param_counts():
    assert sum(p.numel() for p in PPO((9,), (6,), 64).parameters()) == 10061
    # C3D parameter counts at the three grids
    for shape, n in [((4, 67, 43, 70), 153149), ((4, 64, 64, 64), 245309)]:
        assert sum(p.numel() for p in PPO_3DCNN(shape, (6,), 64).parameters()) == n


@pytest.mark.parametrize("spatial,flat", [((67, 43, 70), 2016), ((64, 64, 64), 3456), ((128, 128, 128), 43904),
                                          ((30, 33, 41), None)])
def test_flatten_closed_form(spatial, flat):
    fe = FeaturesExtractor3D((4, *spatial), 64)
    with torch.no_grad():
        dry = fe.cnn(torch.zeros(1, 4, *spatial)).shape[1]
    assert fe.n_flatten == dry
    if flat is not None:
        assert dry == flat


def test_sampling_statistics():
    torch.manual_seed(0)
    agent = PPO((9,), (6,), 64)
    x = torch.zeros(20000, 9)
    with torch.no_grad():
        a, logp, ent, _ = agent.get_action_and_value(x)
        mean = agent.actor_mean(x)
    assert abs((a - mean).std().item() - 1.0) < 0.02
    ref = torch.distributions.Normal(mean, torch.ones_like(mean))
    torch.testing.assert_close(logp, ref.log_prob(a).sum(1), rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(ent, ref.entropy().sum(1), rtol=1e-6, atol=1e-6)


def test_splitk_linear_gradients_match_autograd():
    from ppo_radiotherapy_amd import networks as N

    torch.manual_seed(0)
    lin = N.Linear(64, 64)
    ref = torch.nn.Linear(64, 64)
    ref.load_state_dict(lin.state_dict())
    x = torch.randn(8192, 64, requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    (lin(x) ** 2).sum().backward()
    (ref(x2) ** 2).sum().backward()
    torch.testing.assert_close(lin.weight.grad, ref.weight.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(lin.bias.grad, ref.bias.grad, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-5)
