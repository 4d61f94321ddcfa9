"""Policy evaluation (reference: ppo_eval.py:5-37), on the vectorised env."""
from __future__ import annotations

import torch


@torch.no_grad()
def evaluate(envs, feature_dim: int, model_path: str, eval_episodes: int, Model, device=torch.device("cpu")):
    """Runs the saved agent until `eval_episodes` batches of finished episodes
    were seen; returns the list of their mean episodic returns."""
    observation_shape = envs.single_observation_space.shape
    action_space = envs.single_action_space.shape
    agent = Model(observation_shape, action_space, feature_dim).to(device)
    agent.load_state_dict(torch.load(model_path, map_location=device, weights_only=True))
    agent.eval()
    obs, _ = envs.reset()
    episodic_returns = []
    print("Starting evaluation")
    while len(episodic_returns) < eval_episodes:
        actions, _, _, _ = agent.get_action_and_value(torch.as_tensor(obs, device=device))
        obs, _, _, _, infos = envs.step(actions)
        done = infos["_episode"]
        if bool(done.any()):
            mean_returns = float(infos["episode"]["r"][done].double().mean())
            print(f"eval_episode={len(episodic_returns)}, episodic_return={mean_returns}")
            episodic_returns.append(mean_returns)
    return episodic_returns
