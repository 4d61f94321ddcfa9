"""Drop-in front-end on the GPU: the single-env facade (environment.py
surface), train.py's CLI/outputs, ppo_eval.evaluate, and learning."""
import json
import os

import numpy as np
import pytest

from ppo_radiotherapy_amd import assets

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def test_facade_replays_reference_trajectory(golden):
    from environment import RadiotherapyEnv

    z = golden("env_traj_ref.npz")
    env = RadiotherapyEnv(visionless=True)
    off = 0
    for e in range(3):
        obs, info = env.reset(options={"tumour_id": int(z["tumour_id"][e])})
        assert info == {}
        np.testing.assert_array_equal(obs, z["obs0"][e])  # f64, exact
        for t in range(int(z["ep_len"][e])):
            obs, r, done, trunc, info = env.step(z["actions"][e][t])
            k = off + t
            # f64 obs: position and centroid exact; direction within an ulp (libm sin/cos)
            np.testing.assert_array_equal(obs[[0, 1, 2, 6, 7, 8]], z["step_obs"][k][[0, 1, 2, 6, 7, 8]])
            assert np.abs(obs[3:6] - z["step_obs"][k][3:6]).max() <= 1e-15
            np.testing.assert_array_equal(np.array(info["beam_position"]["translation"]), z["step_pos"][k])
            assert abs(r - z["step_reward"][k]) <= 1e-5 and trunc is False
            assert abs(info["reward_components"]["tumour"] - z["step_tumour"][k]) <= 1e-5
            # doses (environment.py:233-236): the reference's f32 np.sum values, bit-exact
            assert info["doses"]["tumour"] == float(np.float32(z["step_dose_tumour"][k]))
            assert info["doses"]["lung"] == float(np.float32(z["step_dose_lung"][k]))
            assert done == bool(z["step_done"][k])
        off += int(z["ep_len"][e])
        lo, hi = z["dose_off"][e], z["dose_off"][e + 1]
        d = env.dose.ravel()
        nz = np.flatnonzero(d)
        np.testing.assert_array_equal(nz, z["dose_idx"][lo:hi])
        np.testing.assert_array_equal(d[nz], z["dose_val"][lo:hi])
        assert len(env.beams) == int(z["ep_len"][e])
    env.close()


def test_facade_draws_reference_tumour_sequence():
    from environment import RadiotherapyEnv

    names = assets.reference_library().names
    np.random.seed(1)
    env = RadiotherapyEnv(visionless=True)  # __init__ resets once, like the reference
    picks = [env._tumour_id]
    for _ in range(3):
        env.reset()
        picks.append(env._tumour_id)
    np.random.seed(1)
    expect = [names.index(np.random.choice(names)) for _ in range(4)]
    assert picks == expect
    env.close()


def _tiny_cfg(tmp_path, **kw):
    import yaml

    cfg = yaml.safe_load(open(os.path.join(REPO, "configs", "default.yaml")))
    cfg.update(dict(exp_name="tiny", num_envs=64, num_steps=16, total_timesteps=64 * 16 * 3, num_minibatches=4,
                    update_epochs=2, num_saves=1))
    cfg.update(kw)
    p = tmp_path / "tiny.yaml"
    yaml.safe_dump(cfg, open(p, "w"))
    return str(p)


def test_train_cli_outputs(tmp_path):
    import train as train_mod

    out = tmp_path / "out"
    agent = train_mod.main(["--config-file", _tiny_cfg(tmp_path), "--output-dir", str(out)])
    runs = os.listdir(out / "models")
    assert len(runs) == 1
    models = sorted(os.listdir(out / "models" / runs[0]))
    assert models == ["tiny_3.model"]
    sd = torch.load(out / "models" / runs[0] / models[0], weights_only=True)
    ref_keys = {k[4:] for k in np.load(os.path.join(REPO, "tests", "golden", "policy_ref.npz")).files
                if k.startswith("sd::")}
    assert set(sd.keys()) == ref_keys  # loadable by the reference's networks.PPO
    assert os.path.exists(out / runs[0] / "config.yaml")
    tb = out / "tensorboard" / runs[0]
    files = os.listdir(tb)
    if "scalars.jsonl" in files:
        tags = {json.loads(x).get("tag") for x in open(tb / "scalars.jsonl")}
        for t in ["charts/learning_rate", "losses/value_loss", "losses/policy_loss", "losses/entropy",
                  "losses/approx_kl", "losses/clipfrac", "losses/explained_variance", "perf/env_steps_per_s"]:
            assert t in tags, t
    assert all(torch.isfinite(p).all() for p in agent.parameters())


def test_train_checkpoint_resume(tmp_path):
    """SURVEY §5 checkpoint/resume: every save writes a full trainer checkpoint
    beside the model; resume_from continues at the next iteration with the
    agent, Adam moments/step and counters of the checkpoint."""
    import train as train_mod

    out = tmp_path / "out"
    train_mod.main(["--config-file", _tiny_cfg(tmp_path, num_saves=3), "--output-dir", str(out)])
    run = os.listdir(out / "checkpoints")[0]
    cks = sorted(os.listdir(out / "checkpoints" / run))
    assert cks == ["tiny_1.ckpt", "tiny_2.ckpt", "tiny_3.ckpt"]
    c1 = torch.load(out / "checkpoints" / run / "tiny_1.ckpt", weights_only=True)
    assert c1["iteration"] == 1 and c1["global_step"] == 64 * 16
    per_iter = 2 * 4  # update_epochs x num_minibatches optimizer steps
    if "adam" in c1:
        assert c1["adam"]["step"] == per_iter
    out2 = tmp_path / "out2"
    agent = train_mod.main(["--config-file", _tiny_cfg(tmp_path, num_saves=3,
                                                         resume_from=str(out / "checkpoints" / run / "tiny_1.ckpt")),
                            "--output-dir", str(out2)])
    run2 = os.listdir(out2 / "models")[0]
    assert sorted(os.listdir(out2 / "models" / run2)) == ["tiny_2.model", "tiny_3.model"]
    c3 = torch.load(out2 / "checkpoints" / run2 / "tiny_3.ckpt", weights_only=True)
    assert c3["iteration"] == 3 and c3["global_step"] == 3 * 64 * 16
    if "adam" in c3:
        assert c3["adam"]["step"] == 3 * per_iter
    assert all(torch.isfinite(p).all() for p in agent.parameters())


def test_evaluate_reference_checkpoint(tmp_path, golden):
    import ppo_eval
    from networks import PPO
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    z = golden("policy_ref.npz")
    sd = {k[4:]: torch.tensor(v) for k, v in z.items() if k.startswith("sd::")}
    path = tmp_path / "20M.model"
    torch.save(sd, path)
    envs = RadiotherapyVecEnv(256, visionless=True)
    rets = ppo_eval.evaluate(envs, 64, str(path), 2, PPO, device=envs.device)
    assert len(rets) == 2 and all(np.isfinite(rets))
    # the reference's trained agent (20M steps) reaches a clearly positive return
    assert np.mean(rets) > 50.0, rets
    envs.close()


def test_ppo_learns_on_64cubed():
    """A short run improves the mean step reward (tumour dose) markedly."""
    from types import SimpleNamespace

    from ppo_radiotherapy_amd.networks import PPO
    from ppo_radiotherapy_amd.ppo import PPOTrainer
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    lib = assets.synthetic_library((64, 64, 64), 1000, 0)
    env = RadiotherapyVecEnv(1024, library=lib, seed=3)
    torch.manual_seed(0)
    agent = PPO((9,), (6,), 64).cuda()
    cfg = SimpleNamespace(num_steps=64, num_minibatches=8, update_epochs=10, learning_rate=3e-4, anneal_lr=False,
                          gamma=0.99, gae_lambda=0.95, norm_adv=True, clip_coef=0.1, clip_vloss=True, ent_coef=0.0,
                          vf_coef=0.5, max_grad_norm=0.5)
    gen = torch.Generator(device="cuda").manual_seed(0)
    tr = PPOTrainer(cfg, env, agent, "cuda", generator=gen)
    tr.reset()
    first = None
    for it in range(1, 41):
        tr.train_iteration(it, 40)
        r = float(tr.rewards.mean())
        first = r if first is None else first
    assert r > first + 0.3, (first, r)
    env.close()


def test_export_trajectory_format(tmp_path, golden):
    """RadiotherapyEnv.export_trajectory writes environment.py:69-75's npz:
    tumours (f32 volume), dose (f32 volume), beams = [(position, direction)]
    per step as f64 [n, 2, 3]; replaying golden actions gives the golden dose."""
    from environment import RadiotherapyEnv

    z = golden("env_traj_ref.npz")
    env = RadiotherapyEnv(visionless=True)
    env.reset(options={"tumour_id": int(z["tumour_id"][0])})
    n = int(z["ep_len"][0])
    infos = []
    for t in range(n):
        _, _, _, _, info = env.step(z["actions"][0][t])
        infos.append(info)
    path = tmp_path / "traj.npz"
    env.export_trajectory(path)
    d = np.load(path, allow_pickle=False)
    assert set(d.files) == {"tumours", "dose", "beams"}
    assert d["tumours"].dtype == np.float32 and d["tumours"].shape == (67, 43, 70)
    assert d["dose"].dtype == np.float32 and d["dose"].shape == (67, 43, 70)
    assert d["beams"].dtype == np.float64 and d["beams"].shape == (n, 2, 3)
    np.testing.assert_array_equal(d["dose"], env.dose)
    for t, info in enumerate(infos):
        np.testing.assert_array_equal(d["beams"][t, 0], np.array(info["beam_position"]["translation"]))
        np.testing.assert_array_equal(d["beams"][t, 1], np.array(info["beam_position"]["rotation"]))
    nz = np.flatnonzero(d["dose"].ravel())
    np.testing.assert_array_equal(nz, z["dose_idx"][z["dose_off"][0]:z["dose_off"][1]])
    env.close()


@pytest.mark.parametrize("conv_precision", [None, "bf16x3"])
def test_train_cli_vision_reference_grid(tmp_path, capsys, conv_precision):
    """The reference's vision entry point, `python train.py --config-file
    configs/vision.yaml` (train.py:102-106: PPO_3DCNN + agent.summary(),
    configs/vision.yaml.template keys), run through the CLI at the reference
    grid 67x43x70 -- odd dims, so the first pool pads (networks.py:18-20) --
    on the C3D kernels, with the micro-batched update; and with the config key
    conv_precision: bf16x3 (the forward products, rt_conv_layer.precision)."""
    import yaml

    import train as train_mod
    from ppo_radiotherapy_amd import _lib

    cfg = yaml.safe_load(open(os.path.join(REPO, "configs", "vision.yaml")))
    cfg.update(dict(exp_name="vis", num_envs=4, num_steps=8, total_timesteps=64, num_minibatches=2,
                    update_epochs=2, num_saves=1, micro_batch=6))
    if conv_precision:
        cfg["conv_precision"] = conv_precision
    p = tmp_path / "vision.yaml"
    yaml.safe_dump(cfg, open(p, "w"))
    out = tmp_path / "out"
    agent = train_mod.main(["--config-file", str(p), "--output-dir", str(out)])
    want = _lib.CONV_PREC[conv_precision or "f32"]
    assert all(layer.precision == want for layer, _ in agent.features_extractor._plan())
    printed = capsys.readouterr().out
    assert "Observation shape:  (4, 67, 43, 70)" in printed  # agent.summary()
    from ppo_radiotherapy_amd.networks import PPO_3DCNN

    assert isinstance(agent, PPO_3DCNN)
    assert agent.features_extractor.n_flatten == 2016  # the reference's dry-run flatten at 67x43x70
    runs = os.listdir(out / "models")
    assert len(runs) == 1
    assert sorted(os.listdir(out / "models" / runs[0])) == ["vis_2.model"]
    sd = torch.load(out / "models" / runs[0] / "vis_2.model", weights_only=True)
    ref = PPO_3DCNN((4, 67, 43, 70), (6,), 64)
    assert set(sd) == set(ref.state_dict())  # the reference's PPO_3DCNN keys
    for k, v in ref.state_dict().items():
        assert tuple(sd[k].shape) == tuple(v.shape), k
    tb = out / "tensorboard" / runs[0]
    files = os.listdir(tb)
    if "scalars.jsonl" in files:
        tags = {json.loads(x).get("tag") for x in open(tb / "scalars.jsonl")}
        for t in ["charts/learning_rate", "losses/value_loss", "losses/policy_loss", "losses/entropy",
                  "losses/approx_kl", "losses/clipfrac", "losses/explained_variance"]:
            assert t in tags, t
    assert all(torch.isfinite(p).all() for p in agent.parameters())
