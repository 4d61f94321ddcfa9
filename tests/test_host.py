"""Config, logging, assets and the single-env facade's reference RNG draw."""
import json
import os

import numpy as np
import pytest

from ppo_radiotherapy_amd import assets, config, logger

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_config_keys_and_derivation(tmp_path):
    cfg = config.derive(config.load(os.path.join(REPO, "configs", "default.yaml")))
    # train.py:292-297 on default.yaml.template values
    assert cfg.batch_size == 16 * 2048 and cfg.minibatch_size == 1024
    assert cfg.num_iterations == 10000000 // 32768 == 305
    assert cfg.save_frequency_iterations == 61
    assert cfg.visionless is True and cfg.learning_rate == 3e-4
    p = tmp_path / "c.yaml"
    config.save(cfg, str(p))
    again = config.load(str(p))
    assert again.batch_size == cfg.batch_size
    with pytest.raises(ValueError):
        config.derive(config.load(os.path.join(REPO, "configs", "default.yaml")), world=3)
    v = config.derive(config.load(os.path.join(REPO, "configs", "vision.yaml")))
    assert v.visionless is False and v.minibatch_size == 16 * 128 // 2


def test_jsonl_writer(tmp_path):
    w = logger.JsonlWriter(str(tmp_path))
    w.add_scalar("charts/episodic_return", 1.5, 10)
    w.add_text("hyperparameters", "|a|b|")
    w.close()
    rows = [json.loads(x) for x in open(tmp_path / "scalars.jsonl")]
    assert rows[0] == {**rows[0], "tag": "charts/episodic_return", "value": 1.5, "step": 10}


def test_reference_library():
    lib = assets.reference_library()
    assert lib.shape == (67, 43, 70) and lib.n_tumours == 1000
    assert int(lib.lungs.sum()) == 74029
    sizes = np.diff(lib.offsets)
    assert sizes.min() == 16 and sizes.max() == 586
    for k in (0, 17, 999):
        v = lib.tumour_voxels(k)
        assert np.all(np.diff(v) > 0)
    # centroid = mean of np.where coordinates (environment.py:145-148)
    vol = lib.tumour_dense(5)
    np.testing.assert_array_equal(lib.centroid(5), np.mean(np.stack(np.where(vol == 1.0), -1), axis=0))


def test_synthetic_library_64():
    lib = assets.synthetic_library((64, 64, 64), 200, 0)
    sizes = np.diff(lib.offsets)
    assert lib.n_tumours == 200 and sizes.min() >= 8 and sizes.max() <= 1024
    assert 16 <= np.median(sizes) <= 600
    # deterministic and prefix-stable in n_tumours
    small = assets.synthetic_library((64, 64, 64), 20, 0)
    np.testing.assert_array_equal(small.voxels, lib.voxels[:small.offsets[-1]])
    # tumour centres lie in the lung mask
    for k in range(20):
        c = np.round(lib.centroid(k)).astype(int)
        assert lib.lungs[tuple(np.clip(c, 0, 63))] in (0, 1)


def test_facade_draws_tumours_like_the_reference():
    """RadiotherapyEnv.reset draws np.random.choice(len(names)); the reference
    draws np.random.choice(names) (environment.py:90): same stream, same pick."""
    names = assets.reference_library().names
    for seed in range(20):
        np.random.seed(seed)
        a = np.random.choice(names)
        np.random.seed(seed)
        b = names[int(np.random.choice(len(names)))]
        assert a == b


def test_reference_style_generator_against_reference_library():
    """assets.reference_style_library restates graphics.py:110-208: its sphere
    voxelization reproduces the reference voxel sets of the reference names
    (counts, overlap) and its draws follow the reference's distributions."""
    from ppo_radiotherapy_amd import assets

    ref = assets.reference_library()
    J, Q = [], []
    for k in range(0, ref.n_tumours, 4):
        x, y, z, r = (float(t) for t in ref.names[k][:-4].split("_"))
        mine = set(assets._sphere_voxels((x, y, z), r, ref.shape, assets.REF_ORIGIN, assets.REF_PITCH).tolist())
        theirs = set(ref.tumour_voxels(k).tolist())
        J.append(len(mine & theirs) / len(mine | theirs))
        Q.append(len(mine) / len(theirs))
    assert np.mean(J) > 0.6 and 0.9 < np.median(Q) < 1.15, (np.mean(J), np.median(Q))
    lib = assets.reference_style_library(300, seed=3)
    assert lib.shape == ref.shape and lib.n_tumours == 300
    radii = np.array([float(n[:-4].split("_")[3]) for n in lib.names])
    ref_radii = np.array([float(n[:-4].split("_")[3]) for n in ref.names])
    assert radii.min() >= 0.05 and np.allclose(radii, np.round(radii, 2))
    assert abs(radii.mean() - ref_radii.mean()) < 0.01 and abs(radii.std() - ref_radii.std()) < 0.01
    counts = np.diff(lib.offsets)
    ref_counts = np.diff(ref.offsets)
    assert abs(np.median(counts) / np.median(ref_counts) - 1) < 0.25
    inside = np.mean([ref.lungs.ravel()[lib.tumour_voxels(k)].mean() for k in range(lib.n_tumours)])
    assert inside > 0.9
    again = assets.reference_style_library(300, seed=3)
    assert again.names == lib.names and np.array_equal(again.voxels, lib.voxels)
    lib64 = assets.reference_style_library(20, seed=1, shape=(64, 64, 64))
    assert lib64.shape == (64, 64, 64) and lib64.n_tumours == 20


def test_tumour_draw_rng_known_answers():
    """tests/rt_rng.py's Philox4x32-10 (the restated tumour-draw contract the
    headline replay predicts autoresets with) against the Random123 KATs."""
    import rt_rng

    assert rt_rng.philox4x32_10((0, 0, 0, 0), (0, 0)) == (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)
    assert rt_rng.philox4x32_10((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2) == (0x408F276D, 0x41C83B0E, 0xA20BC7C6,
                                                                          0x6D5451FD)
    assert rt_rng.philox4x32_10((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0)) == (
        0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)
    draws = [rt_rng.tumour_draw(5, g, i, 1000) for g in range(50) for i in range(4)]
    assert min(draws) >= 0 and max(draws) < 1000 and len(set(draws)) > 150
