"""The C-ABI library (include/rtenv.h -> librtenv.so) on a host without a GPU:
it loads, exports every declared symbol, its config struct layout matches the
header, and its host-side parity hooks agree with the reference numerics."""
import ctypes
import math
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from ppo_radiotherapy_amd import _lib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "rtenv.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    L = _lib.load()
    decl = declared_functions()
    assert len(decl) >= 15
    for name in decl:
        assert hasattr(L, name), name
    assert sorted(_lib.EXPORTS) == decl
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (rt_\w+)", out))
    assert set(decl) <= exported


def test_library_has_gfx950_code_object():
    # the fat binary embeds the offload bundle for gfx950 (and nothing else)
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data
    assert b"amdgcn-amd-amdhsa--gfx942" not in data


@pytest.mark.parametrize("cname,pyname", [("rt_env_config", "RtEnvConfig"), ("rt_policy_step", "RtPolicyStep"),
                                           ("rt_policy_rollout", "RtPolicyRollout"), ("rt_ppo_batch", "RtPpoBatch"),
                                           ("rt_ppo_hparams", "RtPpoHparams"), ("rt_conv_layer", "RtConvLayer")])
def test_struct_layout_matches_header(tmp_path, cname, pyname):
    """Every ctypes mirror of a header struct has its size and field offsets."""
    cls = getattr(_lib, pyname)
    fields = [f[0] for f in cls._fields_]
    probe = tmp_path / "probe.c"
    body = "\n".join(f'    printf("{f} %zu\\n", offsetof({cname}, {f}));' for f in fields)
    probe.write_text(f'#include <stddef.h>\n#include <stdio.h>\n#include "rtenv.h"\nint main(void) {{\n'
                     f'    printf("sizeof %zu\\n", sizeof({cname}));\n{body}\n    return 0;\n}}\n')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(probe), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                       check=True).stdout.splitlines())
    assert int(got["sizeof"]) == ctypes.sizeof(cls)
    for f in fields:
        assert int(got[f]) == getattr(cls, f).offset, f


def test_config_defaults_are_reference_constants():
    L = _lib.load()
    c = _lib.RtEnvConfig()
    assert L.rt_env_config_default(c) == 0
    assert list(c.grid) == [67, 43, 70] and c.max_time_steps == 100
    assert c.beam_dose == np.float32(0.1) and c.lung_dose_threshold == np.float32(0.2)
    assert c.tumour_dose_threshold == np.float32(0.9) and c.min_angle_z == math.pi / 4
    assert c.movement_speed == 0.2 and c.rotation_speed == 0.5
    assert (c.lung_dose_reward, c.tumour_dose_reward, c.distance_reward) == (-1.0, 10.0, -1.0)
    assert L.rt_abi_version() == 5
    assert c.struct_size == ctypes.sizeof(_lib.RtEnvConfig)


def test_config_size_handshake_rejects_stale_declarations():
    """rt_env_config.struct_size: a declaration without it (ABI 1: the first
    member is grid[0]) or without a trailing member (the round-2 INTEGRATION.md
    snippet lacked step_mode) is refused with RT_EINVAL before anything is
    written -- the bytes past the caller's struct stay untouched."""
    L = _lib.load()
    full = ctypes.sizeof(_lib.RtEnvConfig)
    for size in (0, full - 8, full + 8):
        buf = (ctypes.c_uint8 * (full + 32))()
        ctypes.memset(buf, 0xCD, len(buf))
        c = _lib.RtEnvConfig.from_buffer(buf)
        c.struct_size = size
        assert L.rt_env_config_default(c) == -1, size
        assert b"struct_size" in L.rt_last_error()
        assert bytes(buf)[4:] == b"\xcd" * (len(buf) - 4)
        h = ctypes.c_void_p()
        assert L.rt_env_create(c, 0, h) == -1 and h.value is None


def test_integration_binding_struct_is_the_library_struct():
    """INTEGRATION_binding.py declares rt_env_config by hand (a foreign
    binding): same fields, size and offsets as the production mirror, which
    test_struct_layout_matches_header pins to the header."""
    sys.path.insert(0, REPO)
    import INTEGRATION_binding as B

    assert [f[0] for f in B.RtEnvConfig._fields_] == [f[0] for f in _lib.RtEnvConfig._fields_]
    assert ctypes.sizeof(B.RtEnvConfig) == ctypes.sizeof(_lib.RtEnvConfig)
    for f, _ in B.RtEnvConfig._fields_:
        assert getattr(B.RtEnvConfig, f).offset == getattr(_lib.RtEnvConfig, f).offset
    assert B.RTENV_ABI_VERSION == _lib.load().rt_abi_version()


def test_error_paths_do_not_abort():
    L = _lib.load()
    h = ctypes.c_void_p()
    rc = L.rt_env_create(None, 0, h)
    assert rc == -1 and b"NULL" in L.rt_last_error()
    c = _lib.RtEnvConfig()
    L.rt_env_config_default(c)
    c.num_envs = 0
    assert L.rt_env_create(c, 0, h) == -1
    assert L.rt_gae(0, 1, None, None, None, None, None, 0.99, 0.95, None, None, None) == -1
    with pytest.raises(_lib.RtError):
        _lib.check(-1, "probe")


def test_host_sincos_matches_libm():
    L = _lib.load()
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.uniform(0, 1.3614, 200000), [0.0, 1e-300, 5e-4, 1.3614]])
    s = np.zeros_like(x)
    c = np.zeros_like(x)
    assert L.rt_host_sincos(len(x), x.ctypes.data, s.ctypes.data, c.ctypes.data) == 0
    gs = np.array([math.sin(v) for v in x])
    gc = np.array([math.cos(v) for v in x])
    # glibc is correctly rounded except near rounding midpoints (~0.15 %)
    assert np.mean(s == gs) > 0.995 and np.mean(c == gc) > 0.995
    assert np.all(np.abs(s.view(np.int64) - gs.view(np.int64)) <= 1)
    assert np.all(np.abs(c.view(np.int64) - gc.view(np.int64)) <= 1)


@pytest.mark.parametrize("V", [201670, 262144, 2097152, 1000, 8192 * 3 + 5])
def test_exact_tumour_sum_plan(V):
    """k_finish's plan reproduces np.sum over the dense f32 volume bit-exactly."""
    L = _lib.load()
    rng = np.random.default_rng(V)
    for trial in range(40):
        n = int(rng.integers(1, min(V, 1024)))
        if trial % 3 == 0:  # a compact blob like a tumour
            start = int(rng.integers(0, max(V - 4 * n, 1)))
            idx = np.unique(start + rng.integers(0, 4 * n, n)).astype(np.int32)
            idx = idx[idx < V]
        else:
            idx = np.sort(rng.choice(V, size=n, replace=False)).astype(np.int32)
        vals = (rng.random(idx.size) * rng.choice([1.0, 1e-3, 1e3])).astype(np.float32)
        dense = np.zeros(V, np.float32)
        dense[idx] = vals
        out = np.zeros(1, np.float32)
        assert L.rt_host_tumour_sum(V, idx.size, idx.ctypes.data, vals.ctypes.data, out.ctypes.data) == 0
        assert out[0] == np.sum(dense.reshape(-1)), (V, trial)


def _lung_masks():
    from ppo_radiotherapy_amd import assets

    rng = np.random.default_rng(11)
    ref = assets.reference_library().lungs
    yield "reference 67x43x70", ref
    yield "64^3", assets.resample_nearest(ref, (64, 64, 64)).astype(np.uint8)
    yield "40x36x44", assets.resample_nearest(ref, (40, 36, 44)).astype(np.uint8)
    # partial last buffers of every shape: 65 leaves (8190), tails, < 8 elements
    for shape in [(9, 910, 1), (33, 17, 15), (2, 3, 5), (1, 1, 7), (1, 17, 482), (5, 5, 331), (8, 1023, 1)]:
        yield f"random {shape}", (rng.random(shape) < rng.choice([0.3, 0.7, 1.0])).astype(np.uint8)


def test_exact_lung_sum_plan():
    """rt_host_lung_sum -- the chain / slot / leaf / butterfly / level-plan
    evaluation k_dense + k_finish run for info doses.lung (environment.py:235)
    -- equals np.sum(dose * lungs) bit for bit, and the oracle's restatement,
    on the reference lungs, the BASELINE 64^3 resample and random masks whose
    last numpy buffer is partial (irregular leaf trees, tails, < 8 elements),
    for dense, sparse and beam-like (multiples of 0.1f, clipped) doses."""
    import oracle as O  # tests/conftest.py puts oracle/ on the path (the checker only)

    L = _lib.load()
    rng = np.random.default_rng(5)
    for name, lungs in _lung_masks():
        lf = lungs.astype(np.float32)
        grid = (ctypes.c_int32 * 3)(*lungs.shape)
        lm = np.ascontiguousarray(lungs, dtype=np.uint8)
        for trial in range(6):
            if trial % 3 == 0:
                dose = rng.random(lungs.shape, dtype=np.float32)
            elif trial % 3 == 1:
                dose = (rng.random(lungs.shape, dtype=np.float32) * (rng.random(lungs.shape) < 0.05)).astype(np.float32)
            else:  # beam-like: sums of 0.1f steps, clipped to [0, 1]
                dose = np.minimum(np.float32(1), (rng.integers(0, 12, lungs.shape) * np.float32(0.1))
                                  .astype(np.float32) * (rng.random(lungs.shape) < 0.2)).astype(np.float32)
            out = np.zeros(1, np.float32)
            assert L.rt_host_lung_sum(grid, lm.ctypes.data, dose.ctypes.data, out.ctypes.data) == 0
            want = np.sum(dose * lf)
            assert out[0] == want, (name, trial, out[0], want)
            assert O.np_sum_f32(dose * lf) == want


def test_fast_sincos_matches_plain_double_double(tmp_path):
    """rtdd::sincos_cr (the device path of scipy's from_rotvec half angle)
    returns the bits of the plain 18-term double-double sin/cos
    (tools/check_sincos.cpp; 5e7 arguments were checked when it was written)."""
    import shutil
    import subprocess

    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "check_sincos"
    subprocess.run([gxx, "-O2", "-ffp-contract=off", "-I", os.path.join(REPO, "ppo-radiotherapy_amd", "csrc"),
                    os.path.join(REPO, "tools", "check_sincos.cpp"), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe), "1000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout


def test_ppo_precision_is_per_call():
    """rt_ppo_hparams.precision (ABI 4: per call, no process-wide setting):
    a value other than the two RT_PPO_PREC_* is RT_EINVAL before anything is
    launched (host-only; the dummy pointers are never dereferenced)."""
    L = _lib.load()
    assert not hasattr(L, "rt_ppo_set_precision") and not hasattr(L, "rt_conv_set_precision")
    fake = (ctypes.c_void_p * 13)(*[16 * (i + 1) for i in range(13)])
    batch = _lib.RtPpoBatch(16, 32, 48, 64, 80, 96, 1024)
    hp = _lib.RtPpoHparams(clip_coef=0.1, clip_vloss=1, norm_adv=0, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
                           adam_beta1=0.9, adam_beta2=0.999, adam_eps=1e-5, precision=7)
    rc = L.rt_ppo_grad(fake, fake, ctypes.byref(batch), 128, 256, None, ctypes.byref(hp), 256, 1 << 20, 512,
                       None, None)
    assert rc == -1
    assert b"bad argument" in L.rt_last_error()

def test_conv_mfma_count_hook():
    """rt_conv_mfma_count (host only): the MFMA wave-instructions of the f32
    Winograd launches bench.py's c3d_mfma counts as executed work -- linear in
    the batch, 0 for bf16x3 (direct kernels), -1 for a bad pass; the data
    gradient of conv2 at 64^3 (31^3 input, 16^3 tiles) is 2 groups x 16 tile
    rows x 16 items x 64 xi x 2 channel quads per sample."""
    L = _lib.load()

    def lay(cin, groups, dims, pad, prec="f32"):
        return _lib.RtConvLayer(cin, groups, (ctypes.c_int32 * 3)(*dims), (ctypes.c_int32 * 3)(*pad),
                                _lib.CONV_PREC[prec])

    c1 = lay(4, 1, (64, 64, 64), (0, 0, 0))
    c2 = lay(16, 2, (31, 31, 31), (0, 0, 0))
    n1 = L.rt_conv_mfma_count(ctypes.byref(c1), 1, 0)
    assert n1 > 0 and L.rt_conv_mfma_count(ctypes.byref(c1), 512, 0) == 512 * n1
    # conv1 forward: 31^3 pooled windows in 16-window items of pooled rows, 64 xi, one channel quad
    assert n1 >= 31 * 31 * 31 // 16 * 64
    assert L.rt_conv_mfma_count(ctypes.byref(c2), 3, 1) == 3 * 2 * 16 * 16 * 64 * 2
    assert L.rt_conv_mfma_count(ctypes.byref(c1), 1, 1) == 0  # conv1 has no data gradient
    assert L.rt_conv_mfma_count(ctypes.byref(lay(4, 1, (64, 64, 64), (0, 0, 0), "bf16x3")), 1, 0) == 0
    assert L.rt_conv_mfma_count(ctypes.byref(c1), 1, 2) == -1
