"""Test-side restatement of the library's tumour-draw RNG contract.

The reference draws the tumour of every episode with the global
`np.random.choice(TUMOUR_DIRS)` (environment.py:90); a device-resident env
cannot share numpy's global stream, so the library draws it with a
counter-based Philox4x32-10 (csrc/rtenv.hip `pose_step`, include/rtenv.h
rt_env_config.seed / env_id_base):

    counter = (episode_draw_index, gid & 0xffffffff, gid >> 32, 0x52544e56)
    key     = (seed & 0xffffffff, seed >> 32)
    tumour  = (r.x * K) >> 32

with `gid = env_id_base + e` and `episode_draw_index` counting the env's
Philox draws (explicit tumour ids do not advance it).  This file lets the
oracle replay predict which tumour an env's autoreset picks, so sampled envs
of a large rollout can be replayed on the CPU oracle across episode
boundaries without any device-side bookkeeping.
"""
from __future__ import annotations

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(c, k):
    c0, c1, c2, c3 = (int(x) & MASK for x in c)
    k0, k1 = (int(x) & MASK for x in k)
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & MASK, p1 & MASK, ((p0 >> 32) ^ c3 ^ k1) & MASK, p0 & MASK
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return c0, c1, c2, c3


def tumour_draw(seed: int, gid: int, draw_index: int, n_tumours: int) -> int:
    seed &= 0xFFFFFFFFFFFFFFFF
    r = philox4x32_10((draw_index, gid & MASK, (gid >> 32) & MASK, 0x52544E56), (seed & MASK, seed >> 32))
    return (r[0] * n_tumours) >> 32
