"""C3D stages (networks.py:8-45) as fused HIP kernels vs torch:
Conv3d + ReLU + MaxPool3d values, pool argmax, weight/bias/data gradients."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
F = torch.nn.functional

STAGES = [  # cin, groups, dims, pool_pad, batch
    (4, 1, (64, 64, 64), (0, 0, 0), 3),
    (4, 1, (67, 43, 70), (1, 1, 0), 2),
    (16, 2, (31, 31, 31), (0, 0, 0), 4),
    (16, 4, (14, 14, 14), (0, 0, 0), 5),
    (16, 1, (9, 12, 11), (1, 0, 1), 3),
]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _layer(cin, groups, dims, pad):
    from ppo_radiotherapy_amd import _lib

    return _lib.RtConvLayer(cin, groups, (ctypes.c_int32 * 3)(*dims), (ctypes.c_int32 * 3)(*pad))


def _ref(x, w, b, groups, pad):
    y = F.relu(F.conv3d(x, w, b, groups=groups))
    return F.max_pool3d(y, 2, 2, padding=pad, return_indices=True)


@pytest.mark.parametrize("cin,groups,dims,pad,B", STAGES)
def test_conv_relu_pool_forward(cin, groups, dims, pad, B):
    from ppo_radiotherapy_amd import _lib

    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(cin * 100 + groups)
    x = torch.rand((B + 2, cin, *dims), generator=g)
    if cin == 16:
        x = torch.relu(x - 0.3)   # like a pooled ReLU map
    w = torch.randn((16, cin // groups, 3, 3, 3), generator=g) * (1.0 / np.sqrt(cin // groups * 27))
    b = torch.randn(16, generator=g) * 0.1
    rows = torch.tensor([2, 0, 1, 4, 3, 2, 1][:B], dtype=torch.int64)
    L = _layer(cin, groups, dims, pad)
    od = (ctypes.c_int32 * 3)()
    lib = _lib.load()
    _lib.check(lib.rt_conv_out_dims(ctypes.byref(L), od), "rt_conv_out_dims")
    xd, wd, bd, rd = x.to(dev), w.to(dev), b.to(dev), rows.to(dev)
    y = torch.full((B, 16, *od), float("nan"), device=dev)
    am = torch.zeros((B, 16, *od), dtype=torch.uint8, device=dev)
    _lib.check(lib.rt_conv_relu_pool_fwd(ctypes.byref(L), B, xd.data_ptr(), rd.data_ptr(), wd.data_ptr(),
                                         bd.data_ptr(), y.data_ptr(), am.data_ptr(), None), "rt_conv_relu_pool_fwd")
    torch.cuda.synchronize()
    ref, idx = _ref(x[rows].double(), w.double(), b.double(), groups, pad)
    assert tuple(ref.shape[2:]) == tuple(od)
    torch.testing.assert_close(y.cpu().double(), ref, rtol=0, atol=2e-5)
    # argmax byte -> flat index into the conv output, as torch's return_indices
    a = am.cpu().long()
    k = a & 7
    cd, ch, cw = (d - 2 for d in dims)
    pz, py, px = torch.meshgrid(*[torch.arange(n) for n in od], indexing="ij")
    cz = 2 * pz - pad[0] + (k >> 2)
    cy = 2 * py - pad[1] + ((k >> 1) & 1)
    cx = 2 * px - pad[2] + (k & 1)
    flat = (cz * ch + cy) * cw + cx
    active = (a >> 3) & 1
    assert torch.equal(active.bool(), ref > 0)
    # where the window max is unambiguous (top-2 gap), the index equals torch's
    yfull = F.relu(F.conv3d(x[rows].double(), w.double(), b.double(), groups=groups))
    ypad = F.pad(yfull, (pad[2], pad[2], pad[1], pad[1], pad[0], pad[0]), value=-1.0)
    win = ypad.unfold(2, 2, 2).unfold(3, 2, 2).unfold(4, 2, 2).reshape(*ref.shape, 8)
    top2 = win.topk(2, dim=-1).values
    clear = (top2[..., 0] - top2[..., 1] > 1e-6) & (ref > 0)
    assert clear.float().mean() > 0.5
    assert torch.equal(flat[clear], idx[clear])
