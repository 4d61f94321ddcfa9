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
    (16, 2, (11, 21, 63), (0, 0, 0), 2),  # data-gradient ring: 2-row y band (63-wide planes)
    (16, 1, (12, 13, 10), (0, 0, 0), 3),
    # planes wider than the 80 KiB conv1 ring: the 160 KiB ring, one-row bands
    (4, 1, (6, 10, 160), (0, 0, 0), 2),
    (16, 2, (6, 9, 79), (0, 0, 0), 2),
]


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


_PREC = ["f32"]  # the arithmetic _layer / _check_extractor pass per call (_conv_precision)


def _layer(cin, groups, dims, pad):
    from ppo_radiotherapy_amd import _lib

    return _lib.RtConvLayer(cin, groups, (ctypes.c_int32 * 3)(*dims), (ctypes.c_int32 * 3)(*pad),
                            _lib.CONV_PREC[_PREC[0]])


def _ref(x, w, b, groups, pad):
    y = F.relu(F.conv3d(x, w, b, groups=groups))
    return F.max_pool3d(y, 2, 2, padding=pad, return_indices=True)


@pytest.mark.parametrize("cin,groups,dims,pad,B", STAGES)
def test_conv_relu_pool_forward(cin, groups, dims, pad, B):
    _check_forward(cin, groups, dims, pad, B)


class _conv_precision:
    """rt_conv_layer.precision of the layers this module builds, for the
    duration of a block (the arithmetic is per call)."""

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.prev = _PREC[0]
        _PREC[0] = self.name

    def __exit__(self, *exc):
        _PREC[0] = self.prev


@pytest.mark.parametrize("cin,groups,dims,pad,B", STAGES)
def test_forward_bf16x3(cin, groups, dims, pad, B):
    """bf16x3 products (rt_conv_layer.precision: conv1's ring kernel and the
    grouped stages' z-shift kernels; other stage kernels stay f32): the f32 forward's
    value and activity gates at unchanged tolerances (within 2e-5 of float64
    torch), and torch's argmax on every window whose top-2 gap exceeds the
    arithmetic's error bound: 1e-6 + 2 x 2^-15 x max over the window of
    sum |x||w| (bf16x3 keeps ~2^-15 of each product; with the f32 test's bare
    1e-6, windows whose f64 gap is below the bf16x3 rounding pick the other
    maximum)."""
    from ppo_radiotherapy_amd import _lib

    with _conv_precision("bf16x3"):
        assert _layer(cin, groups, dims, pad).precision == _lib.CONV_PREC["bf16x3"]
        _check_forward(cin, groups, dims, pad, B, prod_err=2.0 ** -15)


def test_conv_precision_rejects_unknown():
    from ppo_radiotherapy_amd import _lib

    L = _lib.load()
    lay = _layer(4, 1, (8, 8, 8), (0, 0, 0))
    lay.precision = 7
    x = torch.zeros((1, 4, 8, 8, 8), device="cuda")
    w = torch.zeros((16, 4, 3, 3, 3), device="cuda")
    b = torch.zeros(16, device="cuda")
    y = torch.empty((1, 16, 3, 3, 3), device="cuda")
    assert L.rt_conv_relu_pool_fwd(ctypes.byref(lay), 1, x.data_ptr(), None, w.data_ptr(), b.data_ptr(),
                                   y.data_ptr(), None, None) == -1  # RT_EINVAL


def _check_forward(cin, groups, dims, pad, B, prod_err=0.0):
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
    # activity = (max > 0): where the f64 window max is within f32 rounding of
    # zero, the f32 conv may land on the other side of the ReLU
    bad = active.bool() != (ref > 0)
    if bad.any():
        worst = float(ref[bad].abs().max())
        assert worst <= 2e-5, (int(bad.sum()), worst)
    # where the window max is unambiguous (top-2 gap), the index equals torch's
    yfull = F.relu(F.conv3d(x[rows].double(), w.double(), b.double(), groups=groups))
    ypad = F.pad(yfull, (pad[2], pad[2], pad[1], pad[1], pad[0], pad[0]), value=-1.0)
    win = ypad.unfold(2, 2, 2).unfold(3, 2, 2).unfold(4, 2, 2).reshape(*ref.shape, 8)
    top2 = win.topk(2, dim=-1).values
    margin = _argmax_margin(x[rows].double(), w.double(), groups, pad, ref.shape, prod_err)
    clear = (top2[..., 0] - top2[..., 1] > margin) & (ref > 0)
    assert clear.float().mean() > 0.5
    assert torch.equal(flat[clear], idx[clear])


def _fwd(lib, L, B, xd, rd, wd, bd, od):
    from ppo_radiotherapy_amd import _lib

    dev = xd.device
    y = torch.empty((B, 16, *od), device=dev)
    am = torch.empty((B, 16, *od), dtype=torch.uint8, device=dev)
    _lib.check(lib.rt_conv_relu_pool_fwd(ctypes.byref(L), B, xd.data_ptr(), _lib.ptr(rd), wd.data_ptr(),
                                         bd.data_ptr(), y.data_ptr(), am.data_ptr(), None), "fwd")
    return y, am


@pytest.mark.parametrize("cin,groups,dims,pad,B", STAGES)
def test_conv_relu_pool_backward_bf16x3_forward(cin, groups, dims, pad, B):
    """The backward gates (float64 autograd routed through the kernel's argmax
    bytes) with the argmax bytes of a bf16x3 forward."""
    with _conv_precision("bf16x3"):
        _check_backward(cin, groups, dims, pad, B, prod_err=2.0 ** -15)


def _argmax_margin(x64, w64, groups, pad, shape, prod_err):
    """Top-2 gap above which a window's argmax must equal torch's: 1e-6, plus
    for bf16x3 products twice the error bound prod_err x sum |x||w| of the
    window's worst position."""
    if not prod_err:
        return 1e-6
    absc = F.conv3d(x64.abs(), w64.abs(), groups=groups) * prod_err
    absc = F.pad(absc, (pad[2], pad[2], pad[1], pad[1], pad[0], pad[0]), value=0.0)
    return 1e-6 + 2 * absc.unfold(2, 2, 2).unfold(3, 2, 2).unfold(4, 2, 2).reshape(*shape, 8).amax(-1)


@pytest.mark.parametrize("cin,groups,dims,pad,B", STAGES)
def test_conv_relu_pool_backward(cin, groups, dims, pad, B):
    _check_backward(cin, groups, dims, pad, B)


def _check_backward(cin, groups, dims, pad, B, prod_err=0.0):
    """rt_conv_relu_pool_wgrad (dW, db) and, for 16-channel stages,
    rt_conv_relu_pool_dgrad (dX) vs float64 autograd of the same stage, the
    pooled gradients routed through the kernel's argmax bytes (equal to
    torch's on every unambiguous window)."""
    from ppo_radiotherapy_amd import _lib

    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(7 + cin + groups)
    x = torch.rand((B, cin, *dims), generator=g)
    if cin == 16:
        x = torch.relu(x - 0.3)
    w = torch.randn((16, cin // groups, 3, 3, 3), generator=g) * (1.0 / np.sqrt(cin // groups * 27))
    b = torch.randn(16, generator=g) * 0.1
    L = _layer(cin, groups, dims, pad)
    od = (ctypes.c_int32 * 3)()
    lib = _lib.load()
    _lib.check(lib.rt_conv_out_dims(ctypes.byref(L), od), "dims")
    xd, wd, bd = x.to(dev), w.to(dev), b.to(dev)
    y, am = _fwd(lib, L, B, xd, None, wd, bd, od)
    gy = torch.randn((B, 16, *od), generator=g)
    gyd = gy.to(dev)
    dw = torch.full_like(wd, float("nan"))
    db = torch.full_like(bd, float("nan"))
    ws = torch.empty(int(lib.rt_conv_wgrad_workspace_floats(ctypes.byref(L), B)), device=dev)
    _lib.check(lib.rt_conv_relu_pool_wgrad(ctypes.byref(L), B, xd.data_ptr(), None, gyd.data_ptr(), am.data_ptr(),
                                           dw.data_ptr(), db.data_ptr(), ws.data_ptr(), ws.numel(), None), "wgrad")
    dx = None
    if cin == 16:
        dx = torch.full_like(xd, float("nan"))
        _lib.check(lib.rt_conv_relu_pool_dgrad(ctypes.byref(L), B, wd.data_ptr(), gyd.data_ptr(), am.data_ptr(),
                                               dx.data_ptr(), None), "dgrad")
    torch.cuda.synchronize()
    # float64 reference.  Each pooled gradient flows to the window position the
    # kernel's argmax byte names: in a near-tie window (top-2 gap within f32
    # rounding of the conv sums) the f32 kernel may legitimately pick the other
    # position than float64 torch, which would move a whole gy entry.  The
    # routing is checked against torch's on every unambiguous window here (and
    # in test_conv_relu_pool_forward); the gradients against float64 autograd
    # of the same routing.
    x64, w64, b64 = x.double(), w.double(), b.double()
    ref_pool, idx = _ref(x64, w64, b64, groups, pad)
    a = am.cpu().long()
    k = a & 7
    cd, ch, cw = (d - 2 for d in dims)
    pz, py, px = torch.meshgrid(*[torch.arange(n) for n in od], indexing="ij")
    flat = ((2 * pz - pad[0] + (k >> 2)) * ch + (2 * py - pad[1] + ((k >> 1) & 1))) * cw + (2 * px - pad[2] + (k & 1))
    active = ((a >> 3) & 1).bool()
    bad = active != (ref_pool > 0)
    if bad.any():
        assert float(ref_pool[bad].abs().max()) <= 2e-5
    yfull = F.relu(F.conv3d(x64, w64, b64, groups=groups))
    ypad = F.pad(yfull, (pad[2], pad[2], pad[1], pad[1], pad[0], pad[0]), value=-1.0)
    top2 = ypad.unfold(2, 2, 2).unfold(3, 2, 2).unfold(4, 2, 2).reshape(*ref_pool.shape, 8).topk(2, dim=-1).values
    margin = _argmax_margin(x64, w64, groups, pad, ref_pool.shape, prod_err)
    clear = (top2[..., 0] - top2[..., 1] > margin) & (ref_pool > 0)
    assert torch.equal(flat[clear], idx[clear])
    dconv = torch.zeros((B, 16, cd * ch * cw), dtype=torch.float64)
    dconv.scatter_(2, flat.clamp(0, cd * ch * cw - 1).reshape(B, 16, -1),
                   torch.where(active, gy.double(), torch.zeros((), dtype=torch.float64)).reshape(B, 16, -1))
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x64, w64, b64))
    F.conv3d(xr, wr, br, groups=groups).backward(dconv.reshape(B, 16, cd, ch, cw))
    # torch's own float32 error on the same data sets the scale of the tolerance
    xq, wq, bq = (t.clone().requires_grad_(True) for t in (x64, w64, b64))
    F.max_pool3d(F.relu(F.conv3d(xq, wq, bq, groups=groups)), 2, 2, padding=pad).backward(gy.double())
    xf, wf, bf = (t.clone().requires_grad_(True) for t in (x, w, b))
    F.max_pool3d(F.relu(F.conv3d(xf, wf, bf, groups=groups)), 2, 2, padding=pad).backward(gy)
    for mine, f32, q64, ref in ((dw, wf.grad, wq.grad, wr.grad), (db, bf.grad, bq.grad, br.grad)):
        err = float((mine.cpu().double() - ref).abs().max())
        err32 = float((f32.double() - q64).abs().max())
        assert err <= 10 * err32 + 1e-6 * float(ref.abs().max()), (err, err32)
    if dx is not None:
        d = (dx.cpu().double() - xr.grad).abs()
        scale = float(xr.grad.abs().max())
        assert float(d.max()) <= 2e-5 * scale, (float(d.max()), scale)
        assert float(d.norm() / xr.grad.norm()) < 1e-5


def test_planes_too_wide_fail_cleanly():
    """Beyond every plane ring and the tile kernel the stage returns RT_ELIMIT
    with a message; nothing is launched.  (The Winograd ring takes conv1
    planes up to ~380 wide in f32 -- one pooled row per band, 6 slots + U in
    160 KiB; the direct ring ~170, the tile kernel less.)"""
    from ppo_radiotherapy_amd import _lib

    L = _layer(4, 1, (5, 7, 402), (1, 1, 0))
    lib = _lib.load()
    x = torch.zeros((1, 4, 5, 7, 402), device="cuda")
    w = torch.zeros((16, 4, 3, 3, 3), device="cuda")
    b = torch.zeros(16, device="cuda")
    y = torch.zeros((1, 16, 2, 3, 200), device="cuda")
    rc = lib.rt_conv_relu_pool_fwd(ctypes.byref(L), 1, x.data_ptr(), None, w.data_ptr(), b.data_ptr(), y.data_ptr(),
                                   None, None)
    assert rc == -5 and b"exceeds LDS" in lib.rt_last_error()
    torch.cuda.synchronize()


@pytest.mark.parametrize("shape,B,prec", [((4, 34, 27, 40), 6, "f32"), ((4, 22, 23, 160), 2, "f32"),
                                          ((4, 64, 64, 64), 2, "f32"), ((4, 34, 27, 40), 6, "bf16x3"),
                                          ((4, 64, 64, 64), 2, "bf16x3")])
def test_features_extractor_matches_torch_modules(shape, B, prec):
    """FeaturesExtractor3D on the GPU (fused kernels) vs its own torch modules
    on the CPU in float64 (the second shape: a grid 160 voxels wide, beyond the
    conv1 ring's 80 KiB band).  Features: vs the plain float64 modules at the
    f32 tolerances, for both precisions (bf16x3: conv1 and the grouped stages'
    forward products in bf16x3, measured 7.6e-7 vs 5e-8 for f32).  Parameter
    gradients: vs float64 autograd of the same modules with every max-pool
    routed through the kernels' argmax bytes, gate 2e-3 of each tensor's max
    for both precisions.  The routing itself equals torch's argmax on every
    window whose top-2 gap exceeds the arithmetic's error bound
    (test_conv_relu_pool_forward / test_forward_bf16x3); inside that bound a
    window may route its gradient to the other voxel, a whole-entry move the
    unrouted comparison misread as a 3.8e-3..4.8e-3 gradient error at 64^3
    in bf16x3 (round 3's 5e-3 gate)."""
    with _conv_precision(prec):
        _check_extractor(shape, B, 2e-3)


def _routed_reference(ref, x64, ams, plan):
    """The float64 extractor with each ReLU + MaxPool3d replaced by a gather
    at the window position the kernel's argmax byte names, times the byte's
    ReLU activity bit -- the ReLU itself routed through the kernel's decision:
    a window whose float64 maximum lies within rounding of 0 may be active on
    one side and not on the other, and the kernel passes the window's whole
    gradient exactly when its byte says active."""
    h = x64
    for conv, am, (layer, od) in zip((ref.cnn[0], ref.cnn[3], ref.cnn[6]), ams, plan):
        y = conv(h)
        B, C, cd, ch, cw = y.shape
        pad = tuple(layer.pool_pad)
        k = am.long() & 7
        pz, py, px = torch.meshgrid(*[torch.arange(n) for n in od], indexing="ij")
        flat = (((2 * pz - pad[0] + (k >> 2)) * ch + (2 * py - pad[1] + ((k >> 1) & 1))) * cw
                + (2 * px - pad[2] + (k & 1)))
        active = ((am.long() >> 3) & 1).to(y.dtype)
        h = y.reshape(B, C, -1).gather(2, flat.reshape(B, C, -1)).reshape(B, C, *od) * active
    return ref.mlp(h.flatten(1))


def _check_extractor(shape, B, gtol):
    from ppo_radiotherapy_amd.networks import FeaturesExtractor3D, _stage_fwd

    torch.manual_seed(0)
    fe = FeaturesExtractor3D(shape, 64, conv_precision=_PREC[0])
    ref = FeaturesExtractor3D(shape, 64).double()
    ref.load_state_dict({k: v.double() for k, v in fe.state_dict().items()})
    fe = fe.cuda()
    x = torch.rand((B, *shape))
    f = fe(x.cuda())
    with torch.no_grad():
        fr = ref(x.double())
    torch.testing.assert_close(f.cpu().double(), fr, rtol=1e-4, atol=1e-5)
    # the argmax bytes of the stages (the same deterministic kernels _C3DStack ran)
    plan = fe._plan()
    ams, h = [], x.cuda()
    with torch.no_grad():
        for (layer, od), conv in zip(plan, (fe.cnn[0], fe.cnn[3], fe.cnn[6])):
            h, am = _stage_fwd(layer, od, h, conv.weight, conv.bias, True)
            ams.append(am.cpu())
    fr_routed = _routed_reference(ref, x.double(), ams, plan)
    torch.testing.assert_close(f.cpu().double(), fr_routed.detach(), rtol=1e-4, atol=1e-5)
    gf = torch.randn_like(fr)
    f.backward(gf.float().cuda())
    fr_routed.backward(gf)
    for (n, p), q in zip(fe.named_parameters(), ref.parameters()):
        err = float((p.grad.cpu().double() - q.grad).abs().max()) / (float(q.grad.abs().max()) + 1e-12)
        assert err < gtol, (n, err)
    with torch.no_grad():
        torch.testing.assert_close(fe(x.cuda()), f.detach())  # inference path (no argmax) = training forward
