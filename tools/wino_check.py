"""CPU emulation (float64) of the Winograd C3D kernels' indexing and transforms:
forward (conv1 with pool padding, grouped stages) and the grouped data gradient,
against torch float64 conv3d / max_pool3d / autograd."""
import numpy as np
import torch
import torch.nn.functional as F
torch.set_default_dtype(torch.float64)
G_ = np.array([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]])
BT = np.array([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], float)
AT = np.array([[1, 1, 1, 0], [0, 1, -1, -1]], float)

def t3(M, X):  # apply M along the last 3 axes
    X = np.einsum('ai,...ijk->...ajk', M, X)
    X = np.einsum('bj,...ajk->...abk', M, X)
    return np.einsum('ck,...abk->...abc', M, X)

def fwd_wino(x, w, b, groups, pad):
    B, CIN, D, H, W = x.shape
    cpg = CIN // groups; cog = 16 // groups
    cd, ch, cw = D - 2, H - 2, W - 2
    PD, PH, PW = [(c + 2 * p - 2) // 2 + 1 for c, p in zip((cd, ch, cw), pad)]
    U = t3(G_, w)  # [16][cpg][4][4][4]
    y = np.zeros((B, 16, PD, PH, PW)); am = np.zeros((B, 16, PD, PH, PW), int)
    for pz in range(PD):
        for py in range(PH):
            for px in range(PW):
                z0, y0, x0 = 2 * pz - pad[0], 2 * py - pad[1], 2 * px - pad[2]
                zi = np.clip(np.arange(z0, z0 + 4), 0, D - 1); yi = np.clip(np.arange(y0, y0 + 4), 0, H - 1)
                xi = np.clip(np.arange(x0, x0 + 4), 0, W - 1)
                d = x[:, :, zi][:, :, :, yi][:, :, :, :, xi]  # [B][CIN][4][4][4]
                V = t3(BT, d)
                for grp in range(groups):
                    Vg = V[:, grp * cpg:(grp + 1) * cpg]
                    Ug = U[grp * cog:(grp + 1) * cog]  # [cog][cpg]
                    M = np.einsum('oc...,bc...->bo...', Ug, Vg)
                    Y = t3(AT, M)  # [B][cog][2][2][2]
                    Y = Y + b[grp * cog:(grp + 1) * cog, None, None, None]
                    valid = np.zeros((2, 2, 2), bool)
                    for oz in range(2):
                        for oy in range(2):
                            for ox in range(2):
                                valid[oz, oy, ox] = 0 <= z0 + oz < cd and 0 <= y0 + oy < ch and 0 <= x0 + ox < cw
                    val = np.where(valid, np.maximum(Y, 0), -np.inf).reshape(B, cog, 8)
                    y[:, grp * cog:(grp + 1) * cog, pz, py, px] = val.max(-1)
                    k = val.argmax(-1)
                    am[:, grp * cog:(grp + 1) * cog, pz, py, px] = k | np.where(val.max(-1) > 0, 8, 0)
    return y, am

def dgrad_wino(w, gy, am, groups, dims):
    B = gy.shape[0]; D, H, W = dims
    cpg = 16 // groups
    PD, PH, PW = gy.shape[2:]
    Wf = w[:, :, ::-1, ::-1, ::-1]
    U = t3(G_, Wf)  # [16 co][cpg ci][4][4][4]
    QD, QH, QW = (D + 1) // 2, (H + 1) // 2, (W + 1) // 2
    dx = np.zeros((B, 16, D, H, W))
    for qz in range(QD):
        for qy in range(QH):
            for qx in range(QW):
                e = np.zeros((B, 16, 4, 4, 4))
                for wq in range(8):
                    wz, wy, wx = qz - 1 + (wq >> 2), qy - 1 + ((wq >> 1) & 1), qx - 1 + (wq & 1)
                    if not (0 <= wz < PD and 0 <= wy < PH and 0 <= wx < PW):
                        continue
                    a = am[:, :, wz, wy, wx]; v = gy[:, :, wz, wy, wx]
                    for i in range(8):
                        z, yy, xx = 2 * (wq >> 2) + (i >> 2), 2 * ((wq >> 1) & 1) + ((i >> 1) & 1), 2 * (wq & 1) + (i & 1)
                        e[:, :, z, yy, xx] = np.where((a & 15) == (8 | i), v, 0.0)
                V = t3(BT, e)
                for grp in range(groups):
                    Vg = V[:, grp * cpg:(grp + 1) * cpg]           # [B][co of group]
                    Ug = U[grp * cpg:(grp + 1) * cpg]              # [co][ci]
                    M = np.einsum('oc...,bo...->bc...', Ug, Vg)     # -> [B][ci]
                    Y = t3(AT, M)
                    for o in range(8):
                        z, yy, xx = 2 * qz + (o >> 2), 2 * qy + ((o >> 1) & 1), 2 * qx + (o & 1)
                        if z < D and yy < H and xx < W:
                            dx[:, grp * cpg:(grp + 1) * cpg, z, yy, xx] = Y[:, :, o >> 2, (o >> 1) & 1, o & 1]
    return dx

rng = np.random.default_rng(0)
for cin, groups, dims, pad in [(4, 1, (11, 9, 12), (1, 1, 0)), (4, 1, (10, 10, 10), (0, 0, 0)),
                               (16, 2, (11, 9, 13), (0, 0, 0)), (16, 4, (8, 10, 9), (0, 0, 0))]:
    B = 2
    x = rng.random((B, cin, *dims))
    w = rng.standard_normal((16, cin // groups, 3, 3, 3)) / np.sqrt(cin // groups * 27)
    b = rng.standard_normal(16) * 0.1
    y, am = fwd_wino(x, w, b, groups, pad)
    ref, idx = F.max_pool3d(F.relu(F.conv3d(torch.tensor(x), torch.tensor(w), torch.tensor(b), groups=groups)),
                            2, 2, padding=pad, return_indices=True)
    err = np.abs(y - ref.numpy()).max()
    # argmax -> flat conv index as torch
    k = am & 7
    cd, ch, cw = (d - 2 for d in dims)
    pz, py, px = np.meshgrid(*[np.arange(n) for n in y.shape[2:]], indexing='ij')
    flat = ((2 * pz - pad[0] + (k >> 2)) * ch + (2 * py - pad[1] + ((k >> 1) & 1))) * cw + (2 * px - pad[2] + (k & 1))
    agree = (flat == idx.numpy()).mean()
    print(f"fwd cin={cin} g={groups} dims={dims} pad={pad}: max err {err:.2e}, argmax agree {agree:.4f}")
    if cin == 16:
        gy = rng.standard_normal(y.shape)
        dx = dgrad_wino(w, gy, am, groups, dims)
        # reference: route gy through the (same) argmax into the conv output, autograd
        dconv = np.zeros((B, 16, cd * ch * cw))
        act = (am >> 3) & 1
        np.put_along_axis(dconv, flat.reshape(B, 16, -1), (gy * act).reshape(B, 16, -1), axis=2)
        xr = torch.tensor(x, requires_grad=True)
        F.conv3d(xr, torch.tensor(w), groups=groups).backward(torch.tensor(dconv.reshape(B, 16, cd, ch, cw)))
        print(f"   dgrad max err {np.abs(dx - xr.grad.numpy()).max():.2e} (scale {np.abs(xr.grad.numpy()).max():.2e})")
