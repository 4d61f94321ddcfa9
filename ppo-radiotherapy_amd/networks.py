"""Policy / value networks (reference: networks.py).

`PPO` (networks.py:107-147) is the visionless MLP actor-critic; `PPO_3DCNN`
(networks.py:54-104) puts the C3D-style `FeaturesExtractor3D`
(networks.py:8-45) in front.  Module names and parameter shapes are those of
the reference, so `saves/*.model` state dicts load unchanged.

The Gaussian policy head is written out in closed form instead of going
through `torch.distributions.Normal`: the distribution's argument validation
reduces its inputs to a host bool on every construction (a device->host sync
per rollout step); the math is identical (log N(a; mu, sigma) summed over the
6 action dims, entropy 0.5 + 0.5 log 2pi + log sigma).
"""
from __future__ import annotations

import ctypes
import math

import numpy as np
import torch
from torch import nn

_HALF_LOG_2PI = 0.5 * math.log(2.0 * math.pi)


class _SplitKLinearFn(torch.autograd.Function):
    """y = x W^T + b whose weight gradient W' = dY^T X (a K = batch reduction:
    32768 in the PPO update) is computed as a batched GEMM over `chunks` slices
    of the batch plus one sum, so the reduction runs on many workgroups; the
    GEMM libraries give a K = 32768, 64 x 64 product only a handful."""

    @staticmethod
    def forward(ctx, x, weight, bias, chunks):
        ctx.save_for_backward(x, weight)
        ctx.chunks = chunks
        return torch.addmm(bias, x, weight.t())

    @staticmethod
    def backward(ctx, gy):
        x, weight = ctx.saved_tensors
        gx = gy.mm(weight) if ctx.needs_input_grad[0] else None
        c = ctx.chunks
        B = x.shape[0]
        if c > 1 and B % c == 0:
            gw = torch.bmm(gy.reshape(c, B // c, -1).transpose(1, 2), x.reshape(c, B // c, -1)).sum(0)
        else:
            gw = gy.t().mm(x)
        return gx, gw, gy.sum(0), None


SPLITK_MIN_BATCH = 4096
SPLITK_CHUNK = 512  # rows per slice of the weight-gradient reduction


class Linear(nn.Linear):
    """nn.Linear (same parameters and state-dict keys) with the split-K
    weight gradient for large batches (2-D inputs)."""

    def forward(self, x):
        B = x.shape[0] if x.dim() == 2 else 0
        if x.requires_grad or self.weight.requires_grad:
            if B >= SPLITK_MIN_BATCH and B % SPLITK_CHUNK == 0 and torch.is_grad_enabled():
                return _SplitKLinearFn.apply(x, self.weight, self.bias, B // SPLITK_CHUNK)
        return super().forward(x)


def layer_init(layer: nn.Module, std: float = float(np.sqrt(2)), bias_const: float = 0.0) -> nn.Module:
    """Orthogonal weights, constant bias (networks.py:48-51)."""
    nn.init.orthogonal_(layer.weight, std)
    nn.init.constant_(layer.bias, bias_const)
    return layer


def _tanh_mlp(d_in: int, width: int, d_out: int, head_std: float) -> nn.Sequential:
    # indices 0/2/4 hold the Linear layers, as in the reference's Sequential
    return nn.Sequential(
        layer_init(Linear(d_in, width)), nn.Tanh(),
        layer_init(Linear(width, width)), nn.Tanh(),
        layer_init(Linear(width, d_out), std=head_std),
    )


class GaussianHeadMixin:
    """get_value / get_action_and_value of the reference agents."""

    actor_logstd: nn.Parameter

    def _features(self, x: torch.Tensor) -> torch.Tensor:
        return x

    def get_value(self, x: torch.Tensor) -> torch.Tensor:
        return self.critic(self._features(x))

    def get_action_and_value(self, x: torch.Tensor, action: torch.Tensor | None = None,
                             generator: torch.Generator | None = None):
        f = self._features(x)
        mean = self.actor_mean(f)
        logstd = self.actor_logstd.expand_as(mean)
        std = torch.exp(logstd)
        if action is None:
            noise = torch.randn(mean.shape, dtype=mean.dtype, device=mean.device, generator=generator)
            action = mean + std * noise
        z = (action - mean) / std
        logprob = (-0.5 * z * z - logstd - _HALF_LOG_2PI).sum(1)
        entropy = (0.5 + _HALF_LOG_2PI + logstd).sum(1)
        return action, logprob, entropy, self.critic(f)


class PPO(GaussianHeadMixin, nn.Module):
    """Visionless agent: obs [B, 9] -> MLP 64-64 -> mean [B, 6], value [B, 1]."""

    def __init__(self, observation_shape, action_space, feature_dim: int = 64):
        super().__init__()
        self.feature_dim = feature_dim
        self.observation_shape = tuple(observation_shape)
        self.action_space = tuple(np.atleast_1d(action_space))
        n_obs = int(np.prod(self.observation_shape))
        n_act = int(np.prod(self.action_space))
        self.critic = _tanh_mlp(n_obs, feature_dim, 1, head_std=1.0)
        self.actor_mean = _tanh_mlp(n_obs, feature_dim, n_act, head_std=0.01)
        self.actor_logstd = nn.Parameter(torch.zeros(1, n_act))


def _conv_layer(cin, groups, dims, pad, precision: str = "f32"):
    from . import _lib

    return _lib.RtConvLayer(cin, groups, (ctypes.c_int32 * 3)(*dims), (ctypes.c_int32 * 3)(*pad),
                            _lib.CONV_PREC[precision])


def _stage_fwd(layer, out_dims, x, w, b, train: bool):
    """One fused Conv3d + ReLU + MaxPool3d stage (rt_conv_relu_pool_fwd)."""
    from . import _lib

    L = _lib.load()
    B = x.shape[0]
    y = torch.empty((B, 16, *out_dims), device=x.device, dtype=torch.float32)
    am = torch.empty((B, 16, *out_dims), device=x.device, dtype=torch.uint8) if train else None
    _lib.check(L.rt_conv_relu_pool_fwd(ctypes.byref(layer), B, x.data_ptr(), None, w.data_ptr(), b.data_ptr(),
                                       y.data_ptr(), _lib.ptr(am), _lib.stream_handle()), "rt_conv_relu_pool_fwd")
    return y, am


class _C3DStack(torch.autograd.Function):
    """The three C3D stages (networks.py:13-33) on the HIP kernels of
    csrc/c3d.hip; backward = weight gradients of all stages and the data
    gradients of stages 3 and 2 (the observation needs none)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, w3, b3, plan):
        (l1, d1), (l2, d2), (l3, d3) = plan
        p1, a1 = _stage_fwd(l1, d1, x, w1, b1, True)
        p2, a2 = _stage_fwd(l2, d2, p1, w2, b2, True)
        p3, a3 = _stage_fwd(l3, d3, p2, w3, b3, True)
        ctx.plan = plan
        ctx.save_for_backward(x, w2, w3, p1, a1, p2, a2, a3)
        return p3

    @staticmethod
    def backward(ctx, gp3):
        from . import _lib

        L = _lib.load()
        st = _lib.stream_handle()
        (l1, _), (l2, _), (l3, _) = ctx.plan
        x, w2, w3, p1, a1, p2, a2, a3 = ctx.saved_tensors
        B = x.shape[0]
        gp3 = gp3.contiguous()

        def wgrad(layer, xin, gy, am, cin, groups):
            dw = torch.empty((16, cin // groups, 3, 3, 3), device=x.device)
            db = torch.empty(16, device=x.device)
            ws = torch.empty(int(L.rt_conv_wgrad_workspace_floats(ctypes.byref(layer), B)), device=x.device)
            _lib.check(L.rt_conv_relu_pool_wgrad(ctypes.byref(layer), B, xin.data_ptr(), None, gy.data_ptr(),
                                                 am.data_ptr(), dw.data_ptr(), db.data_ptr(), ws.data_ptr(),
                                                 ws.numel(), st), "rt_conv_relu_pool_wgrad")
            return dw, db

        def dgrad(layer, w, gy, am, like):
            dx = torch.empty_like(like)
            _lib.check(L.rt_conv_relu_pool_dgrad(ctypes.byref(layer), B, w.data_ptr(), gy.data_ptr(), am.data_ptr(),
                                                 dx.data_ptr(), st), "rt_conv_relu_pool_dgrad")
            return dx

        dw3, db3 = wgrad(l3, p2, gp3, a3, 16, 4)
        gp2 = dgrad(l3, w3, gp3, a3, p2)
        dw2, db2 = wgrad(l2, p1, gp2, a2, 16, 2)
        gp1 = dgrad(l2, w2, gp2, a2, p1)
        dw1, db1 = wgrad(l1, x, gp1, a1, int(x.shape[1]), 1)
        return None, dw1, db1, dw2, db2, dw3, db3, None


class FeaturesExtractor3D(nn.Module):
    """C3D-lite encoder (networks.py:8-45): three 3x3x3 convs (groups 1/2/4)
    with ReLU and 2x2x2 max-pools, flatten, Linear -> features_dim, ReLU.
    The first pool pads each axis by (S_i - 2) % 2 (networks.py:18-20).
    On the GPU the three stages run as the fused f32-MFMA kernels of
    csrc/c3d.hip (forward + backward); the Conv3d modules hold the parameters
    (same state-dict keys).  `conv_precision` ("f32", the reference's, or
    "bf16x3") is the arithmetic of the forward products, passed per call in
    each stage's rt_conv_layer (set_conv_precision)."""

    def __init__(self, observation_shape, features_dim: int, conv_precision: str = "f32"):
        super().__init__()
        self.conv_precision = "f32"
        self.set_conv_precision(conv_precision)
        self.observation_shape = tuple(observation_shape)
        c_in, *spatial = self.observation_shape
        pad1 = tuple((s - 2) % 2 for s in spatial)
        self.cnn = nn.Sequential(
            nn.Conv3d(c_in, 16, 3), nn.ReLU(), nn.MaxPool3d(2, 2, padding=pad1),
            nn.Conv3d(16, 16, 3, groups=2), nn.ReLU(), nn.MaxPool3d(2, 2),
            nn.Conv3d(16, 16, 3, groups=4), nn.ReLU(), nn.MaxPool3d(2, 2),
            nn.Flatten(),
        )
        self.n_flatten = self._flat_size(spatial)
        self.mlp = nn.Sequential(nn.Linear(self.n_flatten, features_dim), nn.ReLU())

    @staticmethod
    def _flat_size(spatial) -> int:
        # closed form of the reference's dry run (networks.py:35-37)
        s = [x - 2 for x in spatial]                           # conv1
        s = [(x + 2 * ((sp - 2) % 2) - 2) // 2 + 1 for x, sp in zip(s, spatial)]  # pool1
        s = [(x - 2 - 2) // 2 + 1 for x in s]                  # conv2 + pool2
        s = [(x - 2 - 2) // 2 + 1 for x in s]                  # conv3 + pool3
        return 16 * int(np.prod(s))

    def set_conv_precision(self, precision: str):
        """Arithmetic of the stages' forward products ("f32" or "bf16x3")."""
        if precision not in ("f32", "bf16x3"):
            raise ValueError(f"conv_precision {precision!r}: expected 'f32' or 'bf16x3'")
        if precision != self.conv_precision:
            self.conv_precision = precision
            self._plan_cache = None

    def _plan(self):
        """rt_conv_layer descriptors + pooled dims of the three stages."""
        if getattr(self, "_plan_cache", None) is None:
            from . import _lib

            L = _lib.load()
            c_in, *spatial = self.observation_shape
            pads = [tuple((s - 2) % 2 for s in spatial), (0, 0, 0), (0, 0, 0)]
            dims, plan = tuple(spatial), []
            for (cin, groups), pad in zip([(c_in, 1), (16, 2), (16, 4)], pads):
                layer = _conv_layer(cin, groups, dims, pad, self.conv_precision)
                od = (ctypes.c_int32 * 3)()
                _lib.check(L.rt_conv_out_dims(ctypes.byref(layer), od), "rt_conv_out_dims")
                plan.append((layer, tuple(od)))
                dims = tuple(od)
            self._plan_cache = tuple(plan)
        return self._plan_cache

    def forward(self, observations: torch.Tensor) -> torch.Tensor:
        if observations.device.type != "cuda":
            return self.mlp(self.cnn(observations))  # CPU: the reference's torch modules
        x = observations.contiguous()
        c1, c2, c3 = self.cnn[0], self.cnn[3], self.cnn[6]
        params = (c1.weight, c1.bias, c2.weight, c2.bias, c3.weight, c3.bias)
        plan = self._plan()
        if torch.is_grad_enabled() and any(p.requires_grad for p in params):
            p3 = _C3DStack.apply(x, *params, plan)
        else:
            (l1, d1), (l2, d2), (l3, d3) = plan
            p1, _ = _stage_fwd(l1, d1, x, c1.weight, c1.bias, False)
            p2, _ = _stage_fwd(l2, d2, p1, c2.weight, c2.bias, False)
            p3, _ = _stage_fwd(l3, d3, p2, c3.weight, c3.bias, False)
        return self.mlp(p3.flatten(1))


class PPO_3DCNN(GaussianHeadMixin, nn.Module):
    """Vision agent (networks.py:54-104)."""

    def __init__(self, observation_shape, action_space, feature_dim: int = 64):
        super().__init__()
        self.feature_dim = feature_dim
        self.observation_shape = tuple(observation_shape)
        self.action_space = tuple(np.atleast_1d(action_space))
        n_act = int(np.prod(self.action_space))
        self.features_extractor = FeaturesExtractor3D(self.observation_shape, feature_dim)
        self.critic = _tanh_mlp(feature_dim, feature_dim, 1, head_std=1.0)
        self.actor_mean = _tanh_mlp(feature_dim, feature_dim, n_act, head_std=0.01)
        self.actor_logstd = nn.Parameter(torch.zeros(1, n_act))

    def _features(self, x):
        return self.features_extractor(x)

    def summary(self):
        print("Observation shape: ", self.observation_shape)
        print("Action space: ", self.action_space)
        print("Feature dim: ", self.feature_dim)
        n = sum(p.numel() for p in self.features_extractor.parameters())
        print(f"Features extractor: {self.features_extractor}\n  flatten={self.features_extractor.n_flatten} params={n}")
