"""ctypes binding of librtenv.so (include/rtenv.h).

This is the same binding a maintainer would add to the reference repo (see
INTEGRATION.md).  Device buffers are passed as raw pointers (torch
`tensor.data_ptr()`), the stream as the raw hipStream_t of torch's current
stream.  There is no CPU fallback: if the library is missing or fails to load
every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

from . import build as _build

# RT_LIB_PATH: load another build of the library (kernel-variant experiments)
LIB_PATH = os.environ.get("RT_LIB_PATH") or _build.OUT

INFO_NAMES = {
    "total": 0, "tumour": 1, "lung": 2, "distance_to_tumour": 3, "dose_tumour": 4, "dose_lung": 5,
    "overshoot_t": 6, "overshoot_r": 9, "pos": 10, "dir": 13, "stepped": 16, "ep_done": 17,
    "ep_return": 18, "ep_length": 19,
}
INFO_W = 20
STEP_DENSE, STEP_INCREMENTAL = 0, 1
DP_ID_BYTES, DP_F32, DP_F64 = 128, 0, 1  # RT_DP_ID_BYTES, RT_DP_F32, RT_DP_F64
PPO_PREC = {"f32": 0, "bf16x3": 1}  # RT_PPO_PREC_* (rt_ppo_hparams.precision)
CONV_PREC = {"f32": 0, "bf16x3": 1}  # RT_CONV_PREC_* (rt_conv_layer.precision)

RT_ELIMIT = -5
RT_ERRORS = {0: "RT_OK", -1: "RT_EINVAL", -2: "RT_ENOMEM", -3: "RT_EDEVICE", -4: "RT_ELAUNCH", -5: "RT_ELIMIT"}

# every symbol include/rtenv.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "rt_env_config_default", "rt_env_create", "rt_env_destroy", "rt_env_reset", "rt_env_step",
    "rt_env_set_next_tumours", "rt_env_reseed", "rt_env_dose", "rt_env_dose_index", "rt_env_get_state", "rt_env_set_pose", "rt_env_set_tumours", "rt_env_set_render_source",
    "rt_env_num_envs",
    "rt_env_kernel_timing", "rt_env_kernel_timing_read",
    "rt_debug_beam", "rt_debug_pose", "rt_env_beam_list", "rt_probe_random_rmw", "rt_probe_stream", "rt_host_sincos", "rt_host_tumour_sum", "rt_host_lung_sum", "rt_policy_sample", "rt_gae",
    "rt_env_step_policy", "rt_env_rollout_policy", "rt_env_set_rollout_groups",
    "rt_ppo_workspace_floats", "rt_ppo_num_params", "rt_ppo_grad", "rt_adam_step", "rt_ppo_update", "rt_ppo_status",
    "rt_dp_unique_id", "rt_dp_comm_create", "rt_dp_comm_destroy", "rt_dp_allreduce", "rt_ppo_update_dp",
    "rt_ppo_shuffle", "rt_ppo_shuffle_epochs", "rt_ppo_shuffle_adv", "rt_ppo_adv_stats", "rt_ppo_adv_sums", "rt_ppo_adv_finalize",
    "rt_conv_out_dims", "rt_conv_relu_pool_fwd", "rt_conv_wgrad_workspace_floats", "rt_conv_relu_pool_wgrad", "rt_conv_mfma_count",
    "rt_conv_relu_pool_dgrad",
    "rt_last_error", "rt_abi_version",
]


class RtError(RuntimeError):
    pass


ABI_VERSION = 5  # RTENV_ABI_VERSION of include/rtenv.h


class RtEnvConfig(ctypes.Structure):
    """rt_env_config (include/rtenv.h); struct_size is set on construction
    (the library rejects a config whose struct_size != its sizeof)."""
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("grid", ctypes.c_int32 * 3),
        ("num_envs", ctypes.c_int32),
        ("visionless", ctypes.c_int32),
        ("max_time_steps", ctypes.c_int32),
        ("beam_dose", ctypes.c_float),
        ("lung_dose_threshold", ctypes.c_float),
        ("tumour_dose_threshold", ctypes.c_float),
        ("min_angle_z", ctypes.c_double),
        ("movement_speed", ctypes.c_double),
        ("rotation_speed", ctypes.c_float),
        ("lung_dose_reward", ctypes.c_double),
        ("tumour_dose_reward", ctypes.c_float),
        ("distance_reward", ctypes.c_double),
        ("lungs_h", ctypes.c_void_p),
        ("n_tumours", ctypes.c_int32),
        ("tumour_voxels_h", ctypes.c_void_p),
        ("tumour_offsets_h", ctypes.c_void_p),
        ("seed", ctypes.c_uint64),
        ("env_id_base", ctypes.c_int64),
        ("step_mode", ctypes.c_int32),
    ]

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if not self.struct_size:
            self.struct_size = ctypes.sizeof(self)


class RtPpoBatch(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in ("obs", "actions", "logprobs", "advantages", "returns", "values")] + [
        ("batch_size", ctypes.c_int64)]


class RtPpoHparams(ctypes.Structure):
    _fields_ = [
        ("clip_coef", ctypes.c_float),
        ("clip_vloss", ctypes.c_int32),
        ("norm_adv", ctypes.c_int32),
        ("ent_coef", ctypes.c_float),
        ("vf_coef", ctypes.c_float),
        ("max_grad_norm", ctypes.c_float),
        ("adam_beta1", ctypes.c_double),
        ("adam_beta2", ctypes.c_double),
        ("adam_eps", ctypes.c_float),
        ("precision", ctypes.c_int32),
    ]


class RtPolicyStep(ctypes.Structure):
    _fields_ = [("params", ctypes.POINTER(ctypes.c_void_p)), ("n_params", ctypes.c_int32)] + [
        (k, ctypes.c_void_p) for k in ("obs_in", "done_in", "obs_store", "done_store", "act_store", "logp_store",
                                       "value_store")] + [
        ("seed", ctypes.c_uint64), ("counter", ctypes.c_uint64), ("env_id_base", ctypes.c_int64)]


class RtPolicyRollout(ctypes.Structure):
    _fields_ = [("step", RtPolicyStep), ("n_steps", ctypes.c_int32), ("reward_store", ctypes.c_void_p),
                ("info_store", ctypes.c_void_p)]


class RtConvLayer(ctypes.Structure):
    _fields_ = [("cin", ctypes.c_int32), ("groups", ctypes.c_int32), ("in_dims", ctypes.c_int32 * 3),
                ("pool_pad", ctypes.c_int32 * 3), ("precision", ctypes.c_int32)]


_lib = None


def load(build_if_missing: bool = True):
    """Load librtenv.so (building it first when only sources are present)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch ships its own libamdhip64.so.7; importing it first makes the
    # process use that one runtime (loading ours first would pair the system
    # HIP runtime with torch's HSA runtime and find no device).
    import torch  # noqa: F401
    if build_if_missing and (not os.path.exists(LIB_PATH) or _build.needs_build()):
        try:
            _build.build()
        except Exception as exc:  # pragma: no cover - surfaced to the caller
            if not os.path.exists(LIB_PATH):
                raise RtError(f"librtenv.so is missing and could not be built: {exc}") from exc
    if not os.path.exists(LIB_PATH):
        raise RtError(f"librtenv.so not found at {LIB_PATH}")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, f64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    sig = {
        "rt_env_config_default": ([ctypes.POINTER(RtEnvConfig)], ctypes.c_int),
        "rt_env_create": ([ctypes.POINTER(RtEnvConfig), ctypes.c_int, ctypes.POINTER(vp)], ctypes.c_int),
        "rt_env_destroy": ([vp], None),
        "rt_env_reset": ([vp, vp, vp, vp, vp], ctypes.c_int),
        "rt_env_step": ([vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "rt_env_set_next_tumours": ([vp, vp, vp], ctypes.c_int),
        "rt_env_reseed": ([vp, ctypes.c_uint64, vp], ctypes.c_int),
        "rt_env_dose": ([vp, ctypes.POINTER(i64)], vp),
        "rt_env_dose_index": ([vp], vp),
        "rt_env_get_state": ([vp, vp, vp, vp, vp], ctypes.c_int),
        "rt_env_set_pose": ([vp, vp, vp], ctypes.c_int),
        "rt_env_set_tumours": ([vp, vp, vp], ctypes.c_int),
        "rt_env_set_render_source": ([vp, vp, ctypes.c_int64, vp, ctypes.c_int32], ctypes.c_int),
        "rt_env_num_envs": ([vp], ctypes.c_int),
        "rt_env_kernel_timing": ([vp, i32], ctypes.c_int),
        "rt_env_kernel_timing_read": ([vp, ctypes.POINTER(f64), ctypes.POINTER(i32)], ctypes.c_int),
        "rt_debug_beam": ([ctypes.POINTER(i32), i32, vp, vp, i32, vp, vp, vp, vp], ctypes.c_int),
        "rt_debug_pose": ([ctypes.POINTER(i32), i32, vp, vp, vp, vp, vp], ctypes.c_int),
        "rt_env_beam_list": ([vp, i32, vp, vp, vp, vp], ctypes.c_int),
        "rt_probe_random_rmw": ([vp, i64, i32, i32, ctypes.c_uint64, vp], ctypes.c_int),
        "rt_probe_stream": ([vp, vp, i64, i32, i32, vp], ctypes.c_int),
        "rt_host_sincos": ([i32, vp, vp, vp], ctypes.c_int),
        "rt_host_tumour_sum": ([i64, i32, vp, vp, vp], ctypes.c_int),
        "rt_host_lung_sum": ([ctypes.POINTER(i32), vp, vp, vp], ctypes.c_int),
        "rt_gae": ([i32, i32, vp, vp, vp, vp, vp, f64, f64, vp, vp, vp], ctypes.c_int),
        "rt_policy_sample": ([ctypes.POINTER(vp), i32, i32, vp, vp, vp, vp, vp, vp, vp, ctypes.c_uint64,
                              ctypes.c_uint64, i64, vp], ctypes.c_int),
        "rt_env_step_policy": ([vp, ctypes.POINTER(RtPolicyStep), vp, vp, vp, vp, vp], ctypes.c_int),
        "rt_env_rollout_policy": ([vp, ctypes.POINTER(RtPolicyRollout), vp, vp, vp], ctypes.c_int),
        "rt_env_set_rollout_groups": ([vp, i32], ctypes.c_int),
        "rt_ppo_workspace_floats": ([i32], i64),
        "rt_ppo_num_params": ([], i32),
        "rt_ppo_grad": ([ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(RtPpoBatch), vp, i32, vp,
                         ctypes.POINTER(RtPpoHparams), vp, i64, vp, vp, vp], ctypes.c_int),
        "rt_adam_step": ([i64, vp, vp, vp, vp, i64, f64, ctypes.POINTER(RtPpoHparams), i32, vp, vp], ctypes.c_int),
        "rt_ppo_update": ([ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(RtPpoBatch), vp, i32, i32, vp,
                           ctypes.POINTER(RtPpoHparams), vp, vp, vp, vp, i64, i64, f64, vp, i64, vp, vp, vp],
                          ctypes.c_int),
        "rt_ppo_status": ([], ctypes.c_int),
        "rt_dp_unique_id": ([vp], ctypes.c_int),
        "rt_dp_comm_create": ([vp, i32, i32, ctypes.c_int, ctypes.POINTER(vp)], ctypes.c_int),
        "rt_dp_comm_destroy": ([vp], None),
        "rt_dp_allreduce": ([vp, vp, i64, i32, vp], ctypes.c_int),
        "rt_ppo_update_dp": ([ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(RtPpoBatch), vp, i32, i32, vp,
                              ctypes.POINTER(RtPpoHparams), vp, vp, vp, vp, i64, i64, f64, vp, i64, vp, vp, vp, vp],
                             ctypes.c_int),
        "rt_ppo_shuffle": ([i64, ctypes.c_uint64, vp, vp], ctypes.c_int),
        "rt_ppo_shuffle_epochs": ([i64, i32, vp, vp, vp], ctypes.c_int),
        "rt_ppo_shuffle_adv": ([i64, i32, vp, vp, vp, i32, vp, vp, vp, i64, vp], ctypes.c_int),
        "rt_ppo_adv_stats": ([vp, vp, i32, i32, vp, vp, i64, vp], ctypes.c_int),
        "rt_ppo_adv_sums": ([vp, vp, i32, i32, vp, vp, i64, vp], ctypes.c_int),
        "rt_ppo_adv_finalize": ([vp, i64, i32, vp, vp], ctypes.c_int),
        "rt_conv_out_dims": ([ctypes.POINTER(RtConvLayer), ctypes.POINTER(i32)], ctypes.c_int),
        "rt_conv_relu_pool_fwd": ([ctypes.POINTER(RtConvLayer), i32, vp, vp, vp, vp, vp, vp, vp], ctypes.c_int),
        "rt_conv_wgrad_workspace_floats": ([ctypes.POINTER(RtConvLayer), i32], i64),
        "rt_conv_mfma_count": ([ctypes.POINTER(RtConvLayer), i32, i32], i64),
        "rt_conv_relu_pool_wgrad": ([ctypes.POINTER(RtConvLayer), i32, vp, vp, vp, vp, vp, vp, vp, i64, vp],
                                    ctypes.c_int),
        "rt_conv_relu_pool_dgrad": ([ctypes.POINTER(RtConvLayer), i32, vp, vp, vp, vp, vp], ctypes.c_int),
        "rt_last_error": ([], ctypes.c_char_p),
        "rt_abi_version": ([], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.rt_abi_version() != ABI_VERSION:
        raise RtError(f"{LIB_PATH}: ABI {L.rt_abi_version()} != {ABI_VERSION} expected by this package (rebuild it)")
    _lib = L
    return L


def check(rc: int, what: str):
    if rc != 0:
        msg = load().rt_last_error().decode(errors="replace")
        raise RtError(f"{what} failed: {RT_ERRORS.get(rc, rc)}: {msg}")


def ptr(t) -> int | None:
    """Raw device pointer of a torch tensor (None passes NULL)."""
    return None if t is None else t.data_ptr()


def stream_handle(stream=None) -> int | None:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream or None


def grid_arg(grid):
    return (ctypes.c_int32 * 3)(*[int(x) for x in grid])
