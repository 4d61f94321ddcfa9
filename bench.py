#!/usr/bin/env python3
"""Benchmark: env steps/s (whole node) + PPO updates/s, visionless, 64^3.

Workload (BASELINE.json configs[1]; configs[2] at --gpus 8): 4096 envs per
GPU on a 64^3 voxel grid (reference lung mask nearest-resampled, 1000
synthetic spherical tumours), the reference's visionless MLP policy, PPO with
num_steps=64, num_minibatches=8, update_epochs=10 and the
remaining keys of configs/default.yaml.

A bench "step" = one vectorised rollout step of every env on every GPU:
policy forward + Gaussian sample + the HIP env step (k_beam + k_dense +
k_finish), i.e. train.py:143-158, issued by the trainer's rollout call
(rt_env_rollout_policy: in dense mode two env groups pipelined over two
streams, taking turns on a persistent k_dense; --rollout-groups 1 issues
every launch on one stream).  roofline.isolated: k_dense of a one-group
pass over the same workload (the kernel alone on the chip).  `value` = envs x steps / max-over-ranks
wall time.
Also reported:
  ppo_updates_per_s      optimizer steps/s of the PPO update phase
                         (80 minibatch steps of 32768 samples per rank, flat
                         gradient all-reduce per step when n_gpus > 1)
  train_env_steps_per_s  env steps/s of a full PPO iteration
                         (64 rollout steps + GAE + 80 updates)
  update_mfma            the fused update (rt_ppo_update) vs the f32 MFMA peak
  update_precision       the 64x64 layer products of that update: f32
                         (--update-precision, default: the reference's
                         arithmetic) or bf16x3 (split-operand bf16 MFMA, the
                         f64 gates of tests/test_gpu_trainer.py hold);
                         ppo_update_ms_<other> times the other one on the same
                         update
  other_step_mode        the same rollout + iteration with the other env step
                         formulation (incremental, SURVEY §8 f-2: bitwise-equal
                         rewards/termination, touches only the beam's voxels)
  roofline               k_dense (the dominant kernel) vs HBM: HIP events the
                         library records around it on the env stream over
                         the timed region; traffic from the committed PMC run
                         (PMC_FILE), rocprofv3's average from ROCPROF_FILE
  steady_state           >= 101 steps (2 x num_steps) with the envs' episode
                         clocks staggered uniformly, so the window carries the
                         t = 100 truncation autoresets a long run pays
  other_step_mode.roofline
                         the incremental step's transaction model (random
                         128-B line RMWs per env-step) vs a measured random-line
                         RMW ceiling (rt_probe_random_rmw)
  update_allreduce_ms    (n_gpus > 1) the flat-gradient all-reduce alone
  ppo_update_ms_collective_path
                         the data-parallel update path (rt_ppo_update_dp:
                         grad, RCCL all-reduce, clip + Adam per minibatch in
                         one library call); at n_gpus 1 over a world-1 RCCL
                         group
  cpu_baseline           op-for-op NumPy port of the reference step on one
                         pinned host core, BASELINE.md §3 config C1 (reference
                         grid and tumours, seed 1, default_rng(0) actions;
                         bounded sample); beside it the same on the box's core
                         share and the scalar C port
  roofline.measured_read_ceiling_GBps / measured_copy_ceiling_GBps
                         HBM stream ceilings measured in the same run
                         (rt_probe_stream: k_dense's non-temporal float4
                         read sweep alone, and a float4 copy)
  c3d_mfma               configs[3]'s C3D feature extractor (the MFMA path,
                         north_star): its stage kernels on 512 vision
                         observations at 64^3, inference forward and the
                         training pass; EXECUTED work (Winograd MFMA
                         wave-instructions, = SQ_INSTS_MFMA; the sparse weight
                         gradients' VALU FMAs) over kernel time vs the f32
                         peak, the committed PMC MFMA-busy per stage beside it,
                         and the direct-conv FLOP rate as `effective_*` (HIP
                         events on the kernels' stream)

Run:  python bench.py [--gpus N --steps K --warmup W]
      (N > 1: one rank per GPU under torch.distributed.run -- started by the
      caller, or by bench.py itself when it runs outside one; add
      --rehearse-same-device to run the N ranks on cuda:0 over gloo)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "env steps/sec (whole node) + PPO updates/sec, visionless 64³ voxel, 1/2/4/8 GPU"
HBM_PEAK = 8.0e12  # MI355X HBM3E, B/s (MI355X_MICROARCH.md)
F32_MFMA_PEAK = 157.3e12  # dense f32 MFMA (= f32 vector) peak, FLOP/s (MI355X_MICROARCH.md)


def c3d_fwd_flop(grid) -> int:
    """Convolution FLOPs of one C3D forward (networks.py:13-33) on `grid`
    (0.999 GFLOP at 64^3, 8.56 at 128^3)."""
    dims, total = list(grid), 0
    for k, (cin_per_group, pad) in enumerate([(4, None), (8, 0), (4, 0)]):
        conv = [d - 2 for d in dims]
        total += 2 * 16 * cin_per_group * 27 * int(np.prod(conv))
        pads = [(d - 2) % 2 for d in dims] if pad is None else [0, 0, 0]
        dims = [(c + 2 * p - 2) // 2 + 1 for c, p in zip(conv, pads)]
    return total
WINO_USEFUL = 64 / 216  # F(2x2x2, 3x3x3): products per window and channel pair / direct MACs
UPDATE_MACS_PER_SAMPLE = (9 * 64 + 64 * 64 + 64 * 6) + (9 * 64 + 64 * 64 + 64) \
    + (2 * 64 * 6 + 2 * 64 * 64 + 9 * 64) + (2 * 64 + 2 * 64 * 64 + 9 * 64)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--envs", type=int, default=4096, help="envs per GPU")
    ap.add_argument("--grid", type=int, default=64)
    ap.add_argument("--num-steps", type=int, default=64)
    ap.add_argument("--num-minibatches", type=int, default=8)
    ap.add_argument("--update-epochs", type=int, default=10)
    ap.add_argument("--cpu-seconds", type=float, default=8.0,
                    help="CPU-baseline sample budget per leg (4 legs: numpy/C x 1/all cores)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-update", action="store_true")
    ap.add_argument("--no-c3d", action="store_true", help="skip the C3D MFMA stage timing (c3d_mfma)")
    ap.add_argument("--no-steady", action="store_true", help="skip the >= 101-step steady-state window")
    ap.add_argument("--env-only", action="store_true", help="time rt_env_step alone (profiling)")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--vision", action="store_true",
                    help="BASELINE configs[3]: C3D policy on 4-channel volume observations (512 envs, 64^3)")
    ap.add_argument("--micro-batch", type=int, default=0)
    ap.add_argument("--step-mode", choices=["dense", "incremental"], default="dense",
                    help="env step formulation measured as `value` (the other is reported beside it)")
    ap.add_argument("--rollout-groups", type=int, default=2, choices=[1, 2, 3, 4],
                    help="dense mode: env groups of the rollout call (2 = two pipelined streams, "
                         "1 = the stepwise launches on one stream)")
    ap.add_argument("--update-minibatches", type=int, default=0,
                    help="time only this many minibatch steps of the update (0 = all)")
    ap.add_argument("--conv-precision", choices=["f32", "bf16x3"], default="f32",
                    help="vision: conv1's forward products (rt_conv_layer.precision) in the rollout and the update")
    ap.add_argument("--update-precision", choices=["f32", "bf16x3"], default="f32",
                    help="the fused update's 64x64 layer products (ppo_update_ms); the other is timed beside it")
    ap.add_argument("--rocprof-stats", default=None,
                    help="rocprofv3 --stats kernel_stats.csv of this same command (roofline.rocprof cross-check); "
                         "default: the committed stats, labelled historical")
    ap.add_argument("--rehearse-same-device", action="store_true",
                    help="multi-rank rehearsal on one GPU: every rank on cuda:0, gloo instead of RCCL")
    a = ap.parse_args()
    if a.vision:
        # 512 envs, 64^3, num_steps 16, vision.yaml minibatching
        # micro-batches of the update: the C3D kernels run 16 % faster per sample
        # at 1024 than at 128 (64^3: 145 vs 172 ms per 4096-sample minibatch,
        # flat from 1024 to 4096); at 128^3 (32 MiB of observation per sample)
        # 512 (1226 vs 1265 ms)
        mb = 1024 if a.grid <= 64 else 512
        for k, v in dict(envs=512, num_steps=16, num_minibatches=2, micro_batch=mb, update_minibatches=2).items():
            if getattr(a, k) == ap.get_default(k):
                setattr(a, k, v)
    return a


def trainer_cfg(a):
    # configs/default.yaml keys; C2 rollout/update shape
    return SimpleNamespace(num_steps=a.num_steps, num_minibatches=a.num_minibatches, update_epochs=a.update_epochs,
                           learning_rate=3e-4, anneal_lr=False, gamma=0.99, gae_lambda=0.95, norm_adv=True,
                           clip_coef=0.1, clip_vloss=True, ent_coef=0.0, vf_coef=0.5, max_grad_norm=0.5,
                           micro_batch=a.micro_batch, update_precision=a.update_precision,
                           **({"conv_precision": a.conv_precision} if a.vision else {}))


def cpu_baseline(seconds: float):
    """The reference's single-env step on the host cores (oracle/cpu_bench.py,
    run as a child process) on BASELINE.md §3's config C1 (reference grid and
    tumours, np.random.seed(1), default_rng(0) actions): the op-for-op NumPy
    port on one pinned core is `value`; the same on the box's core share (one
    pinned process each) and the scalar C restatement are reported beside it."""
    import subprocess

    cmd = [sys.executable, os.path.join(REPO, "oracle", "cpu_bench.py"), "--grid", "0",
           "--seconds", str(seconds), "--kinds", "numpy,c"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=20 * seconds + 300)
    if r.returncode != 0:
        return {"error": r.stderr[-2000:]}
    d = json.loads(r.stdout.strip().splitlines()[-1])
    one = d["numpy"]["one_core"]
    out = {"value": one["value"], "unit": "env steps/s", "cores": 1, "kind": "port",
           "sample": f"{one['steps']} visionless steps of one env, {d['config']} (oracle/numpy_env.py, "
                     f"calibrated to the reference: tools/calibrate_cpu.py), {one['seconds']:.1f} s on 1 pinned "
                     f"host core ({d['cpu_model']}), allocator pinned (the reference's fault-free regime)",
           "cpu_model": d["cpu_model"], "cores_available": d["cores_available"], "cores_cap": d["cores_cap"]}
    if "all_cores" in d["numpy"]:
        out["all_cores"] = {k: d["numpy"]["all_cores"][k] for k in ("value", "cores", "steps")}
    out["c_port"] = {"one_core": d["c"]["one_core"]["value"],
                     "all_cores": d["c"].get("all_cores", {}).get("value"),
                     "cores": d["c"].get("all_cores", {}).get("cores", 1)}
    return out


def run_steps(tr, k: int):
    """k vectorised rollout steps through the trainer, continuing the storage
    ring (row = step mod T): runs of consecutive rows go to tr.rollout_steps,
    which is one persistent launch per run where the env supports it
    (incremental step mode) and one launch per step otherwise."""
    i = 0
    while i < k:
        s = i % tr.T
        c = min(tr.T - s, k - i)
        tr.rollout_steps(s, c)
        i += c


def stagger_phases(tr, env, dev):
    """Spread the envs' episode clocks uniformly over the 100-step episode: a
    100-step pre-roll resets the envs with e % 100 == k at pre-roll step k
    (masked rt_env_reset), so from then on every rollout step carries ~1 % of
    the envs through the t = 100 truncation autoreset (a RESET zeroes the
    env's whole dose row) -- the steady state of a long run (train.py:138-161
    with every env autoresetting inside the rollout), which a window started
    right after reset() never reaches."""
    import torch

    N = env.num_envs
    e_idx = torch.arange(N, device=dev)
    for k in range(100):
        env.reset(options={"mask": (e_idx % 100) == k})
        tr.rollout_steps(k % tr.T, 1)


_MARK_BUF = {}


def window_marker(dev):
    """A one-block rt_probe_stream launch on the current stream, issued just
    before a timed window's opening synchronise: it marks the window in a
    rocprofv3 kernel trace (tools/window_kernels.py, tools/call_cost_trace.py)
    and costs the window nothing."""
    import torch

    from ppo_radiotherapy_amd import _lib

    buf = _MARK_BUF.get(dev)
    if buf is None:
        buf = _MARK_BUF[dev] = torch.zeros(4, device=dev)
    _lib.check(_lib.load().rt_probe_stream(buf.data_ptr(), buf.data_ptr(), 4, 0, 1, _lib.stream_handle()), "marker")


def steady_state(tr, env, dev, barrier, max_over_ranks, total_envs, calls: int = 2):
    """Env steps/s over three back-to-back windows of calls x T (>= 101)
    rollout steps each, on the staggered episode phases stagger_phases set up
    before the warmup (the phases stay staggered: every env autoresets on its
    own clock).  Nothing but the rollout calls runs inside the timed windows;
    the autoreset count and the kernel times come from a fourth, instrumented
    window.  A one-block rt_probe_stream launch before each window marks it in
    a rocprofv3 kernel trace (tools/window_kernels.py)."""
    import torch

    def mark():
        window_marker(dev)

    T = tr.T
    K = calls * T
    # three back-to-back windows (the phases stay staggered); the median is reported
    dts = []
    for _ in range(3):
        mark()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(calls):
            tr.rollout_steps(0, T)
        torch.cuda.synchronize()
        barrier()
        dts.append(max_over_ranks(time.perf_counter() - t0))
    mark()
    dt = sorted(dts)[1]
    # kernel times and the autoreset count: a fourth window of the same length, with HIP events
    resets = torch.zeros((), dtype=torch.int64, device=dev)
    env.kernel_timing(2 * K)
    for _ in range(calls):
        tr.rollout_steps(0, T)
        resets += (tr.infos[..., 16] == 0).sum()  # autoresets in these T steps
    torch.cuda.synchronize()
    kms, kcalls = env.kernel_timing_read()
    env.kernel_timing(0)
    return {"steps": K, "ms_per_step": 1000 * dt / K, "env_steps_per_s": total_envs * K / dt,
            "windows_env_steps_per_s": [total_envs * K / d for d in dts],
            "kernel_ms_per_step": {k: v * kcalls / K for k, v in kms.items()},
            "autoresets_in_window": int(resets.item()),
            "episode_phase": "staggered uniformly over the 100-step episode (stagger_phases before the warmup)"}


def march_lines(env):
    """Distinct 128-B dose lines the march read-modify-writes per env-step
    (draw_line.py:49-100 splats applied by environment.py:107-110), counted on
    the beams the envs applied last (rt_env_beam_list), at the dose-row
    positions the library stores them (lung-first rows: rt_env_dose_index).
    Envs whose last call was a reset count 0 (they marched nothing)."""
    import torch

    idx, _, cnt = env.beam_list()
    cap = idx.shape[1]
    valid = torch.arange(cap, device=idx.device)[None, :] < cnt.clamp_min(0)[:, None]
    pos = env.dose_index()
    if pos is not None:
        idx = pos.long()[idx.long().clamp(0, pos.numel() - 1)]
    lines = torch.where(valid, idx.long() // 32, torch.full_like(idx.long(), -1))
    lines, _ = lines.sort(dim=1)
    distinct = ((lines[:, 1:] != lines[:, :-1]) & (lines[:, 1:] >= 0)).sum(1) + (lines[:, 0] >= 0).long()
    return float(distinct.double().mean())


def incremental_transactions(env, lib):
    """Transaction model of one incremental env-step: the
    march read-modify-writes the distinct 128-B dose lines its splats touch,
    the finish reads the lines of the tumour's voxels.  Counted on the beams
    the envs applied last (rt_env_beam_list) and their current tumours."""
    import torch

    idx, _, cnt = env.beam_list()
    cap = idx.shape[1]
    valid = torch.arange(cap, device=idx.device)[None, :] < cnt.clamp_min(0)[:, None]
    lines = torch.where(valid, idx // 32, torch.full_like(idx, -1))
    lines, _ = lines.sort(dim=1)
    distinct = ((lines[:, 1:] != lines[:, :-1]) & (lines[:, 1:] >= 0)).sum(1) + (lines[:, 0] >= 0).long()
    beam_lines = float(distinct.double().mean())
    _, _, tum = env.get_state()
    per_tumour = np.array([len(np.unique(lib.tumour_voxels(k) // 32)) for k in range(lib.n_tumours)], np.float64)
    tumour_lines = float(per_tumour[tum.cpu().numpy()].mean())
    return beam_lines, tumour_lines


def random_rmw_ceiling(dev, lib_obj, floats: int, lanes: int = 1 << 18, lines_per_lane: int = 64):
    """Random 128-B line read-modify-writes per second (rt_probe_random_rmw:
    one float per lane and line, 4 lines in flight per lane) over a buffer of
    the dose array's size."""
    import torch

    from ppo_radiotherapy_amd import _lib

    buf = torch.zeros(floats, dtype=torch.float32, device=dev)
    st = _lib.stream_handle()
    _lib.check(lib_obj.rt_probe_random_rmw(buf.data_ptr(), floats, lanes, lines_per_lane, 1, st), "probe")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record()
    for r in range(reps):
        _lib.check(lib_obj.rt_probe_random_rmw(buf.data_ptr(), floats, lanes, lines_per_lane, 2 + r, st), "probe")
    e1.record()
    torch.cuda.synchronize()
    sec = e0.elapsed_time(e1) * 1e-3
    del buf
    torch.cuda.empty_cache()
    return reps * lanes * lines_per_lane / sec


def stream_ceilings(dev, lib_obj, gib: float = 4.0, reps: int = 8) -> dict:
    """Measured HBM stream ceilings in the same run (rt_probe_stream, HIP
    events on the stream the probe runs on): a READ sweep of non-temporal 16-B
    loads -- k_dense's access shape, the ceiling its `frac_of_measured_ceiling`
    is against -- and a COPY (read + write bytes), over a buffer 16x the
    256 MiB Infinity Cache; best of three grid sizes."""
    import torch

    from ppo_radiotherapy_amd import _lib

    n = int(gib * (1 << 30)) // 4
    src = torch.ones(n, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    st = _lib.stream_handle()
    out = {}
    for mode, name, traffic in ((0, "read", 4 * n), (1, "copy", 8 * n)):
        best = 0.0
        for blocks in (1024, 2048, 4096):
            def once():
                _lib.check(lib_obj.rt_probe_stream(src.data_ptr(), dst.data_ptr(), n, mode, blocks, st), "probe")
            once()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                once()
            e1.record()
            torch.cuda.synchronize()
            best = max(best, traffic * reps / (e0.elapsed_time(e1) * 1e-3))
        out[name] = best
    del src, dst
    torch.cuda.empty_cache()
    return out


PMC_FILE = os.path.join(REPO, "profiles", "r06", "r06_final_k_dense_pmc.json")
# rocprofv3 --kernel-trace --stats of this bench's default command, committed
# with a sidecar <csv>.meta.json naming the commit of the tree it was measured
# on; used (labelled "historical") when --rocprof-stats does not name the
# stats of the current run
ROCPROF_FILE = os.path.join(REPO, "profiles", "r06", "r06_final_kernel_stats.csv")
# the lung-first stream kernel (k_dense<true> gathers from C-order rows)
DENSE_KERNEL = "k_dense<false>"


def load_rocprof(kernel: str, path: str | None = None):
    """Average duration (ms) and call count of `kernel` in rocprofv3 --stats
    output: `path` (the stats of THIS run, --rocprof-stats) or the committed
    file of the default command (historical, with the commit it was measured
    on).  None when the kernel is not in it."""
    import csv

    src = path or ROCPROF_FILE
    try:
        for r in csv.DictReader(open(src)):
            if kernel in r["Name"]:
                out = {"avg_ms": float(r["AverageNs"]) / 1e6, "calls": int(r["Calls"]),
                       "source": os.path.relpath(src, REPO) if src.startswith(REPO) else src}
                if path is None:
                    try:
                        with open(src + ".meta.json") as f:
                            meta = json.load(f)
                    except OSError:
                        meta = {}
                    out["historical"] = True
                    out["measured_at_commit"] = meta.get("commit")
                    out["note"] = ("committed stats of this command on an earlier tree (not this run); pass "
                                   "--rocprof-stats <kernel_stats.csv> of the current run to cross-check it")
                else:
                    out["historical"] = False
                return out
    except Exception:
        return None
    return None


def load_pmc(grid, envs, pipelined=False, kernel="k_dense"):
    """Per-launch HBM traffic (bytes) of the dense stream from the committed
    rocprofv3 PMC runs, gfx950 FETCH_SIZE x2 correction applied there: the
    pipelined rollout (k_dense over 2048 envs per launch) from
    tools/probe_dense_pmc.py + tools/dense_pmc_segments.py on the current
    kernel -> {"value_window": B, "steady_window": B}; the older single-run
    files (profiles/{kernel}_pmc.json) otherwise.  None when no run matches."""
    if pipelined:
        try:
            with open(PMC_FILE) as f:
                d = json.load(f)
            if tuple(d["grid"]) == tuple(grid) and int(d["envs_per_launch"]) == envs:
                seg = d["segments"]
                return {"value_window": seg["value_window_20_steps"]["hbm_bytes_median"],
                        "steady_window": seg["steady_window_64_steps"]["hbm_bytes_median"],
                        "source": os.path.relpath(PMC_FILE, REPO)}
        except Exception:
            return None
        return None
    p = os.path.join(REPO, "profiles", f"{kernel}_pmc.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if (tuple(d.get("grid", ())) == tuple(grid) and int(d.get("envs", -1)) == envs
                and d.get("layout") == "lung_first"):
            return d.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


C3D_PMC_FILE = os.path.join(REPO, "profiles", "r05", "r05_c3d_pmc_b512.json")
MFMA_F32_FLOP = 2 * 16 * 16 * 4  # one v_mfma_f32_16x16x4_f32 wave-instruction


def load_c3d_pmc():
    """Per-kernel PMC of the C3D stage kernels at batch 512 (rocprofv3 --pmc
    over tools/c3d_pmc_driver.py, tools/c3d_pmc_summary.py): SQ_INSTS_MFMA,
    MFMA-busy fraction of the SIMD cycles at the measured clock, the clock.
    None when the committed file is absent."""
    try:
        with open(C3D_PMC_FILE) as f:
            d = json.load(f)
    except OSError:
        return None
    out = {}
    for k, v in d["kernels"].items():
        short = k.replace("void ", "").replace(" ", "")
        out[short] = v
    return {"kernels": out, "source": os.path.relpath(C3D_PMC_FILE, REPO)}


def c3d_roofline(dev, lib, grid, batch: int = 512, reps: int = 5):
    """BASELINE configs[3]'s C3D (north_star: "MFMA utilisation on the 3D-conv
    against gfx950 peak"): the feature extractor's three fused stage kernels
    on `batch` observations of a vision env at `grid` (a rollout step of 512
    envs), timed with HIP events on the stream they run on: inference forward
    (the rollout policy) and the training pass (forward with argmax bytes,
    weight gradients of the three stages, data gradients of stages 3 and 2).

    Work is counted as EXECUTED: the f32 forward and the grouped data
    gradients run Winograd F(2x2x2, 3x3x3) on v_mfma_f32_16x16x4_f32 -- their
    MFMA wave-instructions come from the launch planner (rt_conv_mfma_count,
    = rocprofv3's SQ_INSTS_MFMA, checked against the committed PMC run), 2,048
    FLOP each, zero-padded channel lanes included; the weight gradients gather
    one argmax patch per (channel, pooled window) -- 1/8 of the dense MACs --
    as f32 FMAs on the VALU, priced against the VALU peak (= the f32 MFMA
    peak, 157.3 TFLOP/s).  `frac` = executed FLOP / kernel time / peak (at
    the 2.4 GHz spec clock); `pmc_mfma_busy` = SQ_INSTS_MFMA x 32 cycles over
    the SIMD cycles at the clock the kernel ran at (GRBM_GUI_ACTIVE), so frac
    = busy x clock / 2.4 GHz.  The direct-convolution FLOPs (the reference's
    cuDNN work, 0.999 GFLOP per 64^3 forward) over the same time are reported
    beside them as `effective_*`: not a utilisation (Winograd executes 3.4x
    fewer products, the sparse weight gradient 8x fewer)."""
    import ctypes

    import torch

    from ppo_radiotherapy_amd import _lib
    from ppo_radiotherapy_amd.networks import FeaturesExtractor3D
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    env = RadiotherapyVecEnv(batch, visionless=False, library=lib, device=dev, seed=7)
    env.reset()
    g = torch.Generator(device=dev).manual_seed(3)
    for _ in range(6):
        env.step(torch.rand((batch, 6), device=dev, generator=g) * 2 - 1)
    obs = env.obs.clone()
    env.close()
    torch.manual_seed(0)
    fe = FeaturesExtractor3D((4, *grid), 64).to(dev)
    convs = [m for m in fe.modules() if isinstance(m, torch.nn.Conv3d)]
    L = _lib.load()
    st = _lib.stream_handle()
    names = ["conv1", "conv2", "conv3"]
    cins = [4, 16, 16]
    pmc = load_c3d_pmc() if tuple(grid) == (64, 64, 64) and batch == 512 else None

    def timed(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    def run_stages(prec):
        fe.set_conv_precision(prec)
        plan = fe._plan()
        acts, ams, grads = [obs], [], []
        for layer, od in plan:
            acts.append(torch.empty((batch, 16, *od), device=dev))
            ams.append(torch.empty((batch, 16, *od), dtype=torch.uint8, device=dev))
            grads.append(torch.randn((batch, 16, *od), device=dev) * 1e-3)
        stages, tot = {}, {"fwd_ms": 0.0, "train_ms": 0.0, "fwd_exec": 0, "train_mfma": 0, "train_valu": 0,
                           "fwd_eff": 0, "train_eff": 0, "train_useful": 0}
        dims = list(grid)
        for k, (layer, od) in enumerate(plan):
            cpg = cins[k] // int(layer.groups)
            direct = 2 * batch * 16 * cpg * 27 * int(np.prod([d - 2 for d in dims]))  # dense conv FLOP
            dims = list(od)
            w, bb = convs[k].weight.detach().contiguous(), convs[k].bias.detach().contiguous()

            def fwd(am):
                return lambda: _lib.check(L.rt_conv_relu_pool_fwd(ctypes.byref(layer), batch, acts[k].data_ptr(),
                                                                  None, w.data_ptr(), bb.data_ptr(),
                                                                  acts[k + 1].data_ptr(), _lib.ptr(am), st), "fwd")
            t_inf = timed(fwd(None))
            t_trn = timed(fwd(ams[k]))
            dw, db = torch.empty_like(w), torch.empty_like(bb)
            ws = torch.empty(int(L.rt_conv_wgrad_workspace_floats(ctypes.byref(layer), batch)), device=dev)
            t_wg = timed(lambda: _lib.check(L.rt_conv_relu_pool_wgrad(
                ctypes.byref(layer), batch, acts[k].data_ptr(), None, grads[k].data_ptr(), ams[k].data_ptr(),
                dw.data_ptr(), db.data_ptr(), ws.data_ptr(), ws.numel(), st), "wgrad"))
            n_fwd = int(L.rt_conv_mfma_count(ctypes.byref(layer), batch, 0))
            f_fwd = n_fwd * MFMA_F32_FLOP
            # sparse weight gradient: one 27-tap patch per (output channel, pooled window, input channel)
            f_wg = 2 * batch * 16 * int(np.prod(od)) * cpg * 27
            row = {"forward_ms": t_inf, "train_forward_ms": t_trn, "wgrad_ms": t_wg,
                   "forward_effective_tflops": direct / t_inf / 1e9, "wgrad_effective_tflops": direct / t_wg / 1e9,
                   "wgrad_valu_flop": f_wg, "wgrad_valu_tflops": f_wg / t_wg / 1e9,
                   "wgrad_valu_frac": f_wg / (t_wg * 1e-3) / F32_MFMA_PEAK}
            if n_fwd > 0:
                row.update({"forward_mfma_insts": n_fwd, "forward_executed_tflops": f_fwd / t_inf / 1e9,
                            "forward_frac": f_fwd / (t_inf * 1e-3) / F32_MFMA_PEAK,
                            "train_forward_frac": f_fwd / (t_trn * 1e-3) / F32_MFMA_PEAK})
            t_dg, f_dg = 0.0, 0
            if k > 0:
                dx = torch.empty_like(acts[k])
                t_dg = timed(lambda: _lib.check(L.rt_conv_relu_pool_dgrad(
                    ctypes.byref(layer), batch, w.data_ptr(), grads[k].data_ptr(), ams[k].data_ptr(),
                    dx.data_ptr(), st), "dgrad"))
                n_dg = int(L.rt_conv_mfma_count(ctypes.byref(layer), batch, 1))
                f_dg = n_dg * MFMA_F32_FLOP
                row.update({"dgrad_ms": t_dg, "dgrad_effective_tflops": direct / t_dg / 1e9})
                if n_dg > 0:
                    row.update({"dgrad_mfma_insts": n_dg, "dgrad_executed_tflops": f_dg / t_dg / 1e9,
                                "dgrad_frac": f_dg / (t_dg * 1e-3) / F32_MFMA_PEAK})
            stages[names[k]] = row
            tot["fwd_ms"] += t_inf
            tot["train_ms"] += t_trn + t_wg + t_dg
            tot["fwd_exec"] += f_fwd
            tot["train_mfma"] += f_fwd + f_dg
            tot["train_valu"] += f_wg
            tot["fwd_eff"] += direct
            tot["train_eff"] += 2 * direct + (direct if k > 0 else 0)
            # useful Winograd work: 64 products per 2x2x2 window and channel pair against
            # the direct form's 8 x 27 = 216 (no zero-padded rows or channel lanes)
            tot["train_useful"] += direct * WINO_USEFUL * (2 if k > 0 else 1) + f_wg
        return stages, tot, [a for a in acts[1:]]

    stages, tot, y32 = run_stages("f32")
    y32 = [t.clone() for t in y32]
    # PMC per stage kernel (committed run of the same kernels at this batch)
    if pmc is not None:
        # kernel-name prefixes (the training forward, whose argmax bytes the PMC driver requests)
        kern = {"conv1": ("k_conv_wino<4,16,", None), "conv2": ("k_conv_wino<8,8,", "k_dgrad_wino<8,"),
                "conv3": ("k_conv_wino<4,4,", "k_dgrad_wino<4,")}
        for nm, (kf, kd) in kern.items():
            for key, prefix, count_key in (("forward", kf, "forward_mfma_insts"), ("dgrad", kd, "dgrad_mfma_insts")):
                hits = [k for k in pmc["kernels"] if prefix and k.startswith(prefix)
                        and (key == "dgrad" or k.endswith(",true>"))]
                if not hits:
                    continue
                kname = hits[0]
                v = pmc["kernels"][kname]
                stages[nm][f"{key}_pmc"] = {
                    "kernel": kname, "mfma_busy": v.get("mfma_busy_frac"), "clock_GHz": v.get("clock_GHz"),
                    "valu_per_mfma": v.get("valu_per_mfma"), "kernel_ms": v.get("kernel_ms"),
                    "SQ_INSTS_MFMA": v.get("SQ_INSTS_MFMA"),
                    "count_matches_planner": int(v.get("SQ_INSTS_MFMA", -1)) == stages[nm].get(count_key),
                    "busy_x_clock_over_2.4GHz": (v["mfma_busy_frac"] * v["clock_GHz"] / 2.4
                                                 if v.get("mfma_busy_frac") is not None and v.get("clock_GHz") else None)}
    # bf16x3 forward products (direct ring kernels): time per stage, outputs vs f32
    st_bf, tot_bf, _ = run_stages("bf16x3")
    dmax = {}
    fe.set_conv_precision("bf16x3")
    for k, (layer, od) in enumerate(fe._plan()):
        w, bb = convs[k].weight.detach().contiguous(), convs[k].bias.detach().contiguous()
        yb = torch.empty_like(y32[k])
        _lib.check(L.rt_conv_relu_pool_fwd(ctypes.byref(layer), batch, (obs if k == 0 else y32[k - 1]).data_ptr(),
                                           None, w.data_ptr(), bb.data_ptr(), yb.data_ptr(), None, st), "fwd")
        torch.cuda.synchronize()
        dmax[names[k]] = float((yb - y32[k]).abs().max())
    fe.set_conv_precision("f32")
    bf = {"stages": {k: {kk: vv for kk, vv in v.items() if kk.endswith("_ms")} for k, v in st_bf.items()},
          "forward_ms": tot_bf["fwd_ms"], "train_pass_ms": tot_bf["train_ms"], "max_abs_diff_vs_f32": dmax,
          "forward_effective_tflops": tot_bf["fwd_eff"] / tot_bf["fwd_ms"] / 1e9,
          "train_pass_effective_tflops": tot_bf["train_eff"] / tot_bf["train_ms"] / 1e9,
          "note": "forward products in bf16x3 (hi*hi + hi*lo + lo*hi, f32 accumulate) on the direct ring kernels "
                  "(conv1, the grouped stages' forward and data gradient); weight gradients f32; "
                  "effective = direct-conv FLOP / time (not a utilisation)"}
    fwd_frac = tot["fwd_exec"] / (tot["fwd_ms"] * 1e-3) / F32_MFMA_PEAK
    fwd_useful = tot["fwd_eff"] * WINO_USEFUL
    exec_train = tot["train_mfma"] + tot["train_valu"]
    return {"bound": "mfma", "workload": f"C3D extractor stages, {batch} observations at {grid[0]}^3 "
                                         "(BASELINE configs[3] rollout step), f32",
            "peak": F32_MFMA_PEAK / 1e12, "unit": "TFLOP/s",
            "forward": {"ms": tot["fwd_ms"], "executed_flop": tot["fwd_exec"],
                        "achieved": tot["fwd_exec"] / tot["fwd_ms"] / 1e9, "frac": fwd_frac, "executed_frac": fwd_frac,
                        "useful_flop": fwd_useful, "useful_frac": fwd_useful / (tot["fwd_ms"] * 1e-3) / F32_MFMA_PEAK,
                        "effective_flop": tot["fwd_eff"],
                        "effective_tflops": tot["fwd_eff"] / tot["fwd_ms"] / 1e9,
                        "work": "Winograd MFMA wave-instructions x 2,048 FLOP (rt_conv_mfma_count = SQ_INSTS_MFMA)"},
            "train_pass": {"ms": tot["train_ms"], "executed_flop": exec_train,
                           "executed_mfma_flop": tot["train_mfma"], "executed_valu_flop": tot["train_valu"],
                           "achieved": exec_train / tot["train_ms"] / 1e9,
                           "frac": exec_train / (tot["train_ms"] * 1e-3) / F32_MFMA_PEAK,
                           "executed_frac": exec_train / (tot["train_ms"] * 1e-3) / F32_MFMA_PEAK,
                           "useful_flop": tot["train_useful"],
                           "useful_frac": tot["train_useful"] / (tot["train_ms"] * 1e-3) / F32_MFMA_PEAK,
                           "effective_flop": tot["train_eff"],
                           "effective_tflops": tot["train_eff"] / tot["train_ms"] / 1e9,
                           "work": "MFMA: training forward + grouped data gradients (Winograd); VALU: the sparse "
                                   "weight gradients (one 27-tap argmax patch per channel pair and pooled window)"},
            "stages": stages, "bf16x3": bf,
            "pmc_source": pmc["source"] if pmc else None,
            "frac_note": "frac = executed_frac: the MFMA wave-instructions the kernels issue (zero-padded rows and "
                         "channel lanes included, since round 5); useful_frac: the Winograd products the "
                         "convolution needs (direct FLOP x 64/216) plus the sparse weight gradients' FMAs",
            "timing": "HIP events on the kernels' stream, mean of 5 back-to-back launches"}


def needs_spawn(gpus: int, environ) -> bool:
    """--gpus N > 1 outside a torch.distributed.run rank (no WORLD_SIZE)."""
    return gpus > 1 and "WORLD_SIZE" not in environ


def launcher_cmd(gpus: int, port: int, argv) -> list:
    """The single-node launcher of the driver's own N-GPU command line."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(REPO, "bench.py"), *argv]


def spawn_ranks(gpus: int, argv) -> int:
    """Run `gpus` ranks of this same command under torch.distributed.run as a
    child process (one rank per GPU; with --rehearse-same-device all on cuda:0
    over gloo) and return its exit status.  Rank 0 prints the JSON line.  No
    exec: the child is a new process, this one has not initialised the GPU."""
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.call(launcher_cmd(gpus, port, argv), env=env)


def collective_update_ms(tr, dist, dev) -> float:
    """ms per minibatch of the trainer's data-parallel update path over a
    world-1 RCCL group (the update the 8-GPU run makes, minus the xGMI
    traffic): rt_ppo_update_dp with the library's own communicator."""
    import socket

    import torch

    own = not dist.is_initialized()
    if own:
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    keep = tr.collective
    tr.collective = True
    try:
        tr.update()  # warm: the communicator, RCCL's first launch
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = tr.update()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert tr._dp_comm, "the update did not take the library's RCCL path"
    finally:
        tr.collective = keep
        if own:
            dist.destroy_process_group()
    return 1000 * dt / n


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if needs_spawn(a.gpus, os.environ):
        # started directly with --gpus N > 1: the N ranks run as children of a
        # torch.distributed.run started HERE, before this process touches the GPU
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    if a.gpus != world:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)

    import torch
    import torch.distributed as dist

    import _rtpkg  # noqa: F401
    from ppo_radiotherapy_amd import _lib, assets
    from ppo_radiotherapy_amd.networks import PPO, PPO_3DCNN
    from ppo_radiotherapy_amd.ppo import PPOTrainer, broadcast_parameters
    from ppo_radiotherapy_amd.vec_env import RadiotherapyVecEnv

    if a.rehearse_same_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if a.rehearse_same_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    grid = (a.grid,) * 3
    lib = assets.synthetic_library(grid, 1000, 0)
    env = RadiotherapyVecEnv(a.envs, visionless=not a.vision, library=lib, device=dev, seed=a.seed + rank,
                             env_id_base=rank * a.envs, step_mode=a.step_mode)
    if not a.vision and a.step_mode == "dense":
        env.set_rollout_groups(a.rollout_groups)
    torch.manual_seed(a.seed)
    if a.vision:  # conv1's arithmetic: the trainer sets it from cfg.conv_precision
        agent = PPO_3DCNN((4, *grid), (6,), 64).to(dev)
    else:
        agent = PPO((9,), (6,), 64).to(dev)
    broadcast_parameters(agent)
    gen = torch.Generator(device=dev)
    gen.manual_seed(a.seed * 1000 + rank)
    cfg = trainer_cfg(a)
    tr = PPOTrainer(cfg, env, agent, dev, rank, world, gen)
    tr.reset()
    T = tr.T
    if not a.vision and not a.env_only:
        # every timed window below runs on staggered episode phases, as a long
        # run does (autoresets and their dose-row zeroing inside the window)
        stagger_phases(tr, env, dev)

    # ---------------- warmup: W untimed rollout steps around one untimed
    # update (its kernels warm too), so the timed pass follows rollout steps
    # as it does in a long run
    if a.update_minibatches:
        tr.max_minibatches = a.update_minibatches
    w1 = a.warmup // 2 if not a.no_update and not a.env_only else a.warmup
    run_steps(tr, w1)
    if not a.no_update and not a.env_only:
        tr.compute_gae()
        tr.update()
        run_steps(tr, a.warmup - w1)
    torch.cuda.synchronize()

    # ---------------- timed rollout (or env-only)
    K = a.steps
    actions = torch.rand((a.envs, 6), device=dev, generator=gen) * 2 - 1

    def rollout_pass():
        if a.env_only:
            for i in range(K):
                env.step(actions, info_out=tr.infos[i % T])
        else:
            run_steps(tr, K)

    # `value`: the uninstrumented pass (the library's timing events, recorded
    # between kernels, cost ~4 % of the pipelined step)
    window_marker(dev)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rollout_pass()
    torch.cuda.synchronize()
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0)
    # kernel times: an identical pass with HIP events around k_beam / k_dense /
    # k_finish (one slot per env group and step; one per persistent launch)
    env.kernel_timing(2 * K)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rollout_pass()
    torch.cuda.synchronize()
    barrier()
    dt_timed = max_over_ranks(time.perf_counter() - t0)
    kms, kcalls = env.kernel_timing_read()
    kms = {k: v * kcalls / K for k, v in kms.items()}  # per step (a persistent rollout launch spans many)
    env.kernel_timing(0)
    # the march's dose lines on the beams of this pass's last step (roofline.march)
    mlines = march_lines(env) if (not a.vision and not a.env_only and a.step_mode == "dense") else None
    kms = {k: max_over_ranks(v) for k, v in kms.items()}
    env_ms = sum(kms.values())  # k_beam start -> k_finish end, per step
    total_envs = a.envs * world
    steps_per_s = total_envs * K / dt

    # ---------------- k_dense alone on the chip (one env group), same workload
    iso = None
    if not a.vision and not a.env_only and a.step_mode == "dense" and a.rollout_groups > 1:
        env.set_rollout_groups(1)
        run_steps(tr, 4)
        env.kernel_timing(2 * K)
        run_steps(tr, K)
        torch.cuda.synchronize()
        ki, ci = env.kernel_timing_read()
        env.kernel_timing(0)
        env.set_rollout_groups(a.rollout_groups)
        iso = {k: max_over_ranks(v) for k, v in ki.items()}  # per launch (one per step)

    # ---------------- steady state: >= 101 steps, staggered episode phases
    steady = None
    if not a.env_only and not a.vision and not a.no_steady:
        steady = steady_state(tr, env, dev, barrier, max_over_ranks, total_envs)
        steady["vs_value"] = steady["env_steps_per_s"] / steps_per_s

    # ---------------- PPO update phase + one full iteration
    upd = {}
    if not a.no_update and not a.env_only:
        tr.compute_gae()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        n_upd = tr.update()
        torch.cuda.synchronize()
        barrier()
        du = max_over_ranks(time.perf_counter() - t0)
        barrier()
        t0 = time.perf_counter()
        tr.rollout()
        tr.compute_gae()
        full_mb = int(cfg.update_epochs) * int(cfg.num_minibatches)
        capped = bool(tr.max_minibatches) and tr.max_minibatches < full_mb
        if not capped:
            tr.update()
        torch.cuda.synchronize()
        barrier()
        di = max_over_ranks(time.perf_counter() - t0)
        if capped:  # vision: rollout + GAE measured, the update's full_mb steps at the timed per-step cost
            di += full_mb * du / n_upd
        if world > 1:  # the per-minibatch flat-gradient all-reduce alone (included in the update above)
            barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(n_upd):
                dist.all_reduce(tr.flat_grad)
            torch.cuda.synchronize()
            dar = max_over_ranks(time.perf_counter() - t0)
        upd = {"ppo_updates_per_s": n_upd / du, "ppo_update_ms": 1000 * du / n_upd,
               "minibatch_size_per_gpu": tr.minibatch_size, "update_minibatches_timed": n_upd,
               "train_env_steps_per_s": total_envs * T / di, "train_iteration_s": di,
               "train_iteration": (f"rollout + GAE measured, {full_mb} minibatch steps at the timed "
                                   f"{1000 * du / n_upd:.3f} ms each" if capped else "measured whole")}
        if world > 1:
            upd["update_allreduce_ms"] = 1000 * dar / n_upd
            upd["update_allreduce_bytes"] = 4 * tr.flat_grad.numel()
        if tr.fused_update:
            # MLP forward + backward of both heads: 28,224 MACs per sample
            # (DESIGN.md §3); whole minibatch step (grad + reduce + clip/Adam + epoch overheads)
            fl = 2 * UPDATE_MACS_PER_SAMPLE * tr.minibatch_size
            upd["update_precision"] = a.update_precision
            upd["update_mfma"] = {"bound": "mfma", "flop_per_minibatch": fl,
                                  "achieved": fl / (du / n_upd) / 1e12, "peak": F32_MFMA_PEAK / 1e12,
                                  "unit": "TFLOP/s", "frac": fl / (du / n_upd) / F32_MFMA_PEAK,
                                  "peak_note": "f32 MFMA peak (the f32-equivalent rate, also for bf16x3)"}
            # the other precision of the 64x64 layer products, same update (parameters move on)
            other = "bf16x3" if a.update_precision == "f32" else "f32"
            keep = tr._update_prec
            tr._update_prec = _lib.PPO_PREC[other]
            tr.update()  # warm (first launch of the other kernel instantiation)
            torch.cuda.synchronize()
            barrier()
            t0 = time.perf_counter()
            n2 = tr.update()
            torch.cuda.synchronize()
            barrier()
            d2 = max_over_ranks(time.perf_counter() - t0)
            tr._update_prec = keep
            upd[f"ppo_update_ms_{other}"] = 1000 * d2 / n2
            # the data-parallel update path (rt_ppo_update_dp: grad, RCCL all-reduce
            # of the flat gradient, clip + Adam per minibatch, one library call):
            # at world > 1 that is what ppo_update_ms timed; at world 1 it runs
            # through a world-1 RCCL group (the all-reduce an identity)
            if world > 1:
                upd["ppo_update_ms_collective_path"] = upd["ppo_update_ms"]
            elif not a.rehearse_same_device:
                upd["ppo_update_ms_collective_path"] = collective_update_ms(tr, dist, dev)
            if "ppo_update_ms_collective_path" in upd:
                upd["collective_path_vs_fused"] = upd["ppo_update_ms_collective_path"] / upd["ppo_update_ms"]

    # ---------------- roofline of the dominant kernel, k_dense
    V = int(np.prod(grid))
    Vl = int(np.count_nonzero(lib.lungs))
    # k_dense reads each env's lung segment (the first Vl floats of its
    # lung-first dose row) once: the voxels the lung reductions sum over
    bytes_launch = a.envs * 4 * Vl
    bytes_model = f"4 B x {Vl} lung voxels x envs (lung-first dose rows; {Vl / V:.3f} of the volume)"
    if a.vision:  # k_dense_vis: read the C-order dose row, write the lungs and dose channels
        bytes_launch = a.envs * 20 * V
        bytes_model = ("20 B x V x envs (k_dense_vis: dose read, the four observation channels written -- "
                       "lungs and dose, tumour and beam-view zeroed for k_finish's scatter)")
    launches = max(kcalls, 1) / K  # launches per step (2: pipelined env groups)
    dense_ms = kms["k_dense"]  # per step: the launches of all env groups
    kernel_name = "k_dense"
    if launches > 1.5:  # pipelined: k_dense over half the envs per launch (tools/r06/gpu_final.sh)
        traffic = load_pmc(grid, a.envs // 2, pipelined=True)
    else:  # whole-handle grid launches (tools/archive/gpu_dense_pmc.sh, bench.py --env-only)
        traffic = load_pmc(grid, a.envs)
    achieved = bytes_launch / (dense_ms * 1e-3)  # = per-launch bytes / per-launch duration (per step)
    traffic_steady = traffic_src = None
    if isinstance(traffic, dict):
        traffic, traffic_steady, traffic_src = traffic["value_window"], traffic["steady_window"], traffic["source"]
    roof = {"bound": "hbm", "kernel": kernel_name, "achieved": achieved / 1e9,
            "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
            "traffic": traffic, "traffic_steady_window": traffic_steady, "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": bytes_launch / launches,
            "kernel_ms": dense_ms / launches, "launches_per_step": launches, "k_dense_ms_per_step": dense_ms,
            "kernel_calls_timed": kcalls, "kernel_ms_all": kms, "env_step_ms": env_ms,
            "bytes_model": bytes_model,
            "env_step_frac_of_hbm": bytes_launch / (env_ms * 1e-3) / HBM_PEAK,
            "survey_model_bytes_per_env_step": 8 * V,
            "survey_model_frac": a.envs * 8 * V / (env_ms * 1e-3) / HBM_PEAK}
    if kernel_name == "k_dense" and launches > 1.5 and a.envs == 4096 and a.grid == 64:
        # the same kernel in the committed rocprofv3 stats of this command: the
        # HIP-event interval above also spans the dispatch after the turn
        # hand-off (~9 us), rocprofv3 times the kernel alone
        rp = load_rocprof(DENSE_KERNEL, a.rocprof_stats)
        if rp is not None:
            rp["achieved"] = bytes_launch / launches / (rp["avg_ms"] * 1e-3) / 1e9
            rp["frac"] = rp["achieved"] * 1e9 / HBM_PEAK
            roof["rocprof"] = rp
    if iso is not None:
        iso_ach = a.envs * 4 * Vl / (iso["k_dense"] * 1e-3)
        roof["isolated"] = {"kernel_ms": iso["k_dense"], "achieved": iso_ach / 1e9, "frac": iso_ach / HBM_PEAK,
                            "kernel_ms_all": iso, "note": "k_dense over all envs, one launch per step, "
                                                          "nothing co-running (one-group pass)"}
    roof["step_frac_of_hbm"] = a.envs * 4 * Vl / (dt / K) / HBM_PEAK if not a.vision else None
    roof["timed_pass_ms_per_step"] = 1000 * dt_timed / K  # the instrumented pass (kernel times above)
    rmw_ceil = None
    if rank == 0 and not a.env_only:
        from ppo_radiotherapy_amd import _lib

        cel = stream_ceilings(dev, _lib.load())
        roof["measured_read_ceiling_GBps"] = cel["read"] / 1e9
        roof["measured_copy_ceiling_GBps"] = cel["copy"] / 1e9
        roof["measured_ceiling_probe"] = ("rt_probe_stream over 4 GiB: non-temporal 16-B loads, 8 in flight per lane "
                                          "(read: reduced; copy: + plain 16-B stores, read+write bytes)")
        roof["frac_of_measured_ceiling"] = achieved / cel["read"]
        rmw_ceil = random_rmw_ceiling(dev, _lib.load(), a.envs * V)
        if mlines is not None:
            # the beam march (draw_line.py:49-100 + environment.py:107-110) runs in
            # k_step_policy (policy + pose + march, one wave per env): its random
            # 128-B line read-modify-writes against the measured random-RMW rate
            kp_ms = kms["k_beam"]  # per step: the k_step_policy launches of all env groups
            rate = a.envs * mlines / (kp_ms * 1e-3)
            roof["march"] = {
                "kernel": "k_step_policy", "bound": "random-line RMW (latency/transactions)",
                "model": "per env-step: the distinct 128-B dose lines the beam's splats touch, each read and written "
                         "(2 x 128 B); the policy MLP and the f64 pose update run in the same kernel",
                "lines_per_env_step": mlines, "kernel_ms_per_step": kp_ms, "line_rmw_per_s": rate,
                "achieved_GBps": rate * 256 / 1e9, "frac_of_hbm_peak": rate * 256 / HBM_PEAK,
                "probe_line_rmw_per_s": rmw_ceil, "frac": rate / rmw_ceil,
                "timing": "library HIP events around k_step_policy on the env-group streams, instrumented pass"}
            rpm = load_rocprof("k_step_policy", a.rocprof_stats)
            if rpm is not None and launches > 1.5:
                rpm["line_rmw_per_s"] = a.envs / launches * mlines / (rpm["avg_ms"] * 1e-3)
                rpm["frac"] = rpm["line_rmw_per_s"] / rmw_ceil
                roof["march"]["rocprof"] = rpm

    # ---------------- the other step formulation, same workload (policy in the loop)
    other = None
    if not a.vision and not a.env_only:
        other_mode = "incremental" if a.step_mode == "dense" else "dense"
        env.close()
        env2 = RadiotherapyVecEnv(a.envs, visionless=True, library=lib, device=dev, seed=a.seed + rank,
                                  env_id_base=rank * a.envs, step_mode=other_mode)
        tr.env = env2
        tr.reset()
        run_steps(tr, a.warmup)
        env2.kernel_timing(2 * K)
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        run_steps(tr, K)
        torch.cuda.synchronize()
        barrier()
        d2 = max_over_ranks(time.perf_counter() - t0)
        k2, c2 = env2.kernel_timing_read()
        k2 = {k: v * c2 / K for k, v in k2.items()}
        env2.kernel_timing(0)
        env_ms2 = sum(max_over_ranks(v) for v in k2.values())
        other = {"step_mode": other_mode, "env_steps_per_s": total_envs * K / d2, "ms_per_step": 1000 * d2 / K,
                 "env_kernels_ms": k2, "env_only_kernel_steps_per_s": total_envs / (env_ms2 * 1e-3)}
        if other_mode == "incremental" and rank == 0:
            from ppo_radiotherapy_amd import _lib

            bl, tl = incremental_transactions(env2, lib)
            ceil = rmw_ceil
            sps = a.envs * K / d2  # this rank's env steps/s
            ach_lines = sps * bl
            ach_bytes = sps * 128 * (2 * bl + tl)
            other["roofline"] = {
                "bound": "random-line RMW (latency/transactions)", "kernel": "k_rollout_policy",
                "model": "per env-step: the march read-modify-writes the distinct 128-B dose lines its splats "
                         "touch (2 x 128 B each), the finish reads the tumour's lines (128 B each)",
                "beam_lines_per_step": bl, "tumour_lines_per_step": tl,
                "bytes_per_env_step": 128 * (2 * bl + tl), "achieved_GBps": ach_bytes / 1e9,
                "frac_of_hbm_peak": ach_bytes / HBM_PEAK,
                "line_rmw_per_s": ach_lines, "probe_line_rmw_per_s": ceil,
                "probe": "rt_probe_random_rmw: 2^18 lanes x 64 random lines (one float per lane and line, 4 in "
                         "flight) over a buffer the size of the dose array",
                "frac": ach_lines / ceil}
        if not a.no_update:
            barrier()
            t0 = time.perf_counter()
            tr.rollout()
            tr.compute_gae()
            tr.update()
            torch.cuda.synchronize()
            barrier()
            di2 = max_over_ranks(time.perf_counter() - t0)
            other.update({"train_env_steps_per_s": total_envs * T / di2, "train_iteration_s": di2})
        env = env2
    if a.vision:
        roof["note"] = "vision: the env kernel above is k_dense_vis; the policy is C3D on f32 MFMA (c3d_mfma)"
        # C3D forward of one rollout step (512 envs), timed separately on the
        # same agent: executed Winograd MFMA work (rt_conv_mfma_count) and the
        # direct-conv FLOPs as `effective`
        fe = agent.features_extractor
        xo = env.obs
        with torch.no_grad():
            fe(xo)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(4):
                fe(xo)
            torch.cuda.synchronize()
        dfe = (time.perf_counter() - t0) / 4
        import ctypes

        L = _lib.load()
        n_mfma = sum(int(L.rt_conv_mfma_count(ctypes.byref(layer), a.envs, 0)) for layer, _ in fe._plan())
        fx = n_mfma * MFMA_F32_FLOP
        fl = c3d_fwd_flop(grid) * a.envs
        roof["c3d_mfma"] = {"bound": "mfma", "forward_ms": dfe * 1e3, "executed_flop": fx,
                            "achieved": fx / dfe / 1e12, "peak": F32_MFMA_PEAK / 1e12, "unit": "TFLOP/s",
                            "frac": fx / dfe / F32_MFMA_PEAK, "effective_flop": fl,
                            "effective_tflops": fl / dfe / 1e12,
                            "conv_precision": fe.conv_precision,
                            "note": "executed = Winograd MFMA wave-instructions x 2,048 FLOP (0 under bf16x3: direct "
                                    "kernels); effective = direct-conv FLOPs / time"}
    out = {"metric": METRIC, "value": steps_per_s, "unit": "env steps/s", "n_gpus": world, "steps": K,
           "warmup": a.warmup, "ms_per_step": 1000 * dt / K, "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f32", "data": "synthetic",
           "config": {"workload": (f"vision C3D, {a.envs} envs/GPU, {a.grid}^3 voxel grid (BASELINE "
                                   + ("configs[3])" if a.grid == 64 else "configs[4], per-GPU share)")
                                   if a.vision else
                                   f"visionless MLP, {a.envs} envs/GPU, {a.grid}^3 voxel grid "
                                   f"(BASELINE configs[{1 if world == 1 else 2}])") + (" env-only" if a.env_only else ""),
                      "envs_per_gpu": a.envs, "global_envs": total_envs, "grid": list(grid),
                      "num_steps": T, "num_minibatches": a.num_minibatches, "update_epochs": a.update_epochs,
                      "parallelism": f"dp{world}",
                      "episode_phases": ("lockstep (all envs reset together)" if (a.vision or a.env_only) else
                                         "staggered: env e's episode clock offset by e mod 100, ~1 % of the envs "
                                         "autoreset (and zero their dose rows) in every timed step")},
           "env_only_kernel_steps_per_s": total_envs / (env_ms * 1e-3)}
    out.update(upd)
    if steady is not None:
        out["steady_state"] = steady
    out["step_mode"] = a.step_mode
    if a.vision:
        out["conv_precision"] = a.conv_precision
        if a.conv_precision != "f32":
            out["dtype"] = "f32 (conv1 forward bf16x3)"
    out["rollout_groups"] = a.rollout_groups if a.step_mode == "dense" and not a.vision else 1
    if other is not None:
        out["other_step_mode"] = other
    out["roofline"] = roof
    if rank == 0 and not a.no_c3d and not a.env_only:
        out["c3d_mfma"] = c3d_roofline(dev, lib, grid)
    if rank == 0 and world == 1 and not a.no_cpu:
        out["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
