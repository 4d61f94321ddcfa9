/*
 * rtenv.h -- C-ABI of librtenv.so, the MI355X-native vectorised radiotherapy
 * environment (HIP kernels for gfx950).
 *
 * Drop-in boundary for the reference's hot path (rmaguado/ppo-radiotherapy):
 *
 *   reference                                   | this ABI
 *   --------------------------------------------+---------------------------------
 *   RadiotherapyEnv.__init__  environment.py:34 | rt_env_create (N envs at once)
 *   RadiotherapyEnv.reset     environment.py:77 | rt_env_reset
 *   RadiotherapyEnv.step      environment.py:193| rt_env_step (+ gymnasium 1.0
 *     + SyncVectorEnv.step / NEXT_STEP autoreset|   SyncVectorEnv autoreset and
 *     + RecordEpisodeStatistics (train.py:32-39)|   RecordEpisodeStatistics)
 *   beam_voxels               draw_line.py:4    | rt_debug_beam (parity hook)
 *   apply_rotation/translation transforms.py:7,62| rt_debug_pose (parity hook)
 *   GAE loop                  train.py:163-181  | rt_gae
 *   agent.get_action_and_value train.py:143-149 | rt_policy_sample (visionless agent)
 *   rollout step (policy + env) train.py:143-158 | rt_env_step_policy (fused)
 *   rollout loop              train.py:138-161  | rt_env_rollout_policy (persistent)
 *   PPO minibatch step        train.py:197-246  | rt_ppo_grad + rt_adam_step / rt_ppo_update
 *   FeaturesExtractor3D.cnn   networks.py:8-45  | rt_conv_relu_pool_fwd (+ backward kernels)
 *
 * Conventions
 *  - Plain pointers and sizes only; `*_d` arguments are DEVICE pointers
 *    (caller-owned, e.g. torch tensors), host pointers are named `*_h`.
 *  - All device work is enqueued on the caller's stream (a hipStream_t passed
 *    as `void*`; NULL = the legacy default stream); no call synchronises the
 *    device, allocates, or frees after rt_env_create -> the step and reset
 *    calls are hipGraph-capturable.
 *  - Return 0 on success or a negative RT_E* code; never abort.  The message of
 *    the last failure on the calling thread is in rt_last_error().
 *  - One host thread per handle (a handle is not thread-safe); handles are
 *    independent, typically one per GPU / process.
 */
#ifndef RTENV_H
#define RTENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTENV_ABI_VERSION 5  /* 2: rt_env_config.struct_size (first member); 3: rt_adam_step grad_div,
                                rt_env_set_dense_handoff removed; 4: arithmetic per call
                                (rt_ppo_hparams.precision, rt_conv_layer.precision) instead of the
                                process-wide rt_ppo_/rt_conv_set_precision; 5: RT_ROLLOUT_FLOW and
                                the dense persistent rollout (groups 0 on dense handles) removed,
                                rt_ppo_status, rt_host_lung_sum and the RCCL
                                data-parallel update (rt_dp_*, rt_ppo_update_dp) added, dense-mode
                                doses.lung in numpy's exact order */

enum {
    RT_OK = 0,
    RT_EINVAL = -1,   /* bad argument / config */
    RT_ENOMEM = -2,   /* device or host allocation failed */
    RT_EDEVICE = -3,  /* HIP runtime error (no device, bad device id, ...) */
    RT_ELAUNCH = -4,  /* kernel launch failed */
    RT_ELIMIT = -5    /* a compile-time capacity was exceeded (grid, tumour size) */
};

/* info[N][RT_INFO_W] float layout written by rt_env_step (environment.py:222-241
 * plus the RecordEpisodeStatistics / autoreset fields of gymnasium 1.0). */
enum {
    RT_INFO_TOTAL = 0,        /* reward_components.total                       */
    RT_INFO_TUMOUR = 1,       /* reward_components.tumour                      */
    RT_INFO_LUNG = 2,         /* reward_components.lung                        */
    RT_INFO_DISTANCE = 3,     /* reward_components.distance_to_tumour          */
    RT_INFO_DOSE_TUMOUR = 4,  /* doses.tumour  = sum(dose * tumour)            */
    RT_INFO_DOSE_LUNG = 5,    /* doses.lung    = sum(dose * lungs)             */
    RT_INFO_OVERSHOOT_T = 6,  /* overshoot.translation[3]  (6,7,8)             */
    RT_INFO_OVERSHOOT_R = 9,  /* overshoot.rotation                            */
    RT_INFO_POS = 10,         /* beam_position.translation[3] (10,11,12)       */
    RT_INFO_DIR = 13,         /* beam_position.rotation[3]    (13,14,15)       */
    RT_INFO_STEPPED = 16,     /* 1: env stepped; 0: this call was its autoreset */
    RT_INFO_EP_DONE = 17,     /* 1: an episode finished on this step ("_r")    */
    RT_INFO_EP_RETURN = 18,   /* episode.r (sum of step rewards)               */
    RT_INFO_EP_LENGTH = 19,   /* episode.l                                     */
    RT_INFO_W = 20
};

typedef struct rt_env rt_env; /* opaque */

/* rt_env_config.step_mode */
enum {
    RT_STEP_DENSE = 0,       /* the reference's formulation: every step re-reduces each env's
                                whole dose volume (k_dense, HBM-bound) */
    RT_STEP_INCREMENTAL = 1  /* visionless only: the lung over-threshold count and lung dose sum
                                are updated on the voxels the beam touches;
                                rewards and termination identical, doses.lung an f64 running
                                sum rounded once (the dense mode's is numpy's f32 order) */
};

typedef struct {
    /* size handshake: the caller sets struct_size = sizeof(rt_env_config) BEFORE
     * rt_env_config_default / rt_env_create; both return RT_EINVAL without
     * touching the struct when it differs, so a binding with a stale (shorter or
     * longer) declaration is rejected instead of overrun. */
    uint32_t struct_size;
    /* geometry */
    int32_t grid[3];          /* D, H, W (LUNG_SHAPE, environment.py:30) */
    int32_t num_envs;         /* envs owned by this handle */
    int32_t visionless;       /* 1: obs f32[9]; 0: obs f32[4,D,H,W] (environment.py:54-57) */
    /* constants (environment.py:16-26); rt_env_config_default fills the reference values */
    int32_t max_time_steps;   /* 100 */
    float beam_dose;          /* 0.1 */
    float lung_dose_threshold;   /* 0.2 */
    float tumour_dose_threshold; /* 0.9 */
    double min_angle_z;       /* pi/4 */
    double movement_speed;    /* 0.2 */
    float rotation_speed;     /* 0.5 (applied in f32, environment.py:141) */
    double lung_dose_reward;  /* -1.0 */
    float tumour_dose_reward; /* 10.0 (applied in f32, environment.py:169) */
    double distance_reward;   /* -1.0 */
    /* assets (host memory; copied to HBM by rt_env_create) */
    const uint8_t* lungs_h;          /* u8[D*H*W] in {0,1}, C order */
    int32_t n_tumours;               /* library size K */
    const int32_t* tumour_voxels_h;  /* concat of sorted flat C-order indices */
    const int64_t* tumour_offsets_h; /* [K+1] */
    /* RNG for tumour sampling on autoreset (np.random.choice, environment.py:90) */
    uint64_t seed;
    int64_t env_id_base;      /* global id of env 0 of this handle (rank * N) */
    int32_t step_mode;        /* RT_STEP_DENSE (default) or RT_STEP_INCREMENTAL */
} rt_env_config;

/* Fill the reference's constants (environment.py:16-30); cfg->struct_size must
 * already hold sizeof(rt_env_config) (kept; everything else is overwritten). */
int rt_env_config_default(rt_env_config* cfg);

int rt_env_create(const rt_env_config* cfg, int device, rt_env** out);
void rt_env_destroy(rt_env* env);

/* Reset the envs selected by mask_d (u8[N], NULL = all).  tumour_ids_d
 * (i32[N], NULL = sample) picks library tumours; a negative entry samples.
 * Writes obs for ALL envs (unselected envs report their current obs). */
int rt_env_reset(rt_env* env, const uint8_t* mask_d, const int32_t* tumour_ids_d, float* obs_d,
                 void* stream);

/* One vectorised step with gymnasium-1.0 NEXT_STEP autoreset: an env whose
 * previous step terminated ignores its action, resets, and returns the reset
 * obs with reward 0 and terminated 0 (info[RT_INFO_STEPPED] = 0).
 * actions_d f32[N,6]; obs_d f32[N,9] (visionless) or f32[N,4,D,H,W];
 * reward_d f32[N]; terminated_d u8[N]; info_d f32[N,RT_INFO_W] (may be NULL). */
int rt_env_step(rt_env* env, const float* actions_d, float* obs_d, float* reward_d,
                uint8_t* terminated_d, float* info_d, void* stream);

/* Tumours used by the NEXT autoreset of each env (i32[N]; negative = sample).
 * Parity mode: replays the reference's np.random.choice draws. */
int rt_env_set_next_tumours(rt_env* env, const int32_t* tumour_ids_d, void* stream);

/* Re-key the tumour-sampling stream (gymnasium reset(seed=...); replaces
 * SyncVectorEnv.reset(seed) -> RadiotherapyEnv.reset(seed), train.py:136,
 * environment.py:77): later Philox draws use key `seed` and every env's
 * episode counter restarts at 0 (ordered on `stream`), so the tumour sequence
 * depends only on (seed, global env id) -- not on the handle's history. */
int rt_env_reseed(rt_env* env, uint64_t seed, void* stream);

/* State access (device pointers into library-owned memory; valid until
 * rt_env_destroy).  dose is f32[N][dose_stride]; the first D*H*W floats of a
 * row hold the env's dose volume, in C order or -- dense-mode visionless
 * handles, whose k_dense streams only the lung voxels -- lung-first: voxel v
 * (C-order flat index) sits at row position rt_env_dose_index(env)[v]
 * (device i32[D*H*W]); rt_env_dose_index returns NULL for C-order rows. */
float* rt_env_dose(rt_env* env, int64_t* dose_stride);
const int32_t* rt_env_dose_index(rt_env* env);
int rt_env_get_state(rt_env* env, double* pose_d /* f64[N,6] pos,dir */, int32_t* t_d,
                     int32_t* tumour_d, void* stream);
int rt_env_set_pose(rt_env* env, const double* pose_d /* f64[N,6] */, void* stream);
/* Current tumour of each env (i32[N]; out-of-range entries leave it), without
 * a reset.  With rt_env_set_pose, a copy into rt_env_dose and rt_env_reset
 * with an all-zero mask, a handle re-renders the observation of any stored
 * (dose, pose, tumour) state -- the vision rollout's compact storage (SURVEY
 * §8 f-3). */
int rt_env_set_tumours(rt_env* env, const int32_t* tumour_d, void* stream);
/* Vision handles: the NEXT rt_env_reset re-emits the observation of each env
 * e < n_rows that the reset leaves unselected (mask 0) from row rows_d[e] of
 * a dose store (f32, C order, row stride store_stride >= the padded volume,
 * 16-B aligned) instead of from its own dose row, which stays as it was; the
 * reset clears the setting.  The re-render of stored states without copying
 * their doses into the handle first (the trainer's compact vision storage). */
int rt_env_set_render_source(rt_env* env, const float* dose_store_d, int64_t store_stride,
                             const int64_t* rows_d /* i64[n_rows] */, int32_t n_rows);
int rt_env_num_envs(const rt_env* env);

/* Live kernel timing.  rt_env_kernel_timing(env, K) creates HIP events for
 * the next K step launches (0 disables; not graph-capturable while on): each
 * step/reset call -- and each env group of each step of a dense-mode
 * rt_env_rollout_policy -- takes one slot and records events on its stream
 * around its three kernels (beam or policy+beam, k_dense, k_finish).
 * rt_env_kernel_timing_read waits for them and returns the summed
 * milliseconds of the three (ms_out[3]) over `steps` slots, then clears the
 * ring. */
int rt_env_kernel_timing(rt_env* env, int32_t capacity);
int rt_env_kernel_timing_read(rt_env* env, double* ms_out /* [3] */, int32_t* steps);

/* Parity hooks (same device code as the step kernels). */
/* beam_voxels for M poses: raw splats in march order, idx_d i32[M,cap],
 * w_d f32[M,cap], count_d i32[M] (-1 = ValueError: direction norm < eps). */
int rt_debug_beam(const int32_t grid[3], int32_t m, const double* pos_d, const double* dir_d,
                  int32_t cap, int32_t* idx_d, float* w_d, int32_t* count_d, void* stream);
/* map_translation/apply_translation/map_rotation/apply_rotation for M
 * (pos,dir,action) triples: out_d f64[M,10] = new pos[3], new dir[3],
 * overshoot_t[3], overshoot_r. */
int rt_debug_pose(const int32_t grid[3], int32_t m, const double* pos_d, const double* dir_d,
                  const float* action_d, double* out_d, void* stream);

/* The beam each env applied on its last step (draw_line.py:4-102 called
 * from environment.py:107-110 on the post-update pose): raw splats in march
 * order as rt_debug_beam -- idx_d i32[N,cap] C-order flat voxel indices,
 * w_d f32[N,cap] weights (a voxel can appear twice; the env adds both),
 * count_d i32[N] (0: the env's last call was its reset, no beam applied;
 * > cap: truncated).  Replaces reading `beam_voxels(...)` back in a debugger. */
int rt_env_beam_list(rt_env* env, int32_t cap, int32_t* idx_d, float* w_d, int32_t* count_d, void* stream);

/* Measurement hook (bench.py): `lanes` threads each read-modify-write
 * `lines_per_lane` pseudo-random 128-B lines of buf_d (one float per line,
 * 4 in flight) -- the access shape of the incremental step's march -- so the
 * caller can time the random-line RMW ceiling of the device. */
int rt_probe_random_rmw(float* buf_d, int64_t n_floats, int32_t lanes, int32_t lines_per_lane, uint64_t seed,
                        void* stream);

/* Measurement hook (bench.py): the HBM stream ceilings k_dense is priced
 * against -- `blocks` x 256 threads sweep src_d (n_floats, 16-B aligned) with
 * non-temporal 16-B loads, 8 in flight per lane.  mode 0 (READ): reduced to
 * 4 * blocks floats written to dst_d; mode 1 (COPY): stored to dst_d (plain
 * 16-B stores).  Time it with events on `stream`. */
int rt_probe_stream(const float* src_d, float* dst_d, int64_t n_floats, int32_t mode, int32_t blocks, void* stream);

/* Host-side evaluation of the correctly rounded sin/cos the pose kernel uses
 * for scipy's from_rotvec half angle (no device needed; parity hook). */
int rt_host_sincos(int32_t n, const double* x_h, double* sin_h, double* cos_h);

/* Host-side evaluation of the exact-order plan k_finish uses for
 * np.sum(dose * tumours) over a V-voxel volume whose nonzeros are vals_h at
 * the sorted flat indices idx_h (no device needed; parity hook). */
int rt_host_tumour_sum(int64_t V, int32_t n, const int32_t* idx_h, const float* vals_h, float* out_h);

/* Host-side evaluation of the plan k_dense + k_finish use for info doses.lung
 * = np.sum(dose * lungs) (environment.py:235) in numpy's exact order, on a
 * C-order f32 volume dose_h with the u8 mask lungs_h (no device needed;
 * parity hook). */
int rt_host_lung_sum(const int32_t grid[3], const uint8_t* lungs_h, const float* dose_h, float* out_h);

/* Fused rollout policy step of the visionless agent (networks.py PPO,
 * feature_dim 64): for every env, obs -> actor/critic MLPs -> Gaussian sample
 * (Philox; key seed, counter `counter`, env id env_id_base + e) -> action,
 * log_prob(action).sum, value; also copies obs and done (u8 -> f32; NULL = 0)
 * into the rollout storage slices.  params_d: the 13 f32 parameter tensors
 * in the order actor_mean.{0,2,4}.{weight,bias}, actor_logstd,
 * critic.{0,2,4}.{weight,bias}.  Replaces train.py:143-149 per step. */
int rt_policy_sample(const float* const* params_d, int32_t n_params_tensors, int32_t n_envs,
                     const float* obs_d, const uint8_t* done_d, float* obs_out_d, float* done_out_d,
                     float* act_out_d, float* logp_out_d, float* value_out_d, uint64_t seed,
                     uint64_t counter, int64_t env_id_base, void* stream);

/* Fused rollout step of the visionless agent (train.py:143-158): the
 * policy sample of rt_policy_sample (same arithmetic, same bits) and
 * rt_env_step in ONE launch per step in incremental step mode (policy, pose
 * update, beam march and finish on one wave per env), two more (k_dense,
 * k_finish) in dense mode.  The env acts on the sampled actions
 * (act_store_d); outputs as rt_env_step.  obs_in_d may be obs_d (the env's
 * observation buffer of the previous step). */
typedef struct rt_policy_step {
    const float* const* params;   /* 13 device pointers, rt_policy_sample order (host array) */
    int32_t n_params;             /* 13 */
    const float* obs_in;          /* [N][9] observation acted on (next_obs) */
    const uint8_t* done_in;       /* [N] next_done (env terminated) or NULL */
    float* obs_store;             /* [N][9] storage obs[step] */
    float* done_store;            /* [N]    storage dones[step] */
    float* act_store;             /* [N][6] storage actions[step] */
    float* logp_store;            /* [N]    storage logprobs[step] */
    float* value_store;           /* [N]    storage values[step] */
    uint64_t seed;                /* Philox key */
    uint64_t counter;             /* Philox call counter (one per step) */
    int64_t env_id_base;          /* global id of env 0 (rank * N) */
} rt_policy_step;

int rt_env_step_policy(rt_env* env, const rt_policy_step* step, float* obs_d, float* reward_d,
                       uint8_t* terminated_d, float* info_d, void* stream);

/* n_steps consecutive rollout steps (train.py:138-161).  Incremental step
 * mode: ONE persistent launch -- each env's wave runs its policy sample, env
 * step and finish n_steps times back to back, with no grid-wide
 * synchronisation between steps (envs are independent).  Dense step mode:
 * the envs are split in two groups on two library streams that take turns
 * on the HBM-bound k_dense (a persistent variant that leaves CU slots free),
 * so one group's latency-bound policy/beam and finish kernels run beside the
 * other's dose stream (fork/join with `stream` by events);
 * rt_env_set_rollout_groups(env, 1) issues the three launches of
 * rt_env_step_policy per step on `stream` instead.  Step s (0-based)
 * writes the storage slices step.X_store + s * (row floats * N) -- i.e.
 * step.X_store is row `first` of contiguous [T][N][...] storage -- plus
 * reward_store[s * N + e] and info_store[(s * N + e) * RT_INFO_W] (info_store
 * may be NULL), with Philox counter step.counter + s.  Step 0 acts on
 * step.obs_in / step.done_in; later steps on the env's own outputs, which
 * are left in obs_d / terminated_d after the last step.  Same bits as
 * n_steps calls of rt_env_step_policy.  RT_EINVAL for a vision handle;
 * RT_ELIMIT if the persistent kernel's LDS layout cannot be built (callers
 * then step with rt_env_step_policy; not reached for the visionless MLP --
 * tumours above its LDS share keep their sum plan in global scratch). */
typedef struct rt_policy_rollout {
    rt_policy_step step;          /* storage row of the first step, its counter */
    int32_t n_steps;
    float* reward_store;          /* [n_steps][N] */
    float* info_store;            /* [n_steps][N][RT_INFO_W] or NULL */
} rt_policy_rollout;

int rt_env_rollout_policy(rt_env* env, const rt_policy_rollout* rollout, float* obs_d, uint8_t* terminated_d,
                          void* stream);
/* Env groups of the rollout call.  Dense step mode: 2..4 (pipelined library
 * streams taking turns on k_dense in a ring; default 2) or 1 (every launch on
 * the caller's stream).  Incremental step mode: 0, its one persistent launch
 * (the only value it takes).  RT_EINVAL on any other value. */
int rt_env_set_rollout_groups(rt_env* env, int32_t groups);

/* GAE reverse scan (train.py:163-181), one lane per env, f32 in [T][N] layout:
 * adv[t] = delta + gamma*lambda*(1-done[t+1])*adv[t+1]; ret = adv + values. */
int rt_gae(int32_t T, int32_t N, const float* rewards_d, const float* values_d,
           const float* dones_d, const float* next_value_d, const float* next_done_d,
           double gamma, double gae_lambda, float* adv_d, float* ret_d, void* stream);

/* ---- fused PPO update of the visionless agent (train.py:183-246) ----------
 * The rollout batch, flattened [T*N] (rows of obs are 9 floats, of actions 6). */
typedef struct rt_ppo_batch {
    const float* obs;
    const float* actions;
    const float* logprobs;
    const float* advantages;
    const float* returns;
    const float* values;
    int64_t batch_size;
} rt_ppo_batch;

/* train.py:200-246 hyper-parameters (config keys of the same names). */
typedef struct rt_ppo_hparams {
    float clip_coef;
    int32_t clip_vloss;
    int32_t norm_adv;   /* adv_stats_d ([mean, std] per minibatch) required when set */
    float ent_coef;
    float vf_coef;
    float max_grad_norm; /* <= 0: no clipping */
    double adam_beta1, adam_beta2;
    float adam_eps;
    int32_t precision;   /* RT_PPO_PREC_*: the two 64x64 layer products (below); 0 = f32 */
} rt_ppo_hparams;

/* Floats of workspace rt_ppo_grad / rt_ppo_update need for a minibatch. */
int64_t rt_ppo_workspace_floats(int32_t minibatch_size);
/* Parameters of the fused agent (10,061). */
int32_t rt_ppo_num_params(void);

/* rt_ppo_hparams.precision: arithmetic of the two 64x64 layer products in
 * rt_ppo_grad / rt_ppo_update (forward and data gradient), per call.  F32 (0):
 * exact f32 MFMA, the reference's arithmetic (torch f32 Linear, TF32 off:
 * train.py:200-238 via networks.py).  BF16X3: each f32 operand split into bf16
 * hi + lo, products hi*hi + hi*lo + lo*hi accumulated in f32 (relative error
 * <= ~2^-15 per product); the same f64-autograd gates hold
 * (tests/test_gpu_trainer.py).  RT_EINVAL on another value. */
#define RT_PPO_PREC_F32 0
#define RT_PPO_PREC_BF16X3 1

/* Gradient of the minibatch PPO loss (train.py:200-238: clipped surrogate,
 * [clipped] value loss * vf_coef, - ent_coef * entropy; advantages normalised
 * with adv_stats_d when norm_adv) w.r.t. the 13 parameter tensors (order of
 * rt_policy_sample), written (not accumulated) into grads_d[13].  mb_idx_d:
 * the minibatch's rows of the batch.  stats_d[6] = pg_loss, v_loss, entropy,
 * old_approx_kl, approx_kl, clipfrac of the minibatch (train.py:206-211);
 * stats_accum_d[6] (optional) += the same. */
int rt_ppo_grad(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* batch,
                const int64_t* mb_idx_d, int32_t mb_size, const float* adv_stats_d,
                const rt_ppo_hparams* hp, float* workspace_d, int64_t workspace_floats, float* stats_d,
                float* stats_accum_d, void* stream);

/* nn.utils.clip_grad_norm_(max_grad_norm) + torch.optim.Adam step number
 * `step` (foreach op order) over flat parameter / gradient / state buffers.
 * grad_div >= 1: the gradient is first divided by it (IEEE division, as
 * torch's grad.div_(grad_div)): the world size after a data-parallel SUM
 * all-reduce, so the average needs no kernel of its own; 1 = as is.  grad_d
 * holds the divided, clipped gradient afterwards.  workspace_d: >= 256 floats
 * of device scratch (the norm partials). */
int rt_adam_step(int64_t n, float* param_d, float* grad_d, float* exp_avg_d, float* exp_avg_sq_d,
                 int64_t step, double lr, const rt_ppo_hparams* hp, int32_t grad_div, float* workspace_d,
                 void* stream);

/* n_minibatches consecutive optimizer steps (rt_ppo_grad + rt_adam_step) on
 * the minibatches perm_d[i*mb_size, (i+1)*mb_size) -- of one epoch, or of
 * several whose permutations lie back to back in perm_d (rt_ppo_shuffle_epochs),
 * adv_stats_d then holding [n_minibatches][2] (single process; data-parallel
 * callers interleave rt_ppo_grad, the all-reduce and rt_adam_step themselves).
 * params_d / grads_d are views of flat_param_d / flat_grad_d; the first step
 * is numbered step0. */
int rt_ppo_update(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* batch,
                  const int64_t* perm_d, int32_t mb_size, int32_t n_minibatches, const float* adv_stats_d,
                  const rt_ppo_hparams* hp, float* flat_param_d, float* flat_grad_d, float* exp_avg_d,
                  float* exp_avg_sq_d, int64_t n_flat, int64_t step0, double lr, float* workspace_d,
                  int64_t workspace_floats, float* stats_d, float* stats_accum_d, void* stream);

/* ---- data-parallel update (train.py:183-248 at world > 1) -----
 * One process per GPU.  The library holds its own RCCL communicator: rank 0
 * draws an id (rt_dp_unique_id), the caller broadcasts the RT_DP_ID_BYTES
 * bytes (e.g. torch.distributed), every rank calls rt_dp_comm_create with
 * them (a collective: all ranks at once).  RCCL is loaded on the first call
 * (the copy already mapped in the process, e.g. torch's, else ROCm's). */
typedef struct rt_dp_comm rt_dp_comm; /* opaque */
#define RT_DP_ID_BYTES 128
#define RT_DP_F32 0
#define RT_DP_F64 1
int rt_dp_unique_id(uint8_t* id_h /* [RT_DP_ID_BYTES] */);
int rt_dp_comm_create(const uint8_t* id_h, int32_t nranks, int32_t rank, int device, rt_dp_comm** out);
void rt_dp_comm_destroy(rt_dp_comm* comm);
/* In-place SUM all-reduce of count elements (RT_DP_F32 / RT_DP_F64) on `stream`. */
int rt_dp_allreduce(rt_dp_comm* comm, void* buf_d, int64_t count, int32_t dtype, void* stream);
/* rt_ppo_update across the ranks of `comm`: per minibatch rt_ppo_grad, the SUM
 * all-reduce of flat_grad_d over RCCL, then rt_adam_step with grad_div =
 * nranks (clip on the global gradient, every replica the same step) -- the
 * whole update in one call, enqueued on `stream`.  adv_stats_d: the global
 * per-minibatch statistics (rt_ppo_adv_sums -> all-reduce ->
 * rt_ppo_adv_finalize).  At nranks 1 the all-reduce is an identity and the
 * result equals rt_ppo_grad + rt_adam_step. */
int rt_ppo_update_dp(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* batch,
                     const int64_t* perm_d, int32_t mb_size, int32_t n_minibatches, const float* adv_stats_d,
                     const rt_ppo_hparams* hp, float* flat_param_d, float* flat_grad_d, float* exp_avg_d,
                     float* exp_avg_sq_d, int64_t n_flat, int64_t step0, double lr, float* workspace_d,
                     int64_t workspace_floats, float* stats_d, float* stats_accum_d, rt_dp_comm* comm,
                     void* stream);

/* RT_OK, or RT_EDEVICE when an rt_ppo_update on the current device lost the
 * grid arrival of its fused reduce + Adam launch (the grid was not
 * co-resident): that launch and every later one of the update then wrote no
 * parameter, moment or gradient, so the state is the last complete
 * minibatch's.  Sticky; every later rt_ppo_* call also returns RT_EDEVICE.
 * Trainers call it after synchronising the update's stream, before saving a
 * checkpoint. */
int rt_ppo_status(void);

/* Per-epoch helpers of the update: perm_d[i] = a keyed pseudo-random
 * permutation of [0, n) (train.py:195's shuffle); stats_d[n_mb][2] = mean and
 * unbiased std of adv over each minibatch perm[i*mb, (i+1)*mb) (train.py:215-218),
 * using workspace_d (>= 128 * n_minibatches floats; rt_ppo_update's workspace
 * serves). */
int rt_ppo_shuffle(int64_t n, uint64_t key, int64_t* perm_d, void* stream);
/* n_epochs permutations in one launch: perm_d[e*n .. (e+1)*n) = rt_ppo_shuffle
 * with keys_h[e] (host array) -- every epoch's shuffle of an update at once. */
int rt_ppo_shuffle_epochs(int64_t n, int32_t n_epochs, const uint64_t* keys_h, int64_t* perm_d, void* stream);
int rt_ppo_adv_stats(const float* adv_d, const int64_t* perm_d, int32_t mb_size, int32_t n_minibatches,
                     float* stats_d, float* workspace_d, int64_t workspace_floats, void* stream);
/* rt_ppo_shuffle_epochs + the advantage statistics of all their minibatches
 * (mb_size divides n) in one pass: perm_d[e*n .. (e+1)*n) as rt_ppo_shuffle_epochs,
 * and either stats_d[n_epochs * n/mb_size][2] = rt_ppo_adv_stats of those
 * minibatches (single process) or sums_d[..][2] = rt_ppo_adv_sums (data
 * parallel: the caller all-reduces, then rt_ppo_adv_finalize) -- exactly one
 * of the two non-NULL; bitwise the separate calls' results.  workspace_d:
 * >= 128 * min(n_epochs, 32) * n/mb_size floats. */
int rt_ppo_shuffle_adv(int64_t n, int32_t n_epochs, const uint64_t* keys_h, int64_t* perm_d, const float* adv_d,
                       int32_t mb_size, double* sums_d, float* stats_d, float* workspace_d,
                       int64_t workspace_floats, void* stream);
/* Data-parallel form of rt_ppo_adv_stats (train.py:215-218 over the union
 * of the ranks' minibatches): rt_ppo_adv_sums writes this rank's per-minibatch
 * (sum, sum of squares) of adv, f64 sums_d[n_mb][2] (same workspace rule);
 * the caller all-reduces sums_d (SUM) across ranks, then rt_ppo_adv_finalize
 * turns it into stats_d[n_mb][2] = (mean, unbiased std) over `count` rows per
 * minibatch (mb_size x world size). */
int rt_ppo_adv_sums(const float* adv_d, const int64_t* perm_d, int32_t mb_size, int32_t n_minibatches,
                    double* sums_d, float* workspace_d, int64_t workspace_floats, void* stream);
int rt_ppo_adv_finalize(const double* sums_d, int64_t count, int32_t n_minibatches, float* stats_d, void* stream);

/* ---- C3D feature extractor of the vision agent (networks.py:8-45) ----------
 * One stage = Conv3d(cin, 16, 3, groups) + ReLU + MaxPool3d(2, 2, pool_pad):
 * stage 1 (4, 1, pad (S_i - 2) % 2), stage 2 (16, 2, 0), stage 3 (16, 4, 0).
 * Tensors are NCDHW f32; weights as torch ([16][cin/groups][3][3][3], [16]). */
typedef struct rt_conv_layer {
    int32_t cin;          /* 4 or 16 */
    int32_t groups;       /* 1 (cin 4); 1, 2 or 4 (cin 16) */
    int32_t in_dims[3];   /* D, H, W of the input */
    int32_t pool_pad[3];  /* 0 or 1 per axis */
    int32_t precision;    /* RT_CONV_PREC_* of this call's forward products (below); 0 = f32 */
} rt_conv_layer;

/* rt_conv_layer.precision: arithmetic of the C3D forward products, per call
 * (the vision trainer's conv_precision config key).  F32 (0): f32 throughout
 * (the reference's torch Conv3d in f32; its cuDNN default allowed TF32) --
 * the forward of every stage and the grouped stages' data gradient in the
 * Winograd form F(2x2x2, 3x3x3) (f32 transforms, products on exact f32 MFMA).
 * BF16X3: conv1's forward and the grouped stages' (groups 2 and 4) forward and
 * data gradient as the direct ring kernels, every operand split into bf16 hi
 * + lo (round to nearest even), products hi*hi + hi*lo + lo*hi accumulated in
 * f32 (relative error <= ~2^-15 per product).  The weight gradients stay f32.
 * RT_EINVAL on another value. */
#define RT_CONV_PREC_F32 0
#define RT_CONV_PREC_BF16X3 1

/* Pooled output dims of a stage. */
int rt_conv_out_dims(const rt_conv_layer* layer, int32_t* out_dims);

/* y[b] = maxpool(relu(conv(x[rows[b]]) + bias)) for b < batch (rows_d NULL:
 * row b).  argmax_d (u8, shape of y, NULL for inference): bits 0-2 = index of
 * the window's first maximum in (z, y, x) order, bit 3 = max > 0. */
int rt_conv_relu_pool_fwd(const rt_conv_layer* layer, int32_t batch, const float* x_d, const int64_t* rows_d,
                          const float* w_d, const float* b_d, float* y_d, uint8_t* argmax_d, void* stream);

/* Weight/bias gradient of a stage from the pooled-output gradient dy_d and the
 * forward's argmax bytes: dW [16][cin/groups][27], db [16] (written).
 * workspace_d: rt_conv_wgrad_workspace_floats(layer, batch) floats. */
int64_t rt_conv_wgrad_workspace_floats(const rt_conv_layer* layer, int32_t batch);
int rt_conv_relu_pool_wgrad(const rt_conv_layer* layer, int32_t batch, const float* x_d, const int64_t* rows_d,
                            const float* dy_d, const uint8_t* argmax_d, float* dw_d, float* db_d,
                            float* workspace_d, int64_t workspace_floats, void* stream);

/* Measurement hook (bench.py c3d_mfma): the v_mfma_f32_16x16x4_f32
 * wave-instructions (2,048 FLOP each) the f32 Winograd kernel of a pass
 * issues for `batch` samples -- pass 0: rt_conv_relu_pool_fwd, 1:
 * rt_conv_relu_pool_dgrad -- zero-padded rows and channel lanes included, i.e.
 * what rocprofv3's SQ_INSTS_MFMA counts; 0 when that pass runs no Winograd
 * kernel (bf16x3, the dense or tile fallbacks), -1 on a bad argument.  Host
 * only (the launch planner's arithmetic; nothing is launched). */
int64_t rt_conv_mfma_count(const rt_conv_layer* layer, int32_t batch, int32_t pass);

/* Gradient w.r.t. the stage input (cin 16 stages): dx [B][16][D][H][W]. */
int rt_conv_relu_pool_dgrad(const rt_conv_layer* layer, int32_t batch, const float* w_d, const float* dy_d,
                            const uint8_t* argmax_d, float* dx_d, void* stream);

const char* rt_last_error(void);
int rt_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* RTENV_H */
