// policy.hip -- fused rollout-side policy step for the visionless agent.
//
// Reference: networks.py:107-147 (PPO: actor_mean / critic MLPs 9 -> 64 -> 64
// -> {6, 1}, tanh, state-independent actor_logstd; Normal(mean, exp(logstd)),
// log_prob summed over the action dims) as called per rollout step by
// train.py:143-149 (`get_action_and_value(next_obs)` + the stores into the
// rollout buffers).
//
// One wave per env, 16 envs per 1024-thread block (the arithmetic lives in
// policy_core.h, shared with the fused policy + env step of rtenv.hip); the
// parameters are staged in LDS once per block.  Writes the step's slices of
// the rollout storage (obs, done, action, logprob, value) directly.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

#include "rtenv.h"
#include "rt_trace.h"
#include "policy_core.h"

extern "C" int rt_internal_fail(int code, const char* msg);

namespace {

using namespace rtpol;

constexpr int kEnvsPerBlock = 16;          // one wave per env
constexpr int kThreads = 64 * kEnvsPerBlock;

struct PolicyParams {
    Weights w;
    int32_t N;
    const float* obs;          // [N][9]   next_obs
    const uint8_t* done_u8;    // [N]      next_done (env terminated) or null
    float* obs_out;            // [N][9]   storage obs[step]
    float* done_out;           // [N]      storage dones[step]
    float* act_out;            // [N][6]   storage actions[step]
    float* logp_out;           // [N]
    float* value_out;          // [N]
    uint64_t seed;
    uint64_t counter;
    int64_t id_base;
};

__global__ __launch_bounds__(kThreads) void k_policy_sample(PolicyParams P) {
    __shared__ Lds L;
    __shared__ __attribute__((aligned(16))) float h1s[kEnvsPerBlock][H];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int e = blockIdx.x * kEnvsPerBlock + w;
    if (lane == 0) RT_STAMP(e, 0);
    stage(L, P.w, tid, kThreads);
    __syncthreads();
    if (e >= P.N) return;  // wave-uniform, after the block barrier
    if (lane == 0) RT_STAMP(e, 9);
    float x[NOBS];
#pragma unroll
    for (int i = 0; i < NOBS; ++i) x[i] = P.obs[(size_t)e * NOBS + i];
    const Sample smp = policy_env(L, h1s[w], x, lane, P.seed, P.counter, (uint64_t)(P.id_base + e));
    if (lane < NOBS) {
        float xi = x[0];
#pragma unroll
        for (int i = 1; i < NOBS; ++i) xi = lane == i ? x[i] : xi;
        P.obs_out[(size_t)e * NOBS + lane] = xi;
    }
    if (lane == NOBS) P.done_out[e] = P.done_u8 ? (float)P.done_u8[e] : 0.0f;
    if (lane < NACT) P.act_out[(size_t)e * NACT + lane] = smp.action;
    if (lane == 0) {
        P.logp_out[e] = smp.logp;
        P.value_out[e] = smp.value;
        RT_STAMP(e, 1);
    }
}

}  // namespace

RT_TRACE_READ_FN(rt_trace_read_policy)

extern "C" int rt_policy_sample(const float* const* params_d, int32_t n_params_tensors, int32_t n_envs,
                                const float* obs_d, const uint8_t* done_d, float* obs_out_d, float* done_out_d,
                                float* act_out_d, float* logp_out_d, float* value_out_d, uint64_t seed,
                                uint64_t counter, int64_t env_id_base, void* stream) {
    if (!params_d || n_params_tensors != 13 || n_envs < 1 || !obs_d || !obs_out_d || !done_out_d || !act_out_d ||
        !logp_out_d || !value_out_d)
        return rt_internal_fail(RT_EINVAL, "rt_policy_sample: bad argument");
    PolicyParams P{};
    for (int i = 0; i < kTensors; ++i) {
        if (!params_d[i]) return rt_internal_fail(RT_EINVAL, "rt_policy_sample: NULL parameter");
        P.w.p[i] = params_d[i];
    }
    P.N = n_envs;
    P.obs = obs_d;
    P.done_u8 = done_d;
    P.obs_out = obs_out_d;
    P.done_out = done_out_d;
    P.act_out = act_out_d;
    P.logp_out = logp_out_d;
    P.value_out = value_out_d;
    P.seed = seed;
    P.counter = counter;
    P.id_base = env_id_base;
    hipLaunchKernelGGL(k_policy_sample, dim3((n_envs + kEnvsPerBlock - 1) / kEnvsPerBlock), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}
