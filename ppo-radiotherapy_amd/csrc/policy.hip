// policy.hip -- fused rollout-side policy step for the visionless agent.
//
// Reference: networks.py:107-147 (PPO: actor_mean / critic MLPs 9 -> 64 -> 64
// -> {6, 1}, tanh, state-independent actor_logstd; Normal(mean, exp(logstd)),
// log_prob summed over the action dims) as called per rollout step by
// train.py:143-149 (`get_action_and_value(next_obs)` + the stores into the
// rollout buffers).
//
// 16 lanes per env (16 envs per 256-thread block): lane s owns hidden units
// 4s..4s+3 of both layers; the 10,061 parameters (40 KiB f32) are staged in
// LDS per block (layer-2 rows padded to 68 floats so the 16 lanes' float4 row
// reads hit distinct banks); layer-1 activations are exchanged through LDS,
// head sums through 16-lane shuffles.  Gaussian noise: Philox4x32-10 (key = seed, counter = (call,
// env id)) + Box-Muller.  Writes the step's slices of the rollout storage
// (obs, done, action, logprob, value) directly.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

#include "rtenv.h"

extern "C" int rt_internal_fail(int code, const char* msg);

namespace {

constexpr int H = 64;      // feature_dim (networks.py:107 default)
constexpr int NOBS = 9;    // visionless observation
constexpr int NACT = 6;    // action size (environment.py:16)
constexpr int kThreads = 256;

struct Ptrs {
    const float* p[13];
};

struct PolicyParams {
    Ptrs w;
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

__device__ __forceinline__ uint4 philox(uint4 c, uint2 k) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        uint32_t lo0 = c.x * 0xD2511F53u, hi0 = __umulhi(c.x, 0xD2511F53u);
        uint32_t lo1 = c.z * 0xCD9E8D57u, hi1 = __umulhi(c.z, 0xCD9E8D57u);
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ float u01(uint32_t x) {  // (0, 1]
    return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// 16 lanes per env: lane s owns hidden units 4s..4s+3 of both layers.
constexpr int LPE = 16;                 // lanes per env
constexpr int EPB = kThreads / LPE;     // envs per block
constexpr int W2S = H + 4;              // padded LDS row stride of the 64x64 layer-2 weights

__device__ __forceinline__ float group_sum16(float v) {
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ void layer1(const float* w1, const float* b1, const float x[NOBS], int s, float h[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = 4 * s + u;
        float a = b1[j];
#pragma unroll
        for (int i = 0; i < NOBS; ++i) a += w1[j * NOBS + i] * x[i];
        h[u] = tanhf(a);
    }
}

// layer 2 units 4s..4s+3 (h1 of the env in LDS), squashed
__device__ __forceinline__ void layer2(const float* w2p, const float* b2, const float* h1, int s, float t[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int j = 4 * s + u;
        const float4* row = reinterpret_cast<const float4*>(w2p + j * W2S);
        const float4* hv = reinterpret_cast<const float4*>(h1);
        float a = b2[j];
#pragma unroll
        for (int i = 0; i < H / 4; ++i) {
            const float4 r = row[i];
            const float4 q = hv[i];
            a += r.x * q.x + r.y * q.y + r.z * q.z + r.w * q.w;
        }
        t[u] = tanhf(a);
    }
}

__global__ __launch_bounds__(kThreads) void k_policy_sample(PolicyParams P) {
    __shared__ __attribute__((aligned(16))) float aw1[H * NOBS], ab1[H], ab2[H], aw3[NACT * H], ab3[NACT], ls[NACT];
    __shared__ __attribute__((aligned(16))) float cw1[H * NOBS], cb1[H], cb2[H], cw3[H], cb3[4];
    __shared__ __attribute__((aligned(16))) float aw2[H * W2S], cw2[H * W2S];
    __shared__ __attribute__((aligned(16))) float h1s[EPB][H];
    const int tid = threadIdx.x;
    for (int i = tid; i < H * NOBS; i += kThreads) {
        aw1[i] = P.w.p[0][i];
        cw1[i] = P.w.p[7][i];
    }
    for (int i = tid; i < H * H; i += kThreads) {
        aw2[(i / H) * W2S + (i % H)] = P.w.p[2][i];
        cw2[(i / H) * W2S + (i % H)] = P.w.p[9][i];
    }
    for (int i = tid; i < H; i += kThreads) {
        ab1[i] = P.w.p[1][i];
        ab2[i] = P.w.p[3][i];
        cb1[i] = P.w.p[8][i];
        cb2[i] = P.w.p[10][i];
        cw3[i] = P.w.p[11][i];
    }
    for (int i = tid; i < NACT * H; i += kThreads) aw3[i] = P.w.p[4][i];
    if (tid < NACT) {
        ab3[tid] = P.w.p[5][tid];
        ls[tid] = P.w.p[6][tid];
    }
    if (tid == 0) cb3[0] = P.w.p[12][0];
    __syncthreads();

    const int slot = tid / LPE, s = tid % LPE;
    const int e = blockIdx.x * EPB + slot;
    const bool live = e < P.N;
    const int ec = live ? e : 0;
    float x[NOBS];
#pragma unroll
    for (int i = 0; i < NOBS; ++i) x[i] = P.obs[(size_t)ec * NOBS + i];
    if (live) {
        if (s < NOBS) P.obs_out[(size_t)e * NOBS + s] = x[s];
        if (s == NOBS) P.done_out[e] = P.done_u8 ? (float)P.done_u8[e] : 0.0f;
    }
    float h[4], t[4];
    // ---- actor_mean
    layer1(aw1, ab1, x, s, h);
    *reinterpret_cast<float4*>(&h1s[slot][4 * s]) = make_float4(h[0], h[1], h[2], h[3]);
    __syncthreads();
    layer2(aw2, ab2, h1s[slot], s, t);
    float mean[NACT];
#pragma unroll
    for (int k = 0; k < NACT; ++k) {
        float m = 0.0f;
#pragma unroll
        for (int u = 0; u < 4; ++u) m += aw3[k * H + 4 * s + u] * t[u];
        mean[k] = group_sum16(m) + ab3[k];
    }
    __syncthreads();
    // ---- critic
    layer1(cw1, cb1, x, s, h);
    *reinterpret_cast<float4*>(&h1s[slot][4 * s]) = make_float4(h[0], h[1], h[2], h[3]);
    __syncthreads();
    layer2(cw2, cb2, h1s[slot], s, t);
    float v = 0.0f;
#pragma unroll
    for (int u = 0; u < 4; ++u) v += cw3[4 * s + u] * t[u];
    const float value = group_sum16(v) + cb3[0];
    if (!live || s != 0) return;
    // ---- Normal(mean, exp(logstd)).sample(), log_prob(action).sum(1)
    const uint64_t gid = (uint64_t)(P.id_base + e);
    const uint2 key = make_uint2((uint32_t)P.seed, (uint32_t)(P.seed >> 32));
    const uint4 r0 = philox(make_uint4((uint32_t)P.counter, (uint32_t)(P.counter >> 32), (uint32_t)gid,
                                       (uint32_t)(gid >> 32) ^ 0x504f4c31u), key);
    const uint4 r1 = philox(make_uint4((uint32_t)P.counter, (uint32_t)(P.counter >> 32), (uint32_t)gid,
                                       (uint32_t)(gid >> 32) ^ 0x504f4c32u), key);
    const uint32_t u[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    float nrm[NACT];
#pragma unroll
    for (int k = 0; k < NACT; k += 2) {
        const float rad = sqrtf(-2.0f * logf(u01(u[k])));
        const float th = 6.283185307179586f * u01(u[k + 1]);
        nrm[k] = rad * cosf(th);
        nrm[k + 1] = rad * sinf(th);
    }
    float logp = 0.0f;
#pragma unroll
    for (int k = 0; k < NACT; ++k) {
        const float sd = expf(ls[k]);
        const float a = mean[k] + sd * nrm[k];
        P.act_out[(size_t)e * NACT + k] = a;
        const float z = (a - mean[k]) / sd;
        logp += -0.5f * z * z - ls[k] - 0.91893853320467274f;  // 0.5 * log(2 pi)
    }
    P.logp_out[e] = logp;
    P.value_out[e] = value;
}

}  // namespace

extern "C" int rt_policy_sample(const float* const* params_d, int32_t n_params_tensors, int32_t n_envs,
                                const float* obs_d, const uint8_t* done_d, float* obs_out_d, float* done_out_d,
                                float* act_out_d, float* logp_out_d, float* value_out_d, uint64_t seed,
                                uint64_t counter, int64_t env_id_base, void* stream) {
    if (!params_d || n_params_tensors != 13 || n_envs < 1 || !obs_d || !obs_out_d || !done_out_d || !act_out_d ||
        !logp_out_d || !value_out_d)
        return rt_internal_fail(RT_EINVAL, "rt_policy_sample: bad argument");
    PolicyParams P{};
    for (int i = 0; i < 13; ++i) {
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
    hipLaunchKernelGGL(k_policy_sample, dim3((n_envs + EPB - 1) / EPB), dim3(kThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}
