// policy_core.h -- the visionless agent's rollout-side step for ONE env per
// wave: networks.py:107-147 (actor_mean / critic 9 -> 64 -> 64 -> {6, 1},
// tanh, state-independent actor_logstd; Normal(mean, exp(logstd)).sample(),
// log_prob summed over the action dims) as train.py:143-149 calls it.
//
// Shared by k_policy_sample (policy.hip) and the fused policy + env step
// (rtenv.hip), so both produce the same bits.  Lane j owns hidden unit j of
// both layers; the parameters sit in LDS (staged once per block); layer-1
// activations go through 64 floats of wave-private LDS.  Every sum runs in a
// fixed order: unit j's dot products in input order, each head output as
// 16 sequential 4-unit partials combined by a 16-way xor butterfly, the
// log-probability over the 6 dims in order.  Gaussian noise: Philox4x32-10
// (key = seed, counter = (call, env id)) + Box-Muller, one action dim per lane.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace rtpol {

constexpr int H = 64;      // feature_dim (networks.py:107 default)
constexpr int NOBS = 9;    // visionless observation
constexpr int NACT = 6;    // action size (environment.py:16)
constexpr int W2S = H + 4; // padded LDS row stride of the 64x64 layer-2 weights
constexpr int kTensors = 13;

// parameter tensors in PPO.parameters() order
struct Weights {
    const float* p[kTensors];
};

// LDS image of the 10,061 parameters (42.3 KiB)
struct alignas(16) Lds {
    alignas(16) float aw2[H * W2S];
    alignas(16) float cw2[H * W2S];
    alignas(16) float aw1[H * NOBS];
    alignas(16) float cw1[H * NOBS];
    alignas(16) float aw3[NACT * H];
    float ab1[H], ab2[H], cb1[H], cb2[H], cw3[H];
    float ab3[NACT], ls[NACT], cb3[4];
};

// Stage the parameters by LDS DMA (global_load_lds, 4 B per lane, no
// VGPRs): 160 wave-sized pieces -- the 64-float rows of the two 64x64 layers
// at their padded stride, then the small tensors in 64-float pieces -- split
// over the block's waves, every piece in flight at once.  A register copy
// loop (load, store, next) waited out one dependent L2 round trip per
// iteration: 36 us of the pipelined rollout's 44 us policy phase beside the
// dose stream (tools/trace_env.py --pipelined).  Ends with this wave's DMA
// landed; the caller's barrier then publishes the whole image.
typedef __attribute__((address_space(3))) void* stage_lds_t;
typedef __attribute__((address_space(1))) void* stage_glb_t;
constexpr int kStagePieces = 2 * H + 2 * NOBS + NACT + 5 + 3;

__device__ __forceinline__ void stage(Lds& L, const Weights& w, int tid, int nthreads) {
    const int lane = tid & 63, nw = nthreads >> 6;
    for (int p = __builtin_amdgcn_readfirstlane(tid >> 6); p < kStagePieces; p += nw) {
        const float* src;
        float* dst;
        int n = 64;
        if (p < H) {
            src = w.p[2] + p * H;
            dst = L.aw2 + p * W2S;
        } else if (p < 2 * H) {
            src = w.p[9] + (p - H) * H;
            dst = L.cw2 + (p - H) * W2S;
        } else if (p < 2 * H + NOBS) {
            src = w.p[0] + (p - 2 * H) * 64;
            dst = L.aw1 + (p - 2 * H) * 64;
        } else if (p < 2 * H + 2 * NOBS) {
            src = w.p[7] + (p - 2 * H - NOBS) * 64;
            dst = L.cw1 + (p - 2 * H - NOBS) * 64;
        } else if (p < 2 * H + 2 * NOBS + NACT) {
            src = w.p[4] + (p - 2 * H - 2 * NOBS) * 64;
            dst = L.aw3 + (p - 2 * H - 2 * NOBS) * 64;
        } else {
            switch (p - (2 * H + 2 * NOBS + NACT)) {
                case 0: src = w.p[1]; dst = L.ab1; break;
                case 1: src = w.p[3]; dst = L.ab2; break;
                case 2: src = w.p[8]; dst = L.cb1; break;
                case 3: src = w.p[10]; dst = L.cb2; break;
                case 4: src = w.p[11]; dst = L.cw3; break;
                case 5: src = w.p[5]; dst = L.ab3; n = NACT; break;
                case 6: src = w.p[6]; dst = L.ls; n = NACT; break;
                default: src = w.p[12]; dst = L.cb3; n = 1; break;
            }
        }
        if (lane < n) __builtin_amdgcn_global_load_lds((stage_glb_t)(src + lane), (stage_lds_t)dst, 4, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0);  // this wave's pieces have landed (vmcnt 0)
}

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

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ float lane_f(float v, int src) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), src));
}

// Head output from per-lane products p_j (unit j): 16 partials
// (((0 + p_4s) + p_4s+1) + p_4s+2) + p_4s+3, then an xor butterfly over the
// 16 partials (lane distance 32, 16, 8, 4); every lane gets the sum.
__device__ __forceinline__ float head_sum(float p, int lane) {
    const int q = lane & ~3;
    float m = 0.0f;
    m += __shfl(p, q, 64);
    m += __shfl(p, q + 1, 64);
    m += __shfl(p, q + 2, 64);
    m += __shfl(p, q + 3, 64);
#pragma unroll
    for (int off = 32; off >= 4; off >>= 1) m += __shfl_xor(m, off, 64);
    return m;
}

// hidden unit `lane` of layer 2 after layer 1 (h1: the wave's 64 LDS floats)
__device__ __forceinline__ float trunk(const float* w1, const float* b1, const float* w2, const float* b2,
                                      const float x[NOBS], float* h1, int lane) {
    float a = b1[lane];
#pragma unroll
    for (int i = 0; i < NOBS; ++i) a += w1[lane * NOBS + i] * x[i];
    wave_lds_sync();  // previous readers of h1 are done
    h1[lane] = tanhf(a);
    wave_lds_sync();
    const float4* row = reinterpret_cast<const float4*>(w2 + lane * W2S);
    const float4* hv = reinterpret_cast<const float4*>(h1);
    float s = b2[lane];
#pragma unroll
    for (int i = 0; i < H / 4; ++i) {
        const float4 r = row[i];
        const float4 q = hv[i];
        s += r.x * q.x + r.y * q.y + r.z * q.z + r.w * q.w;
    }
    return tanhf(s);
}

struct Sample {
    float action;  // lanes 0..5: action dim `lane`
    float logp;    // every lane
    float value;   // every lane
};

// One env's policy step on one wave.  x: the env's observation (every lane);
// gid: global env id (Philox counter).
__device__ __forceinline__ Sample policy_env(const Lds& L, float* h1, const float x[NOBS], int lane, uint64_t seed,
                                             uint64_t counter, uint64_t gid) {
    Sample out;
    // ---- actor_mean
    const float ta = trunk(L.aw1, L.ab1, L.aw2, L.ab2, x, h1, lane);
    float mean[NACT];
#pragma unroll
    for (int k = 0; k < NACT; ++k) mean[k] = head_sum(L.aw3[k * H + lane] * ta, lane) + L.ab3[k];
    // ---- critic
    const float tc = trunk(L.cw1, L.cb1, L.cw2, L.cb2, x, h1, lane);
    out.value = head_sum(L.cw3[lane] * tc, lane) + L.cb3[0];
    // ---- Normal(mean, exp(logstd)).sample(): dim k on lane k
    const int k = lane < NACT ? lane : NACT - 1;
    const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
    const uint4 r = philox(make_uint4((uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)gid,
                                      (uint32_t)(gid >> 32) ^ (k < 4 ? 0x504f4c31u : 0x504f4c32u)),
                           key);
    const int w = k & 3;
    const uint32_t u = w == 0 ? r.x : (w == 1 ? r.y : (w == 2 ? r.z : r.w));
    const uint32_t u_pair = (uint32_t)__shfl_xor((int)u, 1, 64);  // the other draw of the Box-Muller pair
    const uint32_t ur = (k & 1) ? u_pair : u, ut = (k & 1) ? u : u_pair;
    const float rad = sqrtf(-2.0f * logf(u01(ur)));
    const float th = 6.283185307179586f * u01(ut);
    const float nrm = (k & 1) ? rad * sinf(th) : rad * cosf(th);
    float mk = mean[0];
#pragma unroll
    for (int j = 1; j < NACT; ++j) mk = k == j ? mean[j] : mk;
    const float lsk = L.ls[k];
    const float sd = expf(lsk);
    const float a = mk + sd * nrm;
    const float z = (a - mk) / sd;
    const float term = -0.5f * z * z - lsk - 0.91893853320467274f;  // 0.5 * log(2 pi)
    float logp = 0.0f;
#pragma unroll
    for (int j = 0; j < NACT; ++j) logp += lane_f(term, j);
    out.action = a;
    out.logp = logp;
    return out;
}

}  // namespace rtpol
