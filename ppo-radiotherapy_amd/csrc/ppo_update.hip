// ppo_update.hip -- fused PPO minibatch update for the visionless agent.
//
// Reference: train.py:197-246 (CleanRL continuous PPO: clipped surrogate,
// clipped value loss, entropy bonus, per-minibatch advantage normalisation,
// clip_grad_norm_ + Adam(eps=1e-5)) applied to networks.py:107-147 (PPO:
// actor_mean / critic = Linear(9,64) tanh Linear(64,64) tanh Linear(64,{6,1}),
// state-independent actor_logstd).
//
// The torch formulation of one minibatch step is ~60 small kernels (forward,
// autograd backward, clip, foreach Adam); on a 64-wide MLP every one of them
// is launch- and latency-bound.  Here it is three kernels:
//
//   k_ppo_grad    one 512-thread block per 64 samples: gathers the minibatch
//                 rows, runs both MLPs forward, evaluates the PPO loss and its
//                 derivative per sample in closed form, back-propagates
//                 through both MLPs (all activations in LDS) and writes the
//                 block's partial weight gradients + loss statistics;
//   k_ppo_reduce  sums the block partials column-wise (fixed order:
//                 deterministic) into the flat gradient bucket;
//   k_clip_adam   one block: global grad norm, clip, Adam update over the flat
//                 parameter / state buffers, in torch's foreach-Adam op order.
//
// GEMM shapes per block are 64 x 64 x 64; tiles are mapped so that one
// wavefront shares an 8-sample group (broadcast LDS reads) and each lane owns a
// hidden unit (bank-distinct reads of 68-float padded rows).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "rtenv.h"

extern "C" int rt_internal_fail(int code, const char* msg);

namespace {

constexpr int H = 64;
constexpr int NOBS = 9;
constexpr int NACT = 6;
constexpr int TS = 64;          // samples per block
constexpr int HP = H + 4;       // padded LDS row stride
constexpr int kThreads = 512;             // 8 waves: 2 per SIMD (the LDS footprint allows 1 block per CU)
constexpr int NW = kThreads / 64;          // wavefronts per block
constexpr int SPW = TS / NW;               // samples per wavefront in the sample-major phases
constexpr int LPS = kThreads / TS;         // lanes per sample in the per-sample phases
constexpr int UPL = H / LPS;               // hidden units per lane there
constexpr int CPW = H / NW;                // layer-2 weight-gradient columns per wavefront
constexpr float kHalfLog2Pi = 0.91893853320467274f;

// parameter offsets, policy order (include/rtenv.h RT_PPO_*)
constexpr int O_AW1 = 0, O_AB1 = 576, O_AW2 = 640, O_AB2 = 4736, O_AW3 = 4800, O_AB3 = 5184, O_LS = 5190;
constexpr int O_CW1 = 5196, O_CB1 = 5772, O_CW2 = 5836, O_CB2 = 9932, O_CW3 = 9996, O_CB3 = 10060;
constexpr int NP = 10061;
constexpr int NSTAT = 6;
constexpr int PSTRIDE = 10068;  // NP + NSTAT rounded up to a float4
static_assert(PSTRIDE >= NP + NSTAT, "partial row");
constexpr int kTensorOff[14] = {O_AW1, O_AB1, O_AW2, O_AB2, O_AW3, O_AB3, O_LS,
                                O_CW1, O_CB1, O_CW2, O_CB2, O_CW3, O_CB3, NP};

struct Ptr13 {
    const float* p[13];
};
struct Dst13 {
    float* p[13];
};

struct GradParams {
    Ptr13 w;
    const float* obs;   // [B][9]
    const float* act;   // [B][6]
    const float* logp;  // [B]
    const float* adv;   // [B]
    const float* ret;   // [B]
    const float* val;   // [B]
    const int64_t* idx; // [mb] rows of this minibatch
    const float* adv_stats;  // [2] mean, std, or null (no normalisation)
    int32_t mb;
    float clip_lo, clip_hi, clip;  // ratio clamp [1 - c, 1 + c], c
    int32_t clip_vloss;
    float vf_coef;
    float* ws;  // [gridDim.x][PSTRIDE]
};

// ---- forward of one MLP trunk: H1 = tanh(X W1^T + b1), H2 = tanh(H1 W2^T + b2)
// thread (j = tid % 64, sample group sg = tid / 64: one wavefront per SPW samples)
__device__ __forceinline__ void trunk_fwd(const float* w1, const float* b1, const float* w2, const float* b2,
                                          const float* X, float* H1, float* H2, int tid) {
    const int j = tid & 63, sg = tid >> 6;
    float wr[NOBS];
#pragma unroll
    for (int i = 0; i < NOBS; ++i) wr[i] = w1[j * NOBS + i];
#pragma unroll 4
    for (int v = 0; v < SPW; ++v) {
        const int s = sg * SPW + v;
        float a = 0.0f;
#pragma unroll
        for (int i = 0; i < NOBS; ++i) a += wr[i] * X[s * NOBS + i];
        H1[s * HP + j] = tanhf(a + b1[j]);
    }
    __syncthreads();
    float acc[SPW];
#pragma unroll
    for (int v = 0; v < SPW; ++v) acc[v] = 0.0f;
    for (int i4 = 0; i4 < H / 4; ++i4) {
        const float4 w = *reinterpret_cast<const float4*>(&w2[j * HP + 4 * i4]);
#pragma unroll
        for (int v = 0; v < SPW; ++v) {
            const float4 h = *reinterpret_cast<const float4*>(&H1[(sg * SPW + v) * HP + 4 * i4]);
            acc[v] += w.x * h.x + w.y * h.y + w.z * h.z + w.w * h.w;
        }
    }
#pragma unroll
    for (int v = 0; v < SPW; ++v) H2[(sg * SPW + v) * HP + j] = tanhf(acc[v] + b2[j]);
    __syncthreads();
}

// head outputs of sample s = tid / LPS (its LPS lanes q own units UPL*q .. UPL*q+UPL-1)
template <int NOUT>
__device__ __forceinline__ void head_fwd(const float* w3, const float* b3, const float* H2, int tid, float out[NOUT]) {
    const int s = tid / LPS, q = tid % LPS;
#pragma unroll
    for (int k = 0; k < NOUT; ++k) {
        float p = 0.0f;
#pragma unroll
        for (int c = 0; c < UPL; ++c) p += w3[k * H + UPL * q + c] * H2[s * HP + UPL * q + c];
#pragma unroll
        for (int off = 1; off < LPS; off <<= 1) p += __shfl_xor(p, off, 64);
        out[k] = p + b3[k];
    }
}

// ---- backward of one head + trunk; GOUT[s][k] = dL/d out_k (row stride 8).
// Writes the block's partial gradients of W1 b1 W2 b2 W3 b3 at the given offsets.
// H1 is overwritten by dL/d(pre-activation of layer 1).
template <int NOUT>
__device__ __forceinline__ void trunk_bwd(const float* w2, const float* w3, const float* X, float* H1,
                                          const float* H2, float* G2, const float* GOUT, int tid, float* out,
                                          int o_w1, int o_b1, int o_w2, int o_b2, int o_w3, int o_b3) {
    const int j = tid & 63, wq = tid >> 6;
    // dW3[k][j] = sum_s GOUT[s][k] H2[s][j];  db3[k] = sum_s GOUT[s][k]
    for (int k = wq; k < NOUT; k += NW) {
        float a = 0.0f;
        for (int s = 0; s < TS; ++s) a += GOUT[s * 8 + k] * H2[s * HP + j];
        out[o_w3 + k * H + j] = a;
    }
    if (tid < NOUT) {
        float a = 0.0f;
        for (int s = 0; s < TS; ++s) a += GOUT[s * 8 + tid];
        out[o_b3 + tid] = a;
    }
    // G2[s][j] = (sum_k GOUT[s][k] W3[k][j]) * (1 - H2^2)
    {
        float w3r[NOUT];
#pragma unroll
        for (int k = 0; k < NOUT; ++k) w3r[k] = w3[k * H + j];
#pragma unroll 4
        for (int v = 0; v < SPW; ++v) {
            const int s = wq * SPW + v;
            float g = 0.0f;
#pragma unroll
            for (int k = 0; k < NOUT; ++k) g += GOUT[s * 8 + k] * w3r[k];
            const float h = H2[s * HP + j];
            G2[s * HP + j] = g * (1.0f - h * h);
        }
    }
    __syncthreads();
    // dW2[j][i] = sum_s G2[s][j] H1[s][i]  (lane j, wave wq owns i = CPW*wq ..); db2[j]
    {
        float acc[CPW];
#pragma unroll
        for (int c = 0; c < CPW; ++c) acc[c] = 0.0f;
        float bsum = 0.0f;
        for (int s = 0; s < TS; ++s) {
            const float g = G2[s * HP + j];
            bsum += g;
            const float4* hr = reinterpret_cast<const float4*>(&H1[s * HP + CPW * wq]);
#pragma unroll
            for (int c4 = 0; c4 < CPW / 4; ++c4) {
                const float4 h = hr[c4];
                acc[4 * c4 + 0] += g * h.x;
                acc[4 * c4 + 1] += g * h.y;
                acc[4 * c4 + 2] += g * h.z;
                acc[4 * c4 + 3] += g * h.w;
            }
        }
        float4* dst = reinterpret_cast<float4*>(out + o_w2 + j * H + CPW * wq);  // o_w2 % 4 == 0
#pragma unroll
        for (int c4 = 0; c4 < CPW / 4; ++c4)
            dst[c4] = make_float4(acc[4 * c4], acc[4 * c4 + 1], acc[4 * c4 + 2], acc[4 * c4 + 3]);
        if (wq == 0) out[o_b2 + j] = bsum;
    }
    __syncthreads();
    // G1[s][i] = (sum_j G2[s][j] W2[j][i]) * (1 - H1^2), in place of H1 (lane i, wave = sample group)
    {
        const int i = j;
        float acc[SPW];
#pragma unroll
        for (int v = 0; v < SPW; ++v) acc[v] = 0.0f;
        for (int j4 = 0; j4 < H / 4; ++j4) {
            const float wa = w2[(4 * j4 + 0) * HP + i], wb = w2[(4 * j4 + 1) * HP + i];
            const float wc = w2[(4 * j4 + 2) * HP + i], wd = w2[(4 * j4 + 3) * HP + i];
#pragma unroll
            for (int v = 0; v < SPW; ++v) {
                const float4 g = *reinterpret_cast<const float4*>(&G2[(wq * SPW + v) * HP + 4 * j4]);
                acc[v] += g.x * wa + g.y * wb + g.z * wc + g.w * wd;
            }
        }
#pragma unroll
        for (int v = 0; v < SPW; ++v) {
            const int s = wq * SPW + v;
            const float h = H1[s * HP + i];
            H1[s * HP + i] = acc[v] * (1.0f - h * h);
        }
    }
    __syncthreads();
    // dW1[j][i] = sum_s G1[s][j] X[s][i]  (i = wq, wq+NW, ...); db1[j] (wave NW-1)
    for (int i = wq; i < NOBS; i += NW) {
        float a = 0.0f;
        for (int s = 0; s < TS; ++s) a += H1[s * HP + j] * X[s * NOBS + i];
        out[o_w1 + j * NOBS + i] = a;
    }
    if (wq == NW - 1) {
        float a = 0.0f;
        for (int s = 0; s < TS; ++s) a += H1[s * HP + j];
        out[o_b1 + j] = a;
    }
    __syncthreads();
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__global__ __launch_bounds__(kThreads) void k_ppo_grad(GradParams P) {
    __shared__ __attribute__((aligned(16))) float aw1[H * NOBS], ab1[H], aw2[H * HP], ab2[H], aw3[NACT * H], ab3[8], ls[8];
    __shared__ __attribute__((aligned(16))) float cw1[H * NOBS], cb1[H], cw2[H * HP], cb2[H], cw3[H], cb3[4];
    __shared__ __attribute__((aligned(16))) float X[TS * NOBS], AH1[TS * HP], AH2[TS * HP], CH1[TS * HP],
        CH2[TS * HP], G2[TS * HP];
    __shared__ __attribute__((aligned(16))) float GM[TS * 8], GV[TS * 8];
    __shared__ float red[NW][16];
    const int tid = threadIdx.x;
    for (int i = tid; i < H * NOBS; i += kThreads) {
        aw1[i] = P.w.p[0][i];
        cw1[i] = P.w.p[7][i];
    }
    for (int i = tid; i < H * H; i += kThreads) {
        aw2[(i >> 6) * HP + (i & 63)] = P.w.p[2][i];
        cw2[(i >> 6) * HP + (i & 63)] = P.w.p[9][i];
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
    // lanes LPS*s .. LPS*s+LPS-1 hold sample s
    const int s = tid / LPS, q = tid % LPS;
    const int m = blockIdx.x * TS + s;
    const bool live = m < P.mb;
    const int64_t row = live ? P.idx[m] : 0;
    for (int i = q; i < NOBS; i += LPS) X[s * NOBS + i] = live ? P.obs[row * NOBS + i] : 0.0f;
    __syncthreads();

    trunk_fwd(aw1, ab1, aw2, ab2, X, AH1, AH2, tid);
    float mean[NACT];
    head_fwd<NACT>(aw3, ab3, AH2, tid, mean);
    trunk_fwd(cw1, cb1, cw2, cb2, X, CH1, CH2, tid);
    float value;
    head_fwd<1>(cw3, cb3, CH2, tid, &value);

    // ---- per-sample PPO loss and its derivative (train.py:200-236), every lane of the sample
    float st[NSTAT + NACT];  // pg, vl, ent, -logratio, (r-1)-logratio, clipped, dL/dlogstd[6]
#pragma unroll
    for (int k = 0; k < NSTAT + NACT; ++k) st[k] = 0.0f;
    float gm[NACT] = {0, 0, 0, 0, 0, 0}, gv = 0.0f;
    if (live) {
        const float inv_n = 1.0f / (float)P.mb;
        float z[NACT], sd[NACT], logp = 0.0f, ent = 0.0f;
#pragma unroll
        for (int k = 0; k < NACT; ++k) {
            sd[k] = expf(ls[k]);
            z[k] = (P.act[row * NACT + k] - mean[k]) / sd[k];
            logp += -0.5f * z[k] * z[k] - ls[k] - kHalfLog2Pi;
            ent += 0.5f + kHalfLog2Pi + ls[k];
        }
        const float lr = logp - P.logp[row];
        const float r = expf(lr);
        float A = P.adv[row];
        if (P.adv_stats) A = (A - P.adv_stats[0]) / (P.adv_stats[1] + 1e-8f);
        const float pg1 = -A * r;
        const float rc = fminf(fmaxf(r, P.clip_lo), P.clip_hi);
        const float pg2 = -A * rc;
        // torch.maximum backward: the larger input takes the gradient, ties split it
        const float w1 = pg1 > pg2 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
        const float w2 = pg2 > pg1 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
        const float pass = (r >= P.clip_lo && r <= P.clip_hi) ? 1.0f : 0.0f;  // clamp backward
        const float g_logp = inv_n * (w1 * -A + w2 * -A * pass) * r;
#pragma unroll
        for (int k = 0; k < NACT; ++k) {
            gm[k] = g_logp * z[k] / sd[k];
            st[NSTAT + k] = g_logp * (z[k] * z[k] - 1.0f);
        }
        const float R = P.ret[row], V = P.val[row];
        float vl, dv;
        if (P.clip_vloss) {
            const float d = value - V;
            const float vc = V + fminf(fmaxf(d, -P.clip), P.clip);
            const float vu = (value - R) * (value - R), vcc = (vc - R) * (vc - R);
            vl = fmaxf(vu, vcc);
            const float wu = vu > vcc ? 1.0f : (vu == vcc ? 0.5f : 0.0f);
            const float wc = vcc > vu ? 1.0f : (vu == vcc ? 0.5f : 0.0f);
            const float dpass = (d >= -P.clip && d <= P.clip) ? 1.0f : 0.0f;
            dv = wu * 2.0f * (value - R) + wc * 2.0f * (vc - R) * dpass;
        } else {
            vl = (value - R) * (value - R);
            dv = 2.0f * (value - R);
        }
        gv = P.vf_coef * 0.5f * inv_n * dv;
        st[0] = fmaxf(pg1, pg2);
        st[1] = vl;
        st[2] = ent;
        st[3] = -lr;
        st[4] = (r - 1.0f) - lr;
        st[5] = fabsf(r - 1.0f) > P.clip ? 1.0f : 0.0f;
    }
    if (q == 0) {
#pragma unroll
        for (int k = 0; k < NACT; ++k) GM[s * 8 + k] = gm[k];
        GV[s * 8] = gv;
    }
    // block sums of the statistics and dL/dlogstd (one contribution per sample)
#pragma unroll
    for (int k = 0; k < NSTAT + NACT; ++k) {
        const float v = wave_sum(q == 0 ? st[k] : 0.0f);
        if ((tid & 63) == 0) red[tid >> 6][k] = v;
    }
    __syncthreads();
    float* out = P.ws + (size_t)blockIdx.x * PSTRIDE;
    if (tid < NSTAT + NACT) {
        float v = 0.0f;
#pragma unroll
        for (int w = 0; w < NW; ++w) v += red[w][tid];
        if (tid < NSTAT)
            out[NP + tid] = v;
        else
            out[O_LS + tid - NSTAT] = v;
    }
    trunk_bwd<1>(cw2, cw3, X, CH1, CH2, G2, GV, tid, out, O_CW1, O_CB1, O_CW2, O_CB2, O_CW3, O_CB3);
    trunk_bwd<NACT>(aw2, aw3, X, AH1, AH2, G2, GM, tid, out, O_AW1, O_AB1, O_AW2, O_AB2, O_AW3, O_AB3);
}

struct ReduceParams {
    const float* ws;
    int32_t nblk;
    Dst13 grad;
    float* stats;        // [6]
    float* stats_accum;  // [6] or null
    float inv_n;
    float ent_coef;
};

// block: 64 columns; wave w sums rows w, w+4, ... (4 independent chains),
// the 4 wave sums are combined in a fixed order (deterministic)
__global__ __launch_bounds__(256) void k_ppo_reduce(ReduceParams P) {
    __shared__ float part[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int p = blockIdx.x * 64 + lane;
    const bool ok = p < NP + NSTAT;
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f;
    if (ok) {
        int b = w;
        for (; b + 12 < P.nblk; b += 16) {
            a0 += P.ws[(size_t)b * PSTRIDE + p];
            a1 += P.ws[(size_t)(b + 4) * PSTRIDE + p];
            a2 += P.ws[(size_t)(b + 8) * PSTRIDE + p];
            a3 += P.ws[(size_t)(b + 12) * PSTRIDE + p];
        }
        for (; b < P.nblk; b += 4) a0 += P.ws[(size_t)b * PSTRIDE + p];
    }
    part[w][lane] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (w != 0 || !ok) return;
    const float a = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    if (p < NP) {
        int t = 0;
#pragma unroll
        for (int k = 1; k < 13; ++k) t += p >= kTensorOff[k] ? 1 : 0;
        P.grad.p[t][p - kTensorOff[t]] = t == 6 ? a + -P.ent_coef : a;  // d(-ent_coef * mean(entropy)) / d logstd
    } else {
        const int k = p - NP;
        float v = a * P.inv_n;
        if (k == 1) v *= 0.5f;  // v_loss = 0.5 * mean(max(...))
        P.stats[k] = v;
        if (P.stats_accum) P.stats_accum[k] += v;
    }
}

struct AdamParams {
    int64_t n;
    float* param;
    float* grad;
    float* m;
    float* v;
    float max_norm;  // <= 0: no clipping
    float lerp_w;    // 1 - beta1
    float beta2, one_minus_beta2;
    float step_size;  // -lr / (1 - beta1^t)
    float bc2_sqrt;   // sqrt(1 - beta2^t)
    float eps;
};

__global__ __launch_bounds__(1024) void k_clip_adam(AdamParams P) {
    __shared__ float part[16];
    __shared__ float coef_s;
    const int tid = threadIdx.x;
    float coef = 1.0f;
    if (P.max_norm > 0.0f) {
        float acc = 0.0f;
        for (int64_t i = tid; i < P.n; i += 1024) acc += P.grad[i] * P.grad[i];
        acc = wave_sum(acc);
        if ((tid & 63) == 0) part[tid >> 6] = acc;
        __syncthreads();
        if (tid == 0) {
            float t = 0.0f;
            for (int w = 0; w < 16; ++w) t += part[w];
            // clip_grad_norm_: coef = max_norm / (||g|| + 1e-6), clamped to 1
            coef_s = fminf(P.max_norm / (sqrtf(t) + 1e-6f), 1.0f);
        }
        __syncthreads();
        coef = coef_s;
    }
    for (int64_t i = tid; i < P.n; i += 1024) {
        const float g = P.grad[i] * coef;
        P.grad[i] = g;
        float m = P.m[i];
        m = m + P.lerp_w * (g - m);                   // exp_avg.lerp_(grad, 1 - beta1)
        float v = P.v[i] * P.beta2;                   // exp_avg_sq.mul_(beta2)
        v = v + P.one_minus_beta2 * g * g;            //   .addcmul_(grad, grad, 1 - beta2)
        const float denom = sqrtf(v) / P.bc2_sqrt + P.eps;
        P.param[i] = P.param[i] + P.step_size * (m / denom);  // addcdiv_(exp_avg, denom, -step_size)
        P.m[i] = m;
        P.v[i] = v;
    }
}

int ppo_grad_launch(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* b,
                    const int64_t* idx_d, int32_t mb, const float* adv_stats_d, const rt_ppo_hparams* hp,
                    float* ws_d, int64_t ws_floats, float* stats_d, float* accum_d, hipStream_t st) {
    const int nblk = (mb + TS - 1) / TS;
    if ((int64_t)nblk * PSTRIDE > ws_floats) return rt_internal_fail(RT_EINVAL, "rt_ppo_grad: workspace too small");
    GradParams G{};
    ReduceParams R{};
    for (int i = 0; i < 13; ++i) {
        G.w.p[i] = params_d[i];
        R.grad.p[i] = grads_d[i];
    }
    G.obs = b->obs;
    G.act = b->actions;
    G.logp = b->logprobs;
    G.adv = b->advantages;
    G.ret = b->returns;
    G.val = b->values;
    G.idx = idx_d;
    G.adv_stats = hp->norm_adv ? adv_stats_d : nullptr;
    G.mb = mb;
    G.clip = hp->clip_coef;
    G.clip_lo = (float)(1.0 - (double)hp->clip_coef);
    G.clip_hi = (float)(1.0 + (double)hp->clip_coef);
    G.clip_vloss = hp->clip_vloss;
    G.vf_coef = hp->vf_coef;
    G.ws = ws_d;
    hipLaunchKernelGGL(k_ppo_grad, dim3(nblk), dim3(kThreads), 0, st, G);
    R.ws = ws_d;
    R.nblk = nblk;
    R.stats = stats_d;
    R.stats_accum = accum_d;
    R.inv_n = 1.0f / (float)mb;
    R.ent_coef = hp->ent_coef;
    hipLaunchKernelGGL(k_ppo_reduce, dim3((NP + NSTAT + 63) / 64), dim3(256), 0, st, R);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

int adam_launch(int64_t n, float* p, float* g, float* m, float* v, int64_t step, double lr,
                const rt_ppo_hparams* hp, hipStream_t st) {
    AdamParams A{};
    A.n = n;
    A.param = p;
    A.grad = g;
    A.m = m;
    A.v = v;
    A.max_norm = hp->max_grad_norm;
    const double b1 = hp->adam_beta1, b2 = hp->adam_beta2;
    // torch.optim.Adam (foreach): host-side scalars in double, applied in f32
    A.lerp_w = (float)(1.0 - b1);
    A.beta2 = (float)b2;
    A.one_minus_beta2 = (float)(1.0 - b2);
    A.step_size = (float)(-(lr / (1.0 - std::pow(b1, (double)step))));
    A.bc2_sqrt = (float)std::pow(1.0 - std::pow(b2, (double)step), 0.5);
    A.eps = hp->adam_eps;
    hipLaunchKernelGGL(k_clip_adam, dim3(1), dim3(1024), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

bool bad13(const void* const* p) {
    if (!p) return true;
    for (int i = 0; i < 13; ++i)
        if (!p[i]) return true;
    return false;
}

bool bad_batch(const rt_ppo_batch* b) {
    return !b || !b->obs || !b->actions || !b->logprobs || !b->advantages || !b->returns || !b->values ||
           b->batch_size < 1;
}

}  // namespace

extern "C" int64_t rt_ppo_workspace_floats(int32_t minibatch_size) {
    if (minibatch_size < 1) return 0;
    return (int64_t)((minibatch_size + TS - 1) / TS) * PSTRIDE;
}

extern "C" int32_t rt_ppo_num_params(void) { return NP; }

extern "C" int rt_ppo_grad(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* batch,
                           const int64_t* mb_idx_d, int32_t mb_size, const float* adv_stats_d,
                           const rt_ppo_hparams* hp, float* workspace_d, int64_t workspace_floats, float* stats_d,
                           float* stats_accum_d, void* stream) {
    if (bad13(reinterpret_cast<const void* const*>(params_d)) || bad13(reinterpret_cast<const void* const*>(grads_d)) ||
        bad_batch(batch) || !mb_idx_d || mb_size < 1 || !hp || !workspace_d || !stats_d ||
        (hp->norm_adv && !adv_stats_d))
        return rt_internal_fail(RT_EINVAL, "rt_ppo_grad: bad argument");
    return ppo_grad_launch(params_d, grads_d, batch, mb_idx_d, mb_size, adv_stats_d, hp, workspace_d,
                           workspace_floats, stats_d, stats_accum_d, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int rt_adam_step(int64_t n, float* param_d, float* grad_d, float* exp_avg_d, float* exp_avg_sq_d,
                            int64_t step, double lr, const rt_ppo_hparams* hp, void* stream) {
    if (n < 1 || !param_d || !grad_d || !exp_avg_d || !exp_avg_sq_d || step < 1 || !hp)
        return rt_internal_fail(RT_EINVAL, "rt_adam_step: bad argument");
    return adam_launch(n, param_d, grad_d, exp_avg_d, exp_avg_sq_d, step, lr, hp,
                       reinterpret_cast<hipStream_t>(stream));
}

extern "C" int rt_ppo_update(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* batch,
                             const int64_t* perm_d, int32_t mb_size, int32_t n_minibatches,
                             const float* adv_stats_d, const rt_ppo_hparams* hp, float* flat_param_d,
                             float* flat_grad_d, float* exp_avg_d, float* exp_avg_sq_d, int64_t n_flat,
                             int64_t step0, double lr, float* workspace_d, int64_t workspace_floats,
                             float* stats_d, float* stats_accum_d, void* stream) {
    if (bad13(reinterpret_cast<const void* const*>(params_d)) || bad13(reinterpret_cast<const void* const*>(grads_d)) ||
        bad_batch(batch) || !perm_d || mb_size < 1 || n_minibatches < 1 || !hp || !flat_param_d || !flat_grad_d ||
        !exp_avg_d || !exp_avg_sq_d || n_flat != NP || step0 < 1 || !workspace_d || !stats_d ||
        (hp->norm_adv && !adv_stats_d) || (int64_t)mb_size * n_minibatches > batch->batch_size)
        return rt_internal_fail(RT_EINVAL, "rt_ppo_update: bad argument");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    for (int i = 0; i < n_minibatches; ++i) {
        int rc = ppo_grad_launch(params_d, grads_d, batch, perm_d + (int64_t)i * mb_size, mb_size,
                                 adv_stats_d ? adv_stats_d + 2 * i : nullptr, hp, workspace_d, workspace_floats,
                                 stats_d, stats_accum_d, st);
        if (rc) return rc;
        rc = adam_launch(n_flat, flat_param_d, flat_grad_d, exp_avg_d, exp_avg_sq_d, step0 + i, lr, hp, st);
        if (rc) return rc;
    }
    return RT_OK;
}
