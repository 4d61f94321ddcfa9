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
//   k_ppo_grad_mfma  512-thread blocks of 4 (actor, critic) wave pairs over
//                    16-sample tiles: gathers the minibatch rows, runs both MLPs
//                    forward, the PPO loss derivative per sample in closed form
//                    and the backward on MFMA, one partial gradient row per block;
//   k_ppo_reduce     sums the block partials column-wise (fixed order:
//                    deterministic) into the flat gradient bucket, plus the
//                    ||g||^2 partials of the clip;
//   k_adam           clip_grad_norm_ + Adam over the flat parameter / state
//                    buffers, in torch's foreach-Adam op order.
#include "rt_trace.h"
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <type_traits>

#include "rtenv.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

extern "C" int rt_internal_fail(int code, const char* msg);

namespace {

constexpr int H = 64;
constexpr int NOBS = 9;
constexpr int NACT = 6;
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

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// ============================================================================
// k_ppo_grad_mfma: the minibatch gradient on f32 MFMA (v_mfma_f32_16x16x4_f32,
// exact f32 FMA chains; round 1's VALU kernel, 64 samples per block in LDS,
// measured slower and was removed).
//
// The PPO loss separates by head: the clipped surrogate and the entropy depend
// only on actor_mean / actor_logstd, the value loss only on the critic.  A
// block runs 4 wavefront pairs; in each pair one wave back-propagates the
// actor and the other the critic over the same 16-sample tiles, so every SIMD
// holds two independent instruction streams (one wave's MFMAs overlap the
// other's VALU) within 256 registers per wave.
//
// Inside a wave every activation stays in registers in the transposed
// [unit][sample] layout of the MFMA accumulator (lane l: sample c = l & 15,
// units 4g..4g+3 of each 16-row tile, g = l >> 4):
//   forward   Z^T = W . X^T           (sums over the accumulator's ROW index:
//   data grad G1^T = W2^T . G2^T        the previous tile is the B operand as is)
//   weight grad dW = G^T-tile . H       (sums over samples = the lane index: the
//                                        tiles go through wave-private LDS
//                                        scratch [unit][16 samples] and come back
//                                        as ds_read_b128 fragments)
// Weight gradients accumulate in MFMA accumulators across all tiles of the
// wave; the 4 pairs of a block are summed through LDS in a fixed order
// (deterministic) into one partial row.  Layer-1 biases ride in column 9 of an
// augmented W1 (X^T row 9 = 1), so db1 comes out of the dW1 product.
// ============================================================================
typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int MT = 512;   // 8 wavefronts: 4 (actor, critic) pairs, 2 per SIMD
constexpr int NPAIR = MT / 128;
constexpr int WP = 68;    // LDS row stride of W2 (b128 fragment reads 2-way, b32 reads conflict-free)
constexpr int W1P = 12;   // augmented W1 row: 9 weights, bias, 2 zeros
constexpr int SP = 24;    // scratch row stride (16 samples + pad: b128 reads conflict-free)
constexpr int SCR = 136;  // scratch rows per wave: A 0..63, B 64..127, GM^T 128..135
// per-wave tile inputs, copied from the minibatch rows by LDS DMA one tile
// ahead, [column][16 samples]: obs^T [9][16] at 0; actor: actions^T [6][16] at
// 144, logp at 240, adv at 256; critic: returns at 144, values at 160
constexpr int IN_OBS = 0, IN_ACT = 144, IN_LOGP = 240, IN_ADV = 256, IN_RET = 144, IN_VAL = 160, IN_FLOATS = 272;
constexpr int kMaxGradBlocks = 256;

// bf16x3 mode (kPrecBf16x3): each W2 as two bf16 images, hi = bf16(value)
// and lo = bf16(value - hi), rows = output unit j,
// columns = input unit i at wpos(i) (the k order of the 16x16x32 operand
// fragments, below).  80-element rows (128 B + 32 B pad): the ds_read_b128
// row reads are conflict-free, the ds_read_b64_tr_b16 column reads 2-way.
constexpr int WBP = 80;
constexpr int kPrecF32 = 0, kPrecBf16x3 = 1;

struct MfmaLds {
    union {
        float w2[2][H * WP];           // kPrecF32
        uint16_t w2b[2][2][H * WBP];   // kPrecBf16x3: [head][hi, lo]
    };
    float w1[2][H * W1P];
    float b2[2][H];
    float w3[7 * H];  // rows 0..5 actor_mean.4, row 6 critic.4
    float b3[8];
    float ls[8];
    float isd[8];  // 1 / exp(logstd), [6]: 1 / (adv std + 1e-8)
    float scr[MT / 64][SCR * SP];
    float in[MT / 64][IN_FLOATS];
};
static_assert(sizeof(MfmaLds) <= 160 * 1024, "LDS");
constexpr int kW2Region = 2 * H * H;    // reduction phase 1: both W2 of one pair
constexpr int kRestRegion = 1880;       // phase 2: the other 1875 values + dump slot
static_assert(sizeof(MfmaLds) >= NPAIR * kW2Region * sizeof(float), "reduction overlay");

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// lanes of a wavefront exchange data through LDS between these points
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ---- bf16x3 operands --------------------------------------------------------
// x = hi + lo + e with hi = bf16(x), lo = bf16(x - hi) (both round to nearest
// even; x - hi is exact), |lo| <= 2^-8 |x|, |e| <= 2^-17 |x|; a product is
// hi*hi + hi*lo + lo*hi in three bf16 MFMAs (f32 accumulate), dropping lo*lo:
// relative error <= ~2^-15 per product against exact f32's 2^-24, at 3/16 of
// the f32 MFMA's cycles per flop (MI355X_MICROARCH.md cycle constants: 16
// cycles per 16x16x32 bf16, 32 per 16x16x4 f32).
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef float f2v __attribute__((ext_vector_type(2)));
typedef __bf16 b2v __attribute__((ext_vector_type(2)));

// (hi(a), hi(b)) and (lo(a), lo(b)) packed, a in the low halves
__device__ __forceinline__ void bf_split2(float a, float b, uint32_t& hi, uint32_t& lo) {
    hi = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a, b}, b2v));
    const float ha = __uint_as_float(hi << 16), hb = __uint_as_float(hi & 0xFFFF0000u);
    lo = __builtin_bit_cast(uint32_t, __builtin_convertvector((f2v){a - ha, b - hb}, b2v));
}

// The k order of a 64-long contraction in two 16x16x32 steps s: element e of
// lane group g is unit u(s,g,e) = 16(2s + e/4) + 4g + e%4, so that a
// transposed tile in MFMA accumulator layout (lane (c,g) holds rows 4g+r of
// 16-row tile J) is the B operand with no lane movement: elements 0..3 =
// tile 2s, rows 4g..4g+3; 4..7 = tile 2s+1.  wpos(u) = 32s + 8g + e puts a
// lane's 8 elements of a W2 row next to each other.
__device__ __forceinline__ int wpos(int u) {
    return (u & 32) | (((u >> 2) & 3) << 3) | (((u >> 4) & 1) << 2) | (u & 3);
}

__device__ __forceinline__ void split_frag(const f4 v[4], int s, bf8& hi, bf8& lo) {
    u4v h, l;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const int J = 2 * s + (d >> 1), r = 2 * (d & 1);
        uint32_t hh, ll;
        bf_split2(v[J][r], v[J][r + 1], hh, ll);
        h[d] = hh;
        l[d] = ll;
    }
    hi = __builtin_bit_cast(bf8, h);
    lo = __builtin_bit_cast(bf8, l);
}

__device__ __forceinline__ f4 mfma3(bf8 ah, bf8 al, bf8 bh, bf8 bl, f4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

// A operand W2[16J + c][u(s,g,.)] of image img: one 16-B row read
__device__ __forceinline__ bf8 w2_row_frag(const uint16_t* img, int J, int s, int c, int g) {
    return *reinterpret_cast<const bf8*>(img + (16 * J + c) * WBP + 32 * s + 8 * g);
}

// A operand W2^T[16I + c][u(s,g,.)] = W2[u(s,g,e)][16I + c]: two transposed
// reads (ds_read_b64_tr_b16, 4 rows x 16 columns per 16-lane group; lane
// 4q+p of the group addresses row q, columns 16I+4p..+3).  EXEC must be full.
typedef __attribute__((address_space(3))) s4v* lds_s4_t;
__device__ __forceinline__ bf8 w2_col_frag(const uint16_t* img, int I, int s, int c, int g) {
    const int q = c >> 2, p = c & 3;
    const uint16_t* a = img + (32 * s + 4 * g + q) * WBP + 32 * (I >> 1) + 8 * p + 4 * (I & 1);
    const s4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(a));
    const s4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(a + 16 * WBP));
    return __builtin_bit_cast(bf8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
__device__ __forceinline__ float el(const float4& v, int r) { return r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w; }

// tanh(x) = 1 - 2 / (exp(2x) + 1) on v_exp_f32 + v_rcp_f32 (1 ulp each; the
// file's correctly-rounded-division flag would expand a plain reciprocal into
// an 11-instruction division): 5 VALU, branch-free, exact limits (+-1, no
// overflow NaN), absolute error <= ~1.2e-7 everywhere -- relative error grows
// near 0, where only the absolute error reaches the next layer's products and
// 1 - h^2.  The update need not be bit-exact: ratio = exp(new - old logprob)
// moves by ~1e-6 (tests/test_gpu_trainer.py compares against f64 autograd).
__device__ __forceinline__ float tanh_fast(float x) {
    const float e = __builtin_amdgcn_exp2f(x * 2.88539008177792681f);  // e^(2x)
    return __builtin_fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}

__device__ __forceinline__ float sum16(float v) {  // over the 16 lanes c of one g-group
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// index of a parameter in the phase-2 reduction region (everything but the two W2)
__device__ __forceinline__ int rest_slot(int p) {
    return p < O_AW2 ? p : (p < O_CW2 ? O_AW2 + (p - O_AB2) : O_AW2 + (O_CW2 - O_AB2) + (p - O_CB2));
}
constexpr int kRestDump = 1875;

typedef __attribute__((address_space(1))) void* glb_ptr_t;
typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Copy the inputs of tile t (16 minibatch rows: obs, and the actor's actions,
// logp, adv or the critic's returns, values) into the wave's `in` buffer with
// async global->LDS loads (no VGPRs; completion by vmcnt).  The buffer is
// sample-minor ([column][16 samples]), so lane l always copies sample l & 15
// and needs one row index.  Samples past the minibatch read row 0: finite,
// and their loss terms are masked by `live`.
template <int HEAD>
__device__ __forceinline__ void mf_prefetch(const GradParams& P, float* in, int t, int lane) {
    const int m = t * 16 + (lane & 15), hi = lane >> 4;
    const int64_t r = m < P.mb ? P.idx[m] : 0;
    const float* ob = P.obs + r * NOBS + hi;
    __builtin_amdgcn_global_load_lds((glb_ptr_t)ob, (lds_ptr_t)(in + IN_OBS), 4, 0, 0);             // columns 0..3
    __builtin_amdgcn_global_load_lds((glb_ptr_t)(ob + 4), (lds_ptr_t)(in + IN_OBS + 64), 4, 0, 0);  // 4..7
    if (lane < 16) __builtin_amdgcn_global_load_lds((glb_ptr_t)(ob + 8), (lds_ptr_t)(in + IN_OBS + 128), 4, 0, 0);
    if constexpr (HEAD == 0) {
        const float* ac = P.act + r * NACT + hi;
        __builtin_amdgcn_global_load_lds((glb_ptr_t)ac, (lds_ptr_t)(in + IN_ACT), 4, 0, 0);  // columns 0..3
        if (lane < 32) {
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(ac + 4), (lds_ptr_t)(in + IN_ACT + 64), 4, 0, 0);  // 4, 5
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(lane < 16 ? P.logp + r : P.adv + r),
                                             (lds_ptr_t)(in + IN_LOGP), 4, 0, 0);
        }
    } else {
        if (lane < 32)
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(lane < 16 ? P.ret + r : P.val + r), (lds_ptr_t)(in + IN_RET),
                                             4, 0, 0);
    }
}

// ---- bf16x3 dW2: the sum over the tile's 16 samples in v_mfma_f32_16x16x16_bf16
// (lane l: A[l&15][k = 4(l>>4) + j], B[k][l&15]).  G2^T and H1^T go through
// [sample][unit] bf16 images (hi at img, lo at img + IMG_FL; rows of IMG_RS
// elements = 136 B: the lanes' 8-B stores conflict-free, the transposed reads
// 2-way) and come back as 4-sample fragments by ds_read_b64_tr_b16.
constexpr int IMG_RS = 68, IMG_FL = 16 * IMG_RS;
static_assert(2 * IMG_FL * 2 <= 64 * SP * 4, "an image pair fits a 64-row scratch region");

// lane (c,g) stores units 4g..4g+3 of tiles 2s, 2s+1 of sample c: the packed
// dwords split_frag made (dwords 0,1: tile 2s; 2,3: tile 2s+1)
__device__ __forceinline__ void put_img(uint16_t* img, const bf8 hi[2], const bf8 lo[2], int c, int g) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const u4v h = __builtin_bit_cast(u4v, hi[s]), l = __builtin_bit_cast(u4v, lo[s]);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
            uint16_t* a = img + c * IMG_RS + 16 * (2 * s + half) + 4 * g;
            *reinterpret_cast<uint2*>(a) = make_uint2(h[2 * half], h[2 * half + 1]);
            *reinterpret_cast<uint2*>(a + IMG_FL) = make_uint2(l[2 * half], l[2 * half + 1]);
        }
    }
}

// X^T[16J + c][samples 4g..4g+3] from X's [sample][unit] image (16-lane group
// g: lane 4q+p addresses sample 4g+q, units 16J+4p..+3; lane i receives unit 16J+i)
__device__ __forceinline__ s4v img_frag(const uint16_t* img, int J, int c, int g) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4_t)(img + (4 * g + (c >> 2)) * IMG_RS + 16 * J + 4 * (c & 3)));
}

__device__ __forceinline__ f4 mfma3k16(s4v ah, s4v al, s4v bh, s4v bl, f4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(al, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ah, bh, c, 0, 0, 0);
}

// X^T of the augmented first layer (row NOBS = the bias input 1, rows above 0)
__device__ __forceinline__ float xin(const float* in, int row, int smp) {
    return row < NOBS ? in[IN_OBS + row * 16 + smp] : (row == NOBS ? 1.0f : 0.0f);
}

// forward of this wave's trunk for its tile: h1, h2 = tanh layers, transposed tiles
template <int PREC>
__device__ __forceinline__ void mf_fwd(const MfmaLds& S, int h, const float* in, int c, int g, f4 h1[4], f4 h2[4],
                                       uint16_t* img_h1) {
#pragma clang fp contract(fast)
    float xb[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) xb[q] = xin(in, 4 * q + g, c);
#pragma unroll
    for (int J = 0; J < 4; ++J) {
        f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int q = 0; q < 3; ++q) z = mfma4(S.w1[h][(16 * J + c) * W1P + 4 * q + g], xb[q], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) h1[J][r] = tanh_fast(z[r]);
    }
    if constexpr (PREC == kPrecBf16x3) {
        bf8 bh[2], bl[2];
        split_frag(h1, 0, bh[0], bl[0]);
        split_frag(h1, 1, bh[1], bl[1]);
        put_img(img_h1, bh, bl, c, g);  // dW2's H1 operand (read after later wave_syncs)
#pragma unroll
        for (int J = 0; J < 4; ++J) {
            f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int s = 0; s < 2; ++s)
                z = mfma3(w2_row_frag(S.w2b[h][0], J, s, c, g), w2_row_frag(S.w2b[h][1], J, s, c, g), bh[s], bl[s],
                          z);
            const float4 b = ld4(&S.b2[h][16 * J + 4 * g]);
#pragma unroll
            for (int r = 0; r < 4; ++r) h2[J][r] = tanh_fast(z[r] + el(b, r));
        }
        return;
    }
#pragma unroll
    for (int J = 0; J < 4; ++J) {
        f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int T = 0; T < 4; ++T) {
            const float4 a = ld4(&S.w2[h][(16 * J + c) * WP + 16 * T + 4 * g]);
            z = mfma4(a.x, h1[T][0], z);
            z = mfma4(a.y, h1[T][1], z);
            z = mfma4(a.z, h1[T][2], z);
            z = mfma4(a.w, h1[T][3], z);
        }
        const float4 b = ld4(&S.b2[h][16 * J + 4 * g]);
#pragma unroll
        for (int r = 0; r < 4; ++r) h2[J][r] = tanh_fast(z[r] + el(b, r));
    }
}

// per-role accumulators of one wave
template <int HEAD>
struct Acc {
    f4 d2[4][4];       // dW2[16J+4g+r][16T+c]
    f4 d1[4];          // [dW1 | db1][16J+4g+r][c]
    f4 d3[4];          // actor: dW3[4g+r][16J+c] (rows < 6); critic: per-lane dW3 partial [16J+4g+r]
    float db2[16];     // per-lane partial db2[16J+4g+r]
    float sc[HEAD == 0 ? 2 * NACT + 5 : 2];  // actor: db3[6], dlogstd[6], pg, ent, -lr, r-1-lr, clipped; critic: db3, vl
};

// ---- the phases of one 16-sample tile for one head (mf_tile runs them for
// the wave's head).  LDS scratch rows are exchanged between the lanes of the
// wave only at wave_sync points.
#define RT_FP_FAST _Pragma("clang fp contract(fast)")

// head outputs and the per-sample loss derivative w.r.t. them (train.py:200-236)
template <int HEAD>
__device__ __forceinline__ void ph_out_loss(const MfmaLds& S, const GradParams& P, const float* in, int c, int g,
                                            bool live, float inv_n, const f4 h2[4], Acc<HEAD>& acc,
                                            float go[HEAD == 0 ? NACT : 1]) {
    RT_FP_FAST
    constexpr int NOUT = HEAD == 0 ? NACT : 1;
    // partial dots over this lane's 16 units, summed over the sample's 4 g-lanes
    float out[NOUT];
#pragma unroll
    for (int o = 0; o < NOUT; ++o) {
        const int wr = HEAD == 0 ? o : NACT;
        float p = 0.0f;
#pragma unroll
        for (int J = 0; J < 4; ++J) {
            const float4 w = ld4(&S.w3[wr * H + 16 * J + 4 * g]);
            p += w.x * h2[J][0] + w.y * h2[J][1] + w.z * h2[J][2] + w.w * h2[J][3];
        }
        p += __shfl_xor(p, 16, 64);
        p += __shfl_xor(p, 32, 64);
        out[o] = p + S.b3[wr];
    }
#pragma unroll
    for (int o = 0; o < NOUT; ++o) go[o] = 0.0f;
    if (!live) return;
    if constexpr (HEAD == 0) {
        float z[NACT], logp = 0.0f, ent = 0.0f;
#pragma unroll
        for (int k = 0; k < NACT; ++k) {
            z[k] = (in[IN_ACT + k * 16 + c] - out[k]) * S.isd[k];
            logp += -0.5f * z[k] * z[k] - S.ls[k] - kHalfLog2Pi;
            ent += 0.5f + kHalfLog2Pi + S.ls[k];
        }
        const float lr = logp - in[IN_LOGP + c];
        const float r = __expf(lr);
        float Av = in[IN_ADV + c];
        if (P.adv_stats) Av = (Av - P.adv_stats[0]) * S.isd[NACT];
        const float pg1 = -Av * r;
        const float rc = fminf(fmaxf(r, P.clip_lo), P.clip_hi);
        const float pg2 = -Av * rc;
        // torch.maximum backward: the larger input takes the gradient, ties split it
        const float w1 = pg1 > pg2 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
        const float w2 = pg2 > pg1 ? 1.0f : (pg1 == pg2 ? 0.5f : 0.0f);
        const float pass = (r >= P.clip_lo && r <= P.clip_hi) ? 1.0f : 0.0f;  // clamp backward
        const float g_logp = inv_n * (w1 * -Av + w2 * -Av * pass) * r;
#pragma unroll
        for (int k = 0; k < NACT; ++k) go[k] = g_logp * z[k] * S.isd[k];
        if (g == 0) {  // one contribution per sample
#pragma unroll
            for (int k = 0; k < NACT; ++k) {
                acc.sc[k] += go[k];
                acc.sc[NACT + k] += g_logp * (z[k] * z[k] - 1.0f);
            }
            acc.sc[2 * NACT + 0] += fmaxf(pg1, pg2);
            acc.sc[2 * NACT + 1] += ent;
            acc.sc[2 * NACT + 2] += -lr;
            acc.sc[2 * NACT + 3] += (r - 1.0f) - lr;
            acc.sc[2 * NACT + 4] += fabsf(r - 1.0f) > P.clip ? 1.0f : 0.0f;
        }
    } else {
        const float value = out[0];
        const float R = in[IN_RET + c], V = in[IN_VAL + c];
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
        go[0] = P.vf_coef * 0.5f * inv_n * dv;
        if (g == 0) {
            acc.sc[0] += go[0];
            acc.sc[1] += vl;
        }
    }
}

// actor: GM^T -> scratch, H2^T -> A (read back after a wave_sync by ph_dw3)
template <int HEAD>
__device__ __forceinline__ void ph_dw3_pre(float* A, float* GMs, const f4 h2[4], const float* go, int c, int g) {
    if constexpr (HEAD == 0) {
        for (int o = g; o < NACT; o += 4) GMs[o * SP + c] = go[o];
#pragma unroll
        for (int J = 0; J < 4; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) A[(16 * J + 4 * g + r) * SP + c] = h2[J][r];
    }
}

// dW3 += GM^T . H2 over the tile's samples (actor, MFMA); critic: per-lane partials
template <int HEAD>
__device__ __forceinline__ void ph_dw3(const float* A, const float* GMs, const f4 h2[4], const float* go, int c, int g,
                                       Acc<HEAD>& acc) {
    RT_FP_FAST
    if constexpr (HEAD == 0) {
        const float4 ga = c < NACT ? ld4(&GMs[c * SP + 4 * g]) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
        for (int J = 0; J < 4; ++J) {
            const float4 bq = ld4(&A[(16 * J + c) * SP + 4 * g]);
            acc.d3[J] = mfma4(ga.x, bq.x, acc.d3[J]);
            acc.d3[J] = mfma4(ga.y, bq.y, acc.d3[J]);
            acc.d3[J] = mfma4(ga.z, bq.z, acc.d3[J]);
            acc.d3[J] = mfma4(ga.w, bq.w, acc.d3[J]);
        }
    } else {
#pragma unroll
        for (int J = 0; J < 4; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc.d3[J][r] += go[0] * h2[J][r];
    }
}

// G2^T = (W3^T go) * (1 - H2^2); db2 += G2
template <int HEAD>
__device__ __forceinline__ void ph_g2(const MfmaLds& S, const float* go, const f4 h2[4], int g, Acc<HEAD>& acc,
                                      f4 g2[4]) {
    RT_FP_FAST
    constexpr int NOUT = HEAD == 0 ? NACT : 1;
#pragma unroll
    for (int J = 0; J < 4; ++J) {
        f4 a = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int o = 0; o < NOUT; ++o) {
            const float4 w = ld4(&S.w3[(HEAD == 0 ? o : NACT) * H + 16 * J + 4 * g]);
            a[0] += w.x * go[o];
            a[1] += w.y * go[o];
            a[2] += w.z * go[o];
            a[3] += w.w * go[o];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            g2[J][r] = a[r] * (1.0f - h2[J][r] * h2[J][r]);
            acc.db2[4 * J + r] += g2[J][r];
        }
    }
}

// transposed tiles -> scratch rows [unit][16 samples]
__device__ __forceinline__ void ph_put(float* A, const f4 v[4], int c, int g) {
#pragma unroll
    for (int J = 0; J < 4; ++J)
#pragma unroll
        for (int r = 0; r < 4; ++r) A[(16 * J + 4 * g + r) * SP + c] = v[J][r];
}

// dW2 += G2^T . H1 over the tile's samples (G2^T in A, H1^T in Bs)
template <int HEAD>
__device__ __forceinline__ void ph_dw2(const float* A, const float* Bs, int c, int g, Acc<HEAD>& acc) {
    float4 a[4], bq[4];
#pragma unroll
    for (int J = 0; J < 4; ++J) {
        a[J] = ld4(&A[(16 * J + c) * SP + 4 * g]);
        bq[J] = ld4(&Bs[(16 * J + c) * SP + 4 * g]);
    }
#pragma unroll
    for (int J = 0; J < 4; ++J)
#pragma unroll
        for (int T = 0; T < 4; ++T) {
            acc.d2[J][T] = mfma4(a[J].x, bq[T].x, acc.d2[J][T]);
            acc.d2[J][T] = mfma4(a[J].y, bq[T].y, acc.d2[J][T]);
            acc.d2[J][T] = mfma4(a[J].z, bq[T].z, acc.d2[J][T]);
            acc.d2[J][T] = mfma4(a[J].w, bq[T].w, acc.d2[J][T]);
        }
}

// G1^T = (W2^T . G2^T) * (1 - H1^2)   (A operand W2[16J+4g+r][16I+c])
template <int HEAD>
__device__ __forceinline__ void ph_g1(const MfmaLds& S, const f4 g2[4], const f4 h1[4], int c, int g, f4 g1[4]) {
    RT_FP_FAST
#pragma unroll
    for (int I = 0; I < 4; ++I) {
        f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int J = 0; J < 4; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) z = mfma4(S.w2[HEAD][(16 * J + 4 * g + r) * WP + 16 * I + c], g2[J][r], z);
#pragma unroll
        for (int r = 0; r < 4; ++r) g1[I][r] = z[r] * (1.0f - h1[I][r] * h1[I][r]);
    }
}

// bf16x3 G1: the B operand G2^T split once (gh, gl; also the dW2 image)
template <int HEAD>
__device__ __forceinline__ void ph_g1_b(const MfmaLds& S, const bf8 gh[2], const bf8 gl[2], const f4 h1[4], int c,
                                        int g, f4 g1[4]) {
    RT_FP_FAST
#pragma unroll
    for (int I = 0; I < 4; ++I) {
        f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < 2; ++s)
            z = mfma3(w2_col_frag(S.w2b[HEAD][0], I, s, c, g), w2_col_frag(S.w2b[HEAD][1], I, s, c, g), gh[s], gl[s],
                      z);
#pragma unroll
        for (int r = 0; r < 4; ++r) g1[I][r] = z[r] * (1.0f - h1[I][r] * h1[I][r]);
    }
}

// dW2 += G2^T . H1 over the tile's samples; acc.d2[J][T] as in ph_dw2
template <int HEAD>
__device__ __forceinline__ void ph_dw2_b(const uint16_t* ig, const uint16_t* ih, int c, int g, Acc<HEAD>& acc) {
    s4v ah[4], al[4], bh[4], bl[4];
#pragma unroll
    for (int J = 0; J < 4; ++J) {
        ah[J] = img_frag(ig, J, c, g);
        al[J] = img_frag(ig + IMG_FL, J, c, g);
        bh[J] = img_frag(ih, J, c, g);
        bl[J] = img_frag(ih + IMG_FL, J, c, g);
    }
#pragma unroll
    for (int J = 0; J < 4; ++J)
#pragma unroll
        for (int T = 0; T < 4; ++T) acc.d2[J][T] = mfma3k16(ah[J], al[J], bh[T], bl[T], acc.d2[J][T]);
}

// [dW1 | db1] += G1^T . [X | 1]   (G1^T in A)
template <int HEAD>
__device__ __forceinline__ void ph_dw1(const float* A, const float xd[4], int c, int g, Acc<HEAD>& acc) {
#pragma unroll
    for (int J = 0; J < 4; ++J) {
        const float4 a = ld4(&A[(16 * J + c) * SP + 4 * g]);
        acc.d1[J] = mfma4(a.x, xd[0], acc.d1[J]);
        acc.d1[J] = mfma4(a.y, xd[1], acc.d1[J]);
        acc.d1[J] = mfma4(a.z, xd[2], acc.d1[J]);
        acc.d1[J] = mfma4(a.w, xd[3], acc.d1[J]);
    }
}

// [X | 1] operand of the dW1 product (samples 4g..4g+3 of input row c)
__device__ __forceinline__ void load_xd(const float* in, int c, int g, float xd[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) xd[k] = xin(in, c, 4 * g + k);
}

template <int HEAD, int PREC>
__device__ __forceinline__ void mf_tile(const MfmaLds& S, const GradParams& P, float* A, float* Bs, float* in,
                                        float* GMs, int c, int g, int t, int t_next, float inv_n, Acc<HEAD>& acc) {
    constexpr int NOUT = HEAD == 0 ? NACT : 1;
    const bool live = t * 16 + c < P.mb;
    __builtin_amdgcn_s_waitcnt(0);  // this tile's inputs (LDS DMA issued during the previous tile) have landed
    wave_sync();  // ... and the previous tile's reads of the scratch are done
    f4 h1[4], h2[4];
    // bf16x3: the H1 images over B, the G2 images over A once dW3 is done with it
    uint16_t* const img_h1 = reinterpret_cast<uint16_t*>(Bs);
    uint16_t* const img_g2 = reinterpret_cast<uint16_t*>(A);
    mf_fwd<PREC>(S, HEAD, in, c, g, h1, h2, img_h1);
    float xd[4];  // read now: `in` is refilled below
    load_xd(in, c, g, xd);
    float go[NOUT];
    ph_out_loss<HEAD>(S, P, in, c, g, live, inv_n, h2, acc, go);
    // every read of `in` for this tile is done (xd and the loss inputs are in
    // registers): stream the next tile's inputs in beside the backward
    if (t_next >= 0) {
        asm volatile("" ::"v"(xd[0]), "v"(xd[1]), "v"(xd[2]), "v"(xd[3]));
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the LDS reads have returned
        mf_prefetch<HEAD>(P, in, t_next, 16 * g + c);
    }
    ph_dw3_pre<HEAD>(A, GMs, h2, go, c, g);
    if constexpr (HEAD == 0) wave_sync();
    ph_dw3<HEAD>(A, GMs, h2, go, c, g, acc);
    f4 g2[4];
    ph_g2<HEAD>(S, go, h2, g, acc, g2);
    f4 g1[4];
    if constexpr (PREC == kPrecBf16x3) {
        bf8 gh[2], gl[2];
        split_frag(g2, 0, gh[0], gl[0]);
        split_frag(g2, 1, gh[1], gl[1]);
        if constexpr (HEAD == 0) wave_sync();  // dW3's reads of A are done
        put_img(img_g2, gh, gl, c, g);
        wave_sync();
        ph_dw2_b<HEAD>(img_g2, img_h1, c, g, acc);
        ph_g1_b<HEAD>(S, gh, gl, h1, c, g, g1);
    } else {
        wave_sync();
        ph_put(A, g2, c, g);
        ph_put(Bs, h1, c, g);
        wave_sync();
        ph_dw2<HEAD>(A, Bs, c, g, acc);
        ph_g1<HEAD>(S, g2, h1, c, g, g1);
    }
    wave_sync();
    ph_put(A, g1, c, g);
    wave_sync();
    ph_dw1<HEAD>(A, xd, c, g, acc);
}

template <int HEAD, int PREC>
__device__ __forceinline__ void mf_wave(MfmaLds& S, const GradParams& P, int pair, int lane) {
    const int c = lane & 15, g = lane >> 4;
    float* A = S.scr[2 * pair + HEAD];
    float* Bs = A + 64 * SP;
    float* GMs = A + 128 * SP;
    float* in = S.in[2 * pair + HEAD];
    Acc<HEAD> acc;
    const f4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int J = 0; J < 4; ++J) {
#pragma unroll
        for (int T = 0; T < 4; ++T) acc.d2[J][T] = zero;
        acc.d1[J] = acc.d3[J] = zero;
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) acc.db2[k] = 0.0f;
#pragma unroll
    for (int k = 0; k < (int)(sizeof(acc.sc) / sizeof(float)); ++k) acc.sc[k] = 0.0f;
    const float inv_n = 1.0f / (float)P.mb;
    const int ntiles = (P.mb + 15) / 16;
    const int tw = blockIdx.x * (MT / 64) + 2 * pair + HEAD;  // trace row of this wave
    (void)tw;  // used by RT_STAMP in trace builds only
    int nt_done = 0;
    const int tstep = gridDim.x * NPAIR;
    for (int t = blockIdx.x * NPAIR + pair; t < ntiles; t += tstep) {
        mf_tile<HEAD, PREC>(S, P, A, Bs, in, GMs, c, g, t, t + tstep < ntiles ? t + tstep : -1, inv_n, acc);
        if (lane == 0 && nt_done++ == 0) RT_STAMP(tw, 6);
    }
    if (lane == 0) RT_STAMP(tw, 2);

    // ---- per-lane partials reduced over the 16 samples c of each g-group
#pragma unroll
    for (int k = 0; k < 16; ++k) acc.db2[k] = sum16(acc.db2[k]);
    if constexpr (HEAD == 1) {
#pragma unroll
        for (int J = 0; J < 4; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc.d3[J][r] = sum16(acc.d3[J][r]);
    }
#pragma unroll
    for (int k = 0; k < (int)(sizeof(acc.sc) / sizeof(float)); ++k) acc.sc[k] = sum16(acc.sc[k]);
    if (lane == 0) RT_STAMP(tw, 3);
    __syncthreads();
    // ---- phase 1: both W2 of every pair in its own region, summed in pair order
    float* R = reinterpret_cast<float*>(&S);
    {
        float* Rp = R + pair * kW2Region + HEAD * H * H;
#pragma unroll
        for (int J = 0; J < 4; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int T = 0; T < 4; ++T) Rp[(16 * J + 4 * g + r) * H + 16 * T + c] = acc.d2[J][T][r];
    }
    __syncthreads();
    float* out = P.ws + (size_t)blockIdx.x * PSTRIDE;
    const int tid = threadIdx.x;
    // float4 per lane (O_AW2, O_CW2 and PSTRIDE are multiples of 4), stored
    // write-through: the 32 KB of W2 partials per block leave the XCD's L2
    // during the kernel instead of as dirty lines the boundary to the
    // reduction writes back (MI355X_MICROARCH.md, boundary / publish-large)
    static_assert(O_AW2 % 4 == 0 && O_CW2 % 4 == 0 && PSTRIDE % 4 == 0, "float4 partial rows");
    const __amdgpu_buffer_rsrc_t wsrd = __builtin_amdgcn_make_buffer_rsrc(out, 0, PSTRIDE * 4, 0x00020000);
    for (int q = 4 * tid; q < kW2Region; q += 4 * MT) {
        f4 v = *reinterpret_cast<const f4*>(R + q);
#pragma unroll
        for (int pp = 1; pp < NPAIR; ++pp) v += *reinterpret_cast<const f4*>(R + pp * kW2Region + q);
        const int o = (q < H * H ? O_AW2 : O_CW2 - H * H) + q;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), wsrd, 4 * o, 0, 16);  // aux 16: sc1
    }
    if (lane == 0) RT_STAMP(tw, 4);
    __syncthreads();
    // ---- phase 2: everything else (1875 values), same scheme
    {
        float* Rp = R + pair * kRestRegion;
        constexpr int o_w1 = HEAD == 0 ? O_AW1 : O_CW1, o_b1 = HEAD == 0 ? O_AB1 : O_CB1;
        constexpr int o_b2 = HEAD == 0 ? O_AB2 : O_CB2;
#pragma unroll
        for (int J = 0; J < 4; ++J)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int j = 16 * J + 4 * g + r;
                Rp[c < NOBS ? rest_slot(o_w1 + j * NOBS + c) : (c == NOBS ? rest_slot(o_b1 + j) : kRestDump)] =
                    acc.d1[J][r];
                if constexpr (HEAD == 0) {
                    const int o = 4 * g + r;
                    Rp[o < NACT ? rest_slot(O_AW3 + o * H + 16 * J + c) : kRestDump] = acc.d3[J][r];
                } else {
                    Rp[c == 0 ? rest_slot(O_CW3 + j) : kRestDump] = acc.d3[J][r];
                }
                Rp[c == 0 ? rest_slot(o_b2 + j) : kRestDump] = acc.db2[4 * J + r];
            }
        if (lane == 0) {
            if constexpr (HEAD == 0) {
#pragma unroll
                for (int k = 0; k < NACT; ++k) {
                    Rp[rest_slot(O_AB3 + k)] = acc.sc[k];
                    Rp[rest_slot(O_LS + k)] = acc.sc[NACT + k];
                }
                Rp[rest_slot(NP + 0)] = acc.sc[2 * NACT + 0];
                Rp[rest_slot(NP + 2)] = acc.sc[2 * NACT + 1];
                Rp[rest_slot(NP + 3)] = acc.sc[2 * NACT + 2];
                Rp[rest_slot(NP + 4)] = acc.sc[2 * NACT + 3];
                Rp[rest_slot(NP + 5)] = acc.sc[2 * NACT + 4];
            } else {
                Rp[rest_slot(O_CB3)] = acc.sc[0];
                Rp[rest_slot(NP + 1)] = acc.sc[1];
            }
        }
    }
    __syncthreads();
    for (int q = tid; q < kRestDump; q += MT) {
        float v = R[q];
#pragma unroll
        for (int pp = 1; pp < NPAIR; ++pp) v += R[pp * kRestRegion + q];
        const int p = q < O_AW2 ? q : (q < O_AW2 + (O_CW2 - O_AB2) ? q - O_AW2 + O_AB2 : q - O_AW2 - (O_CW2 - O_AB2) + O_CB2);
        out[p] = v;
    }
    if (lane == 0) RT_STAMP(tw, 5);
}

template <int PREC>
__global__ __launch_bounds__(MT) void k_ppo_grad_mfma(GradParams P) {
    __shared__ __attribute__((aligned(16))) MfmaLds S;
    const int tid = threadIdx.x;
    if ((tid & 63) == 0) RT_STAMP(blockIdx.x * (MT / 64) + (tid >> 6), 0);
    // parameter staging: every parameter load is issued before the first wait,
    // so the staging costs one memory round trip (loop-by-loop staging waited
    // ~10 times: 4.8 us per launch)
    constexpr int NW2 = H * H / MT, NW1 = (H * W1P + MT - 1) / MT;
    float w2v[2][NW2], w1v[2][NW1];
    // f32: element tid + MT u; bf16x3: the pair 2 (tid + MT u'), u' < NW2 / 2
#pragma unroll
    for (int u = 0; u < NW2; ++u) {
        const int f = PREC == kPrecF32 ? tid + MT * u : 2 * (tid + MT * (u >> 1)) + (u & 1);
        w2v[0][u] = P.w.p[2][f];
        w2v[1][u] = P.w.p[9][f];
    }
#pragma unroll
    for (int u = 0; u < NW1; ++u) {
        const int i = tid + MT * u, j = i / W1P, k = i % W1P;
        const bool in = i < H * W1P;
        w1v[0][u] = in && k < NOBS ? P.w.p[0][j * NOBS + k] : (in && k == NOBS ? P.w.p[1][j] : 0.0f);
        w1v[1][u] = in && k < NOBS ? P.w.p[7][j * NOBS + k] : (in && k == NOBS ? P.w.p[8][j] : 0.0f);
    }
    float b2a = 0.0f, b2c = 0.0f, w3c = 0.0f, w3a = 0.0f, b3v = 0.0f, lsv = 0.0f, advsd = 0.0f;
    if (tid < H) {
        b2a = P.w.p[3][tid];
        b2c = P.w.p[10][tid];
        w3c = P.w.p[11][tid];
    }
    if (tid < NACT * H) w3a = P.w.p[4][tid];
    if (tid < NACT) {
        b3v = P.w.p[5][tid];
        lsv = P.w.p[6][tid];
    }
    if (tid == NACT) {
        b3v = P.w.p[12][0];
        advsd = P.adv_stats ? P.adv_stats[1] : 0.0f;
    }
    {  // the first tile's inputs stream in while the parameters are staged
        const int wave = tid >> 6, pair = wave & 3, t0 = blockIdx.x * NPAIR + pair;
        if (t0 < (P.mb + 15) / 16) {
            if (wave >= 4)
                mf_prefetch<1>(P, S.in[2 * pair + 1], t0, tid & 63);
            else
                mf_prefetch<0>(P, S.in[2 * pair], t0, tid & 63);
        }
    }
    if constexpr (PREC == kPrecF32) {
#pragma unroll
        for (int u = 0; u < NW2; ++u) {
            const int i = tid + MT * u;
            S.w2[0][(i >> 6) * WP + (i & 63)] = w2v[0][u];
            S.w2[1][(i >> 6) * WP + (i & 63)] = w2v[1][u];
        }
    } else {
#pragma unroll
        for (int u = 0; u < NW2; u += 2) {
            const int f = 2 * (tid + MT * (u >> 1)), o = (f >> 6) * WBP + wpos(f & 63);  // wpos(i + 1) = wpos(i) + 1
#pragma unroll
            for (int hd = 0; hd < 2; ++hd) {
                uint32_t hh, ll;
                bf_split2(w2v[hd][u], w2v[hd][u + 1], hh, ll);
                *reinterpret_cast<uint32_t*>(&S.w2b[hd][0][o]) = hh;
                *reinterpret_cast<uint32_t*>(&S.w2b[hd][1][o]) = ll;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < NW1; ++u) {
        const int i = tid + MT * u;
        if (i < H * W1P) {
            S.w1[0][i] = w1v[0][u];
            S.w1[1][i] = w1v[1][u];
        }
    }
    if (tid < H) {
        S.b2[0][tid] = b2a;
        S.b2[1][tid] = b2c;
        S.w3[NACT * H + tid] = w3c;
    }
    if (tid < NACT * H) S.w3[tid] = w3a;
    if (tid < NACT) {
        S.b3[tid] = b3v;
        S.ls[tid] = lsv;
        S.isd[tid] = 1.0f / expf(lsv);
    }
    if (tid == NACT) {
        S.b3[NACT] = b3v;
        S.isd[NACT] = P.adv_stats ? 1.0f / (advsd + 1e-8f) : 1.0f;
    }
    __syncthreads();
    const int wave = tid >> 6, lane = tid & 63;
    if (lane == 0) RT_STAMP(blockIdx.x * (MT / 64) + wave, 1);
    // waves w and w + 4 share SIMD w (a 512-thread workgroup places two waves
    // per SIMD, in dispatch order): actors are waves 0..3, critics 4..7, so
    // every SIMD pairs an actor with a critic -- and the heavier actor is the
    // older wave, which wins VALU arbitration (MI355X_MICROARCH.md, two waves
    // per SIMD).  (wave & 1 as the role put both actors of two pairs on one SIMD.)
    if (wave >= 4)
        mf_wave<1, PREC>(S, P, wave & 3, lane);
    else
        mf_wave<0, PREC>(S, P, wave & 3, lane);
}

int grad_blocks(int mb) {
    const int tiles = (mb + 15) / 16;
    const int b = (tiles + NPAIR - 1) / NPAIR;
    return b < kMaxGradBlocks ? b : kMaxGradBlocks;
}

constexpr int kReduceCols = 64;
constexpr int kReduceBlocks = (NP + NSTAT + kReduceCols - 1) / kReduceCols;
constexpr int kNormSlots = 256;  // grad-norm partials at the workspace tail
static_assert(kReduceBlocks <= kNormSlots, "norm partials");

struct ReduceParams {
    const float* ws;
    int32_t nblk;
    Dst13 grad;
    float* stats;        // [6]
    float* stats_accum;  // [6] or null
    float* norm_part;    // [kReduceBlocks] sum of squared gradients per block, or null
    float inv_n;
    float ent_coef;
};

// block: 64 columns; wave w of 16 sums rows w, w+16, ..., w+240 (all 16
// loads in flight, then a fixed-order pairwise sum; rows past nblk add 0); the
// 16 wave sums are combined in a fixed order (deterministic).  Also emits the
// block's share of ||grad||^2 for the clip in k_adam.
static_assert(kMaxGradBlocks <= 16 * 16, "k_ppo_reduce covers 256 partial rows");
__global__ __launch_bounds__(1024) void k_ppo_reduce(ReduceParams P) {
    __shared__ float part[16][kReduceCols];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int p = blockIdx.x * kReduceCols + lane;
    const bool ok = p < NP + NSTAT;
    float x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int b = w + 16 * k;
        x[k] = (ok && b < P.nblk) ? P.ws[(size_t)b * PSTRIDE + p] : 0.0f;
    }
#pragma unroll
    for (int h = 8; h > 0; h >>= 1)
#pragma unroll
        for (int k = 0; k < h; ++k) x[k] += x[k + h];
    part[w][lane] = x[0];
    __syncthreads();
    if (w != 0) return;
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) a += part[k][lane];
    float sq = 0.0f;
    if (ok) {
        if (p < NP) {
            int t = 0;
#pragma unroll
            for (int k = 1; k < 13; ++k) t += p >= kTensorOff[k] ? 1 : 0;
            if (t == 6) a += -P.ent_coef;  // d(-ent_coef * mean(entropy)) / d logstd
            P.grad.p[t][p - kTensorOff[t]] = a;
            sq = a * a;
        } else {
            const int k = p - NP;
            float v = a * P.inv_n;
            if (k == 1) v *= 0.5f;  // v_loss = 0.5 * mean(max(...))
            P.stats[k] = v;
            if (P.stats_accum) P.stats_accum[k] += v;
        }
    }
    sq = wave_sum(sq);
    if (lane == 0 && P.norm_part) P.norm_part[blockIdx.x] = sq;
}

// ||grad / div||^2 partials of a flat gradient after a data-parallel SUM
// all-reduce (div = world size: the average, torch's grad.div_(world))
__global__ __launch_bounds__(256) void k_gnorm(const float* g, int64_t n, int64_t per_block, float div,
                                               float* norm_part) {
    __shared__ float part[4];
    float a = 0.0f;
    const int64_t lo = (int64_t)blockIdx.x * per_block, hi = lo + per_block < n ? lo + per_block : n;
    for (int64_t i = lo + threadIdx.x; i < hi; i += 256) {
        const float x = div != 1.0f ? g[i] / div : g[i];
        a += x * x;
    }
    a = wave_sum(a);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = a;
    __syncthreads();
    if (threadIdx.x == 0) norm_part[blockIdx.x] = (part[0] + part[1]) + (part[2] + part[3]);
}

struct AdamParams {
    int64_t n;
    float* param;
    float* grad;
    float* m;
    float* v;
    const float* norm_part;  // [n_part] partial sums of squares
    int32_t n_part;
    float max_norm;  // <= 0: no clipping
    float lerp_w;    // 1 - beta1
    float beta2, one_minus_beta2;
    float step_size;  // -lr / (1 - beta1^t)
    float bc2_sqrt;   // sqrt(1 - beta2^t)
    float eps;
    float grad_div;   // the gradient is divided by this first (1: as is; world size: DP average)
};

// clip_grad_norm_ + torch.optim.Adam (foreach op order), one element per
// thread; every block sums the norm partials in the same fixed order
__global__ __launch_bounds__(256) void k_adam(AdamParams P) {
    __shared__ float coef_s;
    if (threadIdx.x < 64) {
        float t = 0.0f;
        if (P.max_norm > 0.0f)
            for (int k = threadIdx.x; k < P.n_part; k += 64) t += P.norm_part[k];
        t = wave_sum(t);
        // clip_grad_norm_: coef = max_norm / (||g|| + 1e-6), clamped to 1
        if (threadIdx.x == 0) coef_s = P.max_norm > 0.0f ? fminf(P.max_norm / (sqrtf(t) + 1e-6f), 1.0f) : 1.0f;
    }
    __syncthreads();
    const float coef = coef_s;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= P.n) return;
    const float g0 = P.grad_div != 1.0f ? P.grad[i] / P.grad_div : P.grad[i];  // IEEE division
    const float g = g0 * coef;
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

// ---- k_ppo_reduce + clip + Adam in one launch (rt_ppo_update) ---------------
// Every block reduces its 64 columns exactly as k_ppo_reduce does and stores
// them to the gradient; its ||g||^2 partial goes to norm_part[block] by an
// `sc1` store.  After the store has completed (s_waitcnt vmcnt(0)) ONE lane
// adds 1 to an arrival counter (agent scope) and polls it (`sc1` loads) until
// every block of the launch has arrived, then its wave reads the partials
// with `sc1` loads (MI355X_MICROARCH.md hand-off table, first row: no fence)
// and sums them in k_adam's order, so the clip coefficient is bitwise
// k_adam's; the wave then runs clip + Adam on the block's OWN columns only --
// no last-block serialisation (round 3's k_ppo_reduce_adam ran all 10,061
// updates in the last block and lost to the two kernels).  The
// kReduceBlocks blocks (16 waves, 4 KiB LDS each: >= 2 fit a CU) are all
// resident at once on an otherwise idle stream, so the wait completes; a
// bounded poll that runs out leaves the state untouched and raises a sticky
// host-visible flag (every later rt_ppo_* call returns RT_EDEVICE).
// rt_ppo_update checks once per device that the occupancy query admits the
// whole grid at once and otherwise runs k_ppo_reduce + k_adam instead.
// The counter (the workspace's last norm slot) is zeroed by rt_ppo_update
// before its first launch; launch i waits for (i + 1) * kReduceBlocks.
struct ReduceAdamParams {
    ReduceParams R;
    AdamParams A;
    int32_t flat_off[13];  // flat index of each tensor's first element (params_d[t] - flat_param_d)
    unsigned* counter;
    unsigned target;
    unsigned max_polls;  // the bounded wait (1 << 24; RT_PPO_FORCE_LOST_ARRIVAL: 16 and an unreachable target)
    int* fault;      // host-mapped sticky flag (reduce_adam_fault)
    int* dev_fault;  // the same event within this rt_ppo_update call, in device memory
};

__global__ __launch_bounds__(1024) void k_ppo_reduce_adam(ReduceAdamParams Q) {
    __shared__ float part[16][kReduceCols];
    const ReduceParams& P = Q.R;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int p = blockIdx.x * kReduceCols + lane;
    const bool ok = p < NP + NSTAT;
    float x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int b = w + 16 * k;
        x[k] = (ok && b < P.nblk) ? P.ws[(size_t)b * PSTRIDE + p] : 0.0f;
    }
#pragma unroll
    for (int h = 8; h > 0; h >>= 1)
#pragma unroll
        for (int k = 0; k < h; ++k) x[k] += x[k + h];
    part[w][lane] = x[0];
    __syncthreads();
    if (w != 0) return;
    float a = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) a += part[k][lane];
    float sq = 0.0f;
    int t = 0;
    if (ok) {
        if (p < NP) {
#pragma unroll
            for (int k = 1; k < 13; ++k) t += p >= kTensorOff[k] ? 1 : 0;
            if (t == 6) a += -P.ent_coef;  // d(-ent_coef * mean(entropy)) / d logstd
            sq = a * a;
        } else {
            const int k = p - NP;
            float v = a * P.inv_n;
            if (k == 1) v *= 0.5f;  // v_loss = 0.5 * mean(max(...))
            P.stats[k] = v;
            if (P.stats_accum) P.stats_accum[k] += v;
        }
    }
    sq = wave_sum(sq);
    const AdamParams& A = Q.A;
    // the block's own Adam state is loaded before the arrival wait (it does
    // not depend on the clip coefficient): one dependent load round fewer
    const bool upd = ok && p < NP;
    const int64_t i = upd ? Q.flat_off[t] + (p - kTensorOff[t]) : 0;
    float m0 = 0.0f, v0 = 0.0f, w0 = 0.0f;
    if (upd) {
        m0 = A.m[i];
        v0 = A.v[i];
        w0 = A.param[i];
    }
    if (lane == 0) {
        __hip_atomic_store(const_cast<float*>(A.norm_part) + blockIdx.x, sq, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(Q.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the arrival wait: lane 0 polls, the wave follows it in program order
    int arrived = 1;
    if (lane == 0) {
        int spins = 0;
        while (__hip_atomic_load(Q.counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < Q.target) {
            __builtin_amdgcn_s_sleep(1);
            if ((unsigned)++spins > Q.max_polls) {
                arrived = 0;
                break;
            }
        }
    }
    arrived = __shfl(arrived, 0, 64);
    // the partial loads below stay behind the poll (sc1 loads of sc1-stored
    // bytes behind a matched poll: MI355X_MICROARCH.md hand-off table, row 1)
    asm volatile("" ::: "memory");
    // the call's device fault word, loaded beside the partials (no extra round trip)
    const int faulted = __hip_atomic_load(Q.dev_fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float tn = 0.0f;
    if (A.max_norm > 0.0f) {
        // all of a lane's partials in flight at once, summed in k_adam's order
        static_assert(kReduceBlocks <= 4 * 64, "norm partial loads");
        float np[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = lane + 64 * u;
            np[u] = k < A.n_part ? __hip_atomic_load(const_cast<float*>(A.norm_part) + k, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)
                                 : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) tn += np[u];
    }
    tn = wave_sum(tn);
    const float coef = A.max_norm > 0.0f ? fminf(A.max_norm / (sqrtf(tn) + 1e-6f), 1.0f) : 1.0f;
    if (!arrived) {
        // a lost arrival (the grid was not co-resident): no parameter, moment or
        // gradient is written; the call's device word stops every block that
        // arrives later, and the host sees RT_EDEVICE (rt_ppo_status, next call)
        if (lane == 0) {
            __hip_atomic_store(Q.dev_fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(Q.fault, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    // A block of this launch or of an earlier one of the call that gave up set
    // the device word before it left: every block that arrives after it -- late
    // in this launch, or in the call's later launches, which start after it
    // ended -- reads it (above, with its partials) and writes nothing either,
    // so a lost arrival leaves the state as the last complete minibatch left
    // it (never a partly updated parameter set).  (Round 6: the host-mapped
    // flag itself read here cost ~26 us per minibatch -- 158 PCIe reads.)
    if (faulted) return;
    if (!upd) return;
    const float g = a * coef;
    A.grad[i] = g;
    float m = m0;
    m = m + A.lerp_w * (g - m);                   // exp_avg.lerp_(grad, 1 - beta1)
    float v = v0 * A.beta2;                       // exp_avg_sq.mul_(beta2)
    v = v + A.one_minus_beta2 * g * g;            //   .addcmul_(grad, grad, 1 - beta2)
    const float denom = sqrtf(v) / A.bc2_sqrt + A.eps;
    A.param[i] = w0 + A.step_size * (m / denom);  // addcdiv_(exp_avg, denom, -step_size)
    A.m[i] = m;
    A.v[i] = v;
}

// ---- per-epoch shuffle and minibatch advantage statistics ------------------
// A keyed pseudo-random permutation of [0, n): a 4-round Feistel network on
// 2h bits (2^(2h) >= n) with cycle-walking, one index per thread -- replaces
// the device randperm (a multi-kernel radix sort) the reference's
// np.random.permutation maps to (train.py:195).
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ uint32_t feistel_index(uint32_t i, int64_t n, int h, uint64_t key) {
    const uint32_t mask = (1u << h) - 1u;
    const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    uint32_t v = i;
    do {
        uint32_t L = v >> h, R = v & mask;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t f = mix32(R ^ mix32(k0 + 0x9E3779B9U * (uint32_t)(r + 1)) ^ k1) & mask;
            const uint32_t t = L ^ f;
            L = R;
            R = t;
        }
        v = (L << h) | R;
    } while ((int64_t)v >= n);
    return v;
}

__global__ __launch_bounds__(256) void k_shuffle(int64_t n, int h, uint64_t key, int64_t* perm) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) perm[i] = feistel_index((uint32_t)i, n, h, key);
}

// every epoch's permutation in one launch: blockIdx.y = epoch, key keys[y]
constexpr int kShuffleKeys = 32;
struct ShuffleKeys {
    uint64_t k[kShuffleKeys];
};

__global__ __launch_bounds__(256) void k_shuffle_epochs(int64_t n, int h, ShuffleKeys K, int64_t* perm) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) perm[(int64_t)blockIdx.y * n + i] = feistel_index((uint32_t)i, n, h, K.k[blockIdx.y]);
}

// [n_mb][2] = (mean, unbiased std) of adv over each minibatch of perm
// (train.py:215-218), sums in f64.  The gathers adv[perm[j]] are random 4-B
// reads (one cache line each), so they are spread over kAdvParts workgroups
// per minibatch (n_mb x 32 workgroups) instead of one: k_adv_partial writes
// (sum, sum of squares) per part, k_adv_stats adds the parts in order.
constexpr int kAdvParts = 32, kAdvThreads = 256, kAdvBatch = 4;
__global__ __launch_bounds__(kAdvThreads) void k_adv_partial(const float* adv, const int64_t* perm, int mb,
                                                            double* part) {
    __shared__ double ps[kAdvThreads / 64], pq[kAdvThreads / 64];
    const int chunk = (mb + kAdvParts - 1) / kAdvParts;
    const int j0 = blockIdx.x * chunk, j1 = min(j0 + chunk, mb);
    const int64_t base = (int64_t)blockIdx.y * mb;
    double s = 0.0, q = 0.0;
    for (int jb = j0; jb < j1; jb += kAdvThreads * kAdvBatch) {
        int64_t ix[kAdvBatch];
        float a[kAdvBatch];
#pragma unroll
        for (int u = 0; u < kAdvBatch; ++u) {
            const int j = jb + u * kAdvThreads + (int)threadIdx.x;
            ix[u] = j < j1 ? perm[base + j] : -1;
        }
#pragma unroll
        for (int u = 0; u < kAdvBatch; ++u) a[u] = ix[u] >= 0 ? adv[ix[u]] : 0.0f;
#pragma unroll
        for (int u = 0; u < kAdvBatch; ++u) {
            s += (double)a[u];
            q += (double)a[u] * (double)a[u];
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        s += __shfl_xor(s, off, 64);
        q += __shfl_xor(q, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        ps[threadIdx.x >> 6] = s;
        pq[threadIdx.x >> 6] = q;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double S = 0.0, Q = 0.0;
        for (int w = 0; w < kAdvThreads / 64; ++w) {
            S += ps[w];
            Q += pq[w];
        }
        double* o = part + ((size_t)blockIdx.y * kAdvParts + blockIdx.x) * 2;
        o[0] = S;
        o[1] = Q;
    }
}

// rt_ppo_shuffle_adv: the epochs' permutations AND the minibatch advantage
// partial sums in one launch -- k_adv_partial's grid and summation order, each
// position's permuted index computed in place (feistel_index, the k_shuffle
// arithmetic) and stored to perm as it is used, instead of a k_shuffle_epochs
// pass whose output k_adv_partial then re-reads.  blockIdx.y = minibatch k of
// the launch (epoch e0 + k / n_mb); the sums are bitwise k_adv_partial's.
__global__ __launch_bounds__(kAdvThreads) void k_shuffle_adv_partial(const float* adv, int64_t n, int h,
                                                                     ShuffleKeys K, int mb, int n_mb,
                                                                     int64_t* perm, double* part) {
    __shared__ double ps[kAdvThreads / 64], pq[kAdvThreads / 64];
    const int chunk = (mb + kAdvParts - 1) / kAdvParts;
    const int j0 = blockIdx.x * chunk, j1 = min(j0 + chunk, mb);
    const int e = blockIdx.y / n_mb, m = blockIdx.y - e * n_mb;
    const int64_t pos0 = (int64_t)m * mb;
    int64_t* pe = perm + (int64_t)e * n;
    const uint64_t key = K.k[e];
    double s = 0.0, q = 0.0;
    for (int jb = j0; jb < j1; jb += kAdvThreads * kAdvBatch) {
        int64_t ix[kAdvBatch];
        float a[kAdvBatch];
#pragma unroll
        for (int u = 0; u < kAdvBatch; ++u) {
            const int j = jb + u * kAdvThreads + (int)threadIdx.x;
            ix[u] = -1;
            if (j < j1) {
                ix[u] = feistel_index((uint32_t)(pos0 + j), n, h, key);
                pe[pos0 + j] = ix[u];
            }
        }
#pragma unroll
        for (int u = 0; u < kAdvBatch; ++u) a[u] = ix[u] >= 0 ? adv[ix[u]] : 0.0f;
#pragma unroll
        for (int u = 0; u < kAdvBatch; ++u) {
            s += (double)a[u];
            q += (double)a[u] * (double)a[u];
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        s += __shfl_xor(s, off, 64);
        q += __shfl_xor(q, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        ps[threadIdx.x >> 6] = s;
        pq[threadIdx.x >> 6] = q;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double S = 0.0, Q = 0.0;
        for (int w = 0; w < kAdvThreads / 64; ++w) {
            S += ps[w];
            Q += pq[w];
        }
        double* o = part + ((size_t)blockIdx.y * kAdvParts + blockIdx.x) * 2;
        o[0] = S;
        o[1] = Q;
    }
}

__global__ __launch_bounds__(256) void k_adv_stats(const double* part, int mb, int n_mb, float* stats) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_mb) return;
    double S = 0.0, Q = 0.0;
    for (int k = 0; k < kAdvParts; ++k) {
        S += part[((size_t)i * kAdvParts + k) * 2];
        Q += part[((size_t)i * kAdvParts + k) * 2 + 1];
    }
    const double mean = S / mb;
    const double var = mb > 1 ? (Q - S * mean) / (mb - 1) : 0.0;
    stats[2 * i] = (float)mean;
    stats[2 * i + 1] = (float)sqrt(var > 0.0 ? var : 0.0);
}

// Data-parallel split of k_adv_stats: the ranks' (sum, sum of squares) per
// minibatch (fixed-order sums of the parts) are all-reduced by the caller,
// then turned into (mean, unbiased std) over the global minibatch size.
__global__ __launch_bounds__(256) void k_adv_sums(const double* part, int n_mb, double* sums) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_mb) return;
    double S = 0.0, Q = 0.0;
    for (int k = 0; k < kAdvParts; ++k) {
        S += part[((size_t)i * kAdvParts + k) * 2];
        Q += part[((size_t)i * kAdvParts + k) * 2 + 1];
    }
    sums[2 * i] = S;
    sums[2 * i + 1] = Q;
}

__global__ __launch_bounds__(256) void k_adv_finalize(const double* sums, int64_t count, int n_mb, float* stats) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n_mb) return;
    const double S = sums[2 * i], Q = sums[2 * i + 1];
    const double mean = S / (double)count;
    const double var = count > 1 ? (Q - S * mean) / (double)(count - 1) : 0.0;
    stats[2 * i] = (float)mean;
    stats[2 * i + 1] = (float)sqrt(var > 0.0 ? var : 0.0);
}

ReduceParams reduce_params(float* const* grads_d, int32_t mb, const rt_ppo_hparams* hp, float* ws_d,
                           int64_t ws_floats, float* stats_d, float* accum_d) {
    ReduceParams R{};
    for (int i = 0; i < 13; ++i) R.grad.p[i] = grads_d[i];
    R.ws = ws_d;
    R.nblk = grad_blocks(mb);
    R.stats = stats_d;
    R.stats_accum = accum_d;
    R.norm_part = ws_d + (ws_floats - kNormSlots);
    R.inv_n = 1.0f / (float)mb;
    R.ent_coef = hp->ent_coef;
    return R;
}

int ppo_grad_launch(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* b,
                    const int64_t* idx_d, int32_t mb, const float* adv_stats_d, const rt_ppo_hparams* hp,
                    float* ws_d, int64_t ws_floats, float* stats_d, float* accum_d, hipStream_t st,
                    bool with_reduce = true) {
    const int nblk = grad_blocks(mb);
    if ((int64_t)nblk * PSTRIDE + kNormSlots > ws_floats)
        return rt_internal_fail(RT_EINVAL, "rt_ppo_grad: workspace too small");
    GradParams G{};
    ReduceParams R{};
    for (int i = 0; i < 13; ++i) G.w.p[i] = params_d[i];
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
    // arithmetic of the two 64x64 products: per call (rt_ppo_hparams.precision)
    if (hp->precision == RT_PPO_PREC_BF16X3)
        hipLaunchKernelGGL(k_ppo_grad_mfma<kPrecBf16x3>, dim3(nblk), dim3(MT), 0, st, G);
    else
        hipLaunchKernelGGL(k_ppo_grad_mfma<kPrecF32>, dim3(nblk), dim3(MT), 0, st, G);
    R = reduce_params(grads_d, mb, hp, ws_d, ws_floats, stats_d, accum_d);
    if (with_reduce) hipLaunchKernelGGL(k_ppo_reduce, dim3(kReduceBlocks), dim3(1024), 0, st, R);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

// norm_part: the kReduceBlocks partials k_ppo_reduce left (fresh = true), or
// scratch for k_gnorm over the (all-reduced) flat gradient
AdamParams adam_params(int64_t n, float* p, float* g, float* m, float* v, int64_t step, double lr,
                       const rt_ppo_hparams* hp, float* norm_part, float grad_div) {
    AdamParams A{};
    A.n = n;
    A.param = p;
    A.grad = g;
    A.m = m;
    A.v = v;
    A.max_norm = hp->max_grad_norm;
    A.norm_part = norm_part;
    A.n_part = kReduceBlocks;
    const double b1 = hp->adam_beta1, b2 = hp->adam_beta2;
    // torch.optim.Adam (foreach): host-side scalars in double, applied in f32
    A.lerp_w = (float)(1.0 - b1);
    A.beta2 = (float)b2;
    A.one_minus_beta2 = (float)(1.0 - b2);
    A.step_size = (float)(-(lr / (1.0 - std::pow(b1, (double)step))));
    A.bc2_sqrt = (float)std::pow(1.0 - std::pow(b2, (double)step), 0.5);
    A.eps = hp->adam_eps;
    A.grad_div = grad_div;
    return A;
}

int adam_launch(int64_t n, float* p, float* g, float* m, float* v, int64_t step, double lr,
                const rt_ppo_hparams* hp, float* norm_part, bool fresh, float grad_div, hipStream_t st) {
    const AdamParams A = adam_params(n, p, g, m, v, step, lr, hp, norm_part, grad_div);
    if (A.max_norm > 0.0f && !fresh) {
        const int64_t per = (n + kReduceBlocks - 1) / kReduceBlocks;
        hipLaunchKernelGGL(k_gnorm, dim3(kReduceBlocks), dim3(256), 0, st, g, n, per, grad_div, norm_part);
    }
    hipLaunchKernelGGL(k_adam, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

// The sticky fault flag of k_ppo_reduce_adam: one host-mapped int per device
// (a lost grid arrival on that device sets it); nullptr when the host
// allocation failed (rt_ppo_update then runs the two-kernel form)
int* reduce_adam_fault() {
    static std::mutex mu;
    static std::map<int, int*> flags;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> lock(mu);
    const auto f = flags.find(dev);
    if (f != flags.end()) return f->second;
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) p = nullptr;
    if (p) *static_cast<volatile int*>(p) = 0;
    return flags[dev] = static_cast<int*>(p);
}

bool reduce_adam_faulted() {
    int* f = reduce_adam_fault();
    return f && *static_cast<volatile int*>(f) != 0;
}

// Debug knob (tests): RT_PPO_UPDATE_SPLIT=1 makes rt_ppo_update run its
// two-kernel form (k_ppo_grad + k_ppo_reduce, then k_adam) -- the path a
// failed occupancy check or a missing host-mapped flag selects -- so the
// test suite covers it on hardware where the fused form always runs.
bool force_split_update() {
    const char* v = std::getenv("RT_PPO_UPDATE_SPLIT");
    return v && v[0] == '1';
}

// Debug knob (tests): RT_PPO_FORCE_LOST_ARRIVAL=1 makes every block of the
// fused reduce + Adam wait for an arrival count that never comes, with a
// 16-poll budget: the lost-arrival path (no write, device word, sticky
// host flag, RT_EDEVICE from then on) runs as it would on a grid that was
// not co-resident.  The flag is per process: tests run it in a child.
bool force_lost_arrival() {
    const char* v = std::getenv("RT_PPO_FORCE_LOST_ARRIVAL");
    return v && v[0] == '1';
}

// k_ppo_reduce_adam's grid arrival needs all kReduceBlocks blocks resident at
// once: checked per device against the occupancy query (cached)
bool reduce_adam_coresident() {
    static std::mutex mu;
    static std::map<int, bool> ok;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    std::lock_guard<std::mutex> lock(mu);
    const auto f = ok.find(dev);
    if (f != ok.end()) return f->second;
    int per_cu = 0, cus = 0;
    const bool good = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_ppo_reduce_adam, 1024, 0) == hipSuccess &&
                      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
                      (int64_t)per_cu * cus >= kReduceBlocks;
    return ok[dev] = good;
}

bool bad_prec(const rt_ppo_hparams* hp) {
    return hp->precision != RT_PPO_PREC_F32 && hp->precision != RT_PPO_PREC_BF16X3;
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
    return (int64_t)grad_blocks(minibatch_size) * PSTRIDE + kNormSlots;
}

extern "C" int32_t rt_ppo_num_params(void) { return NP; }

extern "C" int rt_ppo_grad(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* batch,
                           const int64_t* mb_idx_d, int32_t mb_size, const float* adv_stats_d,
                           const rt_ppo_hparams* hp, float* workspace_d, int64_t workspace_floats, float* stats_d,
                           float* stats_accum_d, void* stream) {
    if (bad13(reinterpret_cast<const void* const*>(params_d)) || bad13(reinterpret_cast<const void* const*>(grads_d)) ||
        bad_batch(batch) || !mb_idx_d || mb_size < 1 || !hp || bad_prec(hp) || !workspace_d || !stats_d ||
        (hp->norm_adv && !adv_stats_d))
        return rt_internal_fail(RT_EINVAL, "rt_ppo_grad: bad argument");
    if (reduce_adam_faulted())
        return rt_internal_fail(RT_EDEVICE, "rt_ppo_grad: an earlier rt_ppo_update lost its grid arrival");
    return ppo_grad_launch(params_d, grads_d, batch, mb_idx_d, mb_size, adv_stats_d, hp, workspace_d,
                           workspace_floats, stats_d, stats_accum_d, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int rt_adam_step(int64_t n, float* param_d, float* grad_d, float* exp_avg_d, float* exp_avg_sq_d,
                            int64_t step, double lr, const rt_ppo_hparams* hp, int32_t grad_div, float* workspace_d,
                            void* stream) {
    if (n < 1 || !param_d || !grad_d || !exp_avg_d || !exp_avg_sq_d || step < 1 || !hp || !workspace_d ||
        grad_div < 1 || grad_div > (1 << 24))
        return rt_internal_fail(RT_EINVAL, "rt_adam_step: bad argument");
    if (reduce_adam_faulted())
        return rt_internal_fail(RT_EDEVICE, "rt_adam_step: an earlier rt_ppo_update lost its grid arrival");
    return adam_launch(n, param_d, grad_d, exp_avg_d, exp_avg_sq_d, step, lr, hp, workspace_d, false,
                       (float)grad_div, reinterpret_cast<hipStream_t>(stream));
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
        (hp->norm_adv && !adv_stats_d) || mb_size > batch->batch_size || bad_prec(hp))
        return rt_internal_fail(RT_EINVAL, "rt_ppo_update: bad argument");
    if (reduce_adam_faulted())
        return rt_internal_fail(RT_EDEVICE, "rt_ppo_update: an earlier call lost its grid arrival");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    float* norm_part = workspace_d + (workspace_floats - kNormSlots);
    int* fault_h = reduce_adam_fault();
    int* fault_d = nullptr;
    if (fault_h && hipHostGetDevicePointer(reinterpret_cast<void**>(&fault_d), fault_h, 0) != hipSuccess)
        fault_d = nullptr;
    if (!fault_d || !reduce_adam_coresident() || force_split_update()) {
        // the two-kernel form: k_ppo_grad_mfma + k_ppo_reduce, then k_adam
        for (int i = 0; i < n_minibatches; ++i) {
            int rc = ppo_grad_launch(params_d, grads_d, batch, perm_d + (int64_t)i * mb_size, mb_size,
                                     adv_stats_d ? adv_stats_d + 2 * i : nullptr, hp, workspace_d, workspace_floats,
                                     stats_d, stats_accum_d, st, true);
            if (rc) return rc;
            rc = adam_launch(n_flat, flat_param_d, flat_grad_d, exp_avg_d, exp_avg_sq_d, step0 + i, lr, hp, norm_part,
                             true, 1.0f, st);
            if (rc) return rc;
        }
        return RT_OK;
    }
    // the arrival counter of k_ppo_reduce_adam and the call's device fault word:
    // the last two norm slots (unused by the partials)
    static_assert(kReduceBlocks <= kNormSlots - 2, "norm partials vs counter / fault word");
    int* dev_fault = reinterpret_cast<int*>(norm_part + (kNormSlots - 2));
    unsigned* counter = reinterpret_cast<unsigned*>(norm_part + (kNormSlots - 1));
    if (hipMemsetAsync(dev_fault, 0, 2 * sizeof(unsigned), st) != hipSuccess)
        return rt_internal_fail(RT_EDEVICE, "rt_ppo_update: hipMemsetAsync failed");
    ReduceAdamParams Q{};
    for (int t = 0; t < 13; ++t) {
        const int64_t off = params_d[t] - flat_param_d;
        if (off < 0 || off + (kTensorOff[t + 1] - kTensorOff[t]) > n_flat ||
            grads_d[t] - flat_grad_d != off)
            return rt_internal_fail(RT_EINVAL, "rt_ppo_update: params_d / grads_d must be views of the flat buffers");
        Q.flat_off[t] = (int32_t)off;
    }
    Q.counter = counter;
    Q.fault = fault_d;
    Q.dev_fault = dev_fault;
    const bool lost = force_lost_arrival();
    for (int i = 0; i < n_minibatches; ++i) {
        int rc = ppo_grad_launch(params_d, grads_d, batch, perm_d + (int64_t)i * mb_size, mb_size,
                                 adv_stats_d ? adv_stats_d + 2 * i : nullptr, hp, workspace_d, workspace_floats,
                                 stats_d, stats_accum_d, st, false);
        if (rc) return rc;
        Q.R = reduce_params(grads_d, mb_size, hp, workspace_d, workspace_floats, stats_d, stats_accum_d);
        Q.A = adam_params(n_flat, flat_param_d, flat_grad_d, exp_avg_d, exp_avg_sq_d, step0 + i, lr, hp, norm_part,
                          1.0f);
        Q.target = lost ? 0xFFFFFFFFu : (unsigned)((i + 1) * kReduceBlocks);
        Q.max_polls = lost ? 16u : (1u << 24);
        hipLaunchKernelGGL(k_ppo_reduce_adam, dim3(kReduceBlocks), dim3(1024), 0, st, Q);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    }
    return RT_OK;
}

extern "C" int rt_ppo_status(void) {
    if (reduce_adam_faulted())
        return rt_internal_fail(RT_EDEVICE, "rt_ppo_status: an rt_ppo_update on this device lost its grid arrival");
    return RT_OK;
}

extern "C" int rt_ppo_shuffle(int64_t n, uint64_t key, int64_t* perm_d, void* stream) {
    if (n < 1 || n > ((int64_t)1 << 31) || !perm_d) return rt_internal_fail(RT_EINVAL, "rt_ppo_shuffle: bad argument");
    int b = 1;
    while (((int64_t)1 << b) < n) ++b;
    const int h = (b + 1) / 2;
    hipLaunchKernelGGL(k_shuffle, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), n, h, key, perm_d);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_ppo_shuffle_epochs(int64_t n, int32_t n_epochs, const uint64_t* keys_h, int64_t* perm_d,
                                     void* stream) {
    if (n < 1 || n > ((int64_t)1 << 31) || n_epochs < 1 || !keys_h || !perm_d)
        return rt_internal_fail(RT_EINVAL, "rt_ppo_shuffle_epochs: bad argument");
    int b = 1;
    while (((int64_t)1 << b) < n) ++b;
    const int h = (b + 1) / 2;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    for (int e0 = 0; e0 < n_epochs; e0 += kShuffleKeys) {
        const int ne = n_epochs - e0 < kShuffleKeys ? n_epochs - e0 : kShuffleKeys;
        ShuffleKeys K{};
        for (int j = 0; j < ne; ++j) K.k[j] = keys_h[e0 + j];
        hipLaunchKernelGGL(k_shuffle_epochs, dim3((unsigned)((n + 255) / 256), (unsigned)ne), dim3(256), 0, st, n, h,
                           K, perm_d + (int64_t)e0 * n);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_ppo_shuffle_adv(int64_t n, int32_t n_epochs, const uint64_t* keys_h, int64_t* perm_d,
                                  const float* adv_d, int32_t mb_size, double* sums_d, float* stats_d,
                                  float* workspace_d, int64_t workspace_floats, void* stream) {
    if (n < 1 || n > ((int64_t)1 << 31) || n_epochs < 1 || !keys_h || !perm_d || !adv_d || mb_size < 1 ||
        n % mb_size != 0 || n / mb_size > 65535 || (sums_d == nullptr) == (stats_d == nullptr) || !workspace_d)
        return rt_internal_fail(RT_EINVAL, "rt_ppo_shuffle_adv: bad argument");
    const int n_mb = (int)(n / mb_size);
    if (workspace_floats < (int64_t)std::min(n_epochs, kShuffleKeys) * n_mb * kAdvParts * 4 ||
        (int64_t)std::min(n_epochs, kShuffleKeys) * n_mb > 65535)
        return rt_internal_fail(RT_EINVAL, "rt_ppo_shuffle_adv: workspace too small");
    int b = 1;
    while (((int64_t)1 << b) < n) ++b;
    const int h = (b + 1) / 2;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    double* part = reinterpret_cast<double*>(workspace_d);
    for (int e0 = 0; e0 < n_epochs; e0 += kShuffleKeys) {
        const int ne = n_epochs - e0 < kShuffleKeys ? n_epochs - e0 : kShuffleKeys;
        ShuffleKeys K{};
        for (int j = 0; j < ne; ++j) K.k[j] = keys_h[e0 + j];
        const int k = ne * n_mb;  // minibatches of these epochs
        hipLaunchKernelGGL(k_shuffle_adv_partial, dim3(kAdvParts, k), dim3(kAdvThreads), 0, st, adv_d, n, h, K,
                           mb_size, n_mb, perm_d + (int64_t)e0 * n, part);
        if (stats_d)
            hipLaunchKernelGGL(k_adv_stats, dim3((k + 255) / 256), dim3(256), 0, st, part, mb_size, k,
                               stats_d + (int64_t)e0 * n_mb * 2);
        else
            hipLaunchKernelGGL(k_adv_sums, dim3((k + 255) / 256), dim3(256), 0, st, part, k,
                               sums_d + (int64_t)e0 * n_mb * 2);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_ppo_adv_stats(const float* adv_d, const int64_t* perm_d, int32_t mb_size, int32_t n_minibatches,
                                float* stats_d, float* workspace_d, int64_t workspace_floats, void* stream) {
    if (!adv_d || !perm_d || !stats_d || !workspace_d || mb_size < 1 || n_minibatches < 1 ||
        workspace_floats < (int64_t)n_minibatches * kAdvParts * 4)
        return rt_internal_fail(RT_EINVAL, "rt_ppo_adv_stats: bad argument");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    double* part = reinterpret_cast<double*>(workspace_d);
    hipLaunchKernelGGL(k_adv_partial, dim3(kAdvParts, n_minibatches), dim3(kAdvThreads), 0, st, adv_d, perm_d,
                       mb_size, part);
    hipLaunchKernelGGL(k_adv_stats, dim3((n_minibatches + 255) / 256), dim3(256), 0, st, part, mb_size,
                       n_minibatches, stats_d);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_ppo_adv_sums(const float* adv_d, const int64_t* perm_d, int32_t mb_size, int32_t n_minibatches,
                               double* sums_d, float* workspace_d, int64_t workspace_floats, void* stream) {
    if (!adv_d || !perm_d || !sums_d || !workspace_d || mb_size < 1 || n_minibatches < 1 ||
        workspace_floats < (int64_t)n_minibatches * kAdvParts * 4)
        return rt_internal_fail(RT_EINVAL, "rt_ppo_adv_sums: bad argument");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    double* part = reinterpret_cast<double*>(workspace_d);
    hipLaunchKernelGGL(k_adv_partial, dim3(kAdvParts, n_minibatches), dim3(kAdvThreads), 0, st, adv_d, perm_d,
                       mb_size, part);
    hipLaunchKernelGGL(k_adv_sums, dim3((n_minibatches + 255) / 256), dim3(256), 0, st, part, n_minibatches, sums_d);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_ppo_adv_finalize(const double* sums_d, int64_t count, int32_t n_minibatches, float* stats_d,
                                   void* stream) {
    if (!sums_d || !stats_d || count < 1 || n_minibatches < 1)
        return rt_internal_fail(RT_EINVAL, "rt_ppo_adv_finalize: bad argument");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_adv_finalize, dim3((n_minibatches + 255) / 256), dim3(256), 0, st, sums_d, count,
                       n_minibatches, stats_d);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

RT_TRACE_READ_FN(rt_trace_read_update)

// ---------------------------------------------------------------------------
// Data-parallel update over RCCL (train.py:183-248 at world > 1).
// One process per GPU; the library keeps its own RCCL communicator, so the
// per-minibatch sequence -- k_ppo_grad_mfma + k_ppo_reduce, the SUM
// all-reduce of the flat gradient (40 KB for the MLP, in place), k_gnorm +
// k_adam with grad_div = world -- is issued by ONE C call for the whole
// update, with no Python, ctypes or torch.distributed call per minibatch.
// RCCL is loaded at the first communicator (dlopen): the copy torch already
// mapped when there is one (same SONAME), otherwise ROCm's; hosts that never
// build a communicator never load it.
// ---------------------------------------------------------------------------
struct rt_dp_comm {
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0, device = 0;
};

namespace {

struct RcclApi {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string error;
};

const RcclApi& rccl() {
    static RcclApi api = [] {
        RcclApi a;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // torch's copy, when mapped
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            a.error = std::string("librccl.so.1: ") + dlerror();
            return a;
        }
        a.get_unique_id = reinterpret_cast<decltype(a.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
        a.comm_init_rank = reinterpret_cast<decltype(a.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
        a.all_reduce = reinterpret_cast<decltype(a.all_reduce)>(dlsym(h, "ncclAllReduce"));
        a.comm_destroy = reinterpret_cast<decltype(a.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
        a.error_string = reinterpret_cast<decltype(a.error_string)>(dlsym(h, "ncclGetErrorString"));
        if (!a.get_unique_id || !a.comm_init_rank || !a.all_reduce || !a.comm_destroy || !a.error_string)
            a.error = "librccl.so.1: missing symbols";
        return a;
    }();
    return api;
}

int rccl_fail(const char* what, ncclResult_t r) {
    const RcclApi& A = rccl();
    return rt_internal_fail(RT_EDEVICE, (std::string(what) + ": " + (A.error_string ? A.error_string(r) : "RCCL error")).c_str());
}

}  // namespace

extern "C" int rt_dp_unique_id(uint8_t* id_h) {
    if (!id_h) return rt_internal_fail(RT_EINVAL, "rt_dp_unique_id: NULL argument");
    static_assert(sizeof(ncclUniqueId) == RT_DP_ID_BYTES, "RT_DP_ID_BYTES");
    const RcclApi& A = rccl();
    if (!A.error.empty()) return rt_internal_fail(RT_EDEVICE, A.error.c_str());
    ncclUniqueId id;
    const ncclResult_t r = A.get_unique_id(&id);
    if (r != ncclSuccess) return rccl_fail("ncclGetUniqueId", r);
    std::memcpy(id_h, &id, sizeof(id));
    return RT_OK;
}

extern "C" int rt_dp_comm_create(const uint8_t* id_h, int32_t nranks, int32_t rank, int device, rt_dp_comm** out) {
    if (!id_h || !out || nranks < 1 || rank < 0 || rank >= nranks)
        return rt_internal_fail(RT_EINVAL, "rt_dp_comm_create: bad argument");
    *out = nullptr;
    const RcclApi& A = rccl();
    if (!A.error.empty()) return rt_internal_fail(RT_EDEVICE, A.error.c_str());
    int cur = 0;
    (void)hipGetDevice(&cur);
    if (hipSetDevice(device) != hipSuccess) return rt_internal_fail(RT_EDEVICE, "rt_dp_comm_create: bad device");
    ncclUniqueId id;
    std::memcpy(&id, id_h, sizeof(id));
    rt_dp_comm* c = new rt_dp_comm();
    c->nranks = nranks;
    c->rank = rank;
    c->device = device;
    const ncclResult_t r = A.comm_init_rank(&c->comm, nranks, id, rank);
    (void)hipSetDevice(cur);
    if (r != ncclSuccess) {
        delete c;
        return rccl_fail("ncclCommInitRank", r);
    }
    *out = c;
    return RT_OK;
}

extern "C" void rt_dp_comm_destroy(rt_dp_comm* comm) {
    if (!comm) return;
    if (comm->comm && rccl().comm_destroy) (void)rccl().comm_destroy(comm->comm);
    delete comm;
}

extern "C" int rt_dp_allreduce(rt_dp_comm* comm, void* buf_d, int64_t count, int32_t dtype, void* stream) {
    if (!comm || !buf_d || count < 0 || (dtype != RT_DP_F32 && dtype != RT_DP_F64))
        return rt_internal_fail(RT_EINVAL, "rt_dp_allreduce: bad argument");
    const ncclResult_t r = rccl().all_reduce(buf_d, buf_d, (size_t)count, dtype == RT_DP_F32 ? ncclFloat32 : ncclFloat64,
                                             ncclSum, comm->comm, reinterpret_cast<hipStream_t>(stream));
    return r == ncclSuccess ? RT_OK : rccl_fail("ncclAllReduce", r);
}

extern "C" int rt_ppo_update_dp(const float* const* params_d, float* const* grads_d, const rt_ppo_batch* batch,
                                const int64_t* perm_d, int32_t mb_size, int32_t n_minibatches,
                                const float* adv_stats_d, const rt_ppo_hparams* hp, float* flat_param_d,
                                float* flat_grad_d, float* exp_avg_d, float* exp_avg_sq_d, int64_t n_flat,
                                int64_t step0, double lr, float* workspace_d, int64_t workspace_floats,
                                float* stats_d, float* stats_accum_d, rt_dp_comm* comm, void* stream) {
    if (bad13(reinterpret_cast<const void* const*>(params_d)) || bad13(reinterpret_cast<const void* const*>(grads_d)) ||
        bad_batch(batch) || !perm_d || mb_size < 1 || n_minibatches < 1 || !hp || !flat_param_d || !flat_grad_d ||
        !exp_avg_d || !exp_avg_sq_d || n_flat != NP || step0 < 1 || !workspace_d || !stats_d || !comm ||
        (hp->norm_adv && !adv_stats_d) || mb_size > batch->batch_size || bad_prec(hp))
        return rt_internal_fail(RT_EINVAL, "rt_ppo_update_dp: bad argument");
    if (reduce_adam_faulted())
        return rt_internal_fail(RT_EDEVICE, "rt_ppo_update_dp: an earlier rt_ppo_update lost its grid arrival");
    for (int t = 0; t < 13; ++t)
        if (grads_d[t] - flat_grad_d != params_d[t] - flat_param_d || params_d[t] < flat_param_d ||
            params_d[t] - flat_param_d + (kTensorOff[t + 1] - kTensorOff[t]) > n_flat)
            return rt_internal_fail(RT_EINVAL, "rt_ppo_update_dp: params_d / grads_d must be views of the flat buffers");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    float* norm_part = workspace_d + (workspace_floats - kNormSlots);
    const RcclApi& A = rccl();
    for (int i = 0; i < n_minibatches; ++i) {
        int rc = ppo_grad_launch(params_d, grads_d, batch, perm_d + (int64_t)i * mb_size, mb_size,
                                 adv_stats_d ? adv_stats_d + 2 * i : nullptr, hp, workspace_d, workspace_floats,
                                 stats_d, stats_accum_d, st, true);
        if (rc) return rc;
        // SUM over the ranks, in place; the Adam step divides by the world size
        const ncclResult_t r = A.all_reduce(flat_grad_d, flat_grad_d, (size_t)n_flat, ncclFloat32, ncclSum,
                                            comm->comm, st);
        if (r != ncclSuccess) return rccl_fail("ncclAllReduce", r);
        rc = adam_launch(n_flat, flat_param_d, flat_grad_d, exp_avg_d, exp_avg_sq_d, step0 + i, lr, hp, norm_part,
                         false, (float)comm->nranks, st);
        if (rc) return rc;
    }
    return RT_OK;
}
