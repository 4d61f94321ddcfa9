// c3d.hip -- the C3D-lite feature extractor of the vision agent on f32 MFMA.
//
// Reference: networks.py:8-45 (FeaturesExtractor3D.cnn):
//   Conv3d(4, 16, 3)            ReLU  MaxPool3d(2, 2, padding=((S_i - 2) % 2))
//   Conv3d(16, 16, 3, groups=2) ReLU  MaxPool3d(2, 2)
//   Conv3d(16, 16, 3, groups=4) ReLU  MaxPool3d(2, 2)
// Each stage is one fused kernel here: valid 3x3x3 convolution + bias + ReLU +
// 2x2x2 max-pool, writing the pooled map and, for training, a per-output byte
// holding the window index of the maximum (torch's first-max rule) and whether
// the ReLU was active.  The backward kernels (weight gradient, data gradient)
// rebuild the sparse full-resolution gradient from those bytes instead of
// storing the 8x larger pre-pool maps.
//
// MFMA mapping (v_mfma_f32_16x16x4_f32, exact f32 FMA chains): a tile is 16
// conv positions -- a 2(z) x 2(y) x 4(x) box = two pooling windows along x --
// times the 16 output channels.  D[m = out channel][n = position] =
// sum_k W[m][k] * patch[k][n]; k = (input channel, tap).  Lane l (c = l & 15,
// g = l >> 4) supplies A = W[c][k] (registers, loaded once per block) and
// B = the input voxel of position c for k from the block's LDS input tile; in
// k-step s the 4 lane groups g carry 4 input channels of one tap.  Grouped
// convolutions run dense over all 16 input channels with zero A entries
// outside the output channel's group.  The pooled max over a window is three
// DPP max steps (quad_perm + row_ror).
//
// LDS input tile: [cin][zl][yl][xl] with strides YS = 4, ZS = 8, CS = 16
// (mod 32), so the 32 lanes of a ds_read_b32 group (16 positions x 2 channels)
// hit 32 distinct banks.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <climits>
#include <map>
#include <mutex>
#include <tuple>
#include <type_traits>
#include <utility>

#include "rtenv.h"

extern "C" int rt_internal_fail(int code, const char* msg);

namespace {

// blocks the z-shift forward / data-gradient grids aim for when they split z
// into chunks: 2048 (no split at 512 samples) beat 4096 / 8192 -- a block that
// sweeps the whole depth pays its weight load and ring prologue once
constexpr int kZsBlocks = 2048;

constexpr int CO = 16;
constexpr int kThreads = 512;      // weight-gradient kernel: 8 waves = position groups x column groups
// forward / data-gradient kernels: conv1 (4 input channels, 95 VGPRs) runs
// 8-wave blocks (4 waves per SIMD at 2 blocks per CU) on 9-step register
// batches; the 16-channel stages (108 A fragments in registers) 4-wave blocks
// on 27-step batches
template <int CIN>
constexpr int conv_threads() {
    return CIN == 4 ? 512 : 256;
}
template <int CIN>
constexpr int conv_batch() {
    return CIN == 4 ? 9 : 27;
}

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// f4 sums of MFMA results as four scalar v_add / v_sub: the f4 operators
// lower to v_pk_add_f32, which beside MFMAs costs ~4x a scalar add's issue
// (MI355X_MICROARCH.md, 'price of one filler beside MFMAs'); built with
// -fno-slp-vectorize so the SLP pass does not re-pack them
__device__ __forceinline__ f4 add4s(f4 a, f4 b) {
    f4 r;
    r.x = a.x + b.x;
    r.y = a.y + b.y;
    r.z = a.z + b.z;
    r.w = a.w + b.w;
    return r;
}
__device__ __forceinline__ f4 sub4s(f4 a, f4 b) {
    f4 r;
    r.x = a.x - b.x;
    r.y = a.y - b.y;
    r.z = a.z - b.z;
    r.w = a.w - b.w;
    return r;
}

// bf16x3 products (rt_conv_layer.precision = RT_CONV_PREC_BF16X3: the forward and grouped data-gradient ring kernels):
// x = hi + lo + e, hi = bf16(x), lo = bf16(x - hi), both round to nearest even
// (|e| <= 2^-17 |x|); a product is hi*hi + hi*lo + lo*hi in three
// v_mfma_f32_16x16x32_bf16 (16 cycles each, f32 accumulate) against one
// 16x16x4 f32 MFMA (32 cycles) per 4 k: 3/16 of the f32 MFMA cycles per flop.
typedef __bf16 bf8 __attribute__((ext_vector_type(8)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t bf16_bits(float x) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x);
}
// one element as a packed word: hi(x) << 16 | lo(x)
__device__ __forceinline__ uint32_t bf_pack(float x) {
    const uint32_t h = bf16_bits(x);
    return (h << 16) | bf16_bits(x - __uint_as_float(h << 16));
}
__device__ __forceinline__ f4 mfma3(const bf8& ah, const bf8& al, const bf8& bh, const bf8& bl, f4 c) {
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}
// 8 packed words -> the hi and lo bf16x8 operands (element e = word e): one
// v_perm_b32 per element pair and half
__device__ __forceinline__ void bf_unpack8(const uint32_t (&p)[8], bf8& hi, bf8& lo) {
    u4v h, l;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        h[d] = __builtin_amdgcn_perm(p[2 * d + 1], p[2 * d], 0x07060302u);
        l[d] = __builtin_amdgcn_perm(p[2 * d + 1], p[2 * d], 0x05040100u);
    }
    hi = __builtin_bit_cast(bf8, h);
    lo = __builtin_bit_cast(bf8, l);
}

int round_mod(int v, int m) {  // smallest x >= v with x % 32 == m
    int x = v;
    while (((x % 32) + 32) % 32 != m) ++x;
    return x;
}

struct Geom {
    int32_t D, H, W;     // input
    int32_t cd, ch, cw;  // conv output
    int32_t pd, ph, pw;  // pool padding
    int32_t PD, PH, PW;  // pooled output
    int32_t XT;          // x tiles (4 conv positions = 2 windows each)
    int32_t ZL, YL, XL;  // LDS tile extents
    int32_t YS, ZS, CS;  // LDS strides
    int32_t PYB_tiles;   // ring weight gradient: position tiles per pooled row
};

// LDS stride residues (mod 32 dwords): (4, 8, 16) make the forward's reads
// (16 positions x 4 channels per ds_read_b32) conflict-free; the weight
// gradient's B gather (16 (channel, tap) columns x 4 x positions) needs
// (4, 12, 8) -- with (4, 8, 16) it took 2.4-2.6x the conflict-free LDS cycles
// (bank model over every stage geometry; PMC SQ_LDS_BANK_CONFLICT agreed)
template <int PZB, int PYB, int RY = 4, int RZ = 8, int RC = 16>
Geom make_geom(const rt_conv_layer* L) {
    Geom g{};
    g.D = L->in_dims[0];
    g.H = L->in_dims[1];
    g.W = L->in_dims[2];
    g.cd = g.D - 2;
    g.ch = g.H - 2;
    g.cw = g.W - 2;
    g.pd = L->pool_pad[0];
    g.ph = L->pool_pad[1];
    g.pw = L->pool_pad[2];
    g.PD = (g.cd + 2 * g.pd - 2) / 2 + 1;
    g.PH = (g.ch + 2 * g.ph - 2) / 2 + 1;
    g.PW = (g.cw + 2 * g.pw - 2) / 2 + 1;
    g.XT = (g.PW + 1) / 2;
    g.ZL = 2 * PZB + 2;
    g.YL = 2 * PYB + 2;
    g.XL = 4 * g.XT + 2;
    g.YS = round_mod(g.XL, RY);
    g.ZS = round_mod(g.YL * g.YS, RZ);
    g.CS = round_mod(g.ZL * g.ZS, RC);
    return g;
}

// max / min over a pooling window = the 8 lanes of a 16-lane row that share
// bit 1 of the row index (lanes c, c^1 and c+4, c+8, c+12 mod 16): DPP
// quad_perm [1,0,3,2] and row_ror 4, 8 -- full-rate VALU, no LDS crossbar
// (the pooled values are ReLU outputs >= 0 or -inf for masked positions; their
// int bit patterns order as the floats do, so the max runs as a DPP-fused
// integer max)
__device__ __forceinline__ float win_max(float v) {
    int k = __float_as_int(v);
    k = max(k, __builtin_amdgcn_mov_dpp(k, 0xB1, 0xF, 0xF, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, 0x124, 0xF, 0xF, true));
    k = max(k, __builtin_amdgcn_mov_dpp(k, 0x128, 0xF, 0xF, true));
    return __int_as_float(k);
}
__device__ __forceinline__ int win_min(int k) {
    k = min(k, __builtin_amdgcn_mov_dpp(k, 0xB1, 0xF, 0xF, true));
    k = min(k, __builtin_amdgcn_mov_dpp(k, 0x124, 0xF, 0xF, true));
    k = min(k, __builtin_amdgcn_mov_dpp(k, 0x128, 0xF, 0xF, true));
    return k;
}

template <int CIN>
constexpr int nsteps() {
    return CIN == 4 ? 27 : 108;
}

// A fragment of k-step s for lane (c, g): weight of output channel c,
// input channel ci(s, g), tap q(s); zero outside c's group
template <int CIN, int G>
__device__ __forceinline__ float a_frag(const float* w, int s, int c, int g) {
    int q, ci;
    if constexpr (CIN == 4) {
        q = s;
        ci = g;
    } else {
        q = s % 27;
        ci = 4 * (s / 27) + g;
    }
    constexpr int cpg = CIN / G;  // input channels per group
    const int gi = ci / cpg, go = c / (CO / G);
    return gi == go ? w[(c * cpg + (ci - gi * cpg)) * 27 + q] : 0.0f;
}

// LDS offset of k-step s relative to the lane's tap-(0,0,0) address (wave-uniform part)
template <int CIN>
__device__ __forceinline__ int step_off(int s, int YS, int ZS, int CS) {
    const int q = CIN == 4 ? s : s % 27;
    const int dz = q / 9, dy = (q / 3) % 3, dx = q % 3;
    const int j = CIN == 4 ? 0 : s / 27;
    return j * 4 * CS + dz * ZS + dy * YS + dx;
}

struct FwdParams {
    const float* x;
    const int64_t* rows;  // sample b reads x row rows[b] (null: b)
    const float* w;
    const float* bias;
    float* y;
    uint8_t* amax;  // null: inference
    Geom g;
};

// load the block's input region [z0, z0+ZL) x [y0, y0+YL) x [x0, x0+XL) with
// async global->LDS copies (global_load_lds: no VGPRs, all rows in flight);
// wave w takes rows w, w+4, ... of (ci, zz, yy), advanced incrementally.
// Coordinates outside the volume are clamped: those LDS values only feed conv
// positions outside the output (masked), but stay finite for the backward.
typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* glb_ptr_t;

template <int CIN, int NTHREADS>
__device__ __forceinline__ void load_tile(float* xs, const float* xb, const Geom& g, int z0, int y0, int x0) {
    constexpr int NWV = NTHREADS / 64;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    int ci = 0, zz = 0, yy = wave;
    while (yy >= g.YL) {
        yy -= g.YL;
        if (++zz == g.ZL) {
            zz = 0;
            ++ci;
        }
    }
    for (; ci < CIN;) {
        const int gz = min(max(z0 + zz, 0), g.D - 1), gy = min(max(y0 + yy, 0), g.H - 1);
        const float* src = xb + (((size_t)ci * g.D + gz) * g.H + gy) * g.W;
        float* dst = xs + ci * g.CS + zz * g.ZS + yy * g.YS;
        for (int x = 0; x < g.XL; x += 64)
            if (lane < g.XL - x)
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(src + min(max(x0 + x + lane, 0), g.W - 1)),
                                                 (lds_ptr_t)(dst + x), 4, 0, 0);
        yy += NWV;
        while (yy >= g.YL) {
            yy -= g.YL;
            if (++zz == g.ZL) {
                zz = 0;
                ++ci;
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's copies have landed (barrier follows)
}

// The MFMA main loop shared by the forward and the data-gradient kernels: the
// block's LDS tile xs holds a [cin][ZL][YL][XL] input region; rows r of
// (tz, ty) = (r / PYB, r % PYB) times x-tile pairs (tx, tx + 1) are spread
// round-robin over the 4 wavefronts; tile (r, tx) covers the 2x2x4 positions
// at LDS (2tz, 2ty, 4tx).  epi(acc[2], r, xp) consumes the two tiles' D
// (lane (c, g): rows 4g..4g+3, position c).
template <int CIN, int PYB, class Epi>
__device__ __forceinline__ void conv_core(const float* xs, const float (&af)[nsteps<CIN>()], const Geom& g,
                                          int nrows, Epi&& epi) {
    constexpr int NS = nsteps<CIN>();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, gq = lane >> 4;
    const int zc = c >> 3, yc = (c >> 2) & 1, xc = c & 3;
    const int lane_base = gq * g.CS + zc * g.ZS + yc * g.YS + xc;
    const int nxp = (g.XT + 1) / 2;
    int row = 0, xp = wave;
    while (xp >= nxp) {
        xp -= nxp;
        ++row;
    }
    auto tile_base = [&](int r, int tx) { return lane_base + 2 * (r / PYB) * g.ZS + 2 * (r % PYB) * g.YS + 4 * tx; };
    constexpr int CH = conv_batch<CIN>();  // k-steps per register batch (9: one dz slice, 27: a tap set)
    constexpr int NTH = conv_threads<CIN>();
    float bv[2][2][CH];     // [buffer][tile][step]
    int toff[27];           // tap offsets (wave-uniform: scalar registers)
#pragma unroll
    for (int q = 0; q < 27; ++q) toff[q] = (q / 9) * g.ZS + ((q / 3) % 3) * g.YS + q % 3;
    // batch j = k-steps CH*j .. CH*j + CH-1: input-channel quad j / BPQ, taps (j % BPQ) * CH ..
    constexpr int BPQ = 27 / CH;  // batches per input-channel quad
    auto fetch = [&](float (&dst)[2][CH], int r, int xq, int j) {
        const int b0 = tile_base(r, 2 * xq) + (j / BPQ) * 4 * g.CS, b1 = b0 + 4;
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            dst[0][q] = xs[b0 + toff[(j % BPQ) * CH + q]];
            dst[1][q] = xs[b1 + toff[(j % BPQ) * CH + q]];
        }
    };
    constexpr int NJ = NS / CH;  // tap sets (input-channel quads) per tile
    if (row < nrows) fetch(bv[0], row, xp, 0);
    // one work item; buffer parity is compile-time (register arrays stay in registers)
    auto item = [&](auto start) {
        constexpr int S0 = decltype(start)::value;
        f4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
        int nrow = row, nx = xp + NTH / 64;
        while (nx >= nxp) {
            nx -= nxp;
            ++nrow;
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int cb = (S0 + j) & 1;
            // the next batch (next tap set of this item, or the next item) is read
            // two values per MFMA pair, so few LDS reads are ever outstanding
            // (after the last item the "next" batch re-reads this item's tile:
            // unconditional loads, no exec-mask branches in the loop)
            const bool nxt = j + 1 < NJ || nrow < nrows;
            const int fr = j + 1 < NJ ? row : (nxt ? nrow : row), fx = j + 1 < NJ ? xp : (nxt ? nx : xp);
            const int fj = j + 1 < NJ ? j + 1 : 0;
            const int b0 = tile_base(fr, 2 * fx) + (fj / BPQ) * 4 * g.CS, b1 = b0 + 4;
#pragma unroll
            for (int q = 0; q < CH; ++q) {
                {
                    bv[cb ^ 1][0][q] = xs[b0 + toff[(fj % BPQ) * CH + q]];
                    bv[cb ^ 1][1][q] = xs[b1 + toff[(fj % BPQ) * CH + q]];
                }
                acc[0] = mfma4(af[j * CH + q], bv[cb][0][q], acc[0]);
                acc[1] = mfma4(af[j * CH + q], bv[cb][1][q], acc[1]);
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 LDS reads
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMAs
            }
        }
        epi(acc, row, xp);
        row = nrow;
        xp = nx;
    };
    while (row < nrows) {
        item(std::integral_constant<int, 0>{});
        if constexpr (NJ % 2 == 1) {
            if (row >= nrows) break;
            item(std::integral_constant<int, 1>{});
        }
    }
}

template <int CIN, int G, int PZB, int PYB, bool TRAIN>
__global__ __launch_bounds__(conv_threads<CIN>()) void k_conv_relu_pool(FwdParams P) {
    extern __shared__ float xs[];
    constexpr int NS = nsteps<CIN>();
    const Geom& g = P.g;
    const int b = blockIdx.z, pz0 = blockIdx.y * PZB, py0 = blockIdx.x * PYB;
    const int lane = threadIdx.x & 63, c = lane & 15, gq = lane >> 4;
    const int64_t srow = P.rows ? P.rows[b] : b;
    const float* xb = P.x + srow * (int64_t)CIN * g.D * g.H * g.W;
    const int z0 = 2 * pz0 - g.pd, y0 = 2 * py0 - g.ph, x0 = -g.pw;
    load_tile<CIN, conv_threads<CIN>()>(xs, xb, g, z0, y0, x0);
    float af[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) af[s] = a_frag<CIN, G>(P.w, s, c, gq);
    float bias[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[r] = P.bias[4 * gq + r];
    __syncthreads();

    const int zc = c >> 3, yc = (c >> 2) & 1, xc = c & 3;
    const int widx = zc * 4 + yc * 2 + (xc & 1);  // = rank of the lane in its window (0..7)
    const int64_t chan = (int64_t)g.PD * g.PH * g.PW;
    // after the window reduction every lane of a window holds its 4 channels'
    // maxima: the lane of rank i < 4 stores channel 4g + i (one store per lane)
    const int myr = widx & 3;
    const bool storer = widx < 4;
    float* ybase = P.y + ((int64_t)b * CO + 4 * gq + myr) * chan;
    uint8_t* abase = TRAIN ? P.amax + ((int64_t)b * CO + 4 * gq + myr) * chan : nullptr;
    conv_core<CIN, PYB>(xs, af, g, PZB * PYB, [&](const f4 (&acc)[2], int row, int xp) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int tx = 2 * xp + u;
            const int tz = row / PYB, ty = row % PYB;
            const int pz = pz0 + tz, py = py0 + ty;
            const int cz = 2 * pz - g.pd + zc, cy = 2 * py - g.ph + yc, cx = 4 * tx - g.pw + xc;
            const bool valid = cz >= 0 && cz < g.cd && cy >= 0 && cy < g.ch && cx >= 0 && cx < g.cw;
            const int px = 2 * tx + (xc >> 1);
            float mine = 0.0f;
            int kmine = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = valid ? fmaxf(acc[u][r] + bias[r], 0.0f) : -INFINITY;
                const float m = win_max(v);
                mine = r == myr ? m : mine;
                if constexpr (TRAIN) {
                    const int k = win_min(v == m ? widx : 8);  // torch: first maximum in (z, y, x) window order
                    kmine = r == myr ? k : kmine;
                }
            }
            if (storer && tx < g.XT && pz < g.PD && py < g.PH && px < g.PW) {
                const int64_t o = ((int64_t)pz * g.PH + py) * g.PW + px;
                ybase[o] = mine;
                if constexpr (TRAIN) abase[o] = (uint8_t)(kmine | (mine > 0.0f ? 8 : 0));
            }
        }
    });
}

// ---------------------------------------------------------------------------
// Forward, z-ring version (the launched forward).  A block owns a y band of
// PYB pooled rows (full x) of one sample and sweeps a chunk of ZC pooled z
// rows.  Its LDS holds a ring of kRing input z-planes (all CIN channels,
// [ci][yl][xl]); pooled row k needs planes 2k..2k+3 (relative to the pool
// padding), and while the waves compute it the next two planes stream into
// the two free slots by LDS DMA (global_load_lds, VEC floats per lane), so
// the input is read once per chunk (plus 2 halo planes) and its transfer
// overlaps the MFMAs; one barrier per pooled row.  Each item (2 tiles of
// 2x2x4 positions) runs the MFMA chain of 27 k-steps per input-channel quad;
// the epilogue of the PREVIOUS item (bias, ReLU, window max / first argmax,
// stores through a buffer descriptor whose range check drops masked lanes --
// no branches) is issued between this item's MFMAs.
//
// LDS strides (dwords mod 32): row YS = 4, channel CS = 8, slot = 16 (the
// ring wrap too: 6 slots), so the 32 lanes of a ds_read (16 positions x 2
// channels) hit 32 banks.
constexpr int kRing = 6;
// DMA pieces per wave and slot (one source offset register each): conv1's
// 16-B pieces need 2 per wave at 64^3 and 128^3; 4-B pieces up to 8 (conv1
// on unaligned rows) or 12 (16-channel slots)
template <int CIN, int VEC>
constexpr int ring_max_pieces() {
    return VEC == 4 ? 2 : (CIN == 4 ? 8 : 12);
}

struct RingGeom {
    Geom g;            // dims, pool padding, XT; YL, XL, YS; CS = channel stride
    int32_t SLOT;      // floats per plane slot (CIN channels)
    int32_t npiece;    // 64*VEC-float DMA pieces per slot
    int32_t nyb;       // y bands
    int32_t ZC;        // pooled z rows per block (z chunk)
};

// SR = slot stride residue (mod 32 dwords).  The forward relies on 16 (lanes
// of one gather straddle two adjacent slots); the wgrad B gather spans 3 ring
// slots per instruction, where 12 spreads them best (modelled: max bank
// multiplicity 1.26-1.30 vs 1.43-1.56 at 16).
template <int CIN, int PYB, int VEC, int SR = 16>
RingGeom make_ring_geom(const rt_conv_layer* L, int B, int nthreads) {
    RingGeom r{};
    Geom& g = r.g;
    g.D = L->in_dims[0];
    g.H = L->in_dims[1];
    g.W = L->in_dims[2];
    g.cd = g.D - 2;
    g.ch = g.H - 2;
    g.cw = g.W - 2;
    g.pd = L->pool_pad[0];
    g.ph = L->pool_pad[1];
    g.pw = L->pool_pad[2];
    g.PD = (g.cd + 2 * g.pd - 2) / 2 + 1;
    g.PH = (g.ch + 2 * g.ph - 2) / 2 + 1;
    g.PW = (g.cw + 2 * g.pw - 2) / 2 + 1;
    g.XT = (g.PW + 1) / 2;
    g.ZL = 4;
    g.YL = 2 * PYB + 2;
    g.XL = 4 * g.XT + 2;
    g.YS = round_mod((g.XL + VEC - 1) / VEC * VEC, 4);
    g.ZS = 0;
    g.CS = round_mod(g.YL * g.YS, 8);
    r.SLOT = round_mod(CIN * g.CS, SR);
    r.npiece = (r.SLOT + 64 * VEC - 1) / (64 * VEC);
    r.nyb = (g.PH + PYB - 1) / PYB;
    // z chunks: enough blocks to fill the chip a few times over (each chunk
    // re-reads 2 halo planes)
    const int64_t per_chunk = (int64_t)r.nyb * B;
    int nzc = (int)std::min<int64_t>(g.PD, std::max<int64_t>(1, (4096 + per_chunk - 1) / per_chunk));
    r.ZC = (g.PD + nzc - 1) / nzc;
    (void)nthreads;
    return r;
}

// LDS-DMA loader of ring slots: slot = one input z-plane of all CIN channels
// of the block's y band, [ci][yl][xl]; lane l of wave w fills VEC floats of
// piece w + NW*i.  Sources are clamped into the volume (out-of-volume values
// feed masked positions only, and stay finite for the backward).
template <int CIN, int VEC, int NW, int MPX = 0>
struct RingLoader {
    static constexpr int MP = MPX ? MPX : ring_max_pieces<CIN, VEC>();
    int goff[MP];              // per piece: offset within a plane of channel 0
    int npw;                   // pieces of this wave

    __device__ __forceinline__ void init(const RingGeom& rg, int y0, int x0, int wave, int lane) {
        const Geom& g = rg.g;
        const int plane = g.H * g.W;
        npw = (rg.npiece - wave + NW - 1) / NW;
#pragma unroll
        for (int i = 0; i < MP; ++i) {
            int f = ((wave + NW * i) * 64 + lane) * VEC;
            f = min(f, rg.SLOT - VEC);
            int ci = f / g.CS;
            const int rem = f - ci * g.CS;
            int yl = rem / g.YS;
            const int xl = rem - yl * g.YS;
            ci = min(ci, CIN - 1);
            yl = min(yl, g.YL - 1);
            const int gy = min(max(y0 + yl, 0), g.H - 1);
            const int gx = min(max(x0 + xl, 0), g.W - VEC);
            goff[i] = ci * g.D * plane + gy * g.W + gx;
        }
    }
    // relative plane t (input z = t - pd, clamped) -> ring slot.  The pieces
    // are expanded by a fold over a compile-time index sequence (goff stays in
    // registers; a loop the compiler keeps rolled would index it dynamically)
    template <int I>
    __device__ __forceinline__ void piece(const float* src, float* dst, int wave, int lane, int slot_floats) const {
        const int f0 = (wave + NW * I) * 64 * VEC;
        if (I < npw && f0 + lane * VEC < slot_floats) {
            if constexpr (VEC == 4)
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(src + goff[I]), (lds_ptr_t)(dst + f0), 16, 0, 0);
            else
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(src + goff[I]), (lds_ptr_t)(dst + f0), 4, 0, 0);
        }
    }
    template <int... I>
    __device__ __forceinline__ void pieces(const float* src, float* dst, int wave, int lane, int slot_floats,
                                           std::integer_sequence<int, I...>) const {
        (piece<I>(src, dst, wave, lane, slot_floats), ...);
    }
    __device__ __forceinline__ void load(const float* xb, const RingGeom& rg, float* xs, int t, int slot, int wave,
                                         int lane) const {
        const Geom& g = rg.g;
        const int iz = min(max(t - g.pd, 0), g.D - 1);
        pieces(xb + (size_t)iz * g.H * g.W, xs + slot * rg.SLOT, wave, lane, rg.SLOT,
               std::make_integer_sequence<int, MP>{});
    }
};

// One output row of a ring kernel (the 2 conv z-planes of a pooled row, read
// from ring slots sb.., the block's y band, full x): the items (2 tiles of
// 2x2x4 positions: rows r < PYB times x-tile pairs xp) go round-robin to the
// NW waves, each item one MFMA chain of nsteps k-steps in 9-step register
// batches (one (channel quad, dz) each) read from LDS one batch ahead; the
// PREVIOUS item's epilogue (pv) is issued between this item's MFMAs.
struct RingPrev {
    f4 acc[2];
    int r, xp, k;
    bool ok;
};

template <int CIN, int PYB, int NW, class Epi>
__device__ __forceinline__ void ring_row(const float* xs, const float (&af)[nsteps<CIN>()], const Geom& g, int SLOT,
                                         int sb, int k, int wave, int lane, RingPrev& pv, Epi&& epi) {
    constexpr int NB = nsteps<CIN>() / 9;
    const int c = lane & 15, gq = lane >> 4, zc = c >> 3, yc = (c >> 2) & 1, xc = c & 3;
    const int lane_xy = gq * g.CS + yc * g.YS + xc;
    const int nxp = (g.XT + 1) / 2;
    const int NI = (PYB * nxp + NW - 1) / NW;  // item rounds per row (all waves run NI)
    int zoff[3];
#pragma unroll
    for (int dz = 0; dz < 3; ++dz) {
        int sl = sb + zc + dz;
        sl = sl >= kRing ? sl - kRing : sl;
        zoff[dz] = sl * SLOT + lane_xy;
    }
    int r = 0, xp = wave;
    while (xp >= nxp) {
        xp -= nxp;
        ++r;
    }
    for (int it = 0; it < NI; ++it) {
        const bool ok = r < PYB;
        const int rr = ok ? r : PYB - 1;
        const int tb = 2 * rr * g.YS + 8 * xp;
        float bv[2][2][9];
        auto fetch = [&](float (&dst)[2][9], int bj) {
            const int dz = bj % 3, j = bj / 3;
            const int base = zoff[dz] + tb + j * 4 * g.CS;
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    dst[0][dy * 3 + dx] = xs[base + dy * g.YS + dx];
                    dst[1][dy * 3 + dx] = xs[base + dy * g.YS + dx + 4];
                }
        };
        fetch(bv[0], 0);
        epi(pv.acc, pv.r, pv.xp, pv.k, pv.ok);  // the previous item's epilogue, between this item's MFMAs
        f4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
        for (int bj = 0; bj < NB; ++bj) {
            if (bj + 1 < NB) fetch(bv[(bj + 1) & 1], bj + 1);
#pragma unroll
            for (int q = 0; q < 9; ++q) {
                acc[0] = mfma4(af[bj * 9 + q], bv[bj & 1][0][q], acc[0]);
                acc[1] = mfma4(af[bj * 9 + q], bv[bj & 1][1][q], acc[1]);
            }
        }
        pv.acc[0] = acc[0];
        pv.acc[1] = acc[1];
        pv.r = r;
        pv.xp = xp;
        pv.k = k;
        pv.ok = ok;
        xp += NW;
        while (xp >= nxp) {
            xp -= nxp;
            ++r;
        }
    }
}

// ring_row in bf16x3 (conv1 only): the ring slots hold packed words (hi << 16
// | lo, converted in place once per plane, ring_pack_bf); lane (c, g) supplies
// B = 8 taps 8b..8b+7 of input channel g at position c (taps 27..31 zero) and
// A = the same taps of W[c][g] as bf16 hi / lo images in registers, so a
// 2-tile item is 2 x 4 x 3 MFMAs of 16x16x32 in place of 2 x 27 of 16x16x4.
// The accumulator layout is the f32 kernel's: the epilogue is shared.
template <int PYB, int NW, class Epi>
__device__ __forceinline__ void ring_row_bf(const uint32_t* xs, const bf8 (&ah)[4], const bf8 (&al)[4], const Geom& g,
                                            int SLOT, int sb, int k, int wave, int lane, RingPrev& pv, Epi&& epi) {
    const int c = lane & 15, gq = lane >> 4, zc = c >> 3, yc = (c >> 2) & 1, xc = c & 3;
    const int lane_xy = gq * g.CS + yc * g.YS + xc;
    const int nxp = (g.XT + 1) / 2;
    const int NI = (PYB * nxp + NW - 1) / NW;
    int zoff[3];
#pragma unroll
    for (int dz = 0; dz < 3; ++dz) {
        int sl = sb + zc + dz;
        sl = sl >= kRing ? sl - kRing : sl;
        zoff[dz] = sl * SLOT + lane_xy;
    }
    int r = 0, xp = wave;
    while (xp >= nxp) {
        xp -= nxp;
        ++r;
    }
    for (int it = 0; it < NI; ++it) {
        const bool ok = r < PYB;
        const int rr = ok ? r : PYB - 1;
        const int tb = 2 * rr * g.YS + 8 * xp;
        uint32_t pw[2][2][8];
        auto fetch = [&](uint32_t (&dst)[2][8], int b) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int tap = 8 * b + j;
                if (tap < 27) {
                    const int base = zoff[tap / 9] + tb + ((tap / 3) % 3) * g.YS + tap % 3;
                    dst[0][j] = xs[base];
                    dst[1][j] = xs[base + 4];
                } else {
                    dst[0][j] = 0u;
                    dst[1][j] = 0u;
                }
            }
        };
        fetch(pw[0], 0);
        epi(pv.acc, pv.r, pv.xp, pv.k, pv.ok);  // the previous item's epilogue, between this item's MFMAs
        f4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            if (b + 1 < 4) fetch(pw[(b + 1) & 1], b + 1);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                bf8 bh, bl;
                bf_unpack8(pw[b & 1][u], bh, bl);
                acc[u] = mfma3(ah[b], al[b], bh, bl, acc[u]);
            }
        }
        pv.acc[0] = acc[0];
        pv.acc[1] = acc[1];
        pv.r = r;
        pv.xp = xp;
        pv.k = k;
        pv.ok = ok;
        xp += NW;
        while (xp >= nxp) {
            xp -= nxp;
            ++r;
        }
    }
}

// in-place f32 -> packed bf16x3 words of n ring slots from `slot` (after their
// DMA landed and a barrier; a barrier before they are read)
template <int NRING = kRing>
__device__ __forceinline__ void ring_pack_bf(float* xs, int slot, int n, int SLOT) {
    for (int s = 0; s < n; ++s) {
        int sl = slot + s;
        sl = sl >= NRING ? sl - NRING : sl;
        float* p = xs + sl * SLOT;
        uint32_t* q = reinterpret_cast<uint32_t*>(p);
        for (int i = threadIdx.x; i < SLOT; i += blockDim.x) q[i] = bf_pack(p[i]);
    }
}

struct RingParams {
    const float* x;
    const int64_t* rows;  // sample b reads x row rows[b] (null: b)
    const float* w;
    const float* bias;
    float* y;
    uint8_t* amax;  // null: inference
    RingGeom rg;
};

template <int CIN, int G, int PYB, int VEC, int NTH, bool TRAIN, bool BF = false>
__global__ __launch_bounds__(NTH) void k_conv_ring(RingParams P) {
    static_assert(!BF || (CIN == 4 && G == 1), "bf16x3: conv1 only");
    extern __shared__ float xs[];
    constexpr int NS = nsteps<CIN>();
    constexpr int NW = NTH / 64;
    const Geom& g = P.rg.g;
    const int SLOT = P.rg.SLOT;
    const int b = blockIdx.z, py0 = blockIdx.x * PYB;
    const int k0 = blockIdx.y * P.rg.ZC, k1 = min(g.PD, k0 + P.rg.ZC);
    if (k0 >= k1) return;
    const int lane = threadIdx.x & 63, c = lane & 15, gq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t srow = P.rows ? P.rows[b] : b;
    const float* xb = P.x + srow * (int64_t)CIN * g.D * g.H * g.W;
    const int y0 = 2 * py0 - g.ph, x0 = -g.pw;

    RingLoader<CIN, VEC, NW> ld;
    ld.init(P.rg, y0, x0, wave, lane);
    auto load_plane = [&](int t, int slot) { ld.load(xb, P.rg, xs, t, slot, wave, lane); };

    // ---- weights (A fragments), bias, epilogue constants
    float af[BF ? 1 : NS];
    bf8 ah[BF ? 4 : 1], al[BF ? 4 : 1];
    if constexpr (BF) {
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            uint32_t pw[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) pw[j] = 8 * b + j < 27 ? bf_pack(P.w[(c * 4 + gq) * 27 + 8 * b + j]) : 0u;
            bf_unpack8(pw, ah[b], al[b]);
        }
    } else {
#pragma unroll
        for (int s = 0; s < NS; ++s) af[s] = a_frag<CIN, G>(P.w, s, c, gq);
    }
    float bias[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[r] = P.bias[4 * gq + r];
    const int zc = c >> 3, yc = (c >> 2) & 1, xc = c & 3;
    const int widx = zc * 4 + yc * 2 + (xc & 1);  // rank of the lane in its pooling window
    // after the window reduction the lane stores channel 4g + myr: the
    // transposed reduction (below) leaves channel 2 (xc & 1) + yc on it
    const int myr = 2 * (xc & 1) + yc;
    const bool storer = widx < 4;
    const int chan = g.PD * g.PH * g.PW;
    const int cbase = (4 * gq + myr) * chan;       // element offset of this lane's channel in the sample
    const __amdgpu_buffer_rsrc_t ysrd = __builtin_amdgcn_make_buffer_rsrc(
        P.y + (int64_t)b * CO * chan, 0, CO * chan * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t asrd = __builtin_amdgcn_make_buffer_rsrc(
        TRAIN ? (void*)(P.amax + (int64_t)b * CO * chan) : (void*)P.y, 0, TRAIN ? CO * chan : 0, 0x00020000);

    // epilogue of one item (tiles tx = 2xp, 2xp+1 of row r at pooled z pz)
    auto epi = [&](const f4 (&acc)[2], int r, int xp, int pz, bool ok) {
        const int py = py0 + r;
        const int cz = 2 * pz - g.pd + zc, cy = 2 * py - g.ph + yc;
        const bool vzy = ok && cz >= 0 && cz < g.cd && cy >= 0 && cy < g.ch;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int tx = 2 * xp + u;
            const int cx = 4 * tx - g.pw + xc;
            const bool valid = vzy && cx >= 0 && cx < g.cw;
            const int px = 2 * tx + (xc >> 1);
            float mine = 0.0f;
            int kmine = 0;
            // transposed window reduction: each DPP step halves the
            // channels a lane keeps while it reduces over a window bit
            // (bit 0: xor 1; bit 2: row_ror 4, the partner's bit 2 always
            // differs; bit 3: row_ror 8, same channel) -- 3 / 6 DPP moves
            // for the 4 channels instead of 12 / 24.  (value, index) pairs
            // combine as max value, smallest window index among equals:
            // torch's first maximum in (z, y, x) order.
            int vi[4];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
                vi[rr] = __float_as_int(valid ? fmaxf(acc[u][rr] + bias[rr], 0.0f) : -INFINITY);
            const bool b0 = (c & 1) != 0, b2 = ((c >> 2) & 1) != 0;
            auto comb = [](int& v, int& k, int rv, int rk) {
                const int m = max(v, rv);
                k = min(v == m ? k : 8, rv == m ? rk : 8);
                v = m;
            };
            int va = b0 ? vi[2] : vi[0], vb = b0 ? vi[3] : vi[1];
            const int ra = __builtin_amdgcn_mov_dpp(b0 ? vi[0] : vi[2], 0xB1, 0xF, 0xF, true);
            const int rb = __builtin_amdgcn_mov_dpp(b0 ? vi[1] : vi[3], 0xB1, 0xF, 0xF, true);
            int ka = widx, kb = widx;
            if constexpr (TRAIN) {
                comb(va, ka, ra, widx ^ 1);
                comb(vb, kb, rb, widx ^ 1);
            } else {
                va = max(va, ra);
                vb = max(vb, rb);
            }
            int v = b2 ? vb : va, k = b2 ? kb : ka;
            const int rv2 = __builtin_amdgcn_mov_dpp(b2 ? va : vb, 0x124, 0xF, 0xF, true);
            if constexpr (TRAIN) {
                const int rk2 = __builtin_amdgcn_mov_dpp(b2 ? ka : kb, 0x124, 0xF, 0xF, true);
                comb(v, k, rv2, rk2);
                const int rv3 = __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, true);
                const int rk3 = __builtin_amdgcn_mov_dpp(k, 0x128, 0xF, 0xF, true);
                comb(v, k, rv3, rk3);
                kmine = k;
            } else {
                v = max(v, rv2);
                v = max(v, __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, true));
            }
            mine = __int_as_float(v);
            const bool st = ok && storer && tx < g.XT && py < g.PH && px < g.PW;
            const int o = cbase + (pz * g.PH + py) * g.PW + px;
            __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(mine), ysrd, st ? 4 * o : INT32_MIN, 0, 0);
            if constexpr (TRAIN)
                __builtin_amdgcn_raw_buffer_store_b8((uint8_t)(kmine | (mine > 0.0f ? 8 : 0)), asrd,
                                                     st ? o : INT32_MIN, 0, 0);
        }
    };

    // ---- prologue: planes 0..3 of the chunk
#pragma unroll
    for (int i = 0; i < 4; ++i) load_plane(2 * k0 + i, i);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    if constexpr (BF) {
        ring_pack_bf(xs, 0, 4, SLOT);
        __syncthreads();
    }

    RingPrev pv{{{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}}, 0, 0, k0, false};
    int sb = 0;  // ring slot of plane 2k
    for (int k = k0; k < k1; ++k) {
        if (k + 1 < k1) {  // planes of the next pooled row -> the two free slots
            load_plane(2 * k + 4, sb + 4 >= kRing ? sb + 4 - kRing : sb + 4);
            load_plane(2 * k + 5, sb + 5 >= kRing ? sb + 5 - kRing : sb + 5);
        }
        if constexpr (BF)
            ring_row_bf<PYB, NW>(reinterpret_cast<const uint32_t*>(xs), ah, al, g, SLOT, sb, k, wave, lane, pv, epi);
        else
            ring_row<CIN, PYB, NW>(xs, af, g, SLOT, sb, k, wave, lane, pv, epi);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's DMA for the next row has landed
        __syncthreads();                     // ... every wave's; and nobody still reads the slots reloaded next
        sb = sb + 2 >= kRing ? sb + 2 - kRing : sb + 2;
        if constexpr (BF) {
            if (k + 1 < k1) {  // the two planes that just landed, before row k + 1 reads them
                ring_pack_bf(xs, sb + 2 >= kRing ? sb + 2 - kRing : sb + 2, 2, SLOT);
                __syncthreads();
            }
        }
    }
    epi(pv.acc, pv.r, pv.xp, pv.k, pv.ok);
}

template <int CIN, int G, int PYB, int VEC, int NTH, bool BF = false>
int launch_ring(const RingGeom& rg, int32_t B, const float* x, const int64_t* rows, const float* w,
                const float* bias, float* y, uint8_t* amax, hipStream_t st) {
    RingParams P{x, rows, w, bias, y, amax, rg};
    const size_t lds = (size_t)kRing * rg.SLOT * sizeof(float);
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_ring<CIN, G, PYB, VEC, NTH, true, BF>)) return rc_lds;
        if (const int rc_lds = allow_big_lds(&k_conv_ring<CIN, G, PYB, VEC, NTH, false, BF>)) return rc_lds;
        attr = true;
    }
    dim3 grid(rg.nyb, (rg.g.PD + rg.ZC - 1) / rg.ZC, B);
    if (amax)
        hipLaunchKernelGGL((k_conv_ring<CIN, G, PYB, VEC, NTH, true, BF>), grid, dim3(NTH), lds, st, P);
    else
        hipLaunchKernelGGL((k_conv_ring<CIN, G, PYB, VEC, NTH, false, BF>), grid, dim3(NTH), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

// ---------------------------------------------------------------------------
// Forward in the Winograd form F(2x2x2, 3x3x3) on f32 MFMA: conv1 and the
// grouped stages (groups 2 and 4; the launched f32 forward of all three).  A
// 2x2x2 Winograd output tile is exactly one 2x2x2 pooling window, so a
// window's 8 conv outputs come out in ONE lane's registers: the pooling max
// and its first-maximum index are plain register compares (no DPP), and the
// 27 taps of a direct conv output become 64 element-wise products per window:
//   M[xi][co][win] = sum_ci U[xi][co][ci] * V[xi][ci][win],  xi in 4x4x4,
// one v_mfma_f32_16x16x4_f32 per xi, 16 windows and 4 input channels of the
// block's group (K), chained over the group's CPG / 4 channel quads:
//   conv1 (CPG 4, 16 outputs):  64 MFMAs per 16 windows, 216 direct;
//   conv2 (groups 2, CPG 8):   128 per group (rows of the other group's 8
//                              outputs are zero), 2 x 128 against the direct
//                              z-shift form's 576 for both groups;
//   conv3 (groups 4, CPG 4):    64 per group (12 zero rows), 4 x 64 vs 432.
//   U = G w G^T (per axis G = [1 0 0; .5 .5 .5; .5 -.5 .5; 0 0 1]): the
//       filter transform, once per block into LDS (A operand: lane (co = l &
//       15, ci = l >> 4); rows co >= COG hold zeros);
//   V = B^T d B (per axis B^T = [1 0 -1 0; 0 1 1 0; 0 -1 1 0; 0 1 0 -1]): the
//       4x4x4 input patch of the window, per lane (B operand: lane (window n
//       = l & 15, ci = l >> 4)) from the plane ring, adds only;
//   Y = A^T M A (per axis A^T = [1 1 1 0; 0 1 -1 -1]): applied axis by axis
//       as the MFMAs of one (xi_x, xi_y) column complete (z, then y, then x).
// Every operation is f32 (MFMA: exact FMA chains); the result differs from the
// direct sum by rounding only (measured error vs float64 below the direct f32
// kernel's, tools/wino_err.py; tests/test_gpu_c3d.py gates it against float64
// torch like the direct kernels).  The block streams z-planes of its group's
// CPG channels through the 6-slot LDS ring of k_conv_ring (pooled row k needs
// planes 2k..2k+3, the next two load by LDS DMA while the row computes); an
// item is 16 consecutive windows of the block's y band (row-major over
// (py, px)), one per lane group column n.
// ---------------------------------------------------------------------------
#ifndef RT_WINO_C1_NTH
#define RT_WINO_C1_NTH 256
#endif
constexpr int kWinoC1Nth = RT_WINO_C1_NTH;
  // threads per block of conv1's Winograd forward

#ifndef RT_WINO_PATCH_BATCH
#define RT_WINO_PATCH_BATCH 1
#endif

template <int CPG>
constexpr int wino_u_floats() {  // U in LDS: 16 columns x 64 lanes x 4 xi_z x CPG / 4 quads
    return 16 * 64 * 4 * (CPG / 4);
}

// U element (column j, lane, i = xi_z * NS + s) in LDS: float4 q = i / 4 of
// the lane's 4 NS values at ((j NS + q) 64 + lane) 4, so the column's NS
// ds_read_b128 are each 64 lanes x 16 B contiguous (conflict-free; a lane's
// values contiguous put lanes 8 dwords apart at NS = 2: 2-way conflicts)
template <int NS>
__device__ __forceinline__ int wino_u_index(int j, int lane, int i) {
    return ((j * NS + (i >> 2)) * 64 + lane) * 4 + (i & 3);
}

struct WinoParams {
    const float* x;
    const int64_t* rows;  // sample b reads x row rows[b] (null: b)
    const float* w;       // [16][CPG][27]
    const float* bias;
    float* y;
    uint8_t* amax;        // null: inference
    RingGeom rg;          // the group's CPG channels per slot
    int32_t G;            // groups (blockIdx.z = sample * G + group)
    int32_t pyb;          // pooled rows per y band
};

// conv3 (4 channels per group, 4 outputs): 3 waves per SIMD (<= 168 VGPRs,
// no spills; left free the compiler took 150 VGPRs + 44 AGPRs = 2 waves) --
// its 256-thread blocks are small enough for 3 per CU
template <int CPG, int COG, int VEC, int NTH, bool TRAIN>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(CPG == 4 && NTH == 256 ? 3 : 1)))
void k_conv_wino(WinoParams P) {
    extern __shared__ float xs[];
    constexpr int NW = NTH / 64;
    constexpr int NS = CPG / 4;  // channel quads (MFMA k-steps) per xi
    constexpr bool kWinoPrio = CPG == 4 && COG == 16;  // conv1
    constexpr bool kPatchBatch = RT_WINO_PATCH_BATCH && COG != 4;  // (conv3: spills at 3 waves per SIMD)
    const Geom& g = P.rg.g;
    const int SLOT = P.rg.SLOT;
    const int b = blockIdx.z / P.G, grp = blockIdx.z - b * P.G;
    const int PYB = P.pyb, py0 = blockIdx.x * PYB;
    const int k0 = blockIdx.y * P.rg.ZC, k1 = min(g.PD, k0 + P.rg.ZC);
    if (k0 >= k1) return;
    const int lane = threadIdx.x & 63, n = lane & 15, gq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t srow = P.rows ? P.rows[b] : b;
    const int cin = CPG * P.G;
    const float* xb = P.x + (srow * cin + (int64_t)grp * CPG) * g.D * g.H * g.W;
    const int y0 = 2 * py0 - g.ph;

    RingLoader<CPG, VEC, NW, 16> ld;
    ld.init(P.rg, y0, -g.pw, wave, lane);
    auto load_plane = [&](int t, int slot) { ld.load(xb, P.rg, xs, t, slot, wave, lane); };
    // ---- prologue DMA first: the filter transform below runs under it
#pragma unroll
    for (int i = 0; i < 4; ++i) load_plane(2 * k0 + i, i);

    // ---- U = G w G^T for (co = n, ci = 4s + gq), by wave 0 into LDS after the
    // ring: element (j = xy * 4 + xx, lane, xz * NS + s) at wino_u_index (one
    // or two ds_read_b128 per (xi_x, xi_y) column give its 4 xi_z x NS values)
    float* us = xs + kRing * SLOT;
    if (wave == 0) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const bool live = n < COG;
            const float* w = P.w + ((grp * COG + (live ? n : 0)) * CPG + 4 * s + gq) * 27;
            float t[36];  // after the x axis: [kz][ky][xx]
#pragma unroll
            for (int r = 0; r < 9; ++r) {
                const float w0 = live ? w[3 * r] : 0.0f, w1 = live ? w[3 * r + 1] : 0.0f;
                const float w2 = live ? w[3 * r + 2] : 0.0f;
                t[4 * r] = w0;
                t[4 * r + 1] = 0.5f * ((w0 + w1) + w2);
                t[4 * r + 2] = 0.5f * ((w0 - w1) + w2);
                t[4 * r + 3] = w2;
            }
            float sy[48];  // after the y axis: [kz][xy][xx]
#pragma unroll
            for (int kz = 0; kz < 3; ++kz)
#pragma unroll
                for (int xx = 0; xx < 4; ++xx) {
                    const float a0 = t[(kz * 3) * 4 + xx], a1 = t[(kz * 3 + 1) * 4 + xx];
                    const float a2 = t[(kz * 3 + 2) * 4 + xx];
                    sy[(kz * 4) * 4 + xx] = a0;
                    sy[(kz * 4 + 1) * 4 + xx] = 0.5f * ((a0 + a1) + a2);
                    sy[(kz * 4 + 2) * 4 + xx] = 0.5f * ((a0 - a1) + a2);
                    sy[(kz * 4 + 3) * 4 + xx] = a2;
                }
#pragma unroll
            for (int j = 0; j < 16; ++j) {  // j = xy * 4 + xx; along z
                const float a0 = sy[j], a1 = sy[16 + j], a2 = sy[32 + j];
                us[wino_u_index<NS>(j, lane, s)] = a0;
                us[wino_u_index<NS>(j, lane, NS + s)] = 0.5f * ((a0 + a1) + a2);
                us[wino_u_index<NS>(j, lane, 2 * NS + s)] = 0.5f * ((a0 - a1) + a2);
                us[wino_u_index<NS>(j, lane, 3 * NS + s)] = a2;
            }
        }
    }
    float bias[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[r] = 4 * gq + r < COG ? P.bias[grp * COG + 4 * gq + r] : 0.0f;
    const int chan = g.PD * g.PH * g.PW;
    const bool lane_co = 4 * gq < COG;  // this lane group's 4 rows are outputs of the group
    float* ybase = P.y + ((int64_t)b * CO + grp * COG + (lane_co ? 4 * gq : 0)) * chan;
    uint8_t* abase = TRAIN ? P.amax + ((int64_t)b * CO + grp * COG + (lane_co ? 4 * gq : 0)) * chan : nullptr;
    const int nwin = min(PYB, g.PH - py0) * g.PW;  // windows of the band
    const int items = (nwin + 15) >> 4;

    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    int sb = 0;  // ring slot of plane 2k
    for (int k = k0; k < k1; ++k) {
        if (k + 1 < k1) {  // planes of the next pooled row -> the two free slots
            load_plane(2 * k + 4, sb + 4 >= kRing ? sb + 4 - kRing : sb + 4);
            load_plane(2 * k + 5, sb + 5 >= kRing ? sb + 5 - kRing : sb + 5);
        }
        for (int it = wave; it < items; it += NW) {
            const int wi = min(16 * it + n, nwin - 1);  // lanes past the band repeat its last window (not stored)
            const int r = wi / g.PW, px = wi - r * g.PW;
            const int py = py0 + r;
            // ---- in two halves of the x axis (xi_x = 2h, 2h + 1): V = B^T d B
            // of the lane's 4x4x4 patches (channels 4s + gq), then M = U V
            // (MFMA, chained over the NS channel quads) and Y = A^T M A.  (Both
            // halves at once kept all 64 products in flight and spilled.)
            const int xoff = gq * g.CS + 2 * r * g.YS + 2 * px;
            const f4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
            f4 Y[2][2][2];   // [ox][oy][oz]
            f4 Sx[2][2][2];  // [xi_x & 1][oy][oz]: the y-axis sums of a column pair
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float v[NS][32];  // [s][dz][dy][kx] -> [s][xz][xy][kx], xi_x = 2h + kx
                int xo = xoff;
                asm volatile("" : "+v"(xo));  // the halves' patch reads stay separate (no CSE)
                // conv1: the input transform at base issue priority, the MFMA
                // columns raised, so waves in their column phase keep the MFMA
                // pipe fed (conv1 forward 2.32 -> 2.29 ms per 512 samples,
                // training forward 2.32 -> 2.28; conv2's training forward lost
                // 3 % with it: r05_s17)
                if constexpr (kWinoPrio) __builtin_amdgcn_s_setprio(0);
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    // the whole half's patch reads issued before its transform
                    // (one exposed LDS latency instead of one per 2 dy rows)
                    float2 pa[4][4], pc[4][4];
                    if constexpr (kPatchBatch) {
#pragma unroll
                    for (int dz = 0; dz < 4; ++dz) {
                        int sl = sb + dz;
                        sl = sl >= kRing ? sl - kRing : sl;
                        const float* p = xs + sl * SLOT + 4 * s * g.CS + xo;
#pragma unroll
                        for (int dy = 0; dy < 4; ++dy) {
                            pa[dz][dy] = *reinterpret_cast<const float2*>(p + dy * g.YS);
                            pc[dz][dy] = *reinterpret_cast<const float2*>(p + dy * g.YS + 2);
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                    }
#pragma unroll
                    for (int dz = 0; dz < 4; ++dz) {
                        int sl = sb + dz;
                        sl = sl >= kRing ? sl - kRing : sl;
                        const float* p = xs + sl * SLOT + 4 * s * g.CS + xo;
                        (void)p;
#pragma unroll
                        for (int dy = 0; dy < 4; ++dy) {
                            float2 a, c;
                            if constexpr (kPatchBatch) {
                                a = pa[dz][dy];
                                c = pc[dz][dy];
                            } else {
                                a = *reinterpret_cast<const float2*>(p + dy * g.YS);
                                c = *reinterpret_cast<const float2*>(p + dy * g.YS + 2);
                            }
                            float* q = v[s] + (dz * 4 + dy) * 2;
                            if (h == 0) {  // B^T along x, rows 0, 1
                                q[0] = a.x - c.x;
                                q[1] = a.y + c.x;
                            } else {       // rows 2, 3
                                q[0] = c.x - a.y;
                                q[1] = a.y - c.y;
                            }
                        }
                    }
#pragma unroll
                    for (int dz = 0; dz < 4; ++dz)  // along y
#pragma unroll
                        for (int kx = 0; kx < 2; ++kx) {
                            float* q = v[s] + dz * 8 + kx;
                            const float d0 = q[0], d1 = q[2], d2 = q[4], d3 = q[6];
                            q[0] = d0 - d2;
                            q[2] = d1 + d2;
                            q[4] = d2 - d1;
                            q[6] = d1 - d3;
                        }
#pragma unroll
                    for (int j = 0; j < 8; ++j) {  // along z
                        const float d0 = v[s][j], d1 = v[s][8 + j], d2 = v[s][16 + j], d3 = v[s][24 + j];
                        v[s][j] = d0 - d2;
                        v[s][8 + j] = d1 + d2;
                        v[s][16 + j] = d2 - d1;
                        v[s][24 + j] = d1 - d3;
                    }
                }
                // software-pipelined columns (xi_x, xi_y): the MFMAs of column c
                // are issued before the sums of column c - 1, whose results pass
                // through an empty asm so they are formed here (left free, the
                // compiler sinks every column's sums below all the MFMAs and
                // their accumulator registers spill)
                f4 pm[4];
                auto column_sums = [&](const f4 (&m)[4], int xx, int xy) {
                    const f4 t0 = add4s(add4s(m[0], m[1]), m[2]), t1 = sub4s(sub4s(m[1], m[2]), m[3]);  // A^T along z
                    f4(&S)[2][2] = Sx[xx & 1];
                    if (xy == 0) {  // A^T along y: rows (1 1 1 0), (0 1 -1 -1)
                        S[0][0] = t0;
                        S[0][1] = t1;
                    } else if (xy == 1) {
                        S[0][0] = add4s(S[0][0], t0);
                        S[0][1] = add4s(S[0][1], t1);
                        S[1][0] = t0;
                        S[1][1] = t1;
                    } else if (xy == 2) {
                        S[0][0] = add4s(S[0][0], t0);
                        S[0][1] = add4s(S[0][1], t1);
                        S[1][0] = sub4s(S[1][0], t0);
                        S[1][1] = sub4s(S[1][1], t1);
                    } else {
                        S[1][0] = sub4s(S[1][0], t0);
                        S[1][1] = sub4s(S[1][1], t1);
                    }
                    if (xy == 0)
                        asm volatile("" : "+v"(S[0][0]), "+v"(S[0][1]));
                    else
                        asm volatile("" : "+v"(S[0][0]), "+v"(S[0][1]), "+v"(S[1][0]), "+v"(S[1][1]));
                    if (xy == 3) {
#pragma unroll
                        for (int oy = 0; oy < 2; ++oy)
#pragma unroll
                            for (int oz = 0; oz < 2; ++oz) {  // A^T along x
                                if (xx == 0) {
                                    Y[0][oy][oz] = S[oy][oz];
                                } else if (xx == 1) {
                                    Y[0][oy][oz] = add4s(Y[0][oy][oz], S[oy][oz]);
                                    Y[1][oy][oz] = S[oy][oz];
                                } else if (xx == 2) {
                                    Y[0][oy][oz] = add4s(Y[0][oy][oz], S[oy][oz]);
                                    Y[1][oy][oz] = sub4s(Y[1][oy][oz], S[oy][oz]);
                                } else {
                                    Y[1][oy][oz] = sub4s(Y[1][oy][oz], S[oy][oz]);
                                }
                            }
                    }
                };
                if constexpr (kWinoPrio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int c = 0; c <= 8; ++c) {  // column c = kx * 4 + xy of this half
                    f4 m[4];
                    if (c < 8) {
                        const int kx = c >> 2, xy = c & 3, xx = 2 * h + kx;
                        const int j = xy * 4 + xx, jv = xy * 2 + kx;
                        float uc[4 * NS];
#pragma unroll
                        for (int q = 0; q < NS; ++q) {
                            const float4 u4 = *reinterpret_cast<const float4*>(us + wino_u_index<NS>(j, lane, 4 * q));
                            uc[4 * q] = u4.x;
                            uc[4 * q + 1] = u4.y;
                            uc[4 * q + 2] = u4.z;
                            uc[4 * q + 3] = u4.w;
                        }
#pragma unroll
                        for (int xz = 0; xz < 4; ++xz) {
                            m[xz] = mfma4(uc[xz * NS], v[0][xz * 8 + jv], zero);
#pragma unroll
                            for (int s = 1; s < NS; ++s) m[xz] = mfma4(uc[xz * NS + s], v[s][xz * 8 + jv], m[xz]);
                        }
                    }
                    if (c > 0) column_sums(pm, 2 * h + ((c - 1) >> 2), (c - 1) & 3);
                    if (c < 8)
#pragma unroll
                        for (int i = 0; i < 4; ++i) pm[i] = m[i];
                }
            }
            // ---- epilogue: bias, ReLU, the window max + first argmax in (z, y, x) order
            const int cz0 = 2 * k - g.pd, cy0 = 2 * py - g.ph, cx0 = 2 * px - g.pw;
            bool vo[8];
#pragma unroll
            for (int o = 0; o < 8; ++o) {
                const int oz = o >> 2, oy = (o >> 1) & 1, ox = o & 1;
                vo[o] = (unsigned)(cz0 + oz) < (unsigned)g.cd & (unsigned)(cy0 + oy) < (unsigned)g.ch &
                        (unsigned)(cx0 + ox) < (unsigned)g.cw;
            }
            const bool st = lane_co & (16 * it + n < nwin);
            const int oidx = (k * g.PH + py) * g.PW + px;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                float m = -INFINITY;
                int km = 0;
#pragma unroll
                for (int o = 0; o < 8; ++o) {
                    const float val = vo[o] ? fmaxf(Y[o & 1][(o >> 1) & 1][o >> 2][rr] + bias[rr], 0.0f) : -INFINITY;
                    if (TRAIN) km = val > m ? o : km;  // strict: the first maximum keeps its index
                    m = fmaxf(m, val);
                }
                if (st && 4 * gq + rr < COG) {
                    ybase[rr * chan + oidx] = m;
                    if (TRAIN) abase[rr * chan + oidx] = (uint8_t)(km | (m > 0.0f ? 8 : 0));
                }
            }
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's DMA for the next row has landed
        __syncthreads();                     // ... every wave's; and nobody still reads the slots reloaded next
        sb = sb + 2 >= kRing ? sb + 2 - kRing : sb + 2;
    }
}

// LDS-bank cycles of one patch read (ds_read_b64: two 32-lane groups, bank =
// dword mod 64) summed over a band's items: lane (n, gq) reads dwords
// gq CS + 2 r YS + 2 px + {0, 1} of window 16 it + n = (r, px), lanes past
// the band repeating its last window (a broadcast).  The read pattern of
// every (channel quad, dz, dy) of an item is this one shifted by a constant.
int wino_read_cycles(int PW, int nwin, int YS, int CS) {
    int total = 0;
    for (int it = 0; it * 16 < nwin; ++it)
        for (int half = 0; half < 2; ++half) {
            int load[64] = {};
            int seen[32][2];
            int ns = 0;
            for (int l = 32 * half; l < 32 * half + 32; ++l) {
                const int n = l & 15, gq = l >> 4;
                const int wi = std::min(16 * it + n, nwin - 1);
                const int a = gq * CS + 2 * (wi / PW) * YS + 2 * (wi % PW);
                bool dup = false;
                for (int i = 0; i < ns && !dup; ++i) dup = seen[i][0] == a;
                if (dup) continue;
                seen[ns][0] = a;
                seen[ns++][1] = 0;
                ++load[a & 63];
                ++load[(a + 1) & 63];
            }
            total += *std::max_element(load, load + 64);
        }
    return total;
}

// Row stride YS and channel stride CS of the Winograd ring (>= XL and YL YS,
// multiples of the DMA width and of 2 for the float2 patch reads, CS <=
// cs_max: the block's LDS budget) with the fewest patch-read bank cycles,
// then the smallest; cached per shape (the launch planner evaluates every
// band height)
std::pair<int, int> wino_strides(int PW, int nwin, int XL, int YL, int VEC, int cs_max) {
    static std::mutex mu;
    static std::map<std::tuple<int, int, int, int, int, int>, std::pair<int, int>> cache;
    const auto key = std::make_tuple(PW, nwin, XL, YL, VEC, cs_max);
    std::lock_guard<std::mutex> lock(mu);
    const auto f = cache.find(key);
    if (f != cache.end()) return f->second;
    const int step = std::max(VEC, 2);
    const int ys0 = (XL + step - 1) / step * step;
    int best = INT_MAX, bys = ys0, bcs = YL * ys0;
    for (int ys = ys0; ys < ys0 + 32; ys += step) {
        const int cs0 = (YL * ys + step - 1) / step * step;  // even: the float2 patch reads stay 8-B aligned
        for (int cs = cs0; cs < cs0 + 64 && cs <= cs_max; cs += step) {
            const int c = wino_read_cycles(PW, nwin, ys, cs);
            if (c < best || (c == best && cs < bcs)) {
                best = c;
                bys = ys;
                bcs = cs;
            }
        }
    }
    return cache[key] = {bys, bcs};
}

// Ring geometry of the Winograd forward: a y band of pyb pooled rows, XL =
// 2 PW + 2 input columns (the last window's 4-wide patch), row / channel
// strides from wino_strides; z chunks until the grid has ~2048 blocks
template <int CPG, int VEC>
RingGeom make_wino_geom(const rt_conv_layer* L, int B, int G, int pyb, size_t lds_budget = 160 * 1024) {
    RingGeom r{};
    Geom& g = r.g;
    g.D = L->in_dims[0];
    g.H = L->in_dims[1];
    g.W = L->in_dims[2];
    g.cd = g.D - 2;
    g.ch = g.H - 2;
    g.cw = g.W - 2;
    g.pd = L->pool_pad[0];
    g.ph = L->pool_pad[1];
    g.pw = L->pool_pad[2];
    g.PD = (g.cd + 2 * g.pd - 2) / 2 + 1;
    g.PH = (g.ch + 2 * g.ph - 2) / 2 + 1;
    g.PW = (g.cw + 2 * g.pw - 2) / 2 + 1;
    g.XT = (g.PW + 1) / 2;
    g.ZL = 4;
    g.YL = 2 * pyb + 2;
    g.XL = 2 * g.PW + 2;
    const int cs_max = (int)((lds_budget / sizeof(float) - wino_u_floats<CPG>()) / (kRing * CPG));
    const std::pair<int, int> st = wino_strides(g.PW, std::min(pyb, g.PH) * g.PW, g.XL, g.YL, VEC, cs_max);
    g.YS = st.first;
    g.ZS = 0;
    g.CS = st.second;
    r.SLOT = CPG * g.CS;
    r.npiece = (r.SLOT + 64 * VEC - 1) / (64 * VEC);
    r.nyb = (g.PH + pyb - 1) / pyb;
    const int64_t per_chunk = (int64_t)r.nyb * B * G;
    const int nzc = (int)std::min<int64_t>(g.PD, std::max<int64_t>(1, (2048 + per_chunk - 1) / per_chunk));
    r.ZC = (g.PD + nzc - 1) / nzc;
    return r;
}

template <int CPG, int COG, int VEC, int NTH>
int launch_wino_k(const RingGeom& rg, int pyb, int G, int32_t B, const float* x, const int64_t* rows,
                  const float* w, const float* bias, float* y, uint8_t* amax, hipStream_t st) {
    WinoParams P{x, rows, w, bias, y, amax, rg, G, pyb};
    const size_t lds = ((size_t)kRing * rg.SLOT + wino_u_floats<CPG>()) * sizeof(float);
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_wino<CPG, COG, VEC, NTH, true>)) return rc_lds;
        if (const int rc_lds = allow_big_lds(&k_conv_wino<CPG, COG, VEC, NTH, false>)) return rc_lds;
        attr = true;
    }
    dim3 grid(rg.nyb, (rg.g.PD + rg.ZC - 1) / rg.ZC, B * G);
    if (amax)
        hipLaunchKernelGGL((k_conv_wino<CPG, COG, VEC, NTH, true>), grid, dim3(NTH), lds, st, P);
    else
        hipLaunchKernelGGL((k_conv_wino<CPG, COG, VEC, NTH, false>), grid, dim3(NTH), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

// The f32 forward of conv1 and of the grouped stages in the Winograd form: the
// widest y band (up to 2 item rounds per pooled row) whose ring + U fit the
// 160 KiB of one block per CU; RT_ELIMIT when none does or the stage is not
// one of those (groups 1 with 16 channels: the direct ring kernel)
// MFMA wave-instructions of a Winograd forward launch: every pooled z row of
// every (sample, group) runs each band's 16-window items, 64 NS MFMAs each
int64_t wino_fwd_mfma(const RingGeom& rg, int pyb, int B, int G, int NS) {
    int64_t items = 0;
    for (int y = 0; y < rg.g.PH; y += pyb) items += (std::min(pyb, rg.g.PH - y) * rg.g.PW + 15) / 16;
    return (int64_t)B * G * rg.g.PD * items * 64 * NS;
}

// mfma_count (measurement hook): set to the launch's MFMA count, nothing launched
int launch_fwd_wino(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* w,
                    const float* bias, float* y, uint8_t* amax, hipStream_t st, int64_t* mfma_count = nullptr) {
    const int G = L->groups, cpg = L->cin / G;
    if (!(L->cin == 4 || G == 2 || G == 4) || (int64_t)B * G > 65535) return RT_ELIMIT;
    const bool vec4 = cpg == 4 && G == 1 && L->in_dims[2] % 4 == 0 && L->pool_pad[2] == 0 &&
                      (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    // conv1 (and conv3): 256-thread blocks in a third of the LDS, three per
    // CU = 3 waves per SIMD (<= 168 VGPRs), against 2 for one 512-thread
    // block holding the whole LDS
    int nth = (G == 4 || (G == 1 && kWinoC1Nth == 256)) ? 256 : 512;
    size_t lds_budget = nth == 256 ? 160 * 1024 / 3 : 160 * 1024;
    // the band height with the fewest item rounds per pooled row over all
    // bands (a band's 16-window items go round-robin to the NW waves, so 9
    // items on 8 waves cost 2 rounds), plus ~1/4 round per band for its
    // halo planes and prologue; ties go to the taller band
    auto plan = [&](auto cpg_c, auto vec_c, int& pyb_out) -> RingGeom {
        constexpr int CPG_ = decltype(cpg_c)::value, VEC_ = decltype(vec_c)::value;
        RingGeom best{};
        pyb_out = 0;
        const int nw = nth / 64;
        const int ph = (L->in_dims[1] - 2 + 2 * L->pool_pad[1] - 2) / 2 + 1;
        double best_cost = 1e30;
        for (int pyb = 1; pyb <= ph; ++pyb) {
            const RingGeom rg = make_wino_geom<CPG_, VEC_>(L, B, G, pyb, lds_budget);
            const size_t lds = ((size_t)kRing * rg.SLOT + wino_u_floats<CPG_>()) * sizeof(float);
            const int items = (pyb * rg.g.PW + 15) / 16;
            if (lds > lds_budget || (rg.npiece + nw - 1) / nw > 16 || items > 2 * nw || rg.g.W < VEC_) break;
            double cost = 0.25 * rg.nyb;
            for (int y = 0; y < ph; y += pyb) cost += ((std::min(pyb, ph - y) * rg.g.PW + 15) / 16 + nw - 1) / nw;
            if (cost <= best_cost) {
                best_cost = cost;
                best = rg;
                pyb_out = pyb;
            }
        }
        return best;
    };
    int pyb = 0;
    auto counted = [&](const RingGeom& rg, int ns) {
        *mfma_count = wino_fwd_mfma(rg, pyb, B, G, ns);
        return RT_OK;
    };
    if (cpg == 4 && G == 1) {
        // the small blocks when a band fits a third of the LDS, else one
        // 512-thread block per CU (wide planes: 128^3)
        auto conv1 = [&](auto nth_c, int64_t* cnt) -> int {
            constexpr int NT = decltype(nth_c)::value;
            nth = NT;
            lds_budget = NT == 256 ? 160 * 1024 / 3 : 160 * 1024;
            if (vec4) {
                const RingGeom rg = plan(std::integral_constant<int, 4>{}, std::integral_constant<int, 4>{}, pyb);
                if (pyb && cnt) return *cnt = wino_fwd_mfma(rg, pyb, B, G, 1), RT_OK;
                if (pyb) return launch_wino_k<4, 16, 4, NT>(rg, pyb, 1, B, x, rows, w, bias, y, amax, st);
            }
            const RingGeom rg = plan(std::integral_constant<int, 4>{}, std::integral_constant<int, 1>{}, pyb);
            if (pyb && cnt) return *cnt = wino_fwd_mfma(rg, pyb, B, G, 1), RT_OK;
            if (pyb) return launch_wino_k<4, 16, 1, NT>(rg, pyb, 1, B, x, rows, w, bias, y, amax, st);
            return RT_ELIMIT;
        };
        if constexpr (kWinoC1Nth == 256) {
            // the small blocks unless their narrow bands pad the 16-window
            // items by > 10 % more MFMAs than the big block's bands
            int64_t c256 = 0, c512 = 0;
            const int r256 = conv1(std::integral_constant<int, 256>{}, &c256);
            const int r512 = conv1(std::integral_constant<int, 512>{}, &c512);
            if (r256 == RT_OK && (r512 != RT_OK || c256 * 10 <= c512 * 11))
                return conv1(std::integral_constant<int, 256>{}, mfma_count);
        }
        return conv1(std::integral_constant<int, 512>{}, mfma_count);
    } else if (G == 2) {
        const RingGeom rg = plan(std::integral_constant<int, 8>{}, std::integral_constant<int, 1>{}, pyb);
        if (pyb && mfma_count) return counted(rg, 2);
        if (pyb) return launch_wino_k<8, 8, 1, 512>(rg, pyb, 2, B, x, rows, w, bias, y, amax, st);
    } else {
        const RingGeom rg = plan(std::integral_constant<int, 4>{}, std::integral_constant<int, 1>{}, pyb);
        if (pyb && mfma_count) return counted(rg, 1);
        if (pyb) return launch_wino_k<4, 4, 1, 256>(rg, pyb, 4, B, x, rows, w, bias, y, amax, st);
    }
    return RT_ELIMIT;
}

// ---------------------------------------------------------------------------
// Grouped stage (groups = 2) on the plane ring in the z-shift form.  The dense
// ring kernel above multiplies zero weights for the other group's channels
// (2x the useful MFMA work).  Here a block works on ONE group's 8 input
// channels and a tile is D[m = position][n = (co, s)] = sum_k X[m][k] Wext[k][n]:
// rows = a 4(y) x 4(x) patch, columns = the group's 8 output channels x the 2
// conv z-planes s of the pooled row, k = (tz' in 0..3, ci, ty, tx) over the
// row's 4 ring planes; Wext[(tz', ci, ty, tx)][(co, s)] = W[co][ci][tz' - s][ty][tx]
// (zero outside the 3 taps).  72 k-steps per 256 outputs against 108 in the
// dense form: 1.33x the useful work instead of 2x.  A = the patch from the
// ring (lane c: position (c >> 2, c & 3), lane group: input channel; channel
// stride = 16 mod 32 dwords, so a 32-lane read hits 32 banks), B = Wext in
// registers.  Pooling: x pairs are register pairs, y pairs lanes g ^ 1
// (shuffle by 16), z pairs columns s ^ 1 (DPP quad_perm); the argmax byte
// follows torch's first-maximum rule in (z, y, x) window order.
// ---------------------------------------------------------------------------
template <int G, int PYB>
RingGeom make_ring_geom_zs(const rt_conv_layer* L, int B) {
    constexpr int CPG = CO / G;
    RingGeom r{};
    Geom& g = r.g;
    g.D = L->in_dims[0];
    g.H = L->in_dims[1];
    g.W = L->in_dims[2];
    g.cd = g.D - 2;
    g.ch = g.H - 2;
    g.cw = g.W - 2;
    g.pd = L->pool_pad[0];
    g.ph = L->pool_pad[1];
    g.pw = L->pool_pad[2];
    g.PD = (g.cd + 2 * g.pd - 2) / 2 + 1;
    g.PH = (g.ch + 2 * g.ph - 2) / 2 + 1;
    g.PW = (g.cw + 2 * g.pw - 2) / 2 + 1;
    g.XT = (g.PW + 1) / 2;
    g.ZL = 4;
    g.YL = 2 * PYB + 2;
    g.XL = 4 * g.XT + 2;
    g.YS = round_mod(g.XL, 4);
    g.ZS = 0;
    g.CS = round_mod(g.YL * g.YS, 16);
    r.SLOT = round_mod(CPG * g.CS, 16);
    r.npiece = (r.SLOT + 63) / 64;
    r.nyb = (g.PH + PYB - 1) / PYB;
    const int64_t per_chunk = (int64_t)r.nyb * B * G;
    int nzc = (int)std::min<int64_t>(g.PD, std::max<int64_t>(1, (kZsBlocks + per_chunk - 1) / per_chunk));
    r.ZC = (g.PD + nzc - 1) / nzc;
    r.ZC = (r.ZC + G / 2 - 1) / (G / 2) * (G / 2);  // whole tiles (G / 2 pooled rows each) per chunk
    return r;
}

// Arithmetic of the C3D forward products: per call, rt_conv_layer.precision
// (bf16x3 in conv1's ring kernel and the grouped stages' z-shift kernels)
bool layer_bf16x3(const rt_conv_layer* L) { return L->precision == RT_CONV_PREC_BF16X3; }

// ring slots of the z-shift kernel: the G + 2 planes of a tile + the next G
template <int G>
constexpr int ring_zs_slots() {
    return 2 * G + 2;
}

// bf16x3 (BF): lane group g's k values are the list (tz', channel quad q,
// tap) of its input channel 4q + g, 8 per 16x16x32 MFMA (NVB = ZX * QPB * 9 / 8
// rounded up, zero-padded); A = the patch as packed ring words (ring_pack_bf),
// B = Wext hi / lo images in registers; the accumulator layout and the
// epilogue are the f32 kernel's.
template <int G, int PYB, bool TRAIN, bool BF = false>
__global__ __launch_bounds__(512) void k_conv_ring_zs(RingParams P) {
    extern __shared__ float xs[];
    constexpr int CPG = CO / G, NW = 8, ZX = G + 2, KS = CPG * ZX * 9 / 4, NB = KS / 9, NR = ring_zs_slots<G>();
    constexpr int NV = ZX * (CPG / 4) * 9, NVB = (NV + 7) / 8;  // bf16x3: k values per lane group, MFMAs
    constexpr int QPB = CPG / 4;  // channel quads per plane: batch bj = (tz' = bj / QPB, quad bj % QPB)
    static_assert(PYB % 2 == 0, "4-row y tiles");
    const Geom& g = P.rg.g;
    const int SLOT = P.rg.SLOT;
    const int grp = blockIdx.z % G, b = blockIdx.z / G, py0 = blockIdx.x * PYB;
    const int k0 = blockIdx.y * P.rg.ZC, k1 = min(g.PD, k0 + P.rg.ZC);
    if (k0 >= k1) return;
    const int lane = threadIdx.x & 63, c = lane & 15, gq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t srow = P.rows ? P.rows[b] : b;
    const float* xb = P.x + (srow * CO + grp * CPG) * (int64_t)g.D * g.H * g.W;
    const int y0 = 2 * py0 - g.ph, x0 = -g.pw;

    RingLoader<CPG, 1, NW> ld;
    ld.init(P.rg, y0, x0, wave, lane);
    auto load_plane = [&](int t, int slot) { ld.load(xb, P.rg, xs, t, slot, wave, lane); };

    // B = Wext: k-step st = 9 bj + q, batch bj = (tz', channel quad), q = (ty, tx); lane group = ci in the quad
    const int co_l = c / G, sz = c % G;
    float bw[BF ? 1 : KS];
    bf8 bwh[BF ? NVB : 1], bwl[BF ? NVB : 1];
    if constexpr (BF) {
#pragma unroll
        for (int v8 = 0; v8 < NVB; ++v8) {
            uint32_t pw[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int e = 8 * v8 + j, tz = e / (9 * QPB), ci = 4 * ((e / 9) % QPB) + gq, q = e % 9, dz = tz - sz;
                pw[j] = (e < NV && dz >= 0 && dz < 3) ? bf_pack(P.w[((grp * CPG + co_l) * CPG + ci) * 27 + dz * 9 + q])
                                                      : 0u;
            }
            bf_unpack8(pw, bwh[v8], bwl[v8]);
        }
    } else {
#pragma unroll
        for (int st = 0; st < KS; ++st) {
            const int bj = st / 9, q = st % 9, tz = bj / QPB, ci = 4 * (bj % QPB) + gq, dz = tz - sz;
            bw[st] = (dz >= 0 && dz < 3) ? P.w[((grp * CPG + co_l) * CPG + ci) * 27 + dz * 9 + q] : 0.0f;
        }
    }
    const int co = grp * CPG + co_l;
    const float bias = P.bias[co];
    const int64_t chan = (int64_t)g.PD * g.PH * g.PW;
    float* ybase = P.y + ((int64_t)b * CO + co) * chan;
    uint8_t* abase = TRAIN ? P.amax + ((int64_t)b * CO + co) * chan : nullptr;
    const int lane_xy = gq * g.CS + (c >> 2) * g.YS + (c & 3);
    const int rank_zy = (sz & 1) * 4 + (gq & 1) * 2;
    const bool storer = (sz & 1) == 0 && (gq & 1) == 0;
    constexpr int NYT = PYB / 2;
    const int nxp = (g.XT + 1) / 2;
    const int nitem = NYT * nxp;
    const int NI = (nitem + NW - 1) / NW;

    // epilogue of one item: tiles tx = 2xp, 2xp + 1 of y tile yt at pooled rows pz0 .. pz0 + G/2 - 1
    auto epi = [&](const f4 (&acc)[2], int yt, int xp, int pz0, bool ok) {
        const int cz = 2 * pz0 - g.pd + sz, cy = y0 + 4 * yt + gq, pz = pz0 + (sz >> 1);
        const bool vzy = ok && cz >= 0 && cz < g.cd && cy >= 0 && cy < g.ch;
        const int py = py0 + 2 * yt + (gq >> 1);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int tx = 2 * xp + u;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int cx = x0 + 4 * tx + r;
                v[r] = (vzy && cx >= 0 && cx < g.cw) ? fmaxf(acc[u][r] + bias, 0.0f) : -INFINITY;
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                // ReLU outputs or -inf: their int bit patterns order as the floats do
                int m = max(__float_as_int(v[2 * j]), __float_as_int(v[2 * j + 1]));
                m = max(m, __shfl_xor(m, 16, 64));
                m = max(m, __builtin_amdgcn_mov_dpp(m, 0xB1, 0xF, 0xF, true));
                const float M = __int_as_float(m);
                int k = 8;
                if constexpr (TRAIN) {
                    k = v[2 * j + 1] == M ? rank_zy + 1 : 8;
                    k = v[2 * j] == M ? rank_zy : k;
                    k = min(k, __shfl_xor(k, 16, 64));
                    k = min(k, __builtin_amdgcn_mov_dpp(k, 0xB1, 0xF, 0xF, true));
                }
                const int px = 2 * tx + j;
                if (ok && storer && tx < g.XT && px < g.PW && py < g.PH && pz < g.PD) {
                    const int64_t o = ((int64_t)pz * g.PH + py) * g.PW + px;
                    ybase[o] = M;
                    if constexpr (TRAIN) abase[o] = (uint8_t)(k | (M > 0.0f ? 8 : 0));
                }
            }
        }
    };

    // ---- prologue: planes 0 .. G+1 of the chunk
#pragma unroll
    for (int i = 0; i < ZX; ++i) load_plane(2 * k0 + i, i);
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __syncthreads();
    if constexpr (BF) {
        ring_pack_bf<NR>(xs, 0, ZX, SLOT);
        __syncthreads();
    }

    f4 pacc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
    int pyt = 0, pxp = 0, ppz = k0;
    bool pok = false;
    int sb = 0;  // ring slot of plane 2k
    for (int k = k0; k < k1; k += G / 2) {  // one tile row = G conv planes = G/2 pooled rows
        if (k + G / 2 < k1) {  // planes of the next tile row -> the G free slots
#pragma unroll
            for (int i = 0; i < G; ++i) {
                const int sl = sb + ZX + i;
                load_plane(2 * k + ZX + i, sl >= NR ? sl - NR : sl);
            }
        }
        int zoff[ZX];
#pragma unroll
        for (int t = 0; t < ZX; ++t) {
            int sl = sb + t;
            sl = sl >= NR ? sl - NR : sl;
            zoff[t] = sl * SLOT + lane_xy;
        }
        for (int i = 0; i < NI; ++i) {
            const int it = wave + NW * i;
            const bool ok = it < nitem;
            const int itc = ok ? it : nitem - 1;
            const int yt = itc / nxp, xp = itc - yt * nxp;
            const int tb = 4 * yt * g.YS + 8 * xp;
            // wave-uniform padding skips: a y tile past the last pooled row stores
            // nothing (no MFMAs), an item whose second x tile is past XT runs one
            // accumulator
            const bool live = ok && py0 + 2 * yt < g.PH;
            const bool two = 2 * xp + 1 < g.XT;
            float bv[2][2][9];
            auto fetch = [&](float (&dst)[2][9], int bj, auto two_t) {
                const int base = zoff[bj / QPB] + (bj % QPB) * 4 * g.CS + tb;
#pragma unroll
                for (int ty = 0; ty < 3; ++ty)
#pragma unroll
                    for (int tx = 0; tx < 3; ++tx) {
                        dst[0][ty * 3 + tx] = xs[base + ty * g.YS + tx];
                        if constexpr (decltype(two_t)::value) dst[1][ty * 3 + tx] = xs[base + ty * g.YS + tx + 4];
                    }
            };
            if constexpr (!BF) fetch(bv[0], 0, std::true_type{});
            epi(pacc, pyt, pxp, ppz, pok);  // the previous item's epilogue, between this item's MFMAs
            f4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
            auto mloop = [&](auto two_t) {
#pragma unroll
                for (int bj = 0; bj < NB; ++bj) {
                    if (bj + 1 < NB) fetch(bv[(bj + 1) & 1], bj + 1, two_t);
#pragma unroll
                    for (int q = 0; q < 9; ++q) {
                        acc[0] = mfma4(bv[bj & 1][0][q], bw[bj * 9 + q], acc[0]);
                        if constexpr (decltype(two_t)::value) acc[1] = mfma4(bv[bj & 1][1][q], bw[bj * 9 + q], acc[1]);
                    }
                }
            };
            if constexpr (BF) {
                const uint32_t* xu = reinterpret_cast<const uint32_t*>(xs);
                auto fetchb = [&](uint32_t (&dst)[2][8], int v8) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int e = 8 * v8 + j;
                        if (e < NV) {
                            const int q = e % 9;
                            const int a = zoff[e / (9 * QPB)] + ((e / 9) % QPB) * 4 * g.CS + tb + (q / 3) * g.YS + q % 3;
                            dst[0][j] = xu[a];
                            dst[1][j] = xu[a + 4];
                        } else {
                            dst[0][j] = 0u;
                            dst[1][j] = 0u;
                        }
                    }
                };
                if (live) {
                    uint32_t pv[2][2][8];
                    fetchb(pv[0], 0);
#pragma unroll
                    for (int v8 = 0; v8 < NVB; ++v8) {
                        if (v8 + 1 < NVB) fetchb(pv[(v8 + 1) & 1], v8 + 1);
#pragma unroll
                        for (int u = 0; u < 2; ++u) {
                            bf8 ah, al;
                            bf_unpack8(pv[v8 & 1][u], ah, al);
                            acc[u] = mfma3(ah, al, bwh[v8], bwl[v8], acc[u]);
                        }
                    }
                }
            } else if (live) {
                if (two)
                    mloop(std::true_type{});
                else
                    mloop(std::false_type{});
            }
            pacc[0] = acc[0];
            pacc[1] = acc[1];
            pyt = yt;
            pxp = xp;
            ppz = k;
            pok = live;
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // this wave's DMA for the next row has landed
        __syncthreads();                     // ... every wave's; and nobody still reads the slots reloaded next
        sb = sb + G >= NR ? sb + G - NR : sb + G;
        if constexpr (BF) {
            if (k + G / 2 < k1) {  // the G planes that just landed, before the next tile row reads them
                ring_pack_bf<NR>(xs, sb + 2 >= NR ? sb + 2 - NR : sb + 2, G, SLOT);
                __syncthreads();
            }
        }
    }
    epi(pacc, pyt, pxp, ppz, pok);
}

template <int G, int PYB, bool BF>
int launch_ring_zs_kp(const RingGeom& rg, int32_t B, const float* x, const int64_t* rows, const float* w,
                      const float* bias, float* y, uint8_t* amax, hipStream_t st) {
    RingParams P{x, rows, w, bias, y, amax, rg};
    const size_t lds = (size_t)ring_zs_slots<G>() * rg.SLOT * sizeof(float);
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_ring_zs<G, PYB, true, BF>)) return rc_lds;
        if (const int rc_lds = allow_big_lds(&k_conv_ring_zs<G, PYB, false, BF>)) return rc_lds;
        attr = true;
    }
    dim3 grid(rg.nyb, (rg.g.PD + rg.ZC - 1) / rg.ZC, G * B);
    if (amax)
        hipLaunchKernelGGL((k_conv_ring_zs<G, PYB, true, BF>), grid, dim3(512), lds, st, P);
    else
        hipLaunchKernelGGL((k_conv_ring_zs<G, PYB, false, BF>), grid, dim3(512), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

template <int G, int PYB>
int launch_ring_zs_k(const RingGeom& rg, int32_t B, const float* x, const int64_t* rows, const float* w,
                     const float* bias, float* y, uint8_t* amax, bool bf, hipStream_t st) {
    if (bf) return launch_ring_zs_kp<G, PYB, true>(rg, B, x, rows, w, bias, y, amax, st);
    return launch_ring_zs_kp<G, PYB, false>(rg, B, x, rows, w, bias, y, amax, st);
}

// the widest y band whose ring fits 160 KiB (one 8-wave block per CU)
template <int G>
int launch_ring_zs(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* w,
                   const float* bias, float* y, uint8_t* amax, hipStream_t st) {
    auto fits = [&](const RingGeom& rg) {
        return (size_t)ring_zs_slots<G>() * rg.SLOT * sizeof(float) <= 160 * 1024 &&
               (rg.npiece + 7) / 8 <= ring_max_pieces<CO / G, 1>();
    };
    RingGeom rg = make_ring_geom_zs<G, 8>(L, B);
    if (fits(rg)) return launch_ring_zs_k<G, 8>(rg, B, x, rows, w, bias, y, amax, layer_bf16x3(L), st);
    rg = make_ring_geom_zs<G, 4>(L, B);
    if (fits(rg)) return launch_ring_zs_k<G, 4>(rg, B, x, rows, w, bias, y, amax, layer_bf16x3(L), st);
    rg = make_ring_geom_zs<G, 2>(L, B);
    if (fits(rg)) return launch_ring_zs_k<G, 2>(rg, B, x, rows, w, bias, y, amax, layer_bf16x3(L), st);
    return RT_ELIMIT;
}


template <int CIN, int G, int PYB, int VEC, int NTH>
int launch_ring_p(const RingGeom& rg, int32_t B, const float* x, const int64_t* rows, const float* w,
                  const float* bias, float* y, uint8_t* amax, bool bf, hipStream_t st) {
    if constexpr (CIN == 4 && G == 1)
        if (bf) return launch_ring<CIN, G, PYB, VEC, NTH, true>(rg, B, x, rows, w, bias, y, amax, st);
    return launch_ring<CIN, G, PYB, VEC, NTH, false>(rg, B, x, rows, w, bias, y, amax, st);
}

// the forward: the widest y band whose ring fits the LDS budget (80 KiB: two
// 8-wave blocks per CU for conv1; the 16-channel stages hold 2 waves per SIMD
// by registers, one 8-wave block per CU, 160 KiB).  Wider planes: conv1 takes
// the whole 160 KiB (one block per CU), then one-row bands; RT_ELIMIT when even
// that ring does not fit (the caller falls back to the tile kernel).
template <int CIN, int G>
int launch_fwd_ring(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* w,
                    const float* bias, float* y, uint8_t* amax, hipStream_t st) {
    constexpr int NTH = 512;
    const bool vec4 = CIN == 4 && L->in_dims[2] % 4 == 0 && L->pool_pad[2] == 0 &&
                      (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    auto fits = [&](const RingGeom& rg, int vec, size_t budget) {
        return (size_t)kRing * rg.SLOT * sizeof(float) <= budget &&
               (rg.npiece + NTH / 64 - 1) / (NTH / 64) <= (vec == 4 ? ring_max_pieces<CIN, 4>()
                                                                   : ring_max_pieces<CIN, 1>()) &&
               rg.g.W >= vec;
    };
    constexpr int PY_BIG = CIN == 4 ? 4 : 2;
    for (const size_t budget : {(size_t)(CIN == 4 ? 80 : 160) * 1024, (size_t)160 * 1024}) {
        if constexpr (CIN == 4) {
            if (vec4) {
                RingGeom rg = make_ring_geom<CIN, PY_BIG, 4>(L, B, NTH);
                if (fits(rg, 4, budget)) return launch_ring_p<CIN, G, PY_BIG, 4, NTH>(rg, B, x, rows, w, bias, y, amax, layer_bf16x3(L), st);
                rg = make_ring_geom<CIN, PY_BIG / 2, 4>(L, B, NTH);
                if (fits(rg, 4, budget))
                    return launch_ring_p<CIN, G, PY_BIG / 2, 4, NTH>(rg, B, x, rows, w, bias, y, amax, layer_bf16x3(L), st);
            }
        }
        RingGeom rg = make_ring_geom<CIN, PY_BIG, 1>(L, B, NTH);
        if (fits(rg, 1, budget)) return launch_ring_p<CIN, G, PY_BIG, 1, NTH>(rg, B, x, rows, w, bias, y, amax, layer_bf16x3(L), st);
        rg = make_ring_geom<CIN, PY_BIG / 2, 1>(L, B, NTH);
        if (fits(rg, 1, budget)) return launch_ring_p<CIN, G, PY_BIG / 2, 1, NTH>(rg, B, x, rows, w, bias, y, amax, layer_bf16x3(L), st);
        if constexpr (PY_BIG / 4 >= 1) {
            rg = make_ring_geom<CIN, PY_BIG / 4, 1>(L, B, NTH);
            if (fits(rg, 1, budget))
                return launch_ring_p<CIN, G, PY_BIG / 4, 1, NTH>(rg, B, x, rows, w, bias, y, amax, layer_bf16x3(L), st);
        }
        if (CIN != 4) break;  // the 16-channel stages already tried the whole 160 KiB
    }
    return RT_ELIMIT;
}

// ---------------------------------------------------------------------------
struct DgradParams {
    const float* w;    // stage weights [16][16/G][27]
    const float* dP;   // [B][16][PD][PH][PW]
    const uint8_t* am; // same shape
    float* dx;         // [B][16][D][H][W]
    Geom g;            // D,H,W = stage input = dx dims; XT = x tiles of 4 over W
};

// dX[ci][p] = sum_{co, t} W[co][ci][t] dY[co][p - t]: the forward main loop over
// the zero-padded dY region with flipped, transposed weights
template <int G, int PZB, int PYB>
__global__ __launch_bounds__(conv_threads<16>()) void k_conv_dgrad(DgradParams P) {
    extern __shared__ float xs[];
    constexpr int NS = nsteps<16>();
    const Geom& g = P.g;
    const int b = blockIdx.z, z0 = blockIdx.y * 2 * PZB, y0 = blockIdx.x * 2 * PYB;
    const int lane = threadIdx.x & 63, c = lane & 15, gq = lane >> 4;
    // stage dY[co][z0-2 .., y0-2 .., -2 ..] into LDS: zero the tile, then each
    // pooling window that overlaps it scatters its gradient to its recorded
    // maximum (one argmax byte + one gradient load per window, not per position)
    constexpr int NT = conv_threads<16>();
    for (int i = threadIdx.x; i < CO * g.CS; i += NT) xs[i] = 0.0f;
    __syncthreads();
    {
        const int cz0 = z0 - 2, cy0 = y0 - 2, cx0 = -2;  // conv coordinates of LDS (0, 0, 0)
        const int pz_lo = max((cz0 + g.pd) >> 1, 0), pz_hi = min((cz0 + g.ZL - 1 + g.pd) >> 1, g.PD - 1);
        const int py_lo = max((cy0 + g.ph) >> 1, 0), py_hi = min((cy0 + g.YL - 1 + g.ph) >> 1, g.PH - 1);
        const int px_hi = min((cx0 + g.XL - 1 + g.pw) >> 1, g.PW - 1);
        const int nz = pz_hi - pz_lo + 1, ny = py_hi - py_lo + 1, nx = px_hi + 1;
        const int nwin = CO * nz * ny * nx;
        // WU windows per thread in flight: the argmax byte and the gradient of
        // a window are independent loads, so all 2*WU are issued before the
        // first use (one scalar loop iteration per window took two dependent
        // global round trips, and the block's MFMAs wait on this phase)
        constexpr int WU = 8;
        for (int i0 = threadIdx.x; i0 < nwin; i0 += NT * WU) {
            int byte[WU], lds[WU];
            float gv[WU];
#pragma unroll
            for (int u = 0; u < WU; ++u) {
                const int i = i0 + u * NT;
                byte[u] = 0;
                gv[u] = 0.0f;
                lds[u] = 0;
                if (i < nwin) {
                    const int px = i % nx, py = py_lo + (i / nx) % ny, pz = pz_lo + (i / (nx * ny)) % nz,
                              co = i / (nx * ny * nz);
                    const int64_t o = (((int64_t)b * CO + co) * g.PD + pz) * g.PH * g.PW + (int64_t)py * g.PW + px;
                    byte[u] = P.am[o];
                    gv[u] = P.dP[o];
                    // LDS address of the window's (0,0,0) corner relative to the tile
                    lds[u] = co * g.CS + (2 * pz - g.pd - cz0) * g.ZS + (2 * py - g.ph - cy0) * g.YS + (2 * px - g.pw - cx0);
                    // pack the corner's tile coordinates for the range check below
                    byte[u] |= ((2 * pz - g.pd - cz0 + 1) << 8) | ((2 * py - g.ph - cy0 + 1) << 16) |
                               ((2 * px - g.pw - cx0 + 1) << 24);
                }
            }
#pragma unroll
            for (int u = 0; u < WU; ++u) {
                const int bt = byte[u];
                if (!(bt & 8)) continue;
                const int k = bt & 7, kz = k >> 2, ky = (k >> 1) & 1, kx = k & 1;
                const int zz = ((bt >> 8) & 255) - 1 + kz, yy = ((bt >> 16) & 255) - 1 + ky, xx = (bt >> 24) - 1 + kx;
                if (zz >= 0 && zz < g.ZL && yy >= 0 && yy < g.YL && xx >= 0 && xx < g.XL)
                    xs[lds[u] + kz * g.ZS + ky * g.YS + kx] = gv[u];
            }
        }
    }
    float af[NS];
    constexpr int cpg = CO / G;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int q = s % 27, co = 4 * (s / 27) + gq;  // lane group = dY channel, row c = dX channel
        const int gi = c / cpg, go = co / cpg;
        af[s] = gi == go ? P.w[(co * cpg + (c - gi * cpg)) * 27 + (26 - q)] : 0.0f;
    }
    __syncthreads();
    const int zc = c >> 3, yc = (c >> 2) & 1, xc = c & 3;
    conv_core<16, PYB>(xs, af, g, PZB * PYB, [&](const f4 (&acc)[2], int row, int xp) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int tx = 2 * xp + u;
            const int z = z0 + 2 * (row / PYB) + zc, y = y0 + 2 * (row % PYB) + yc, x = 4 * tx + xc;
            if (z < g.D && y < g.H && x < g.W) {
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    P.dx[((((size_t)b * CO + 4 * gq + r) * g.D + z) * g.H + y) * g.W + x] = acc[u][r];
            }
        }
    });
}

// ---------------------------------------------------------------------------
// Weight gradient: D[co][k'] += sum_pos dY[co][pos] * X[ci][pos + tap],
// k' = ci * 27 + tap (column CIN*27 = the constant 1 -> db).  A (dY) is built
// per lane from the pooled gradient + argmax byte: lane (c, g) holds channel
// co = c at the 4 positions n = 4q + g of a tile, which all lie in window
// g >> 1.  B is gathered from the same LDS input tile as the forward.
// Persistent: each block loops over (sample, region) items and keeps its
// column tiles in MFMA accumulators; conv1 splits positions over the 4 waves
// (7 column tiles each, summed through LDS), conv2/3 split the 28 column tiles.
template <int CIN>
constexpr int ncol_tiles() {
    return (CIN * 27 + 1 + 15) / 16;
}
constexpr int kWgradTiles = 7;  // column tiles per wave
struct WgradParams {
    const float* x;
    const int64_t* rows;
    const float* dP;
    const uint8_t* am;
    float* part;  // [gridDim.x][16 * ncol * 16]
    int32_t B;
    int32_t nby, nbz;  // regions per sample (as the forward grid)
    Geom g;
};

template <int CIN, int PZB, int PYB>
__global__ __launch_bounds__(kThreads) void k_conv_wgrad(WgradParams P) {
    extern __shared__ float xs[];
    constexpr int NCT = ncol_tiles<CIN>();
    constexpr int WC = NCT / kWgradTiles;      // column groups (1 for conv1, 4 for conv2/3)
    constexpr int WP = (kThreads / 64) / WC;   // position groups
    static_assert(NCT % kWgradTiles == 0, "column tiles");
    const Geom& g = P.g;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, gq = lane >> 4;
    const int wc = wave % WC, wp = wave / WC;
    const int t0c = wc * kWgradTiles;  // first column tile of this wave
    // per column tile: LDS offset of (ci, tap) of column 16T + c, or a constant
    int koff[kWgradTiles];
    float kconst[kWgradTiles];  // -1: gather; else the constant B value
#pragma unroll
    for (int t = 0; t < kWgradTiles; ++t) {
        const int k = 16 * (t0c + t) + c;
        if (k < CIN * 27) {
            const int ci = k / 27, q = k % 27;
            koff[t] = ci * g.CS + (q / 9) * g.ZS + ((q / 3) % 3) * g.YS + q % 3;
            kconst[t] = -1.0f;
        } else {
            koff[t] = 0;
            kconst[t] = k == CIN * 27 ? 1.0f : 0.0f;
        }
    }
    f4 acc[kWgradTiles];
#pragma unroll
    for (int t = 0; t < kWgradTiles; ++t) acc[t] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const int items = P.B * P.nbz * P.nby;
    const int nxt = g.XT, ntile = PZB * PYB * nxt;
    for (int it = blockIdx.x; it < items; it += gridDim.x) {
        const int b = it / (P.nbz * P.nby), rz = (it / P.nby) % P.nbz, ry = it % P.nby;
        const int pz0 = rz * PZB, py0 = ry * PYB;
        const int64_t srow = P.rows ? P.rows[b] : b;
        __syncthreads();  // the previous item's reads of xs are done
        load_tile<CIN, kThreads>(xs, P.x + srow * (int64_t)CIN * g.D * g.H * g.W, g, 2 * pz0 - g.pd, 2 * py0 - g.ph,
                                 -g.pw);
        __syncthreads();
        const int64_t plane = ((int64_t)b * CO + c) * g.PD * g.PH * g.PW;
        // tiles t = t0, t0 + WP, ...: (tz, ty, tx) advanced incrementally; the
        // next tile's pooled gradient + argmax byte are loaded before this
        // tile's MFMAs, its 28 B values are gathered before the first MFMA
        int tz = 0, ty = 0, tx = wp;
        auto advance = [&](int& z, int& y, int& x) {
            x += WP;
            while (x >= nxt) {
                x -= nxt;
                if (++y == PYB) {
                    y = 0;
                    ++z;
                }
            }
        };
        while (tx >= nxt) {
            tx -= nxt;
            if (++ty == PYB) {
                ty = 0;
                ++tz;
            }
        }
        auto load_a = [&](int z, int y, int x, int& byte, float& d) {
            const int pz = pz0 + z, py = py0 + y, px = 2 * x + (gq >> 1);
            byte = 0;
            d = 0.0f;
            if (z < PZB && pz < g.PD && py < g.PH && px < g.PW) {
                const int64_t o = plane + ((int64_t)pz * g.PH + py) * g.PW + px;
                byte = P.am[o];
                d = P.dP[o];
            }
        };
        int byte, nbyte;
        float d, nd;
        load_a(tz, ty, tx, byte, d);
        for (int t = wp; t < ntile; t += WP) {
            int nz = tz, ny = ty, nx = tx;
            advance(nz, ny, nx);
            const int tb = 2 * tz * g.ZS + 2 * ty * g.YS + 4 * tx + gq;
            float bv[4][kWgradTiles];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int pb = tb + (q >> 1) * g.ZS + (q & 1) * g.YS;
#pragma unroll
                for (int T = 0; T < kWgradTiles; ++T) bv[q][T] = kconst[T] < 0.0f ? xs[pb + koff[T]] : kconst[T];
            }
            load_a(nz, ny, nx, nbyte, nd);
            float a[4];
#pragma unroll
            for (int q = 0; q < 4; ++q)  // position n = 4q + g: zc = q >> 1, yc = q & 1, xc = g
                a[q] = ((byte & 8) && (byte & 7) == ((q >> 1) * 4 + (q & 1) * 2 + (gq & 1))) ? d : 0.0f;
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int T = 0; T < kWgradTiles; ++T) acc[T] = mfma4(a[q], bv[q][T], acc[T]);
            tz = nz;
            ty = ny;
            tx = nx;
            byte = nbyte;
            d = nd;
        }
    }
    // D (lane (c, g)): rows co = 4g + r, column 16T + c; the WP position
    // groups are summed through LDS in a fixed order
    float* out = P.part + (size_t)blockIdx.x * (CO * NCT * 16);
    constexpr int REG = CO * NCT * 16;
    __syncthreads();
    float* R = xs;  // WP regions of 16 x NCT*16 (after the last item)
#pragma unroll
    for (int T = 0; T < kWgradTiles; ++T)
#pragma unroll
        for (int r = 0; r < 4; ++r) R[wp * REG + (4 * gq + r) * (NCT * 16) + 16 * (t0c + T) + c] = acc[T][r];
    __syncthreads();
    for (int i = threadIdx.x; i < REG; i += kThreads) {
        float v = R[i];
#pragma unroll
        for (int k = 1; k < WP; ++k) v += R[k * REG + i];
        out[i] = v;
    }
}

// Weight-gradient ring parameters (k_conv_wgrad_sparse): the forward's plane
// ring over a y band of one sample at a time.
struct WgradRingParams {
    const float* x;
    const int64_t* rows;
    const float* dP;
    const uint8_t* am;
    float* part;  // [nblk][16 * ncol * 16]
    int32_t B;
    RingGeom rg;
};

// ---- weight gradient through the pooling argmax (the launched one) ----------
// dW[co][ci][tap] = sum over pooled windows w of dY[co][w] * X[ci][p(co, w) + tap],
// p = the conv position the window's argmax names; db[co] = sum_w dY[co][w].
// The dense form (an MFMA ring kernel, removed) multiplies every
// conv position's gradient, 7 of 8 of which the max-pool zeroed; here each (co, window) is
// one 27-tap gather of its argmax patch, 1/8 of the multiply-adds, as f32
// FMAs on the VALU with the patch read from the forward's plane ring.
// Thread = (window stream s, output channel co, in-group input channel cig):
// L = 16 * cin/G threads cover one window (one wave for conv1 and conv3, two
// for conv2), NS = 512 / L windows in flight per block; acc[27] per thread,
// summed over the streams through LDS in a fixed order at the end, then over
// the blocks by k_wgrad_reduce (deterministic).  A row's (gradient, argmax)
// pairs of the band are loaded into registers beside the next planes' DMA and
// written to a double-buffered LDS row after the row's gathers, so the
// row's one wait + barrier covers both.  LDS strides: YS = 4, CS = 8, SLOT =
// 2 (mod 32 dwords) put conv1's 4 channels x 8 argmax offsets of a half-wave
// (8 output channels) on 32 distinct banks, ring wrap included.  (Reading the
// patch rows as 8-B pairs from the even x below the patch start -- 2/3 of the
// LDS cycles, but 27 selects and no packed FMAs -- measured slower: conv1
// 2.45 -> 2.94 ms)
// ring geometry of the sparse weight gradient: conv1 and (round 4) the
// groups = 2 stage keep the ring's (YS, CS, SLOT) = (4, 8, 2) residues (mod
// 32 dwords): with a half-wave of 8 output channels x 4 input channels (the
// lane map below) the 4 channels x 8 argmax offsets (dz, dy, dx) of a patch
// read land on 32 distinct banks whatever the argmax bytes; groups = 4 (8
// output channels of two groups per half-wave, 8 input channels) cannot be
// made conflict-free and keeps (2, 4, 0) -- a bank model over random argmax
// variants: 1.54 vs 2.0 mean multiplicity
template <int CIN, int G, int PYB, int NT>
RingGeom make_sparse_geom(const rt_conv_layer* L, int B) {
    RingGeom r = make_ring_geom<CIN, PYB, 1, 2>(L, B, NT);
    if constexpr (CIN == 16 && G != 2) {
        Geom& g = r.g;
        g.YS = round_mod(g.XL, 2);
        g.CS = round_mod(g.YL * g.YS, 4);
        r.SLOT = round_mod(CIN * g.CS, 0);
        r.npiece = (r.SLOT + 63) / 64;
    }
    return r;
}

constexpr int kWgSparseMaxG = 4;  // a band row holds <= NT * 4 (channel, window) entries

// thread li of a window's L = 16 x CPG threads -> (output channel, in-group
// input channel).  groups = 2 (round 4): a 32-lane half-wave holds 8 output
// channels of one group x 4 input channels (li bits: cig & 3, co & 7,
// cig >> 2, co >> 3), so its patch reads are conflict-free on the (4, 8, 2)
// ring (was 4 x 8, 35 % conflict cycles); otherwise co-major
template <int CIN, int G>
__device__ __forceinline__ void sparse_lane(int li, int& co, int& cig) {
    constexpr int CPG = CIN / G;
    if constexpr (CIN == 16 && G == 2) {
        co = ((li >> 6) & 1) * 8 + ((li >> 2) & 7);
        cig = ((li >> 5) & 1) * 4 + (li & 3);
    } else {
        co = li / CPG;
        cig = li - co * CPG;
    }
}

template <int CIN, int G, int PYB, int NT>
__global__ __launch_bounds__(NT) void k_conv_wgrad_sparse(WgradRingParams P) {
    extern __shared__ float xs[];
    constexpr int CPG = CIN / G;   // input channels per group
    constexpr int L = CO * CPG;    // threads per window
    constexpr int NS = NT / L;     // window streams per block
    constexpr int NW = NT / 64;
    static_assert(NS >= 1, "block too small for one window");
    const Geom& g = P.rg.g;
    const int SLOT = P.rg.SLOT;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int sidx = tid / L, li = tid - sidx * L;
    int co, cig;
    sparse_lane<CIN, G>(li, co, cig);
    const int ci = (co / (CO / G)) * CPG + cig;
    const int py0 = blockIdx.x * PYB;
    const int y0 = 2 * py0 - g.ph, x0 = -g.pw;
    const int nwin = PYB * g.PW;  // windows of one pooled row of the band
    const int chan = g.PD * g.PH * g.PW;
    float* gbuf = xs + kRing * SLOT;                                   // [2][CO][nwin] gradient (0: inactive)
    uint8_t* jbuf = reinterpret_cast<uint8_t*>(gbuf + 2 * CO * nwin);  // [2][CO][nwin] argmax index
    RingLoader<CIN, 1, NW, NT == 256 ? 16 : 0> ld;
    ld.init(P.rg, y0, x0, wave, lane);
    float acc[27];
#pragma unroll
    for (int q = 0; q < 27; ++q) acc[q] = 0.0f;
    float dbacc = 0.0f;
    // (gradient, argmax) entries of a band row per thread: entry e = tid + 512 i
    // is (channel e / nwin, window e % nwin); its element offset in a sample
    // is off[i] + k * PH * PW at pooled row k (-1: past the band / volume)
    constexpr int MAXG = kWgSparseMaxG;
    int off[MAXG];
#pragma unroll
    for (int i = 0; i < MAXG; ++i) {
        const int e = tid + NT * i;
        off[i] = -1;
        if (e < CO * nwin) {
            const int c2 = e / nwin, w = e - c2 * nwin, r = w / g.PW, px = w - r * g.PW, py = py0 + r;
            if (py < g.PH) off[i] = c2 * chan + py * g.PW + px;
        }
    }
    const int plane = g.PH * g.PW;
    for (int b = blockIdx.z; b < P.B; b += gridDim.z) {
        const int64_t srow = P.rows ? P.rows[b] : b;
        const float* xb = P.x + srow * (int64_t)CIN * g.D * g.H * g.W;
        const uint8_t* amb = P.am + (int64_t)b * CO * chan;
        const float* dpb = P.dP + (int64_t)b * CO * chan;
        float gv[MAXG];
        int jv[MAXG];
        auto load_row = [&](int k) {
#pragma unroll
            for (int i = 0; i < MAXG; ++i) {
                const int o = off[i] + k * plane;
                const int byte = off[i] >= 0 ? amb[o] : 0;
                gv[i] = off[i] >= 0 ? dpb[o] : 0.0f;
                jv[i] = byte;
            }
        };
        auto store_row = [&](int buf) {
#pragma unroll
            for (int i = 0; i < MAXG; ++i) {
                const int e = tid + NT * i;
                if (e < CO * nwin) {
                    gbuf[buf * CO * nwin + e] = (jv[i] & 8) ? gv[i] : 0.0f;  // inactive window (max <= 0): no gradient
                    jbuf[buf * CO * nwin + e] = (uint8_t)(jv[i] & 7);
                }
            }
        };
        __syncthreads();  // the previous sample's ring and row reads are done
#pragma unroll
        for (int i = 0; i < 4; ++i) ld.load(xb, P.rg, xs, i, i, wave, lane);
        load_row(0);
        store_row(0);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        __syncthreads();
        int sb = 0;
        for (int k = 0; k < g.PD; ++k) {
            const bool more = k + 1 < g.PD;
            if (more) {
                ld.load(xb, P.rg, xs, 2 * k + 4, sb + 4 >= kRing ? sb + 4 - kRing : sb + 4, wave, lane);
                ld.load(xb, P.rg, xs, 2 * k + 5, sb + 5 >= kRing ? sb + 5 - kRing : sb + 5, wave, lane);
                load_row(k + 1);
            }
            const float* grow = gbuf + (k & 1) * CO * nwin + co * nwin;
            const uint8_t* jrow = jbuf + (k & 1) * CO * nwin + co * nwin;
            // ring slots of the row's planes 2k + 0..3 (the patch of argmax dz uses dz .. dz + 2)
            int so[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int sl = sb + t;
                so[t] = (sl >= kRing ? sl - kRing : sl) * SLOT + ci * g.CS;
            }
            // one window: its 27 patch values (registers) and its gradient
            auto gather = [&](int w, int r, int px, float (&v)[27]) {
                const float gw = grow[w];
                const int j = jrow[w];
                const int dz = j >> 2, dy = (j >> 1) & 1, dx = j & 1;
                const int inrow = (2 * r + dy) * g.YS + 2 * px + dx;
                const int zb[3] = {(dz ? so[1] : so[0]) + inrow, (dz ? so[2] : so[1]) + inrow,
                                   (dz ? so[3] : so[2]) + inrow};
#pragma unroll
                for (int tz = 0; tz < 3; ++tz)
#pragma unroll
                    for (int ty = 0; ty < 3; ++ty)
#pragma unroll
                        for (int tx = 0; tx < 3; ++tx) v[tz * 9 + ty * 3 + tx] = xs[zb[tz] + ty * g.YS + tx];
                return gw;
            };
            auto accumulate = [&](float gw, const float (&v)[27]) {
#pragma unroll
                for (int q = 0; q < 27; ++q) acc[q] = fmaf(gw, v[q], acc[q]);
                dbacc += gw;
            };
            auto advance = [&](int& r, int& px) {
                px += NS;
                while (px >= g.PW) {
                    px -= g.PW;
                    ++r;
                }
            };
            int r = 0, px = sidx, w = sidx;
            while (px >= g.PW) {
                px -= g.PW;
                ++r;
            }
            for (; w < nwin; w += NS) {
                if (py0 + r >= g.PH) break;  // uniform: the band's rows past the volume
                float v[27];
                const float gw = gather(w, r, px, v);
                accumulate(gw, v);
                advance(r, px);
            }
            if (more) store_row((k + 1) & 1);
            __builtin_amdgcn_s_waitcnt(0x0F70);
            __syncthreads();
            sb = sb + 2 >= kRing ? sb + 2 - kRing : sb + 2;
        }
    }
    // the NS streams' partial sums through LDS (fixed order), one partial row per block
    const int blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    constexpr int NCOL = CIN * 27 + 1;
    float* out = P.part + (size_t)blk * (CO * NCOL);
    __syncthreads();
    float* R = xs;
#pragma unroll
    for (int q = 0; q < 27; ++q) R[(sidx * L + li) * 28 + q] = acc[q];
    R[(sidx * L + li) * 28 + 27] = dbacc;
    __syncthreads();
    for (int i = tid; i < L * 28; i += NT) {
        const int l2 = i / 28, q = i - l2 * 28;
        float v = R[i];
#pragma unroll
        for (int k = 1; k < NS; ++k) v += R[k * L * 28 + i];
        int co2, cig2;
        sparse_lane<CIN, G>(l2, co2, cig2);
        const int ci2 = (co2 / (CO / G)) * CPG + cig2;
        if (q < 27)
            out[co2 * NCOL + ci2 * 27 + q] = v;
        else if (cig2 == 0)
            out[co2 * NCOL + CIN * 27] = v;
    }
}

// sum of the block partials -> dW [16][cin/G][27] (in-group columns) and db [16].
// A 1024-thread block owns 64 consecutive outputs (lane = output): wave w sums
// the partial rows k = w, w + 16, ... (4 chains, coalesced 64-float rows), the
// 16 wave sums are added in a fixed order (deterministic).  One thread per
// output looping over every partial row (the first version) was latency-bound:
// 147 us per call at 512 ring blocks.
constexpr int kRedWaves = 16;
__global__ __launch_bounds__(64 * kRedWaves) void k_wgrad_reduce(const float* part, int nblk, int cin, int groups,
                                                                 int ncol, float* dw, float* db) {
    __shared__ float red[kRedWaves][64];
    const int cpg = cin / groups, nw = CO * cpg * 27;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + lane;
    const bool ok = i <= nw + CO - 1;
    int co = 0, col = 0;
    if (i < nw) {
        co = i / (cpg * 27);
        const int rem = i % (cpg * 27), cil = rem / 27, q = rem % 27;
        col = ((co / (CO / groups)) * cpg + cil) * 27 + q;
    } else {
        co = i - nw;
        col = cin * 27;
    }
    const float* src = part + (size_t)co * ncol + col;
    const size_t rs = (size_t)CO * ncol;
    float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (ok) {
        int k = w;
        for (; k + 3 * kRedWaves < nblk; k += 4 * kRedWaves) {
#pragma unroll
            for (int u = 0; u < 4; ++u) a[u] += src[(size_t)(k + u * kRedWaves) * rs];
        }
#pragma unroll
        for (int u = 0; u < 3; ++u)
            if (k + u * kRedWaves < nblk) a[u] += src[(size_t)(k + u * kRedWaves) * rs];
    }
    red[w][lane] = (a[0] + a[1]) + (a[2] + a[3]);
    __syncthreads();
    if (w != 0 || !ok) return;
    float t = 0.0f;
#pragma unroll
    for (int k = 0; k < kRedWaves; ++k) t += red[k][lane];
    if (i < nw)
        dw[i] = t;
    else
        db[co] = t;
}

template <class K>
int allow_big_lds(K* kern) {
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return e == hipSuccess ? RT_OK : rt_internal_fail(RT_EDEVICE, hipGetErrorString(e));
}

template <int CIN, int G, int PZB, int PYB>
int launch_fwd(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* w,
               const float* bias, float* y, uint8_t* amax, hipStream_t st) {
    FwdParams P{};
    P.g = make_geom<PZB, PYB>(L);
    P.x = x;
    P.rows = rows;
    P.w = w;
    P.bias = bias;
    P.y = y;
    P.amax = amax;
    const size_t lds = (size_t)CIN * P.g.CS * sizeof(float);
    if (lds > 160 * 1024) return rt_internal_fail(RT_ELIMIT, "rt_conv: input tile exceeds LDS (grid too wide)");
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_relu_pool<CIN, G, PZB, PYB, true>)) return rc_lds;
        if (const int rc_lds = allow_big_lds(&k_conv_relu_pool<CIN, G, PZB, PYB, false>)) return rc_lds;
        attr = true;
    }
    dim3 grid((P.g.PH + PYB - 1) / PYB, (P.g.PD + PZB - 1) / PZB, B);
    if (amax)
        hipLaunchKernelGGL((k_conv_relu_pool<CIN, G, PZB, PYB, true>), grid, dim3(conv_threads<CIN>()), lds, st, P);
    else
        hipLaunchKernelGGL((k_conv_relu_pool<CIN, G, PZB, PYB, false>), grid, dim3(conv_threads<CIN>()), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

template <int PZB, int PYB>
Geom make_dgrad_geom(const rt_conv_layer* L) {
    Geom g = make_geom<PZB, PYB>(L);
    g.XT = (g.W + 3) / 4;
    g.XL = 4 * g.XT + 2;
    g.YS = round_mod(g.XL, 4);
    g.ZS = round_mod(g.YL * g.YS, 8);
    g.CS = round_mod(g.ZL * g.ZS, 16);
    return g;
}


template <int G, int PZB, int PYB>
int launch_dgrad(const rt_conv_layer* L, int32_t B, const float* w, const float* dP, const uint8_t* am, float* dx,
                 hipStream_t st) {
    DgradParams P{};
    P.g = make_dgrad_geom<PZB, PYB>(L);
    P.w = w;
    P.dP = dP;
    P.am = am;
    P.dx = dx;
    const size_t lds = (size_t)CO * P.g.CS * sizeof(float);
    if (lds > 160 * 1024) return rt_internal_fail(RT_ELIMIT, "rt_conv_dgrad: tile exceeds LDS");
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_dgrad<G, PZB, PYB>)) return rc_lds;
        attr = true;
    }
    dim3 grid((P.g.H + 2 * PYB - 1) / (2 * PYB), (P.g.D + 2 * PZB - 1) / (2 * PZB), B);
    hipLaunchKernelGGL((k_conv_dgrad<G, PZB, PYB>), grid, dim3(conv_threads<16>()), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

// ---------------------------------------------------------------------------
// Data gradient, z-ring version (the launched one; pool padding 0, i.e. the
// 16-channel stages).  dX = the full correlation of the sparse conv-output
// gradient dY with the flipped, transposed weights, so the forward's ring
// structure carries over: a block owns a y band of 2*PYB dX rows (full x) of
// one sample and sweeps a chunk of ZC output rows (dX z-plane pairs 2k, 2k+1);
// ring plane t = dY conv plane t - 2 (zero-padded), and the two planes of a
// pair are the two conv planes of ONE pooled row, so a pair is built from
// that row's pooling windows: each window writes its 2x2x2 block (the
// gradient at its recorded maximum, zero elsewhere -- no separate zeroing
// pass).  The argmax bytes and gradients of the next pair are loaded into
// registers before the row's MFMAs and written to the two free slots after
// them, so their latency hides behind the MFMA chains; one barrier per row.
// (The tile version k_conv_dgrad re-staged a 4-plane halo per 2 output
// planes and waited on its scatter before every tile.)
constexpr int kDgMaxWin = 6;  // pooling windows per thread and plane pair

struct DgradRingParams {
    const float* w;     // stage weights [16][16/G][27]
    const float* dP;    // [B][16][PD][PH][PW]
    const uint8_t* am;  // same shape
    float* dx;          // [B][16][D][H][W]
    RingGeom rg;        // g: D,H,W = dX dims, PD,PH,PW = pooled dims, XT = x tiles of 4 over W
};

template <int G, int PYB, int NTH>
__global__ __launch_bounds__(NTH) void k_conv_dgrad_ring(DgradRingParams P) {
    extern __shared__ float xs[];
    constexpr int NS = nsteps<16>(), NW = NTH / 64, MW = kDgMaxWin, cpg = CO / G;
    const Geom& g = P.rg.g;
    const int SLOT = P.rg.SLOT;
    const int b = blockIdx.z, py0 = blockIdx.x * PYB, y0 = 2 * py0;
    const int k0 = blockIdx.y * P.rg.ZC, k1 = min((g.D + 1) / 2, k0 + P.rg.ZC);
    if (k0 >= k1) return;
    const int lane = threadIdx.x & 63, c = lane & 15, gq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pplane = g.PH * g.PW, chan = g.PD * pplane;
    const uint8_t* amb = P.am + (int64_t)b * CO * chan;
    const float* dpb = P.dP + (int64_t)b * CO * chan;

    // this thread's pooling windows of a plane pair (the same for every pair):
    // window (co, pyl, pxw) covers LDS rows 2pyl.. and columns 2pxw..; pooled
    // (py, px) = (py0 - 1 + pyl, pxw - 1), out-of-range windows write zeros
    const int nxw = 2 * g.XT + 1, nwin = CO * (PYB + 1) * nxw;
    int woff[MW], wlds[MW];
#pragma unroll
    for (int u = 0; u < MW; ++u) {
        const int i = threadIdx.x + u * NTH;
        const int pxw = i % nxw, rest = i / nxw, pyl = rest % (PYB + 1), co = rest / (PYB + 1);
        const int px = pxw - 1, py = py0 - 1 + pyl;
        wlds[u] = i < nwin ? co * g.CS + 2 * pyl * g.YS + 2 * pxw : -1;
        woff[u] = i < nwin && px >= 0 && px < g.PW && py >= 0 && py < g.PH ? co * chan + py * g.PW + px : -1;
    }
    int bt[MW];
    float gv[MW];
    auto fetch_pair = [&](int m) {  // pair m = pooled row m - 1 -> registers
        const int pz = m - 1;
        const bool zok = pz >= 0 && pz < g.PD;
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const bool ok = zok && woff[u] >= 0;
            const int o = woff[u] + pz * pplane;
            bt[u] = ok ? amb[o] : 0;
            gv[u] = ok ? dpb[o] : 0.0f;
        }
    };
    auto store_pair = [&](int slot0) {  // registers -> slots slot0, slot0 + 1 (slot0 even: no wrap)
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            if (wlds[u] < 0) continue;
            const int kk = bt[u] & 7;
            const float v = (bt[u] & 8) ? gv[u] : 0.0f;
#pragma unroll
            for (int kz = 0; kz < 2; ++kz)
#pragma unroll
                for (int ky = 0; ky < 2; ++ky) {
                    const int k2 = kz * 4 + ky * 2;
                    *reinterpret_cast<float2*>(xs + (slot0 + kz) * SLOT + wlds[u] + ky * g.YS) =
                        make_float2(kk == k2 ? v : 0.0f, kk == k2 + 1 ? v : 0.0f);
                }
        }
    };

    // A fragments: flipped taps, transposed channels (lane group = dY channel,
    // row c = dX channel); zero across groups
    float af[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int q = s % 27, co = 4 * (s / 27) + gq;
        af[s] = c / cpg == co / cpg ? P.w[(co * cpg + c % cpg) * 27 + 26 - q] : 0.0f;
    }
    const int zc = c >> 3, yc = (c >> 2) & 1, xc = c & 3;
    const int cstride = g.D * g.H * g.W;
    float* dxb = P.dx + ((int64_t)b * CO + 4 * gq) * cstride;
    auto epi = [&](const f4 (&acc)[2], int r, int xp, int k, bool ok) {
        const int z = 2 * k + zc, y = y0 + 2 * r + yc;
        const bool vzy = ok && z < g.D && y < g.H;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int x = 8 * xp + 4 * u + xc;
            if (vzy && x < g.W) {
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) dxb[rr * cstride + (z * g.H + y) * g.W + x] = acc[u][rr];
            }
        }
    };

    fetch_pair(k0);
    store_pair(0);
    fetch_pair(k0 + 1);
    store_pair(2);
    __syncthreads();
    RingPrev pv{{{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}}, 0, 0, k0, false};
    int sb = 0;  // ring slot of plane 2k
    for (int k = k0; k < k1; ++k) {
        const bool more = k + 1 < k1;
        if (more) fetch_pair(k + 2);
        ring_row<16, PYB, NW>(xs, af, g, SLOT, sb, k, wave, lane, pv, epi);
        if (more) store_pair(sb + 4 >= kRing ? sb + 4 - kRing : sb + 4);  // the slots row k - 1 read last
        __syncthreads();
        sb = sb + 2 >= kRing ? sb + 2 - kRing : sb + 2;
    }
    epi(pv.acc, pv.r, pv.xp, pv.k, pv.ok);
}

template <int PYB>
RingGeom make_dgrad_ring_geom(const rt_conv_layer* L, int B) {
    RingGeom r{};
    Geom& g = r.g;
    g.D = L->in_dims[0];
    g.H = L->in_dims[1];
    g.W = L->in_dims[2];
    g.cd = g.D - 2;
    g.ch = g.H - 2;
    g.cw = g.W - 2;
    g.PD = g.cd / 2;
    g.PH = g.ch / 2;
    g.PW = g.cw / 2;
    g.XT = (g.W + 3) / 4;
    g.ZL = 4;
    g.YL = 2 * PYB + 2;
    g.XL = 4 * g.XT + 2;
    g.YS = round_mod(g.XL, 4);
    g.CS = round_mod(g.YL * g.YS, 8);
    r.SLOT = round_mod(CO * g.CS, 16);
    r.nyb = (g.H + 2 * PYB - 1) / (2 * PYB);
    const int KD = (g.D + 1) / 2;
    const int64_t per_chunk = (int64_t)r.nyb * B;
    const int nzc = (int)std::min<int64_t>(KD, std::max<int64_t>(1, (4096 + per_chunk - 1) / per_chunk));
    r.ZC = (KD + nzc - 1) / nzc;
    return r;
}

constexpr int kDgradRingThreads = 512;

template <int G, int PYB>
int launch_dgrad_ring_k(const RingGeom& rg, int32_t B, const float* w, const float* dP, const uint8_t* am, float* dx,
                        hipStream_t st) {
    DgradRingParams P{w, dP, am, dx, rg};
    const size_t lds = (size_t)kRing * rg.SLOT * sizeof(float);
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_dgrad_ring<G, PYB, kDgradRingThreads>)) return rc_lds;
        attr = true;
    }
    dim3 grid(rg.nyb, ((rg.g.D + 1) / 2 + rg.ZC - 1) / rg.ZC, B);
    hipLaunchKernelGGL((k_conv_dgrad_ring<G, PYB, kDgradRingThreads>), grid, dim3(kDgradRingThreads), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

// the widest y band whose ring fits 160 KiB and whose windows fit the threads
template <int G>
int launch_dgrad_ring(const rt_conv_layer* L, int32_t B, const float* w, const float* dP, const uint8_t* am, float* dx,
                      hipStream_t st) {
    auto fits = [&](const RingGeom& rg, int pyb) {
        return (size_t)kRing * rg.SLOT * sizeof(float) <= 160 * 1024 &&
               CO * (pyb + 1) * (2 * rg.g.XT + 1) <= kDgMaxWin * kDgradRingThreads;
    };
    RingGeom rg = make_dgrad_ring_geom<4>(L, B);
    if (fits(rg, 4)) return launch_dgrad_ring_k<G, 4>(rg, B, w, dP, am, dx, st);
    rg = make_dgrad_ring_geom<2>(L, B);
    if (fits(rg, 2)) return launch_dgrad_ring_k<G, 2>(rg, B, w, dP, am, dx, st);
    rg = make_dgrad_ring_geom<1>(L, B);
    if (fits(rg, 1)) return launch_dgrad_ring_k<G, 1>(rg, B, w, dP, am, dx, st);
    return RT_ELIMIT;
}

// Data gradient of the grouped stages in the z-shift form on the same ring:
// one group per block, a tile is D[m = position][n = (ci, s)] over a 4(y) x
// 4(x) patch of the scattered dY planes, columns = the group's dX channels x
// the tile row's G dX z-planes s, k = (tz' in 0..G+1, dY channel quad, ty, tx):
// B = Wext[(tz', co, ty, tx)][(ci, s)] = W[co][ci][2 - (tz' - s)][2 - ty][2 - tx]
// in registers (zero outside the 3 taps) -- the forward z-shift kernel's MFMA
// mapping with flipped, transposed weights (1.33x / 2x the useful work for
// groups 2 / 4 instead of 2x / 4x).  Planes come from the pooling-window
// scatter of k_conv_dgrad_ring, G/2 pooled rows per tile row.
template <int G, int PYB, bool BF = false>
__global__ __launch_bounds__(512) void k_conv_dgrad_ring_zs(DgradRingParams P) {
    extern __shared__ float xs[];
    constexpr int CPG = CO / G, NW = 8, NTH = 512, ZX = G + 2, KS = CPG * ZX * 9 / 4, NB = KS / 9;
    constexpr int NR = ring_zs_slots<G>(), QPB = CPG / 4, MW = kDgMaxWin, HP = G / 2;
    constexpr int NV = ZX * QPB * 9, NVB = (NV + 7) / 8;  // bf16x3 (BF): k values per lane group, MFMAs
    static_assert(PYB % 2 == 0, "4-row y tiles");
    const Geom& g = P.rg.g;
    const int SLOT = P.rg.SLOT;
    const int grp = blockIdx.z % G, b = blockIdx.z / G, py0 = blockIdx.x * PYB, y0 = 2 * py0;
    const int k0 = blockIdx.y * P.rg.ZC, k1 = min((g.D + 1) / 2, k0 + P.rg.ZC);
    if (k0 >= k1) return;
    const int lane = threadIdx.x & 63, c = lane & 15, gq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int pplane = g.PH * g.PW, chan = g.PD * pplane;
    const uint8_t* amb = P.am + ((int64_t)b * CO + grp * CPG) * chan;
    const float* dpb = P.dP + ((int64_t)b * CO + grp * CPG) * chan;

    // this thread's pooling windows of a plane pair (the group's channels)
    const int nxw = 2 * g.XT + 1, nwin = CPG * (PYB + 1) * nxw;
    int woff[MW], wlds[MW];
#pragma unroll
    for (int u = 0; u < MW; ++u) {
        const int i = threadIdx.x + u * NTH;
        const int pxw = i % nxw, rest = i / nxw, pyl = rest % (PYB + 1), co = rest / (PYB + 1);
        const int px = pxw - 1, py = py0 - 1 + pyl;
        wlds[u] = i < nwin ? co * g.CS + 2 * pyl * g.YS + 2 * pxw : -1;
        woff[u] = i < nwin && px >= 0 && px < g.PW && py >= 0 && py < g.PH ? co * chan + py * g.PW + px : -1;
    }
    auto fetch_pair = [&](int m, int (&bt)[MW], float (&gv)[MW]) {  // pair m = pooled row m - 1
        const int pz = m - 1;
        const bool zok = pz >= 0 && pz < g.PD;
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            const bool ok = zok && woff[u] >= 0;
            const int o = woff[u] + pz * pplane;
            bt[u] = ok ? amb[o] : 0;
            gv[u] = ok ? dpb[o] : 0.0f;
        }
    };
    auto store_pair = [&](int slot0, const int (&bt)[MW], const float (&gv)[MW]) {  // slot0 even: no wrap
#pragma unroll
        for (int u = 0; u < MW; ++u) {
            if (wlds[u] < 0) continue;
            const int kk = bt[u] & 7;
            const float v = (bt[u] & 8) ? gv[u] : 0.0f;
#pragma unroll
            for (int kz = 0; kz < 2; ++kz)
#pragma unroll
                for (int ky = 0; ky < 2; ++ky) {
                    const int k2 = kz * 4 + ky * 2;
                    if constexpr (BF)  // packed hi << 16 | lo words (the forward's ring_pack_bf form)
                        *reinterpret_cast<uint2*>(xs + (slot0 + kz) * SLOT + wlds[u] + ky * g.YS) =
                            make_uint2(kk == k2 ? bf_pack(v) : 0u, kk == k2 + 1 ? bf_pack(v) : 0u);
                    else
                        *reinterpret_cast<float2*>(xs + (slot0 + kz) * SLOT + wlds[u] + ky * g.YS) =
                            make_float2(kk == k2 ? v : 0.0f, kk == k2 + 1 ? v : 0.0f);
                }
        }
    };

    // B = Wext: k-step st = 9 bj + q, batch bj = (tz', dY channel quad), q = (ty, tx); lane group = dY channel
    const int ci_l = c / G, sz = c % G;
    float bw[BF ? 1 : KS];
    bf8 bwh[BF ? NVB : 1], bwl[BF ? NVB : 1];
    if constexpr (BF) {  // k list of lane group gq: (tz', dY channel quad, tap) of dY channel 4 quad + gq
#pragma unroll
        for (int v8 = 0; v8 < NVB; ++v8) {
            uint32_t pw[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int e = 8 * v8 + j, tz = e / (9 * QPB), co = 4 * ((e / 9) % QPB) + gq, q = e % 9, dz = tz - sz;
                pw[j] = (e < NV && dz >= 0 && dz < 3)
                            ? bf_pack(P.w[((grp * CPG + co) * CPG + ci_l) * 27 + (2 - dz) * 9 + 8 - q])
                            : 0u;
            }
            bf_unpack8(pw, bwh[v8], bwl[v8]);
        }
    } else {
#pragma unroll
        for (int st = 0; st < KS; ++st) {
            const int bj = st / 9, q = st % 9, tz = bj / QPB, co = 4 * (bj % QPB) + gq, dz = tz - sz;
            bw[st] = (dz >= 0 && dz < 3) ? P.w[((grp * CPG + co) * CPG + ci_l) * 27 + (2 - dz) * 9 + 8 - q] : 0.0f;
        }
    }
    const int cstride = g.D * g.H * g.W;
    float* dxb = P.dx + ((int64_t)b * CO + grp * CPG + ci_l) * cstride;
    const int lane_xy = gq * g.CS + (c >> 2) * g.YS + (c & 3);
    constexpr int NYT = PYB / 2;
    const int nxp = (g.XT + 1) / 2;
    const int nitem = NYT * nxp;
    const int NI = (nitem + NW - 1) / NW;

    // epilogue: lane (c, g) holds dX channel ci_l, plane 2k + sz, row 4yt + g, x = 4tx .. 4tx + 3
    auto epi = [&](const f4 (&acc)[2], int yt, int xp, int k, bool ok) {
        const int z = 2 * k + sz, y = y0 + 4 * yt + gq;
        const bool vzy = ok && z < g.D && y < g.H;
        float* row = dxb + (z * g.H + y) * g.W;
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int x = 8 * xp + 4 * u + r;
                if (vzy && x < g.W) row[x] = acc[u][r];
            }
    };

    {  // prologue: pairs k0 .. k0 + G/2 -> slots 0 .. ZX - 1
        int bt[MW];
        float gv[MW];
#pragma unroll
        for (int j = 0; j <= HP; ++j) {
            fetch_pair(k0 + j, bt, gv);
            store_pair(2 * j, bt, gv);
        }
    }
    __syncthreads();

    int bt[HP][MW];
    float gv[HP][MW];
    f4 pacc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
    int pyt = 0, pxp = 0, pk = k0;
    bool pok = false;
    int sb = 0;  // ring slot of plane 2k
    for (int k = k0; k < k1; k += HP) {  // one tile row = G dX planes
        const bool more = k + HP < k1;
        if (more) {
#pragma unroll
            for (int j = 0; j < HP; ++j) fetch_pair(k + HP + 1 + j, bt[j], gv[j]);
        }
        int zoff[ZX];
#pragma unroll
        for (int t = 0; t < ZX; ++t) {
            int sl = sb + t;
            sl = sl >= NR ? sl - NR : sl;
            zoff[t] = sl * SLOT + lane_xy;
        }
        for (int i = 0; i < NI; ++i) {
            const int it = wave + NW * i;
            const bool ok = it < nitem;
            const int itc = ok ? it : nitem - 1;
            const int yt = itc / nxp, xp = itc - yt * nxp;
            const int tb = 4 * yt * g.YS + 8 * xp;
            float bv[2][2][9];
            auto fetch = [&](float (&dst)[2][9], int bj) {
                const int base = zoff[bj / QPB] + (bj % QPB) * 4 * g.CS + tb;
#pragma unroll
                for (int ty = 0; ty < 3; ++ty)
#pragma unroll
                    for (int tx = 0; tx < 3; ++tx) {
                        dst[0][ty * 3 + tx] = xs[base + ty * g.YS + tx];
                        dst[1][ty * 3 + tx] = xs[base + ty * g.YS + tx + 4];
                    }
            };
            if constexpr (!BF) fetch(bv[0], 0);
            epi(pacc, pyt, pxp, pk, pok);  // the previous item's epilogue, between this item's MFMAs
            f4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
            if constexpr (BF) {
                const uint32_t* xu = reinterpret_cast<const uint32_t*>(xs);
                auto fetchb = [&](uint32_t (&dst)[2][8], int v8) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int e = 8 * v8 + j;
                        if (e < NV) {
                            const int q = e % 9;
                            const int a = zoff[e / (9 * QPB)] + ((e / 9) % QPB) * 4 * g.CS + tb + (q / 3) * g.YS + q % 3;
                            dst[0][j] = xu[a];
                            dst[1][j] = xu[a + 4];
                        } else {
                            dst[0][j] = 0u;
                            dst[1][j] = 0u;
                        }
                    }
                };
                uint32_t pv[2][2][8];
                fetchb(pv[0], 0);
#pragma unroll
                for (int v8 = 0; v8 < NVB; ++v8) {
                    if (v8 + 1 < NVB) fetchb(pv[(v8 + 1) & 1], v8 + 1);
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        bf8 ah, al;
                        bf_unpack8(pv[v8 & 1][u], ah, al);
                        acc[u] = mfma3(ah, al, bwh[v8], bwl[v8], acc[u]);
                    }
                }
            } else {
#pragma unroll
                for (int bj = 0; bj < NB; ++bj) {
                    if (bj + 1 < NB) fetch(bv[(bj + 1) & 1], bj + 1);
#pragma unroll
                    for (int q = 0; q < 9; ++q) {
                        acc[0] = mfma4(bv[bj & 1][0][q], bw[bj * 9 + q], acc[0]);
                        acc[1] = mfma4(bv[bj & 1][1][q], bw[bj * 9 + q], acc[1]);
                    }
                }
            }
            pacc[0] = acc[0];
            pacc[1] = acc[1];
            pyt = yt;
            pxp = xp;
            pk = k;
            pok = ok;
        }
        if (more) {  // the next tile row's pairs -> the slots the previous tile row read last
#pragma unroll
            for (int j = 0; j < HP; ++j) {
                const int sl = sb + ZX + 2 * j;
                store_pair(sl >= NR ? sl - NR : sl, bt[j], gv[j]);
            }
        }
        __syncthreads();
        sb = sb + G >= NR ? sb + G - NR : sb + G;
    }
    epi(pacc, pyt, pxp, pk, pok);
}

template <int G, int PYB>
RingGeom make_dgrad_ring_geom_zs(const rt_conv_layer* L, int B) {
    RingGeom r = make_dgrad_ring_geom<PYB>(L, B);
    Geom& g = r.g;
    g.CS = round_mod(g.YL * g.YS, 16);
    r.SLOT = round_mod(CO / G * g.CS, 16);
    const int KD = (g.D + 1) / 2;
    const int64_t per_chunk = (int64_t)r.nyb * B * G;
    const int nzc = (int)std::min<int64_t>(KD, std::max<int64_t>(1, (kZsBlocks + per_chunk - 1) / per_chunk));
    r.ZC = (KD + nzc - 1) / nzc;
    r.ZC = (r.ZC + G / 2 - 1) / (G / 2) * (G / 2);  // whole tile rows per chunk
    return r;
}

template <int G, int PYB, bool BF>
int launch_dgrad_ring_zs_kp(const RingGeom& rg, int32_t B, const float* w, const float* dP, const uint8_t* am,
                            float* dx, hipStream_t st) {
    DgradRingParams P{w, dP, am, dx, rg};
    const size_t lds = (size_t)ring_zs_slots<G>() * rg.SLOT * sizeof(float);
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_dgrad_ring_zs<G, PYB, BF>)) return rc_lds;
        attr = true;
    }
    dim3 grid(rg.nyb, ((rg.g.D + 1) / 2 + rg.ZC - 1) / rg.ZC, G * B);
    hipLaunchKernelGGL((k_conv_dgrad_ring_zs<G, PYB, BF>), grid, dim3(512), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

template <int G, int PYB>
int launch_dgrad_ring_zs_k(const RingGeom& rg, int32_t B, const float* w, const float* dP, const uint8_t* am,
                           float* dx, bool bf, hipStream_t st) {
    if (bf) return launch_dgrad_ring_zs_kp<G, PYB, true>(rg, B, w, dP, am, dx, st);
    return launch_dgrad_ring_zs_kp<G, PYB, false>(rg, B, w, dP, am, dx, st);
}

template <int G>
int launch_dgrad_ring_zs(const rt_conv_layer* L, int32_t B, const float* w, const float* dP, const uint8_t* am,
                         float* dx, hipStream_t st) {
    auto fits = [&](const RingGeom& rg, int pyb) {
        return (size_t)ring_zs_slots<G>() * rg.SLOT * sizeof(float) <= 160 * 1024 &&
               CO / G * (pyb + 1) * (2 * rg.g.XT + 1) <= kDgMaxWin * 512;
    };
    RingGeom rg = make_dgrad_ring_geom_zs<G, 8>(L, B);
    if (fits(rg, 8)) return launch_dgrad_ring_zs_k<G, 8>(rg, B, w, dP, am, dx, layer_bf16x3(L), st);
    rg = make_dgrad_ring_geom_zs<G, 4>(L, B);
    if (fits(rg, 4)) return launch_dgrad_ring_zs_k<G, 4>(rg, B, w, dP, am, dx, layer_bf16x3(L), st);
    rg = make_dgrad_ring_geom_zs<G, 2>(L, B);
    if (fits(rg, 2)) return launch_dgrad_ring_zs_k<G, 2>(rg, B, w, dP, am, dx, layer_bf16x3(L), st);
    return RT_ELIMIT;
}

constexpr int kWgradBlocks = 512;

template <int CIN, int PZB, int PYB>
int wgrad_blocks(const rt_conv_layer* L, int32_t B) {
    const Geom g = make_geom<PZB, PYB>(L);
    const int64_t items = (int64_t)B * ((g.PD + PZB - 1) / PZB) * ((g.PH + PYB - 1) / PYB);
    return (int)(items < kWgradBlocks ? items : kWgradBlocks);
}

template <int CIN, int PZB, int PYB>
int launch_wgrad(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* dP,
                 const uint8_t* am, float* dw, float* db, float* ws, int64_t ws_floats, hipStream_t st) {
    WgradParams P{};
    P.g = make_geom<PZB, PYB, 4, 12, 8>(L);
    P.x = x;
    P.rows = rows;
    P.dP = dP;
    P.am = am;
    P.B = B;
    P.nby = (P.g.PH + PYB - 1) / PYB;
    P.nbz = (P.g.PD + PZB - 1) / PZB;
    P.part = ws;
    constexpr int NCT = ncol_tiles<CIN>();
    const int nblk = wgrad_blocks<CIN, PZB, PYB>(L, B);
    if ((int64_t)nblk * CO * NCT * 16 > ws_floats) return rt_internal_fail(RT_EINVAL, "rt_conv_wgrad: workspace too small");
    constexpr int WC = NCT / kWgradTiles, WP = (kThreads / 64) / WC;
    const size_t lds = std::max((size_t)CIN * P.g.CS, (size_t)WP * CO * NCT * 16) * sizeof(float);
    if (lds > 160 * 1024) return rt_internal_fail(RT_ELIMIT, "rt_conv_wgrad: tile exceeds LDS");
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_wgrad<CIN, PZB, PYB>)) return rc_lds;
        attr = true;
    }
    hipLaunchKernelGGL((k_conv_wgrad<CIN, PZB, PYB>), dim3(nblk), dim3(kThreads), lds, st, P);
    const int nout = CO * (L->cin / L->groups) * 27 + CO;
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((nout + 63) / 64), dim3(64 * kRedWaves), 0, st, (const float*)ws, nblk, L->cin,
                       L->groups, NCT * 16, dw, db);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

constexpr int kWgradRingBlocks = 512;  // sparse weight-gradient grid (256 / 1024 blocks measured within 1-2 %)

// the sparse weight gradient: two-row bands (one-row for wide 16-channel
// planes), one partial row per block, k_wgrad_reduce over ncol = cin*27 + 1
template <int CIN, int G, int PYB, int NT>
int launch_wgrad_sparse_k(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* dP,
                          const uint8_t* am, float* dw, float* db, float* ws, int64_t ws_floats, hipStream_t st) {
    const RingGeom rg = make_sparse_geom<CIN, G, PYB, NT>(L, B);
    const int nwin = PYB * rg.g.PW;
    const size_t lds = std::max((size_t)kRing * rg.SLOT * 4 + (size_t)2 * CO * nwin * 5, (size_t)NT * 28 * 4);
    if (lds > 160 * 1024 || CO * nwin > NT * kWgSparseMaxG ||
        (rg.npiece + NT / 64 - 1) / (NT / 64) > (NT == 256 ? 16 : ring_max_pieces<CIN, 1>()))
        return RT_ELIMIT;
    const int gz = std::max(1, std::min<int>(B, kWgradRingBlocks * (512 / NT) / std::max(1, rg.nyb)));
    const int nblk = rg.nyb * gz;
    constexpr int NCOL = CIN * 27 + 1;
    if ((int64_t)nblk * CO * NCOL > ws_floats) return rt_internal_fail(RT_EINVAL, "rt_conv_wgrad: workspace too small");
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_conv_wgrad_sparse<CIN, G, PYB, NT>)) return rc_lds;
        attr = true;
    }
    WgradRingParams P{x, rows, dP, am, ws, B, rg};
    hipLaunchKernelGGL((k_conv_wgrad_sparse<CIN, G, PYB, NT>), dim3(rg.nyb, 1, gz), dim3(NT), lds, st, P);
    const int nout = CO * (CIN / G) * 27 + CO;
    hipLaunchKernelGGL(k_wgrad_reduce, dim3((nout + 63) / 64), dim3(64 * kRedWaves), 0, st, (const float*)ws, nblk,
                       CIN, G, NCOL, dw, db);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

// RT_WGS_NT (A/B runs): 512- or 256-thread blocks of the sparse weight gradient
template <int CIN, int G>
int launch_wgrad_sparse(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* dP,
                        const uint8_t* am, float* dw, float* db, float* ws, int64_t ws_floats, hipStream_t st) {
    // 256-thread blocks on one-row bands (512-thread blocks and two-row bands
    // measured 3-4 % slower), the others where those do not fit
    int rc = launch_wgrad_sparse_k<CIN, G, 1, 256>(L, B, x, rows, dP, am, dw, db, ws, ws_floats, st);
    if (rc == RT_ELIMIT) rc = launch_wgrad_sparse_k<CIN, G, 2, 256>(L, B, x, rows, dP, am, dw, db, ws, ws_floats, st);
    if (rc == RT_ELIMIT) rc = launch_wgrad_sparse_k<CIN, G, 2, 512>(L, B, x, rows, dP, am, dw, db, ws, ws_floats, st);
    if (rc == RT_ELIMIT) rc = launch_wgrad_sparse_k<CIN, G, 1, 512>(L, B, x, rows, dP, am, dw, db, ws, ws_floats, st);
    return rc;
}

// ---------------------------------------------------------------------------
// Data gradient of the grouped stages (groups 2 and 4) in the Winograd form
// (the launched f32 data gradient for unpadded pools).  dX is the full
// correlation of the conv-output gradient dC with the flipped weights: per
// axis dX[2Q + o] = sum_t W[2 - t] e[o + t] over the 4-wide patch e[i] =
// dC[2Q - 2 + i], which is exactly the two pooling windows Q - 1 and Q -- so
// an F(2x2x2, 3x3x3) tile of dX reads the 2x2x2 windows (Q-1 .. Q per axis)
// and its patch holds at most one non-zero per window: the pooled gradient at
// the window's argmax when its ReLU was active (argmax byte), zeros elsewhere
// (the max-pool + ReLU backward, built in registers with one compare + select
// per patch entry).  Then, as the forward: V = B^T e B per lane (B operand:
// lane (tile n, co = 4s + l >> 4)), U' = G W' G^T of the flipped weights in LDS
// (A operand: lane (ci = l & 15, co)), M = U' V on f32 MFMA chained over the
// group's output-channel quads, dX tile = A^T M A.  The block holds the pooled
// gradient and the argmax bytes of its group and z chunk (window z rows Qz0 - 1
// .. Qz1 - 1, every y and x) in LDS, loaded once; items are 16 consecutive
// tiles of a tile row (row-major over (Qy, Qx)).  MFMAs per 16 tiles (16 input
// channels): 2 groups x 2 x 64 (groups 2) / 4 x 64 (groups 4) against the
// direct z-shift kernel's 576 / 432.
// ---------------------------------------------------------------------------
struct WinoDgradParams {
    const float* w;     // [16][CPG][27]
    const float* dP;    // [B][16][PD][PH][PW]
    const uint8_t* am;  // same shape
    float* dx;          // [B][16][D][H][W]
    Geom g;             // D, H, W = dX dims; PD, PH, PW = pooled dims
    int32_t G;          // groups (blockIdx.y = sample * G + group)
    int32_t ZC;         // tile rows per block (z chunk)
    int32_t QD, QH, QW; // tiles per axis = ceil(dims / 2)
};

template <int CPG>
constexpr int wino_dg_u_floats() {
    return 16 * 64 * 4 * (CPG / 4);
}

// groups 4 (conv3): 4 waves per SIMD (<= 128 VGPRs, no spills; left free the
// compiler took 130 and 3 waves); groups 2 stays at 2 (167 VGPRs, two
// 4-wave blocks per CU by LDS: 6-wave blocks for 3 per SIMD ran slower, §10)
template <int CPG, int NTH>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(CPG == 4 ? 4 : 1))) void k_dgrad_wino(
    WinoDgradParams P) {
    extern __shared__ float xs[];
    constexpr int NW = NTH / 64;
    constexpr int COG = CPG;     // groups 2 / 4: 8 / 4 output channels per group, as many inputs
    constexpr int NS = COG / 4;  // output-channel quads (MFMA k-steps) per xi
    const Geom& g = P.g;
    const int b = blockIdx.y / P.G, grp = blockIdx.y - b * P.G;
    const int q0 = blockIdx.x * P.ZC, q1 = min(P.QD, q0 + P.ZC);
    if (q0 >= q1) return;
    const int lane = threadIdx.x & 63, n = lane & 15, gq = lane >> 4;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // ---- the block's windows: rows wz0 .. wz1 - 1 of its group's channels
    const int wz0 = max(q0 - 1, 0), wz1 = min(q1, g.PD);
    const int nz = wz1 - wz0;
    const int plane = g.PH * g.PW;
    const int chw = nz * plane;  // window values per channel
    // LDS channel stride = 16 (mod 32): the two channels of a 32-lane group
    // read 16 consecutive windows each on disjoint banks (ds_read_b32: bank =
    // dword mod 32), the argmax bytes likewise
    const int chs = chw + ((48 - chw % 32) & 31);
    float* us = xs;
    float* dps = xs + wino_dg_u_floats<CPG>();
    uint8_t* ams = reinterpret_cast<uint8_t*>(dps + COG * chs);
    {
        // 8 loads in flight per thread (a load-then-store loop waited out one
        // HBM round trip per element)
        constexpr int U = 8;
        const size_t pchan = (size_t)g.PD * plane;
        const float* src = P.dP + ((size_t)b * CO + grp * COG) * pchan + (size_t)wz0 * plane;
        const uint8_t* asrc = P.am + ((size_t)b * CO + grp * COG) * pchan + (size_t)wz0 * plane;
        const int tot = COG * chw;
        for (int i0 = threadIdx.x; i0 < tot; i0 += NTH * U) {
            float v[U];
            int a[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = min(i0 + u * NTH, tot - 1);
                const int c = i / chw, rem = i - c * chw;
                v[u] = src[c * pchan + rem];
                a[u] = asrc[c * pchan + rem];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = i0 + u * NTH;
                if (i < tot) {
                    const int c = i / chw, li = i + c * (chs - chw);
                    dps[li] = v[u];
                    ams[li] = (uint8_t)a[u];
                }
            }
        }
    }
    // ---- U' = G W' G^T, W' = the flipped filter, for (ci = n, co = 4s + gq)
    if (wave == 0) {
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            const bool live = n < CPG;
            const int co = grp * COG + 4 * s + gq;
            const float* w = P.w + (co * CPG + (live ? n : 0)) * 27;
            float t[36];  // after the x axis: [kz][ky][xx] of the flipped taps
#pragma unroll
            for (int r = 0; r < 9; ++r) {
                const int fr = 8 - r;  // (kz, ky) flipped
                const float w0 = live ? w[3 * fr + 2] : 0.0f, w1 = live ? w[3 * fr + 1] : 0.0f;
                const float w2 = live ? w[3 * fr] : 0.0f;
                t[4 * r] = w0;
                t[4 * r + 1] = 0.5f * ((w0 + w1) + w2);
                t[4 * r + 2] = 0.5f * ((w0 - w1) + w2);
                t[4 * r + 3] = w2;
            }
            float sy[48];
#pragma unroll
            for (int kz = 0; kz < 3; ++kz)
#pragma unroll
                for (int xx = 0; xx < 4; ++xx) {
                    const float a0 = t[(kz * 3) * 4 + xx], a1 = t[(kz * 3 + 1) * 4 + xx];
                    const float a2 = t[(kz * 3 + 2) * 4 + xx];
                    sy[(kz * 4) * 4 + xx] = a0;
                    sy[(kz * 4 + 1) * 4 + xx] = 0.5f * ((a0 + a1) + a2);
                    sy[(kz * 4 + 2) * 4 + xx] = 0.5f * ((a0 - a1) + a2);
                    sy[(kz * 4 + 3) * 4 + xx] = a2;
                }
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const float a0 = sy[j], a1 = sy[16 + j], a2 = sy[32 + j];
                us[wino_u_index<NS>(j, lane, s)] = a0;
                us[wino_u_index<NS>(j, lane, NS + s)] = 0.5f * ((a0 + a1) + a2);
                us[wino_u_index<NS>(j, lane, 2 * NS + s)] = 0.5f * ((a0 - a1) + a2);
                us[wino_u_index<NS>(j, lane, 3 * NS + s)] = a2;
            }
        }
    }
    __syncthreads();
    const int ntile = P.QH * P.QW;
    const int items = (ntile + 15) >> 4;
    const int64_t xchan = (int64_t)g.D * g.H * g.W;
    const bool lane_ci = 4 * gq < CPG;
    float* dxb = P.dx + ((int64_t)b * CO + grp * CPG + (lane_ci ? 4 * gq : 0)) * xchan;
    // the chunk's (tile row, item) pairs flattened over the waves: no wave
    // takes more than one item beyond any other (conv3: 4 items per row on 4
    // waves is even either way; the flat loop also lets it run 4 waves per SIMD)
    const int nwork = (q1 - q0) * items;
    for (int k = wave; k < nwork; k += NW) {
        {
            const int qz = q0 + k / items, it = k - (qz - q0) * items;
            const int ti = min(16 * it + n, ntile - 1);
            const int qy = ti / P.QW, qx = ti - qy * P.QW;
            const f4 zero = {0.0f, 0.0f, 0.0f, 0.0f};
            f4 Y[2][2][2];
            f4 Sx[2][2][2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                float v[NS][32];
                int base = 0;
                __builtin_amdgcn_s_setprio(0);  // patch + input transform (conv2 1.357 -> 1.335, conv3 0.150 -> 0.144 ms: r05_s18)
                asm volatile("" : "+v"(base));  // the halves' window reads stay separate (no CSE)
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const int c = 4 * s + gq;  // output channel of the group
                    // the 8 windows (Qz-1..Qz, Qy-1..Qy, Qx-1..Qx): value, and argmax byte
                    // with the active bit (0 outside the pooled volume)
                    float wv[8];
                    int wa[8];
#pragma unroll
                    for (int wq = 0; wq < 8; ++wq) {
                        const int wz = qz - 1 + (wq >> 2), wy = qy - 1 + ((wq >> 1) & 1), wx = qx - 1 + (wq & 1);
                        const bool in = (unsigned)wz < (unsigned)g.PD & (unsigned)wy < (unsigned)g.PH &
                                        (unsigned)wx < (unsigned)g.PW;
                        const int li = base + c * chs + ((in ? wz : wz0) - wz0) * plane + (in ? wy : 0) * g.PW +
                                       (in ? wx : 0);
                        wv[wq] = dps[li];
                        wa[wq] = in ? (int)ams[li] : 0;
                    }
#pragma unroll
                    for (int dz = 0; dz < 4; ++dz)
#pragma unroll
                        for (int dy = 0; dy < 4; ++dy) {
                            // patch row (dz, dy): x 0, 1 from window x Qx-1, x 2, 3 from Qx
                            const int w0 = ((dz >> 1) << 2) | ((dy >> 1) << 1), w1 = w0 | 1;
                            const int kb = 8 | ((dz & 1) << 2) | ((dy & 1) << 1);
                            const float e0 = (wa[w0] & 15) == kb ? wv[w0] : 0.0f;
                            const float e1 = (wa[w0] & 15) == (kb | 1) ? wv[w0] : 0.0f;
                            const float e2 = (wa[w1] & 15) == kb ? wv[w1] : 0.0f;
                            const float e3 = (wa[w1] & 15) == (kb | 1) ? wv[w1] : 0.0f;
                            float* q = v[s] + (dz * 4 + dy) * 2;
                            if (h == 0) {  // B^T along x, rows 0, 1
                                q[0] = e0 - e2;
                                q[1] = e1 + e2;
                            } else {       // rows 2, 3
                                q[0] = e2 - e1;
                                q[1] = e1 - e3;
                            }
                        }
#pragma unroll
                    for (int dz = 0; dz < 4; ++dz)
#pragma unroll
                        for (int kx = 0; kx < 2; ++kx) {
                            float* q = v[s] + dz * 8 + kx;
                            const float d0 = q[0], d1 = q[2], d2 = q[4], d3 = q[6];
                            q[0] = d0 - d2;
                            q[2] = d1 + d2;
                            q[4] = d2 - d1;
                            q[6] = d1 - d3;
                        }
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float d0 = v[s][j], d1 = v[s][8 + j], d2 = v[s][16 + j], d3 = v[s][24 + j];
                        v[s][j] = d0 - d2;
                        v[s][8 + j] = d1 + d2;
                        v[s][16 + j] = d2 - d1;
                        v[s][24 + j] = d1 - d3;
                    }
                }
                __builtin_amdgcn_s_setprio(1);  // the MFMA columns at raised issue priority (as conv1's forward)
                f4 pm[4];
                auto column_sums = [&](const f4 (&m)[4], int xx, int xy) {
                    const f4 t0 = add4s(add4s(m[0], m[1]), m[2]), t1 = sub4s(sub4s(m[1], m[2]), m[3]);
                    f4(&S)[2][2] = Sx[xx & 1];
                    if (xy == 0) {
                        S[0][0] = t0;
                        S[0][1] = t1;
                    } else if (xy == 1) {
                        S[0][0] = add4s(S[0][0], t0);
                        S[0][1] = add4s(S[0][1], t1);
                        S[1][0] = t0;
                        S[1][1] = t1;
                    } else if (xy == 2) {
                        S[0][0] = add4s(S[0][0], t0);
                        S[0][1] = add4s(S[0][1], t1);
                        S[1][0] = sub4s(S[1][0], t0);
                        S[1][1] = sub4s(S[1][1], t1);
                    } else {
                        S[1][0] = sub4s(S[1][0], t0);
                        S[1][1] = sub4s(S[1][1], t1);
                    }
                    if (xy == 0)
                        asm volatile("" : "+v"(S[0][0]), "+v"(S[0][1]));
                    else
                        asm volatile("" : "+v"(S[0][0]), "+v"(S[0][1]), "+v"(S[1][0]), "+v"(S[1][1]));
                    if (xy == 3) {
#pragma unroll
                        for (int oy = 0; oy < 2; ++oy)
#pragma unroll
                            for (int oz = 0; oz < 2; ++oz) {
                                if (xx == 0) {
                                    Y[0][oy][oz] = S[oy][oz];
                                } else if (xx == 1) {
                                    Y[0][oy][oz] = add4s(Y[0][oy][oz], S[oy][oz]);
                                    Y[1][oy][oz] = S[oy][oz];
                                } else if (xx == 2) {
                                    Y[0][oy][oz] = add4s(Y[0][oy][oz], S[oy][oz]);
                                    Y[1][oy][oz] = sub4s(Y[1][oy][oz], S[oy][oz]);
                                } else {
                                    Y[1][oy][oz] = sub4s(Y[1][oy][oz], S[oy][oz]);
                                }
                            }
                    }
                };
#pragma unroll
                for (int cc = 0; cc <= 8; ++cc) {
                    f4 m[4];
                    if (cc < 8) {
                        const int kx = cc >> 2, xy = cc & 3, xx = 2 * h + kx;
                        const int j = xy * 4 + xx, jv = xy * 2 + kx;
                        float uc[4 * NS];
#pragma unroll
                        for (int q = 0; q < NS; ++q) {
                            const float4 u4 = *reinterpret_cast<const float4*>(us + wino_u_index<NS>(j, lane, 4 * q));
                            uc[4 * q] = u4.x;
                            uc[4 * q + 1] = u4.y;
                            uc[4 * q + 2] = u4.z;
                            uc[4 * q + 3] = u4.w;
                        }
#pragma unroll
                        for (int xz = 0; xz < 4; ++xz) {
                            m[xz] = mfma4(uc[xz * NS], v[0][xz * 8 + jv], zero);
#pragma unroll
                            for (int s = 1; s < NS; ++s) m[xz] = mfma4(uc[xz * NS + s], v[s][xz * 8 + jv], m[xz]);
                        }
                    }
                    if (cc > 0) column_sums(pm, 2 * h + ((cc - 1) >> 2), (cc - 1) & 3);
                    if (cc < 8)
#pragma unroll
                        for (int i = 0; i < 4; ++i) pm[i] = m[i];
                }
            }
            // ---- store the tile: dX[ci = 4 gq + r][2Qz + oz][2Qy + oy][2Qx + ox]
            if (lane_ci && 16 * it + n < ntile) {
#pragma unroll
                for (int o = 0; o < 8; ++o) {
                    const int z = 2 * qz + (o >> 2), y = 2 * qy + ((o >> 1) & 1), x = 2 * qx + (o & 1);
                    if (z < g.D && y < g.H && x < g.W) {
                        const int64_t off = ((int64_t)z * g.H + y) * g.W + x;
#pragma unroll
                        for (int r = 0; r < 4; ++r)
                            if (4 * gq + r < CPG) dxb[r * xchan + off] = Y[o & 1][(o >> 1) & 1][o >> 2][r];
                    }
                }
            }
        }
    }
}

template <int CPG, int NTH>
int launch_dgrad_wino_k(const rt_conv_layer* L, int32_t B, const float* w, const float* dP, const uint8_t* am,
                        float* dx, hipStream_t st, int64_t* mfma_count) {
    WinoDgradParams P{};
    P.g = make_geom<1, 1>(L);
    P.w = w;
    P.dP = dP;
    P.am = am;
    P.dx = dx;
    P.G = L->groups;
    P.QD = (P.g.D + 1) / 2;
    P.QH = (P.g.H + 1) / 2;
    P.QW = (P.g.W + 1) / 2;
    // z chunk: equal chunks whose window rows fit half the LDS beside U' (two
    // blocks per CU: one block's load phase runs beside the other's MFMAs),
    // else the whole LDS; then split further while the grid has fewer than
    // ~2048 blocks
    const size_t per_row = (size_t)CPG * P.g.PH * P.g.PW * 5;
    const size_t u_bytes = (size_t)wino_dg_u_floats<CPG>() * 4 + 64 + (size_t)CPG * 31 * 5;  // + stride padding
    auto rows_fit = [&](size_t lds) { return lds > u_bytes ? (int)((lds - u_bytes) / per_row) - 1 : 0; };
    int zmax = rows_fit(80 * 1024);
    if (zmax < 2) zmax = rows_fit(160 * 1024);
    if (zmax < 1) return RT_ELIMIT;
    int chunks = (P.QD + zmax - 1) / zmax;
    while (chunks < P.QD && (int64_t)B * P.G * chunks < 2048) ++chunks;
    const int zc = (P.QD + chunks - 1) / chunks;
    P.ZC = zc;
    if (mfma_count) {  // every tile row of every (sample, group): its 16-tile items, 64 NS MFMAs each
        *mfma_count = (int64_t)B * P.G * P.QD * ((P.QH * P.QW + 15) / 16) * 64 * (CPG / 4);
        return RT_OK;
    }
    const size_t lds = (size_t)wino_dg_u_floats<CPG>() * 4 + (size_t)(zc + 1) * per_row + (size_t)CPG * 31 * 5 + 16;
    static bool attr = false;
    if (!attr) {
        if (const int rc_lds = allow_big_lds(&k_dgrad_wino<CPG, NTH>)) return rc_lds;
        attr = true;
    }
    dim3 grid((P.QD + zc - 1) / zc, B * P.G);
    hipLaunchKernelGGL((k_dgrad_wino<CPG, NTH>), grid, dim3(NTH), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

int launch_dgrad_wino(const rt_conv_layer* L, int32_t B, const float* w, const float* dP, const uint8_t* am,
                      float* dx, hipStream_t st, int64_t* mfma_count = nullptr) {
    if ((int64_t)B * L->groups > 65535) return RT_ELIMIT;
    if (L->groups == 2) return launch_dgrad_wino_k<8, 256>(L, B, w, dP, am, dx, st, mfma_count);
    if (L->groups == 4) return launch_dgrad_wino_k<4, 256>(L, B, w, dP, am, dx, st, mfma_count);
    return RT_ELIMIT;
}

bool bad_layer(const rt_conv_layer* L) {
    if (!L) return true;
    if (!((L->cin == 4 && L->groups == 1) || (L->cin == 16 && (L->groups == 1 || L->groups == 2 || L->groups == 4))))
        return true;
    for (int a = 0; a < 3; ++a)
        if (L->in_dims[a] < 4 || L->pool_pad[a] < 0 || L->pool_pad[a] > 1) return true;
    return L->precision != RT_CONV_PREC_F32 && L->precision != RT_CONV_PREC_BF16X3;
}

// the one-region-per-block tile kernels (before the plane rings; kept as the
// fallback for planes too wide for a ring and for A/B builds)
int fwd_tile(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* w,
             const float* bias, float* y, uint8_t* amax, hipStream_t st) {
    if (L->cin == 4) return launch_fwd<4, 1, 2, 4>(L, B, x, rows, w, bias, y, amax, st);
    if (L->groups == 1) return launch_fwd<16, 1, 1, 2>(L, B, x, rows, w, bias, y, amax, st);
    if (L->groups == 2) return launch_fwd<16, 2, 1, 2>(L, B, x, rows, w, bias, y, amax, st);
    return launch_fwd<16, 4, 1, 2>(L, B, x, rows, w, bias, y, amax, st);
}

int64_t wgrad_tile_ws(const rt_conv_layer* L, int32_t B) {
    if (L->cin == 4) return (int64_t)wgrad_blocks<4, 2, 4>(L, B) * CO * ncol_tiles<4>() * 16;
    return (int64_t)wgrad_blocks<16, 1, 2>(L, B) * CO * ncol_tiles<16>() * 16;
}

int wgrad_tile(const rt_conv_layer* L, int32_t B, const float* x, const int64_t* rows, const float* dy,
               const uint8_t* am, float* dw, float* db, float* ws, int64_t ws_floats, hipStream_t st) {
    if (L->cin == 4) return launch_wgrad<4, 2, 4>(L, B, x, rows, dy, am, dw, db, ws, ws_floats, st);
    return launch_wgrad<16, 1, 2>(L, B, x, rows, dy, am, dw, db, ws, ws_floats, st);
}

}  // namespace

extern "C" int rt_conv_out_dims(const rt_conv_layer* L, int32_t* out_dims) {
    if (bad_layer(L) || !out_dims) return rt_internal_fail(RT_EINVAL, "rt_conv_out_dims: bad layer");
    const Geom g = make_geom<1, 1>(L);
    out_dims[0] = g.PD;
    out_dims[1] = g.PH;
    out_dims[2] = g.PW;
    return RT_OK;
}

extern "C" int rt_conv_relu_pool_fwd(const rt_conv_layer* L, int32_t batch, const float* x_d, const int64_t* rows_d,
                                     const float* w_d, const float* b_d, float* y_d, uint8_t* argmax_d,
                                     void* stream) {
    if (bad_layer(L) || batch < 1 || batch > 65535 || !x_d || !w_d || !b_d || !y_d)
        return rt_internal_fail(RT_EINVAL, "rt_conv_relu_pool_fwd: bad argument");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int rc = RT_ELIMIT;
    // f32: the Winograd kernel (conv1 and the grouped stages); bf16x3, groups 1
    // with 16 channels and planes too wide for its ring: the direct kernels
    if (!layer_bf16x3(L)) rc = launch_fwd_wino(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
    if (rc != RT_ELIMIT) return rc;
    if (L->cin == 4) {
        rc = launch_fwd_ring<4, 1>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
    } else if (L->groups == 1) {
        rc = launch_fwd_ring<16, 1>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
    } else {
        // grouped stages: the z-shift ring kernel, else the dense ring kernel
        if ((int64_t)batch * L->groups <= 65535)
            rc = L->groups == 2 ? launch_ring_zs<2>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st)
                                : launch_ring_zs<4>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
        if (rc == RT_ELIMIT)
            rc = L->groups == 2 ? launch_fwd_ring<16, 2>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st)
                                : launch_fwd_ring<16, 4>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
    }
    if (rc != RT_ELIMIT) return rc;
    // planes too wide for any plane ring: the one-region-per-block tile kernel
    // (its region is 2 pooled z rows x 4 or 2 pooled y rows, so it fits where
    // the 6-plane ring does not)
    return fwd_tile(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
}

extern "C" int64_t rt_conv_mfma_count(const rt_conv_layer* L, int32_t batch, int32_t pass) {
    if (bad_layer(L) || batch < 1 || batch > 65535 || (pass != 0 && pass != 1)) return -1;
    if (layer_bf16x3(L)) return 0;
    int64_t n = 0;
    int rc;
    if (pass == 0) {
        // the forward's input alignment decides conv1's DMA width (same count either way)
        rc = launch_fwd_wino(L, batch, reinterpret_cast<const float*>(16), nullptr, nullptr, nullptr, nullptr, nullptr,
                             nullptr, &n);
    } else {
        const bool pad0 = L->pool_pad[0] == 0 && L->pool_pad[1] == 0 && L->pool_pad[2] == 0;
        if (!pad0 || L->groups == 1 || L->cin != 16) return 0;
        rc = launch_dgrad_wino(L, batch, nullptr, nullptr, nullptr, nullptr, nullptr, &n);
    }
    return rc == RT_OK ? n : 0;
}

extern "C" int64_t rt_conv_wgrad_workspace_floats(const rt_conv_layer* L, int32_t batch) {
    if (bad_layer(L) || batch < 1) return 0;
    // the sparse ring kernel: at most 2 x kWgradRingBlocks partial rows (256-thread
    // blocks); the tile kernel (fallback for planes too wide for the ring) may need more
    const int64_t sparse = (int64_t)2 * kWgradRingBlocks * CO * (L->cin * 27 + 1);
    return std::max(sparse, wgrad_tile_ws(L, batch));
}

extern "C" int rt_conv_relu_pool_wgrad(const rt_conv_layer* L, int32_t batch, const float* x_d, const int64_t* rows_d,
                                       const float* dy_d, const uint8_t* argmax_d, float* dw_d, float* db_d,
                                       float* ws_d, int64_t ws_floats, void* stream) {
    if (bad_layer(L) || batch < 1 || !x_d || !dy_d || !argmax_d || !dw_d || !db_d || !ws_d)
        return rt_internal_fail(RT_EINVAL, "rt_conv_relu_pool_wgrad: bad argument");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // the gather through the pooling argmax; planes too wide for its ring: the tile kernel
    int rc = RT_ELIMIT;
    if (L->cin == 4)
        rc = launch_wgrad_sparse<4, 1>(L, batch, x_d, rows_d, dy_d, argmax_d, dw_d, db_d, ws_d, ws_floats, st);
    else if (L->groups == 1)
        rc = launch_wgrad_sparse<16, 1>(L, batch, x_d, rows_d, dy_d, argmax_d, dw_d, db_d, ws_d, ws_floats, st);
    else if (L->groups == 2)
        rc = launch_wgrad_sparse<16, 2>(L, batch, x_d, rows_d, dy_d, argmax_d, dw_d, db_d, ws_d, ws_floats, st);
    else
        rc = launch_wgrad_sparse<16, 4>(L, batch, x_d, rows_d, dy_d, argmax_d, dw_d, db_d, ws_d, ws_floats, st);
    if (rc != RT_ELIMIT) return rc;
    return wgrad_tile(L, batch, x_d, rows_d, dy_d, argmax_d, dw_d, db_d, ws_d, ws_floats, st);
}

extern "C" int rt_conv_relu_pool_dgrad(const rt_conv_layer* L, int32_t batch, const float* w_d, const float* dy_d,
                                       const uint8_t* argmax_d, float* dx_d, void* stream) {
    if (bad_layer(L) || L->cin != 16 || batch < 1 || batch > 65535 || !w_d || !dy_d || !argmax_d || !dx_d)
        return rt_internal_fail(RT_EINVAL, "rt_conv_relu_pool_dgrad: bad argument");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // grouped stages: the Winograd kernel (f32), the z-shift ring kernel
    // (bf16x3 products, or where the Winograd kernel's LDS does not fit); then
    // the dense ring kernel; the tile kernel for padded pools
    const bool pad0 = L->pool_pad[0] == 0 && L->pool_pad[1] == 0 && L->pool_pad[2] == 0;
    if (pad0 && L->groups > 1 && !layer_bf16x3(L)) {
        const int rc = launch_dgrad_wino(L, batch, w_d, dy_d, argmax_d, dx_d, st);
        if (rc != RT_ELIMIT) return rc;
    }
    if (pad0 && L->groups > 1 && (int64_t)batch * L->groups <= 65535) {
        const int rc = L->groups == 2 ? launch_dgrad_ring_zs<2>(L, batch, w_d, dy_d, argmax_d, dx_d, st)
                                      : launch_dgrad_ring_zs<4>(L, batch, w_d, dy_d, argmax_d, dx_d, st);
        if (rc != RT_ELIMIT) return rc;
    }
    if (pad0) {
        const int rc = L->groups == 1   ? launch_dgrad_ring<1>(L, batch, w_d, dy_d, argmax_d, dx_d, st)
                       : L->groups == 2 ? launch_dgrad_ring<2>(L, batch, w_d, dy_d, argmax_d, dx_d, st)
                                        : launch_dgrad_ring<4>(L, batch, w_d, dy_d, argmax_d, dx_d, st);
        if (rc != RT_ELIMIT) return rc;
    }
    if (L->groups == 1) return launch_dgrad<1, 1, 2>(L, batch, w_d, dy_d, argmax_d, dx_d, st);
    if (L->groups == 2) return launch_dgrad<2, 1, 2>(L, batch, w_d, dy_d, argmax_d, dx_d, st);
    return launch_dgrad<4, 1, 2>(L, batch, w_d, dy_d, argmax_d, dx_d, st);
}
