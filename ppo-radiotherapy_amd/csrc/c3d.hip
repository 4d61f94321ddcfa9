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
#include <cstdint>
#include <type_traits>

#include "rtenv.h"

extern "C" int rt_internal_fail(int code, const char* msg);

namespace {

constexpr int CO = 16;
constexpr int kThreads = 256;

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
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
};

template <int PZB, int PYB>
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
    g.YS = round_mod(g.XL, 4);
    g.ZS = round_mod(g.YL * g.YS, 8);
    g.CS = round_mod(g.ZL * g.ZS, 16);
    return g;
}

// max / min over a pooling window = the 8 lanes of a 16-lane row that share
// bit 1 of the row index (lanes c, c^1 and c+4, c+8, c+12 mod 16): DPP
// quad_perm [1,0,3,2] and row_ror 4, 8 -- full-rate VALU, no LDS crossbar
__device__ __forceinline__ float win_max(float v) {
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, false)));
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false)));
    return v;
}
__device__ __forceinline__ int win_min(int k) {
    k = min(k, __builtin_amdgcn_mov_dpp(k, 0xB1, 0xF, 0xF, false));
    k = min(k, __builtin_amdgcn_mov_dpp(k, 0x124, 0xF, 0xF, false));
    k = min(k, __builtin_amdgcn_mov_dpp(k, 0x128, 0xF, 0xF, false));
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

template <int CIN>
__device__ __forceinline__ void load_tile(float* xs, const float* xb, const Geom& g, int z0, int y0, int x0) {
    constexpr int NWV = kThreads / 64;
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

template <int CIN, int G, int PZB, int PYB>
__global__ __launch_bounds__(kThreads) void k_conv_relu_pool(FwdParams P) {
    extern __shared__ float xs[];
    constexpr int NS = nsteps<CIN>();
    const Geom& g = P.g;
    const int b = blockIdx.z, pz0 = blockIdx.y * PZB, py0 = blockIdx.x * PYB;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, c = lane & 15, gq = lane >> 4;
    const int64_t srow = P.rows ? P.rows[b] : b;
    const float* xb = P.x + srow * (int64_t)CIN * g.D * g.H * g.W;
    const int z0 = 2 * pz0 - g.pd, y0 = 2 * py0 - g.ph, x0 = -g.pw;
    load_tile<CIN>(xs, xb, g, z0, y0, x0);
    float af[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) af[s] = a_frag<CIN, G>(P.w, s, c, gq);
    float bias[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[r] = P.bias[4 * gq + r];
    __syncthreads();

    const int zc = c >> 3, yc = (c >> 2) & 1, xc = c & 3;
    const int widx = zc * 4 + yc * 2 + (xc & 1);
    const int lane_base = gq * g.CS + zc * g.ZS + yc * g.YS + xc;
    // work items: pairs of x-adjacent tiles (tx, tx + 1) of one (tz, ty) row,
    // distributed round-robin over the 4 wavefronts; (row, xp) advance incrementally
    const int nxp = (g.XT + 1) / 2, nrows = PZB * PYB;
    int row = 0, xp = wave;
    while (xp >= nxp) {
        xp -= nxp;
        ++row;
    }
    auto tile_base = [&](int r, int tx) { return lane_base + 2 * (r / PYB) * g.ZS + 2 * (r % PYB) * g.YS + 4 * tx; };
    constexpr int CH = 27;  // k-steps per register batch (one tap set)
    float bv[2][2][CH];     // [buffer][tile][step]
    auto fetch = [&](float (&dst)[2][CH], int r, int xq, int j) {
        const int b0 = tile_base(r, 2 * xq) + j * 4 * g.CS, b1 = b0 + 4;
#pragma unroll
        for (int q = 0; q < CH; ++q) {
            const int off = (q / 9) * g.ZS + ((q / 3) % 3) * g.YS + q % 3;
            dst[0][q] = xs[b0 + off];
            dst[1][q] = xs[b1 + off];
        }
    };
    constexpr int NJ = NS / CH;  // tap sets (input-channel quads) per tile
    if (row < nrows) fetch(bv[0], row, xp, 0);
    // one work item; buffer parity is compile-time (register arrays stay in registers)
    auto item = [&](auto start) {
        constexpr int S0 = decltype(start)::value;
        f4 acc[2] = {{0.0f, 0.0f, 0.0f, 0.0f}, {0.0f, 0.0f, 0.0f, 0.0f}};
        int nrow = row, nx = xp + kThreads / 64;
        while (nx >= nxp) {
            nx -= nxp;
            ++nrow;
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int cb = (S0 + j) & 1;
            // the next batch (next tap set of this item, or the next item) is read
            // two values per MFMA pair, so few LDS reads are ever outstanding
            const bool pf = j + 1 < NJ || nrow < nrows;
            const int fr = j + 1 < NJ ? row : nrow, fx = j + 1 < NJ ? xp : nx, fj = j + 1 < NJ ? j + 1 : 0;
            const int b0 = tile_base(fr, 2 * fx) + fj * 4 * g.CS, b1 = b0 + 4;
#pragma unroll
            for (int q = 0; q < CH; ++q) {
                if (pf) {
                    const int off = (q / 9) * g.ZS + ((q / 3) % 3) * g.YS + q % 3;
                    bv[cb ^ 1][0][q] = xs[b0 + off];
                    bv[cb ^ 1][1][q] = xs[b1 + off];
                }
                acc[0] = mfma4(af[j * CH + q], bv[cb][0][q], acc[0]);
                acc[1] = mfma4(af[j * CH + q], bv[cb][1][q], acc[1]);
                __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);  // 2 LDS reads
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);  // 2 MFMAs
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int tx = 2 * xp + u;
            const int tz = row / PYB, ty = row % PYB;
            const int pz = pz0 + tz, py = py0 + ty;
            const int cz = 2 * pz - g.pd + zc, cy = 2 * py - g.ph + yc, cx = 4 * tx - g.pw + xc;
            const bool valid = cz >= 0 && cz < g.cd && cy >= 0 && cy < g.ch && cx >= 0 && cx < g.cw;
            const int px = 2 * tx + (xc >> 1);
            const bool writer = (c & 0xD) == 0 && tx < g.XT && pz < g.PD && py < g.PH && px < g.PW;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float v = valid ? fmaxf(acc[u][r] + bias[r], 0.0f) : -INFINITY;
                const float m = win_max(v);
                const int k = win_min(v == m ? widx : 8);  // torch: first maximum in (z, y, x) window order
                if (writer) {
                    const size_t o = ((((size_t)b * CO + 4 * gq + r) * g.PD + pz) * g.PH + py) * g.PW + px;
                    P.y[o] = m;
                    if (P.amax) P.amax[o] = (uint8_t)(k | (m > 0.0f ? 8 : 0));
                }
            }
        }
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
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_conv_relu_pool<CIN, G, PZB, PYB>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr = true;
    }
    dim3 grid((P.g.PH + PYB - 1) / PYB, (P.g.PD + PZB - 1) / PZB, B);
    hipLaunchKernelGGL((k_conv_relu_pool<CIN, G, PZB, PYB>), grid, dim3(kThreads), lds, st, P);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_internal_fail(RT_ELAUNCH, hipGetErrorString(e));
    return RT_OK;
}

bool bad_layer(const rt_conv_layer* L) {
    if (!L) return true;
    if (!((L->cin == 4 && L->groups == 1) || (L->cin == 16 && (L->groups == 1 || L->groups == 2 || L->groups == 4))))
        return true;
    for (int a = 0; a < 3; ++a)
        if (L->in_dims[a] < 4 || L->pool_pad[a] < 0 || L->pool_pad[a] > 1) return true;
    return false;
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
    if (L->cin == 4) return launch_fwd<4, 1, 2, 4>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
    if (L->groups == 1) return launch_fwd<16, 1, 1, 2>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
    if (L->groups == 2) return launch_fwd<16, 2, 1, 2>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
    return launch_fwd<16, 4, 1, 2>(L, batch, x_d, rows_d, w_d, b_d, y_d, argmax_d, st);
}
