// rtenv.hip -- MI355X (gfx950) vectorised radiotherapy environment.
//
// Hot path of rmaguado/ppo-radiotherapy re-designed for CDNA4:
//   environment.py:193-243 RadiotherapyEnv.step   -> k_beam + k_dense + k_finish
//   transforms.py:7-69     apply_rotation/translation -> pose_update (k_beam lane 0)
//   draw_line.py:4-102     beam_voxels            -> beam_setup + march_splats (k_beam)
//   environment.py:107-110 add_beam               -> k_beam in-place dose update
//   environment.py:164-191 rewards / termination  -> k_dense (lung reductions) + k_finish
//   environment.py:77-105  reset                  -> RESET mode of the same kernels
//   gymnasium 1.0 SyncVectorEnv NEXT_STEP autoreset + RecordEpisodeStatistics
//   train.py:163-181       GAE                    -> k_gae
//
// Numerics: the reference runs numpy 2.x (NEP 50: its beam code is pure f32),
// scipy's Rotation (f64) and OpenBLAS dot kernels (fused f64 norms).  This file
// is compiled with -ffp-contract=off and IEEE-correct f32/f64 division and
// sqrt so every operation rounds exactly where the reference rounds; fma() is
// written out where OpenBLAS fuses.  See DESIGN.md "Numerics".
//
// Data layout in HBM (per handle = one GPU):
//   dose      f32[N][Vpad]   rows 4 KiB aligned; dense visionless: lung-first rows
//                            (the lung segment in the lung sum plan's chain order
//                            with its zero pad slots, then the other voxels; Vpad =
//                            round_up(its length, 1024)), so k_dense streams only
//                            the lung segment; otherwise C order (Vpad =
//                            round_up(D*H*W, 1024))
//   pose      f64[N][6]      beam position + direction
//   lung_bits u32[Vpad/32]   shared lung mask, 1 bit per voxel (L2-resident)
//   tumour library: sorted C-order voxel lists + per-tumour sum plans
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rtenv.h"
#include "rt_ddmath.h"
#include "rt_trace.h"
#include "policy_core.h"

namespace {

constexpr int kStepThreads = 256;
// k_dense blocks per CU in the pipelined dense rollout: all its 5 resident
// blocks (16-row fetches; blocks per CU 4 / 5 at 16 rows: 11.3 / 12.25 M env
// steps/s; variant builds override this for sweeps)
#ifndef RT_PIPE_DENSE_BPC
#define RT_PIPE_DENSE_BPC 5
#endif

// Library events order work between the library's own streams on one device
// (the pipelined rollout's fork / turns / join) or time kernels; neither needs
// the system-scope release + acquire (L2 writeback and invalidate) a default
// event record performs.  Kernel boundaries keep their device-scope release.
constexpr unsigned kEventNoSysFence = hipEventDisableSystemFence;
constexpr int kSliceVec = 8192;          // k_dense slice: 8192 float4 = 128 KiB of dose
constexpr int kMaxTumourVoxels = 16384;  // tumour voxels (op slots n + n-1 < 2^16; k_finish LDS per wave)
constexpr int kMaxGridDim = 1024;
constexpr int kMaxPlanLevels = 64;       // levels of a tumour's sum plan (LDS copy in k_finish)
constexpr float kEpsF = 1e-6f;           // draw_line.py:4 (f32 under NEP 50)

enum : int32_t { MODE_NOOP = 0, MODE_STEP = 1, MODE_RESET = 2 };
enum : int32_t { FLAG_NEEDS_RESET = 1 };

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define RT_HIP(call)                                                                          \
    do {                                                                                      \
        hipError_t _e = (call);                                                               \
        if (_e != hipSuccess)                                                                 \
            return fail(RT_EDEVICE, std::string(#call) + ": " + hipGetErrorString(_e));       \
    } while (0)

#define RT_LAUNCH_CHECK(name)                                                                 \
    do {                                                                                      \
        hipError_t _e = hipGetLastError();                                                    \
        if (_e != hipSuccess)                                                                 \
            return fail(RT_ELAUNCH, std::string(name) + ": " + hipGetErrorString(_e));        \
    } while (0)

// ---------------------------------------------------------------------------
// Per-env beam record: written by k_beam, read by k_dense / k_finish.  (64 B)
// ---------------------------------------------------------------------------
struct alignas(16) BeamSetup {
    int32_t mode;      // MODE_*
    int32_t niter;     // march iterations (0 = empty beam)
    int32_t start;     // first dominant-axis voxel
    int32_t stepdir;   // +1 / -1
    int32_t dom, o0, o1;
    int32_t tumour;    // tumour id after this call
    float intery0, interz0, sgy, sgz;
    float os_t[3];     // overshoot.translation (f32 copy for info)
    float os_r;        // overshoot.rotation
};

struct TumourMeta {
    int32_t vox_base;    // into tumour voxel array
    int32_t n;           // voxel count
    int32_t op_base;     // into op array
    int32_t lvl_base;    // into level-end array
    int32_t nlev;
    int32_t result;      // slot of the final sum (-1: empty -> 0)
    float T;             // np.sum(tumours) (exact integer in f32)
    float obs_c[3];      // centroid observation (environment.py:261)
    double lung_total;   // np.sum(lungs * (1 - tumours)) (exact)
};

struct Geom {
    int32_t g[3];
    int32_t V;
    int32_t Vpad;
    double S[3];
    double normS;       // np.linalg.norm(LUNG_SHAPE) (ddot: fused)
};

struct Consts {
    int32_t max_t;
    float beam_dose, lung_thr, tum_thr;
    double min_angle, cos_min_angle, move_speed;
    float rot_speed, tum_reward;
    double lung_reward, dist_reward;
    float pi_f;
};

struct EnvState {
    float* dose;          // [N][Vpad]
    double* pose;         // [N][6]
    int32_t* t;
    int32_t* tumour;
    int32_t* flags;
    uint32_t* episode;
    double* ep_return;
    int32_t* ep_len;
    int32_t* next_tumour;
    BeamSetup* setup;
    uint8_t* mode_b;      // [N] setup[e].mode as a byte (k_dense scans a group's modes)
    int32_t* lung_cnt;    // incremental mode: # lung voxels with dose > threshold
    double* lung_sum;     // incremental mode: sum of dose over lung voxels
};

struct Library {
    const uint32_t* lung_bits;
    const int32_t* dose_pos;  // voxel -> position in a dose row (lung-first layout), null = C order
    const int32_t* vox;
    const int32_t* vpos;      // per tumour voxel: its dose-row position (= vox in C order)
    const uint32_t* coord;   // per tumour voxel: lung << 31 | x << 20 | y << 10 | z (no divisions, no
                             // lung-mask lookup in k_finish)
    const uint32_t* ops;     // packed (a | b << 16); dst = n + op index
    const int32_t* lvl_end;  // per level: op index end (relative to op_base)
    const TumourMeta* meta;
    int32_t K;
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef __attribute__((address_space(1))) void* glb_ptr_t;

// ---------------------------------------------------------------------------
// Device numerics helpers
// ---------------------------------------------------------------------------

// np.linalg.norm(f64[n]) = sqrt(ddot) with the OpenBLAS tail loop fused.
__device__ __forceinline__ double ddot_norm3(double a, double b, double c) {
    return sqrt(fma(c, c, fma(b, b, a * a)));
}

// np.linalg.norm(f32[3]): OpenBLAS sdot sums fl32 products in a double, then
// numpy applies sqrtf to the float result.
__device__ __forceinline__ float sdot_norm3(float a, float b, float c) {
    float p0 = a * a, p1 = b * b, p2 = c * c;
    double acc = 0.0;
    acc += (double)p0;
    acc += (double)p1;
    acc += (double)p2;
    return sqrtf((float)acc);
}

__device__ __forceinline__ float clip01(float x) {
    x = x < 0.0f ? 0.0f : x;
    return x > 1.0f ? 1.0f : x;
}

// Philox4x32-10 (counter-based RNG for tumour sampling on autoreset).
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
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

// ---------------------------------------------------------------------------
// transforms.py / environment.py:112-143 (f64 pose update, one lane)
// ---------------------------------------------------------------------------
// libm sin/cos of the rotation half-angle (scipy from_rotvec): correctly
// rounded in double-double on the range the env produces (<= 1.361).
__device__ __forceinline__ void half_sincos(double x, double* s, double* c) {
    if (x <= 1.6) {
        rtdd::sincos_cr(x, s, c);
    } else {
        *s = sin(x);
        *c = cos(x);
    }
}

struct PoseOut {
    double pos[3], dir[3], os_t[3], os_r;
};

__device__ void pose_update(const Geom& G, const Consts& C, const double pos[3], const double dir[3],
                            const float a[6], PoseOut& o) {
    // map_translation (environment.py:122-126) + apply_translation (transforms.py:62-69)
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float c = a[i] < -1.0f ? -1.0f : (a[i] > 1.0f ? 1.0f : a[i]);
        double tr = ((double)c * G.S[i]) * C.move_speed;
        double raw = pos[i] + tr;
        double cl = raw < 0.0 ? 0.0 : raw;
        cl = cl > G.S[i] ? G.S[i] : cl;
        o.pos[i] = cl;
        o.os_t[i] = fabs(raw - cl);
    }
    // map_rotation (environment.py:139-143): f32 under NEP 50
    double r[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        float c = a[3 + i] < -1.0f ? -1.0f : (a[3 + i] > 1.0f ? 1.0f : a[3 + i]);
        r[i] = (double)((c * C.pi_f) * C.rot_speed);
    }
    // apply_rotation (transforms.py:7-59); scipy Rotation.from_rotvec().apply()
    double n0 = ddot_norm3(dir[0], dir[1], dir[2]);
    double d0 = dir[0] / n0, d1 = dir[1] / n0, d2 = dir[2] / n0;
    double ang = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    double sh, ch;
    half_sincos(ang / 2.0, &sh, &ch);
    double s;
    if (ang <= 1e-3) {
        double a2 = ang * ang;
        s = 0.5 - a2 / 48.0 + a2 * a2 / 3840.0;
    } else {
        s = sh / ang;
    }
    double qx = s * r[0], qy = s * r[1], qz = s * r[2], qw = ch;
    double x2 = qx * qx, y2 = qy * qy, z2 = qz * qz, w2 = qw * qw;
    double xy = qx * qy, zw = qz * qw, xz = qx * qz, yw = qy * qw, yz = qy * qz, xw = qx * qw;
    double m00 = x2 - y2 - z2 + w2, m01 = 2.0 * (xy - zw), m02 = 2.0 * (xz + yw);
    double m10 = 2.0 * (xy + zw), m11 = -x2 + y2 - z2 + w2, m12 = 2.0 * (yz - xw);
    double m20 = 2.0 * (xz - yw), m21 = 2.0 * (yz + xw), m22 = -x2 - y2 + z2 + w2;
    // einsum row order on the reference host: (m0*v0 + m2*v2) + m1*v1
    double rd0 = (m00 * d0 + m02 * d2) + m01 * d1;
    double rd1 = (m10 * d0 + m12 * d2) + m11 * d1;
    double rd2 = (m20 * d0 + m22 * d2) + m21 * d1;
    double n1 = ddot_norm3(rd0, rd1, rd2);
    rd0 = rd0 / n1;
    rd1 = rd1 / n1;
    rd2 = rd2 / n1;
    double zc = rd0 < -1.0 ? -1.0 : (rd0 > 1.0 ? 1.0 : rd0);
    double sgn = zc > 0.0 ? 1.0 : (zc < 0.0 ? -1.0 : 0.0);
    double angz = acos(zc);
    if (sgn < 0.0) angz = M_PI - angz;
    double nd0, nd1, nd2;
    if (fabs(angz) < C.min_angle) {
        double tz = sgn * C.cos_min_angle;
        double txy = sqrt(1.0 - tz * tz);
        double x = rd1, y = rd2;
        double nxy = sqrt(fma(y, y, x * x));
        if (nxy < 1e-8) {
            x = 1.0;
            y = 0.0;
        } else {
            x = x / nxy;
            y = y / nxy;
        }
        nd0 = tz;
        nd1 = x * txy;
        nd2 = y * txy;
    } else {
        nd0 = rd0;
        nd1 = rd1;
        nd2 = rd2;
    }
    double n2 = ddot_norm3(nd0, nd1, nd2);
    o.dir[0] = nd0 / n2;
    o.dir[1] = nd1 / n2;
    o.dir[2] = nd2 / n2;
    double os = C.min_angle - angz;
    o.os_r = os > 0.0 ? os : 0.0;
}

// ---------------------------------------------------------------------------
// draw_line.py:17-66 (f32): ray/box clip and march parameters.
// Returns -1 on the ValueError path (norm < eps), else 0 (niter may be 0).
// ---------------------------------------------------------------------------
__device__ int beam_setup(const int32_t g[3], const double pos_d[3], const double dir_d[3],
                          BeamSetup& s) {
    float p[3], d[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        p[i] = (float)pos_d[i];
        d[i] = (float)dir_d[i];
    }
    s.niter = 0;
    float nrm = sdot_norm3(d[0], d[1], d[2]);
    if (nrm < kEpsF) return -1;
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] = d[i] / nrm;
    float tmin[3], tmax[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (fabsf(d[i]) > kEpsF) {
            float t1 = (-p[i]) / d[i];
            float t2 = ((float)(g[i] - 1) - p[i]) / d[i];
            tmin[i] = (t2 < t1) ? t2 : t1;
            tmax[i] = (t2 > t1) ? t2 : t1;
        } else {
            if (p[i] < 0.0f || p[i] > (float)(g[i] - 1)) return 0;
            tmin[i] = -INFINITY;
            tmax[i] = INFINITY;
        }
    }
    float te = tmin[0], tx = tmax[0];
#pragma unroll
    for (int i = 1; i < 3; ++i) {
        if (tmin[i] > te) te = tmin[i];
        if (tmax[i] < tx) tx = tmax[i];
    }
    if (te > tx) return 0;
    float a0 = fabsf(d[0]), a1 = fabsf(d[1]), a2 = fabsf(d[2]);
    int dom = 0;
    float am = a0;
    if (a1 > am) { dom = 1; am = a1; }
    if (a2 > am) { dom = 2; am = a2; }
    int o0 = dom == 0 ? 1 : 0;
    int o1 = dom == 2 ? 1 : 2;
    int step = d[dom] > 0.0f ? 1 : -1;
    float pd = p[dom], dd = d[dom];
    float e_pt = pd + te * dd;
    float x_pt = pd + tx * dd;
    int start = (int)floorf(e_pt);
    int end = (int)floorf(x_pt);
    int niter = (end - start) * step + 1;
    if (niter < 0) niter = 0;
    if (niter > kMaxGridDim + 2) niter = kMaxGridDim + 2;  // unreachable guard
    float po0 = o0 == 0 ? p[0] : p[1];
    float po1 = o1 == 1 ? p[1] : p[2];
    float do0 = o0 == 0 ? d[0] : d[1];
    float do1 = o1 == 1 ? d[1] : d[2];
    s.intery0 = po0 + te * do0;
    s.interz0 = po1 + te * do1;
    float den = dd + kEpsF;
    float gy = do0 / den, gz = do1 / den;
    s.sgy = gy * (float)step;
    s.sgz = gz * (float)step;
    s.start = start;
    s.stepdir = step;
    s.dom = dom;
    s.o0 = o0;
    s.o1 = o1;
    s.niter = niter;
    return 0;
}

// Splats of march iteration k given its intery/interz (draw_line.py:69-100).
// Slot q = 2*dy + dz (the reference's order) holds the flat index and weight,
// or index -1 when the voxel is outside the grid.  Fixed slots keep the
// arrays in registers (a compacted list would be indexed dynamically and
// spill to scratch).
__device__ __forceinline__ void march_splats(const int32_t g[3], const BeamSetup& s, int k, float y, float z,
                                             int32_t idx[4], float w[4]) {
    int x = s.start + k * s.stepdir;
    int yf = (int)floorf(y), zf = (int)floorf(z);
    float yfr = y - (float)yf;
    float zfr = z - (float)zf;
    // idx[dom] = x, idx[o0] = y_floor, idx[o1] = z_floor (draw_line.py:73-82)
    const int b0 = s.dom == 0 ? x : yf;
    const int b1 = s.dom == 1 ? x : (s.dom == 0 ? yf : zf);
    const int b2 = s.dom == 2 ? x : zf;
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
#pragma unroll
        for (int dz = 0; dz < 2; ++dz) {
            float wy = dy == 0 ? (1.0f - yfr) : yfr;
            float ww = wy * (dz == 0 ? (1.0f - zfr) : zfr);
            // draw_line.py:88-90: +dy/+dz always on axes 1/2
            int ix = b0, iy = b1 + dy, iz = b2 + dz;
            const bool in = ix >= 0 && ix < g[0] && iy >= 0 && iy < g[1] && iz >= 0 && iz < g[2];
            idx[2 * dy + dz] = in ? (ix * g[1] + iy) * g[2] + iz : -1;
            w[2 * dy + dz] = ww;
        }
    }
}

__device__ __forceinline__ void no_splats(int32_t idx[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) idx[q] = -1;
}

struct BeamParams {
    Geom G;
    Consts C;
    EnvState st;
    Library lib;
    const float* actions;         // [N][6] (STEP)
    const uint8_t* reset_mask;    // RESET call: NULL = all
    const int32_t* reset_ids;     // RESET call: NULL = sample
    int32_t N;                    // envs [e_begin, N) of the handle take part
    int32_t e_begin;              //   (an env group of the pipelined dense rollout)
    int32_t is_reset_call;
    int32_t incremental;          // RT_STEP_INCREMENTAL (visionless only)
    uint64_t seed;
    int64_t env_id_base;
};

// ---------------------------------------------------------------------------
// One env's control step (a single lane): NEXT_STEP autoreset decision,
// tumour sampling on reset (environment.py:86-105), f64 pose update
// (environment.py:196-210) and the f32 beam setup (draw_line.py:17-66).
// ---------------------------------------------------------------------------
__device__ BeamSetup pose_step(const BeamParams& P, int e, const float* act) {
    const EnvState& st = P.st;
    BeamSetup s{};
    int32_t flags = st.flags[e];
    int mode;
    if (P.is_reset_call) {
        bool sel = P.reset_mask == nullptr || P.reset_mask[e] != 0;
        mode = sel ? MODE_RESET : MODE_NOOP;
        if (sel && P.reset_ids) st.next_tumour[e] = P.reset_ids[e];
    } else {
        mode = (flags & FLAG_NEEDS_RESET) ? MODE_RESET : MODE_STEP;
    }
    s.mode = mode;
    double* pose = st.pose + (size_t)e * 6;
    if (mode == MODE_RESET) {
        int32_t tid = st.next_tumour[e];
        if (tid < 0 || tid >= P.lib.K) {
            uint32_t ep = st.episode[e]++;
            uint64_t gid = (uint64_t)(P.env_id_base + e);
            uint4 r = philox4x32(make_uint4(ep, (uint32_t)gid, (uint32_t)(gid >> 32), 0x52544e56u),
                                 make_uint2((uint32_t)P.seed, (uint32_t)(P.seed >> 32)));
            tid = (int32_t)(((uint64_t)r.x * (uint64_t)P.lib.K) >> 32);
        }
        st.next_tumour[e] = -1;
        st.tumour[e] = tid;
        s.tumour = tid;
        pose[0] = P.G.S[0] / 2.0;
        pose[1] = P.G.S[1] / 2.0;
        pose[2] = P.G.S[2] / 2.0;
        pose[3] = 0.0;
        pose[4] = 1.0;
        pose[5] = 0.0;
        st.t[e] = 0;
        st.flags[e] = flags & ~FLAG_NEEDS_RESET;
        st.ep_return[e] = 0.0;
        st.ep_len[e] = 0;
    } else if (mode == MODE_STEP) {
        s.tumour = st.tumour[e];
        float a[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) a[i] = act ? act[i] : P.actions[(size_t)e * 6 + i];
        double pos[3] = {pose[0], pose[1], pose[2]};
        double dir[3] = {pose[3], pose[4], pose[5]};
#ifdef RT_TRACE
        if (pos[0] + dir[0] + a[0] == 12345.0) pose[0] = 0.0;  // consume the loads before the stamp
#endif
        RT_STAMP(e, 10);
        PoseOut o;
        pose_update(P.G, P.C, pos, dir, a, o);
#ifdef RT_TRACE
        if (o.dir[0] == 12345.0) pose[0] = 0.0;
#endif
        RT_STAMP(e, 11);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            pose[i] = o.pos[i];
            pose[3 + i] = o.dir[i];
            s.os_t[i] = (float)o.os_t[i];
        }
        s.os_r = (float)o.os_r;
        st.t[e] = st.t[e] + 1;
        beam_setup(P.G.g, o.pos, o.dir, s);  // a renormalised direction never takes the ValueError path
    } else {
        s.tumour = st.tumour[e];
    }
    return s;
}

__device__ __forceinline__ int rfl_i(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ float rfl_f(float x) {
    return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(x)));
}

// ---------------------------------------------------------------------------
// k_beam: one wave per env (4 envs per 256-thread block).
// Lane 0 runs pose_step; then lane k marches iteration k (k, k+64, ...) and
// applies add_beam (environment.py:107-109) to the voxels it owns:
//   dose[v] = clip(dose[v] + fl32(b[v] * 0.1f), 0, 1),  b[v] = sum of splats.
// Only voxels the beam touches change, so the update is done in place on
// those <= 4*(D+1) voxels.  A voxel receives at most two splats, and only from
// consecutive iterations (draw_line.py:88-90 puts the +1 offsets on axes 1/2,
// which is the march axis when dom != 0), so the lane of the lower iteration
// owns the voxel and adds its neighbour's weight: fl32(w_k + w_k+1) is exactly
// the reference's `output[...] += weight` sequence (IEEE add commutes).
// ---------------------------------------------------------------------------
// act: the env's 6 action floats in registers (fused policy step) or null
// (read from P.actions).
__device__ int beam_env(const BeamParams& P, int e, int lane, const float* act) {
    BeamSetup s{};
    if (lane == 0) {
        RT_STAMP(e, 2);
        s = pose_step(P, e, act);
        P.st.setup[e] = s;
        P.st.mode_b[e] = (uint8_t)s.mode;
        RT_STAMP(e, 3);
    }
    if (lane == 0) RT_STAMP(e, 12);
    const int mode = rfl_i(s.mode);
    if (P.incremental && mode == MODE_RESET) {
        // reset_dose (environment.py:104) when no k_dense runs (incremental step,
        // persistent rollouts): the env's own wave zeroes its row
        typedef float nf4 __attribute__((ext_vector_type(4)));
        nf4* d4 = reinterpret_cast<nf4*>(P.st.dose + (size_t)e * P.G.Vpad);
        const nf4 z = {0.f, 0.f, 0.f, 0.f};
        const int nvec = P.G.Vpad >> 2;
        for (int q = lane; q < nvec; q += 64) __builtin_nontemporal_store(z, d4 + q);
        if (lane == 0) {
            P.st.lung_cnt[e] = 0;
            P.st.lung_sum[e] = 0.0;
        }
        return mode;
    }
    if (mode != MODE_STEP) return mode;
    BeamSetup b;
    b.niter = rfl_i(s.niter);
    b.start = rfl_i(s.start);
    b.stepdir = rfl_i(s.stepdir);
    b.dom = rfl_i(s.dom);
    b.o0 = rfl_i(s.o0);
    b.o1 = rfl_i(s.o1);
    b.intery0 = rfl_f(s.intery0);
    b.interz0 = rfl_f(s.interz0);
    b.sgy = rfl_f(s.sgy);
    b.sgz = rfl_f(s.sgz);
    const int niter = b.niter;
    if (niter <= 0) return mode;  // (incremental counters unchanged: the beam missed the box)
    float* dose = P.st.dose + (size_t)e * P.G.Vpad;
    const float bd = P.C.beam_dose;
    const bool pairs = b.dom != 0;
    // running march state: (ya, za) = iteration max(k-1, 0)
    const uint32_t* lbits = P.lib.lung_bits;
    const float thr = P.C.lung_thr;
    int dcnt = 0;       // incremental: change of the lung over-threshold count
    double dsum = 0.0;  // incremental: change of the lung dose sum
    float ya = b.intery0, za = b.interz0;
    int k = lane;
    for (int j = 0; j < k - 1; ++j) {
        ya = ya + b.sgy;
        za = za + b.sgz;
    }
    for (; k < niter; k += 64) {
        float yk = ya, zk = za;
        if (k > 0) {
            yk = ya + b.sgy;
            zk = za + b.sgz;
        }
        int32_t ci[4], pi[4], ni[4];
        float cw[4], pw[4], nw[4];
        march_splats(P.G.g, b, k, yk, zk, ci, cw);
        if (pairs && k > 0) march_splats(P.G.g, b, k - 1, ya, za, pi, pw);
        else no_splats(pi);
        if (pairs && k + 1 < niter) march_splats(P.G.g, b, k + 1, yk + b.sgy, zk + b.sgz, ni, nw);
        else no_splats(ni);
        // the lane's owned voxels (<= 4, distinct): every load of the
        // iteration is issued before the first store -- written as a
        // load-modify-store per voxel the compiler kept each store ahead of
        // the next voxel's loads (it cannot prove the rows do not alias), so
        // a lane paid 4 (lung-first rows: 8) dependent HBM round trips
        bool own[4];
        float wv[4];
        int32_t pv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int32_t v = ci[i];
            bool owned = v >= 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) owned = owned && (pi[j] != v);
            float w = cw[i];
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (ni[j] == v) w = w + nw[j];
            own[i] = owned;
            wv[i] = w;
            pv[i] = owned ? v : 0;
        }
        if (P.lib.dose_pos) {
#pragma unroll
            for (int i = 0; i < 4; ++i) pv[i] = own[i] ? P.lib.dose_pos[pv[i]] : 0;
        }
        float old_d[4];
        uint32_t lb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            old_d[i] = own[i] ? dose[pv[i]] : 0.0f;
            lb[i] = (P.incremental && own[i]) ? lbits[ci[i] >> 5] : 0u;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (!own[i]) continue;
            const float new_d = clip01(old_d[i] + wv[i] * bd);
            dose[pv[i]] = new_d;
            if (P.incremental && ((lb[i] >> (ci[i] & 31)) & 1u)) {
                dcnt += (new_d > thr ? 1 : 0) - (old_d[i] > thr ? 1 : 0);
                dsum += (double)new_d - (double)old_d[i];
            }
        }
        // advance (ya, za) to iteration k + 63
        const int adds = k == 0 ? 63 : 64;
        for (int j = 0; j < adds; ++j) {
            ya = ya + b.sgy;
            za = za + b.sgz;
        }
    }
    if (P.incremental) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            dcnt += __shfl_xor(dcnt, off, 64);
            dsum += __shfl_xor(dsum, off, 64);
        }
        if (lane == 0) {
            P.st.lung_cnt[e] += dcnt;
            P.st.lung_sum[e] += dsum;
        }
    }
    if (lane == 0) RT_STAMP(e, 4);
    return mode;
}

__global__ __launch_bounds__(256) void k_beam(BeamParams P) {
    const int lane = threadIdx.x & 63;
    const int e = P.e_begin + blockIdx.x * 4 + (threadIdx.x >> 6);
    if (e >= P.N) return;  // wave-uniform
    beam_env(P, e, lane, nullptr);
}

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

__device__ __forceinline__ void lds_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    __builtin_amdgcn_wave_barrier();
}

// Executes an exact-order sum plan (a tumour's, or a partial numpy buffer's
// leaf tree) over the slots `tv` (leaves
// 0..n-1 filled; op o writes slot n+o) level by level; returns the final sum
// (0 for an empty tumour).  Every lane returns it.
__device__ __forceinline__ float run_plan(float* tv, const uint32_t* ops, const int32_t* lev, int nt, int nlev,
                                          int result, int lane) {
    int lo = 0;
    for (int l = 0; l < nlev; ++l) {
        lds_wave_sync();
        const int hi = lev[l];
        for (int o = lo + lane; o < hi; o += 64) {
            const uint32_t ab = ops[o];
            tv[nt + o] = tv[ab & 0xffffu] + tv[ab >> 16];
        }
        lo = hi;
    }
    lds_wave_sync();
    return result >= 0 ? tv[result] : 0.0f;
}

// ---------------------------------------------------------------------------
// The lung sum plan: np.sum(dose * lungs) (info doses.lung, environment.py:235)
// in numpy's exact order.  numpy reduces a contiguous f32 volume in 8192-element
// buffers, sequentially, each by pairwise summation: a buffer is split at
// n/2 rounded down to a multiple of 8 until a part has <= 128 elements, and a
// part (a "leaf") keeps 8 accumulators -- element i of the leaf goes to r[i % 8]
// for the first n - n % 8 elements -- combined as ((r0+r1)+(r2+r3))+((r4+r5)+
// (r6+r7)), then the n % 8 tail elements are added one by one (oracle/
// rt_oracle.c:pairwise_f32).  Non-lung terms are exact zeros, and adding +0 to
// a non-negative sum is exact, so each accumulator r[j] is the sequential sum of
// its leaf's LUNG voxels of class j (a "chain", <= 16 long), a tail voxel is a
// chain of one, and everything above the chains is a fixed tree.
//
// Dense visionless handles keep each dose row lung-first; the host builder
// (build_lung_plan) orders the lung segment by numpy buffer ("chunk") and, inside
// a chunk, by chain: the chains sorted by length, 256 per group -- lane l of a
// wave owns chains 4l..4l+3 -- group rows stored ragged: row k holds element k
// of the group's first nk[k] chains, contiguously, padded with zero slots to a
// whole number of 64-B sectors (no sector holds two rows).  A wave streams a chunk
// with coalesced 16-B loads (element k of its four chains per lane, a group's
// rows in flight: up to 16 KiB per wave), each lane summing its chains in
// order.  The chain
// sums go to LDS slots [leaf][class]; lane = leaf then combines its 8 slots,
// and a whole 8192-element buffer (64 leaves of 128, a perfect tree) finishes
// with a 6-step xor butterfly (IEEE addition commutes, so both lanes of a pair
// form the same sum).  A partial buffer (the last one of a volume whose size
// is not a multiple of 8192) has an irregular tree: its leaves add their tail
// voxels and run a level plan (run_plan).  The chunk sums go to
// part_sum[e][chunk]; k_finish adds them in chunk order from 0.0f -- numpy's
// outer loop (chunks without lung voxels add +0).
// Vision handles keep C-order rows: the same plan, each segment position
// gathered through lpos (segment position -> voxel, -1 for a pad slot).
// ---------------------------------------------------------------------------
constexpr int kLungChunk = 8192;        // numpy's reduction buffer
constexpr int kLungLeafMax = 65;        // leaves of a buffer of <= 8192 elements (65 at 8185..8191)
constexpr int kLungSlotFloats = 528;    // [leaf][8 classes], 16-B padded
constexpr int kLungWaveFloats = kLungSlotFloats;  // a partial buffer's plan slots (2 x leaves) alias the slots
constexpr int kLungGroup = 256;         // chains per group (4 per lane)
#ifndef RT_LUNG_ROW_ALIGN
#define RT_LUNG_ROW_ALIGN 16
#endif
constexpr int kLungRowAlign = RT_LUNG_ROW_ALIGN;  // floats a lung row is padded to (16: one 64-B sector)
constexpr uint16_t kNoSlot = 0xFFFFu;

struct LChunk {          // one numpy buffer holding lung voxels
    int32_t seg_base;    // segment position of its first chain element (a multiple of kLungRowAlign)
    int32_t grp_base;    // its first chain group
    int32_t n_grp;
    int32_t gen;         // -1: a whole 8192-element buffer (butterfly); else its LGeneric record
};
struct LGroup {          // 256 chains (lane l: chains 4l..4l+3), sorted by length
    uint32_t row[16];    // row k: its first slot relative to the chunk's seg_base | the lanes
                         // whose float4 holds one of its elements (ceil(nk / 4); non-increasing
                         // in k; 0 past the longest chain) << 16
};
struct LGeneric {        // a partial buffer's leaf tree
    int32_t n_leaf, op_base, lvl_base, nlev, result, tail_base;
};
struct LungParams {
    const LChunk* chunk;
    const LGroup* grp;
    const uint64_t* slot;     // [group][64]: lane's 4 chains' slots (leaf * 8 + class; kNoSlot: tail
                              // voxel / no chain), 16 bits each
    const LGeneric* gen;
    const uint32_t* ops;      // partial buffers' leaf trees: (a | b << 16), dst = n_leaf + op
    const int32_t* lvl_end;
    const int32_t* tail_off;  // per partial buffer: [n_leaf + 1] into tail_pos
    const int32_t* tail_pos;  // segment positions of each leaf's tail voxels, C order
    const int32_t* lpos;      // C-order rows (vision): segment position -> voxel (-1: pad); null: lung-first
    int32_t n_chunk;
};

struct DenseParams {
    Geom G;
    float lung_thr;
    EnvState st;
    const uint32_t* lung_bits;
    LungParams L;
    int32_t* part_cnt;     // [N][L.n_chunk] lung voxels above the threshold per numpy buffer
    float* part_sum;       // [N][L.n_chunk] np.sum order partial of each numpy buffer
    int32_t slices;        // k_dense_vis: row slices per env
    int32_t vec_per_slice; // k_dense_vis: float4 per slice
    int32_t e_begin;       // first env (env group of the pipelined rollout)
};

// ---------------------------------------------------------------------------
// k_dense: the full-volume reductions of lungs_dose_reward
// (environment.py:173-182) and info doses.lung (environment.py:235) for every
// env: count(dose > 0.2) over the lung voxels (tumour voxels are corrected in
// k_finish) and np.sum(dose * lungs) in numpy's order (the lung sum plan
// above).  Only lung voxels contribute and the rows are laid out lung-first,
// so the reduction is a read-only stream of each row's lung segment with no
// per-voxel mask; the work item is (env, numpy buffer), one wave each.
// RESET envs' rows are zeroed instead (reset_dose, environment.py:104), by
// zero_reset_share.
// ---------------------------------------------------------------------------
// Non-temporal loads: the 1.6 GB of lung segments a step reads far exceed L2
// and the Infinity Cache, and are read once (plain loads: 6.1 TB/s, nt: the
// 6.3-6.6 TB/s regime; profiles/r01_v3..v6).
__device__ __forceinline__ float4 load_nt(const float4* p) {
    typedef float nf4 __attribute__((ext_vector_type(4)));
    const nf4 t = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p));
    return make_float4(t.x, t.y, t.z, t.w);
}

// The plan is read-only while k_dense runs: read through the constant address
// space so the compiler issues scalar loads (one s_load_dwordx16 per group)
// instead of per-lane loads whose results gate the row addresses.
#if defined(__HIP_DEVICE_COMPILE__)
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* cst(const T* p) {
    return (const __attribute__((address_space(4))) T*)p;
}
#else  // the host pass of the device functions (never executed)
template <typename T>
__device__ __forceinline__ const T* cst(const T* p) {
    return p;
}
#endif

typedef float lf4 __attribute__((ext_vector_type(4)));

// One chain group: element k of the lane's 4 chains -> x[k] (zero where the
// lane holds no element of row k: an exact no-op for the sums and the count;
// pad slots are zeros in memory).  Only the group's rows are loaded (a uniform
// branch per row: the profile of round 6 had the texture-address unit 73 %
// busy when every group issued all 16 rows); buffer loads, the row offset in
// an SGPR.
// Rows per fetch: a group's 16 rows at once, at 88 VGPRs = 5 waves per SIMD.
// (8-row halves at 57 VGPRs and 8 waves per SIMD: 11.4 M env steps/s in the
// pipelined rollout, the stream holding every wave slot of the CU; 10 rows at
// 8 waves, 12 at 7: no better; 16 rows at 5 waves: 12.25 M, the other group's
// chain finds its slots again -- profiles/r06/r06_s18_fetch_rows_sweep.txt.)
// The half index h stays for a fetch size below 16.
constexpr int kLungHalf = 16;
constexpr int kDenseWavesPerSimd = 5;

template <bool GATHER>
__device__ __forceinline__ void lung_fetch(const DenseParams& P, __amdgpu_buffer_rsrc_t rsrc, const float* row,
                                           int seg_base, int g, int h, int lane, lf4 (&x)[kLungHalf]) {
    const auto G = cst(P.L.grp) + g;
    uint32_t ri[kLungHalf];
#pragma unroll
    for (int k = 0; k < kLungHalf; ++k) ri[k] = h * kLungHalf + k < 16 ? G->row[h * kLungHalf + k] : 0u;  // one s_load_dwordx16, one wait
#pragma unroll
    for (int k = 0; k < kLungHalf; ++k) {
        const int nl = (int)(ri[k] >> 16);
        if (nl == 0) {  // wave-uniform: past the group's longest chain
            x[k] = lf4{0.0f, 0.0f, 0.0f, 0.0f};
            continue;
        }
        const int r0 = seg_base + (int)(ri[k] & 0xffffu);
        lf4 v;
        if constexpr (GATHER) {
            const int4 lp = *reinterpret_cast<const int4*>(P.L.lpos + r0 + 4 * lane);
            v = lf4{lp.x >= 0 ? row[lp.x] : 0.0f, lp.y >= 0 ? row[lp.y] : 0.0f, lp.z >= 0 ? row[lp.z] : 0.0f,
                    lp.w >= 0 ? row[lp.w] : 0.0f};
            x[k] = lane < nl ? v : lf4{0.0f, 0.0f, 0.0f, 0.0f};
        } else {
            // only the row's nl lanes load (exec-masked: the lanes past it take no
            // texture-address cycles and fetch no line of the next row); aux 2:
            // non-temporal (streamed once)
            lf4 v = lf4{0.0f, 0.0f, 0.0f, 0.0f};
            if (lane < nl) v = __builtin_bit_cast(lf4, __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * lane, 4 * r0, 2));
            x[k] = v;
        }
    }
}

// the fetched rows of the lane's 4 chains in order (numpy's r[j] += a[i]
// sequences) onto acc, and their over-threshold count
__device__ __forceinline__ void lung_consume(const DenseParams& P, int g, int h, const lf4 (&x)[kLungHalf], lf4& acc,
                                             float thr, int& cnt) {
    const auto G = cst(P.L.grp) + g;
#pragma unroll
    for (int k = 0; k < kLungHalf; ++k) {
        if (h * kLungHalf + k < 16 && (G->row[h * kLungHalf + k] >> 16)) {  // wave-uniform: a row of this group
            acc.x = acc.x + x[k].x;
            acc.y = acc.y + x[k].y;
            acc.z = acc.z + x[k].z;
            acc.w = acc.w + x[k].w;
            cnt += (x[k].x > thr ? 1 : 0) + (x[k].y > thr ? 1 : 0) + (x[k].z > thr ? 1 : 0) + (x[k].w > thr ? 1 : 0);
        }
    }
}

// the group's 4 chain sums of the lane into their LDS slots
__device__ __forceinline__ void lung_emit(uint64_t slot, const lf4& acc, float* slots) {
    const uint32_t s0 = (uint32_t)slot & 0xffffu, s1 = (uint32_t)(slot >> 16) & 0xffffu;
    const uint32_t s2 = (uint32_t)(slot >> 32) & 0xffffu, s3 = (uint32_t)(slot >> 48);
    if (s0 != kNoSlot) slots[s0] = acc.x;
    if (s1 != kNoSlot) slots[s1] = acc.y;
    if (s2 != kNoSlot) slots[s2] = acc.z;
    if (s3 != kNoSlot) slots[s3] = acc.w;
}

// LDS order inside one wave: its DS instructions execute in issue order, so a
// lane reads what another lane of the same wave wrote earlier with no wait on
// memory -- only the compiler must keep the order (the workgroup fence of
// lds_wave_sync would also wait for every vector load in flight).
__device__ __forceinline__ void lds_wave_order() {
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// Item i of a launch -> env e_begin + i / n_chunk, chunk (i + h(env)) mod
// n_chunk with h a multiplicative hash: env-major, so the waves in flight at
// once read neighbouring buffers of a few hundred dose rows, and the rotation
// makes a wave's strided items (stride = the grid's waves, a multiple of the
// chunk count) visit every chunk size -- without it each wave keeps one chunk
// index: a 250x spread of bytes per wave (4.1 TB/s alone), and the chunk-major
// order (the waves on the same buffer of every row) streamed 5.5 against 5.7
// TB/s alone (rocprofv3, round 6).
__device__ __forceinline__ void lung_item_of(const LungParams& L, int e_begin, int i, int& e, int& j) {
    const int r = i / L.n_chunk;
    e = e_begin + r;
    j = (int)(((uint32_t)(i - r * L.n_chunk) + (((uint32_t)r * 2654435761u) >> 16)) % (uint32_t)L.n_chunk);
}

// The (env, chunk) items of envs [e_begin, e_begin + n_env) a wave takes:
// first, first + stride, ... (lung_item_of).  Per item: its groups'
// loads and chain sums, then -- with the NEXT item's first group already in
// flight -- the combine (leaf formula, butterfly or level plan) and the
// partials, written for STEP envs only (a RESET env's row may be zeroed by
// zero_reset_share meanwhile; its values are dropped).  `wl`: the wave's
// kLungWaveFloats of LDS.
template <bool GATHER>
__device__ void lung_stream(const DenseParams& P, int n_env, int first, int stride, int lane, float* wl) {
    const int n_items = n_env * P.L.n_chunk;
    if (first >= n_items) return;
    float* slots = wl;
    // a partial buffer's leaf values and plan slots overwrite the class slots:
    // lane L reads leaf L's 8 slots (all lanes in one instruction) before it
    // writes leafv[L], and leaf L + 64 (lane 0's second pass) lies above 64
    float* leafv = wl;
    const float thr = P.lung_thr;
    auto row_of = [&](int e) { return P.st.dose + (size_t)e * P.G.Vpad; };
    auto rsrc_of = [&](const float* r) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(r), 0, P.G.Vpad * 4, 0x00020000);
    };
    int it = first;
    int e, j;
    lung_item_of(P.L, P.e_begin, it, e, j);
    LChunk c = cst(P.L.chunk)[j];
    const float* row = row_of(e);
    __amdgpu_buffer_rsrc_t rsrc = rsrc_of(row);
    lf4 x[kLungHalf];
    lung_fetch<GATHER>(P, rsrc, row, c.seg_base, c.grp_base, 0, lane, x);
    for (int i = lane; i < kLungSlotFloats / 4; i += 64) reinterpret_cast<lf4*>(slots)[i] = lf4{0.f, 0.f, 0.f, 0.f};
    lds_wave_order();
    for (;;) {
        int cnt = 0;
        for (int g = c.grp_base; g < c.grp_base + c.n_grp; ++g) {
            const uint64_t sl = P.L.slot[(size_t)g * 64 + lane];
            lf4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
            if (g > c.grp_base) lung_fetch<GATHER>(P, rsrc, row, c.seg_base, g, 0, lane, x);
            lung_consume(P, g, 0, x, acc, thr, cnt);
            if (kLungHalf < 16 && (cst(P.L.grp)[g].row[kLungHalf % 16] >> 16)) {  // wave-uniform: the group has a second half
                lung_fetch<GATHER>(P, rsrc, row, c.seg_base, g, 1, lane, x);
                lung_consume(P, g, 1, x, acc, thr, cnt);
            }
            lung_emit(sl, acc, slots);
        }
        lds_wave_order();
        // the next item's first group in flight during this item's combine
        const int nit = it + stride;
        int ne = e, nj = j;
        LChunk nc = c;
        const float* nrow = row;
        __amdgpu_buffer_rsrc_t nrsrc = rsrc;
        if (nit < n_items) {
            lung_item_of(P.L, P.e_begin, nit, ne, nj);
            nc = cst(P.L.chunk)[nj];
            nrow = row_of(ne);
            nrsrc = rsrc_of(nrow);
            lung_fetch<GATHER>(P, nrsrc, nrow, nc.seg_base, nc.grp_base, 0, lane, x);
        }
        float v;
        if (c.gen < 0) {
            // a whole buffer: lane = leaf (64 x 128 elements), leaf formula, then
            // the perfect tree over the 64 leaves as an xor butterfly
            const lf4 a = reinterpret_cast<const lf4*>(slots)[2 * lane];
            const lf4 b = reinterpret_cast<const lf4*>(slots)[2 * lane + 1];
            v = ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) v = v + __shfl_xor(v, off, 64);
        } else {
            const LGeneric q = cst(P.L.gen)[c.gen];
            for (int L = lane; L < q.n_leaf; L += 64) {
                const lf4 a = reinterpret_cast<const lf4*>(slots)[2 * L];
                const lf4 b = reinterpret_cast<const lf4*>(slots)[2 * L + 1];
                float t = ((a.x + a.y) + (a.z + a.w)) + ((b.x + b.y) + (b.z + b.w));
                const int t0 = P.L.tail_off[q.tail_base + L], t1 = P.L.tail_off[q.tail_base + L + 1];
                for (int i = t0; i < t1; ++i) {
                    const int p = P.L.tail_pos[i];
                    t = t + (GATHER ? row[P.L.lpos[p]] : row[p]);
                }
                leafv[L] = t;
            }
            v = run_plan(leafv, P.L.ops + q.op_base, P.L.lvl_end + q.lvl_base, q.n_leaf, q.nlev, q.result, lane);
        }
        cnt = wave_sum_i(cnt);
        if (lane == 0 && cst(P.st.mode_b)[e] == MODE_STEP) {
            P.part_cnt[(size_t)e * P.L.n_chunk + j] = cnt;
            P.part_sum[(size_t)e * P.L.n_chunk + j] = v;
        }
        if (nit >= n_items) break;
        lds_wave_order();  // the combine has read the slots
        for (int i = lane; i < kLungSlotFloats / 4; i += 64)
            reinterpret_cast<lf4*>(slots)[i] = lf4{0.f, 0.f, 0.f, 0.f};
        lds_wave_order();
        it = nit;
        e = ne;
        j = nj;
        c = nc;
        row = nrow;
        rsrc = nrsrc;
    }
}

// reset_dose (environment.py:104) of the RESET envs is not done by their own
// slice blocks/items: a row is 2.7x the bytes of the lung segment a slice
// streams, so a block that drew a reset env's slice ran long and, near the
// end of a launch, set its length.  The zeroing is spread instead: blocks
// count the group's resets (one mode byte per env, block prefix sum), take an
// equal share of the concatenated reset rows [0, R x row) and locate the
// reset envs of that share by rank.
__device__ __forceinline__ int block_excl_scan(int v, int* s_w, int* total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
    }
    if (lane == 63) s_w[wid] = x;
    __syncthreads();
    int base = 0, tot = 0;
    for (int w = 0; w < kStepThreads / 64; ++w) {
        base += w < wid ? s_w[w] : 0;
        tot += s_w[w];
    }
    *total = tot;
    __syncthreads();  // s_w reused by the caller's next scan
    return base + x - v;
}

constexpr int kZeroBlocks = 256;  // grid k_dense: blocks that zero RESET rows (one per CU)

// zero_reset_share: part `part` of n_parts of the zeroing of the RESET rows
// among envs [e_begin, e_begin + n_env) (reset_dose, environment.py:104).
__device__ void zero_reset_share(const DenseParams& P, int e_begin, int n_env, int part, int n_parts) {
    __shared__ int s_w[kStepThreads / 64];
    __shared__ int s_env;
    const int tid = threadIdx.x;
    const int per = (n_env + kStepThreads - 1) / kStepThreads;
    const int a0 = min(tid * per, n_env), a1 = min(a0 + per, n_env);
    const uint8_t* mb = P.st.mode_b + e_begin;
    int c = 0;
    for (int e = a0; e < a1; ++e) c += mb[e] == MODE_RESET;
    int R;
    const int pre = block_excl_scan(c, s_w, &R);
    if (R == 0) return;  // block-uniform
    const int64_t rowv = P.G.Vpad >> 2;  // float4 per row
    const int64_t tot = (int64_t)R * rowv;
    const int64_t share = ((tot + n_parts - 1) / n_parts + 63) / 64 * 64;
    const int64_t z0 = (int64_t)part * share, z1 = min(z0 + share, tot);
    if (z0 >= z1) return;
    for (int64_t r = z0 / rowv; r <= (z1 - 1) / rowv; ++r) {
        if (r >= pre && r < pre + c) {  // this thread's env range holds reset rank r
            int k = (int)(r - pre);
            for (int e = a0; e < a1; ++e) {
                if (mb[e] == MODE_RESET && k-- == 0) {
                    s_env = e_begin + e;
                    break;
                }
            }
        }
        __syncthreads();
        const int e = s_env;
        __syncthreads();
        const int64_t q0 = max(z0, r * rowv) - r * rowv, q1 = min(z1, (r + 1) * rowv) - r * rowv;
        typedef float nf4 __attribute__((ext_vector_type(4)));
        nf4* d4 = reinterpret_cast<nf4*>(P.st.dose + (size_t)e * P.G.Vpad);
        const nf4 z = {0.f, 0.f, 0.f, 0.f};
        for (int64_t q = q0 + tid; q < q1; q += kStepThreads) __builtin_nontemporal_store(z, d4 + q);
    }
}

// k_dense: waves stride over the (env, chunk) items of envs [e_begin,
// e_begin + n_env) (lung_stream), then every block zeroes its share of the
// RESET envs' rows.  A fixed grid of a few blocks per CU: the pipelined dense
// rollout's dose stream leaves CU slots free for the other env group's
// latency-bound kernels; the stepwise / one-group launches fill the chip.
// Items: lung_item_of.
// GATHER: C-order rows (vision handles, after k_dense_vis; no zeroing).
template <bool GATHER>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kDenseWavesPerSimd))) void k_dense(DenseParams P,
                                                                                                    int n_env) {
    __shared__ __attribute__((aligned(16))) float dsm[4 * kLungWaveFloats];
    // wave-uniform (readfirstlane): the item, its chunk and group records then
    // live in SGPRs and the plan is read by scalar loads
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    lung_stream<GATHER>(P, n_env, blockIdx.x * 4 + w, gridDim.x * 4, lane, dsm + w * kLungWaveFloats);
    if (!GATHER) zero_reset_share(P, P.e_begin, n_env, blockIdx.x, gridDim.x);
}

constexpr int kMaxRolloutGroups = 4;

// Store 4 consecutive voxels [v0, v0+4) of one obs channel row.
__device__ __forceinline__ void store4(float* row, int v0, int V, bool aligned4, float a, float b, float c,
                                       float d) {
    if (aligned4) {
        *reinterpret_cast<float4*>(row + v0) = make_float4(a, b, c, d);
    } else {
        if (v0 < V) row[v0] = a;
        if (v0 + 1 < V) row[v0 + 1] = b;
        if (v0 + 2 < V) row[v0 + 2] = c;
        if (v0 + 3 < V) row[v0 + 3] = d;
    }
}

struct DenseVisParams {
    DenseParams d;
    float* obs;   // [N][4][V]
    // render source (rt_env_set_render_source): a NOOP env e < src_n re-emits
    // its observation from src + src_rows[e] * src_stride (C order) instead
    // of its own dose row
    const float* src;
    const int64_t* src_rows;
    int64_t src_stride;
    int32_t src_n;
};

// ---------------------------------------------------------------------------
// k_dense_vis: the dense channels of the vision observation
// (environment.py:252-257, get_volumes): channel 0 = clip(lungs), channel 2 =
// clip(dose) (dose is already in [0,1]); channels 1 (tumour) and 3 (beam view)
// are zeroed here and scattered by k_finish.  Runs for every mode: RESET
// zeroes the dose, NOOP (a reset call's unselected envs) only re-emits the
// observation.  The STEP envs' lung reductions follow as k_dense<true> (the
// lung sum plan gathered from the C-order row).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_dense_vis(DenseVisParams PV) {
    const DenseParams& P = PV.d;
    const int sl = blockIdx.x, e = P.e_begin + blockIdx.y;
    const int tid = threadIdx.x;
    const int mode = P.st.setup[e].mode;
    float4* d4 = reinterpret_cast<float4*>(P.st.dose + (size_t)e * P.G.Vpad);
    if (mode == MODE_NOOP && e < PV.src_n)  // (the source rows are 16-B aligned: checked by the setter)
        d4 = reinterpret_cast<float4*>(const_cast<float*>(PV.src) + PV.src_rows[e] * PV.src_stride);
    const int nvec = P.G.Vpad >> 2;
    const int V = P.G.V;
    const bool al4 = (V & 3) == 0;
    float* o0 = PV.obs + (size_t)e * 4 * V;
    float* o1 = o0 + V;
    float* o2 = o1 + V;
    float* o3 = o2 + V;
    const int q0 = sl * P.vec_per_slice;
    const int q1 = min(q0 + P.vec_per_slice, nvec);
    const uint32_t* lbits = P.lung_bits;
    for (int q = q0 + tid; q < q1; q += kStepThreads) {
        const int v0 = q << 2;
        float4 v;
        if (mode == MODE_RESET) {
            v = make_float4(0.f, 0.f, 0.f, 0.f);
            d4[q] = v;
        } else {
            v = d4[q];
        }
        const uint32_t lb = (lbits[q >> 3] >> ((q & 7) << 2)) & 0xFu;
        if (v0 < V) {
            store4(o0, v0, V, al4, (float)(lb & 1u), (float)((lb >> 1) & 1u), (float)((lb >> 2) & 1u),
                   (float)((lb >> 3) & 1u));
            store4(o1, v0, V, al4, 0.f, 0.f, 0.f, 0.f);
            store4(o2, v0, V, al4, v.x, v.y, v.z, v.w);
            store4(o3, v0, V, al4, 0.f, 0.f, 0.f, 0.f);
        }
    }
}

// LDS hash (flat voxel -> summed weight) for the beam-view channel.
__device__ __forceinline__ uint32_t hslot(int32_t key, uint32_t mask) {
    return ((uint32_t)key * 2654435761u >> 7) & mask;
}

__device__ __forceinline__ void hash_add(int32_t* keys, float* vals, uint32_t mask, int32_t key, float w) {
    uint32_t h = hslot(key, mask);
    while (true) {
        const int32_t old = atomicCAS(&keys[h], -1, key);
        if (old == -1 || old == key) {
            atomicAdd(&vals[h], w);
            return;
        }
        h = (h + 1) & mask;
    }
}

struct FinishParams {
    Geom G;
    Consts C;
    EnvState st;
    Library lib;
    float* obs;          // [N][9]
    float* reward;       // [N]
    uint8_t* terminated; // [N]
    float* info;         // [N][RT_INFO_W] or null
    const int32_t* part_cnt;  // [N][n_chunk] (k_dense)
    const float* part_sum;    // [N][n_chunk]
    int32_t n_chunk;          // numpy buffers holding lung voxels
    int32_t max_tvox;    // per-wave LDS holds the sum plan of tumours up to max_tvox voxels
    float* gscratch;     // larger tumours (k_rollout_policy's smaller LDS share): plan slots
    int64_t gscratch_stride;  //   here, gscratch + e * stride, operands read from the library
    int32_t N;           // envs [e_begin, N) take part
    int32_t e_begin;
    int32_t vision;      // obs is f32 [N][4][V]
    int32_t incremental; // lung count / sum from the k_beam-maintained counters
    uint32_t hash_mask;  // vision: beam-view hash slots - 1
    int32_t wave_lds;    // bytes of LDS per wave
    int32_t wpb;         // envs (waves) per block: 4, or fewer when big tumours need the LDS
};

// np.sum(dose * lungs) from the env's chunk partials (lane u of pv[k] holds
// chunk 64 k + u): numpy's outer loop, sequential in chunk order from 0.0f
// (buffers without lung voxels add +0, an exact no-op).
constexpr int kPartPF = 4;  // chunk partials per lane loaded ahead of the tumour gather (<= 256 chunks)
__device__ __forceinline__ float chunk_fold(const float (&pv)[kPartPF], const FinishParams& P, int e, int lane) {
    float acc = 0.0f;
    const int n = P.n_chunk;
#pragma unroll
    for (int k = 0; k < kPartPF; ++k)
        for (int u = 0; u < 64 && 64 * k + u < n; ++u)
            acc = acc + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pv[k]), u));
    for (int j0 = 64 * kPartPF; j0 < n; j0 += 64) {  // > 256 chunks (grids above ~2.1 M voxels)
        const float x = j0 + lane < n ? P.part_sum[(size_t)e * n + j0 + lane] : 0.0f;
        for (int u = 0; u < 64 && j0 + u < n; ++u)
            acc = acc + __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), u));
    }
    return acc;
}

__device__ __forceinline__ void write_obs9(float* obs, const Geom& G, int e, const double* pose,
                                           const TumourMeta& m) {
    float* o = obs + (size_t)e * 9;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        o[i] = (float)(pose[i] / G.S[i] * 2.0 - 1.0);
        o[3 + i] = (float)pose[3 + i];
        o[6 + i] = m.obs_c[i];
    }
}


// Splats of one beam into the wave's LDS hash (lane k: iterations k, k+64, ...).
__device__ void hash_beam(const Geom& G, const BeamSetup& b, int lane, int32_t* keys, float* vals,
                          uint32_t mask) {
    for (int k = lane; k < b.niter; k += 64) {
        float y = b.intery0, z = b.interz0;
        for (int j = 0; j < k; ++j) {  // the reference's sequential f32 accumulation
            y = y + b.sgy;
            z = z + b.sgz;
        }
        int32_t idx[4];
        float w[4];
        march_splats(G.g, b, k, y, z, idx, w);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (idx[i] >= 0) hash_add(keys, vals, mask, idx[i], w[i]);
    }
}

__device__ BeamSetup wave_beam_setup(const Geom& G, const double pos[3], const double dir[3], int lane) {
    BeamSetup s{};
    if (lane == 0) beam_setup(G.g, pos, dir, s);
    BeamSetup b;
    b.niter = rfl_i(s.niter);
    b.start = rfl_i(s.start);
    b.stepdir = rfl_i(s.stepdir);
    b.dom = rfl_i(s.dom);
    b.o0 = rfl_i(s.o0);
    b.o1 = rfl_i(s.o1);
    b.intery0 = rfl_f(s.intery0);
    b.interz0 = rfl_f(s.interz0);
    b.sgy = rfl_f(s.sgy);
    b.sgz = rfl_f(s.sgz);
    return b;
}

// Vision observation, sparse channels (environment.py:245-257): channel 1 =
// clip(tumours) = 1 on the tumour voxels; channel 3 = clip(beam(pos, dir) +
// beam(pos, [1,0,0])), built as the reference adds the two dense beams: the
// first beam's splats are summed (pairs), THEN the horizontal beam is added.
__device__ void vision_scatter(const FinishParams& P, int e, int lane, const double* pose, const TumourMeta& m,
                               unsigned char* wave_lds) {
    const int V = P.G.V;
    float* row = P.obs + (size_t)e * 4 * V;
    const int32_t* tv = P.lib.vox + m.vox_base;
    for (int i = lane; i < m.n; i += 64) row[V + tv[i]] = 1.0f;
    const uint32_t slots = P.hash_mask + 1;
    int32_t* keys = reinterpret_cast<int32_t*>(wave_lds + (size_t)P.max_tvox * 2 * sizeof(float));
    float* vals = reinterpret_cast<float*>(keys + slots);
    for (uint32_t i = lane; i < slots; i += 64) {
        keys[i] = -1;
        vals[i] = 0.0f;
    }
    const double pos[3] = {pose[0], pose[1], pose[2]};
    const double dir[3] = {pose[3], pose[4], pose[5]};
    const double hdir[3] = {1.0, 0.0, 0.0};
    const BeamSetup b1 = wave_beam_setup(P.G, pos, dir, lane);
    const BeamSetup b2 = wave_beam_setup(P.G, pos, hdir, lane);
    lds_wave_sync();
    hash_beam(P.G, b1, lane, keys, vals, P.hash_mask);
    lds_wave_sync();
    hash_beam(P.G, b2, lane, keys, vals, P.hash_mask);
    lds_wave_sync();
    float* view = row + 3 * (size_t)V;
    for (uint32_t i = lane; i < slots; i += 64) {
        const int32_t k = keys[i];
        if (k >= 0) view[k] = clip01(vals[i]);
    }
}

// ---------------------------------------------------------------------------
// k_finish: one wave per env (4 per block).
//  - tumour voxels: gather the updated dose, lung-voxel threshold correction
//    (lungs * (1 - tumours)), distance argmin (environment.py:150-162, f64,
//    np.argmin first-index tie rule)
//  - np.sum(dose * tumours) in numpy's exact order via the tumour's level plan
//  - combine k_dense slices; rewards (environment.py:164-191), termination,
//    obs (environment.py:259-268), info, episode statistics
// ---------------------------------------------------------------------------
// PF (k_finish): the step's independent scalars (the env's dense partial
// sums, t, episode return / length) are loaded before the tumour gather; the
// nearest tumour voxel's packed coordinates travel with the distance argmin,
// so the tail issues no dependent load (each one a few us beside the dose
// stream).
constexpr int kGatherU = 4;  // tumour voxels per lane in flight in the gather
template <bool PF = false>
__device__ void finish_env(const FinishParams& P, int e, int lane, unsigned char* wave_lds) {
    float* tvals = reinterpret_cast<float*>(wave_lds);
    if (lane == 0) RT_STAMP(e, 5);
    const BeamSetup s = P.st.setup[e];
    const TumourMeta m = P.lib.meta[s.tumour];
    const double* pose = P.st.pose + (size_t)e * 6;
    if (s.mode != MODE_STEP) {
        if (lane == 0) {
            if (!P.vision) write_obs9(P.obs, P.G, e, pose, m);
            if (P.reward) P.reward[e] = 0.0f;
            if (P.terminated) P.terminated[e] = 0;
            if (P.info) {
                float* inf = P.info + (size_t)e * RT_INFO_W;
                for (int i = 0; i < RT_INFO_W; ++i) inf[i] = 0.0f;
            }
        }
        if (P.vision) vision_scatter(P, e, lane, pose, m, wave_lds);
        return;
    }
    const float* dose = P.st.dose + (size_t)e * P.G.Vpad;
    const int nt = m.n;
    const int32_t* tp = P.lib.vpos + m.vox_base;
    const uint32_t* tc = P.lib.coord + m.vox_base;
    const double px = pose[0], py = pose[1], pz = pose[2];
    // plan slots (leaves 0..n-1, op o -> n+o): the wave's LDS, or for a
    // tumour above the LDS capacity a global scratch row (L2)
    const bool in_lds = nt <= P.max_tvox;
    float* tg = in_lds ? nullptr : P.gscratch + (size_t)e * P.gscratch_stride;
    // the sum plan's operands and level ends -> LDS by async copies (no VGPRs),
    // in flight during the gather; the plan below then touches only LDS
    uint32_t* ops_s = reinterpret_cast<uint32_t*>(tvals + 2 * P.max_tvox);
    int32_t* lev_s = reinterpret_cast<int32_t*>(ops_s + P.max_tvox);
    if (in_lds) {
        const uint32_t* ops = P.lib.ops + m.op_base;
        const int32_t* lend = P.lib.lvl_end + m.lvl_base;
        const int nops = nt - 1;  // a binary sum tree over nt leaves (checked at create)
        for (int o = 0; o < nops; o += 64)
            if (lane < nops - o)
                __builtin_amdgcn_global_load_lds((glb_ptr_t)(ops + o + lane), (lds_ptr_t)(ops_s + o), 4, 0, 0);
        if (lane < m.nlev)
            __builtin_amdgcn_global_load_lds((glb_ptr_t)(lend + lane), (lds_ptr_t)lev_s, 4, 0, 0);
    }
    // PF: independent loads of the tail, issued before the gather
    int pf_cnt = 0, pf_t = 0, pf_len = 0;
    double pf_ret = 0.0;
    float pv[kPartPF];
#pragma unroll
    for (int k = 0; k < kPartPF; ++k) pv[k] = 0.0f;
    if constexpr (PF) {
        if (!P.incremental) {
#pragma unroll
            for (int k = 0; k < kPartPF; ++k) {
                const int j = 64 * k + lane;
                if (j < P.n_chunk) {
                    pf_cnt += P.part_cnt[(size_t)e * P.n_chunk + j];
                    pv[k] = P.part_sum[(size_t)e * P.n_chunk + j];
                }
            }
            for (int j = 64 * kPartPF + lane; j < P.n_chunk; j += 64) pf_cnt += P.part_cnt[(size_t)e * P.n_chunk + j];
        }
        if (lane == 0) {
            pf_t = P.st.t[e];
            pf_ret = P.st.ep_return[e];
            pf_len = P.st.ep_len[e];
        }
    }
    int ctum = 0;
    double best = INFINITY;
    int bidx = 0x7fffffff;
    uint32_t bc = 0;  // packed coordinates of the nearest voxel
    auto voxel = [&](int i, uint32_t c, float x) {
        if (in_lds) tvals[i] = x;
        else tg[i] = x;
        ctum += ((c >> 31) && x > P.C.lung_thr) ? 1 : 0;
        const int ix = (int)((c >> 20) & 1023u), iy = (int)((c >> 10) & 1023u), iz = (int)(c & 1023u);
        const double d0 = (double)ix - px, d1 = (double)iy - py, d2 = (double)iz - pz;
        const double nn = sqrt((d0 * d0 + d1 * d1) + d2 * d2);  // np.linalg.norm(axis=1) order
        if (nn < best) {  // ascending i per lane: the first minimum
            best = nn;
            bidx = i;
            bc = c;
        }
    };
    // two dependent loads per voxel (its row position and packed coordinates,
    // then its dose): kGatherU voxels per lane in flight (one voxel at a time
    // paid 2 round trips per 64 voxels: ~40 us for the largest tumours beside
    // the dose stream)
    for (int i0 = 0; i0 < nt; i0 += 64 * kGatherU) {
        int pos[kGatherU];
        uint32_t cc[kGatherU];
        float x[kGatherU];
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const int i = i0 + 64 * u + lane;
            pos[u] = i < nt ? tp[i] : 0;
            cc[u] = i < nt ? tc[i] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const int i = i0 + 64 * u + lane;
            x[u] = i < nt ? dose[pos[u]] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < kGatherU; ++u) {
            const int i = i0 + 64 * u + lane;
            if (i < nt) voxel(i, cc[u], x[u]);
        }
    }
    ctum = wave_sum_i(ctum);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double ob = __shfl_xor(best, off, 64);
        const int oi = __shfl_xor(bidx, off, 64);
        const uint32_t oc = (uint32_t)__shfl_xor((int)bc, off, 64);
        if (ob < best || (ob == best && oi < bidx)) {
            best = ob;
            bidx = oi;
            bc = oc;
        }
    }
    if (lane == 0) RT_STAMP(e, 6);
    // exact np.sum(dose * tumours): level plan
    float S;
    if (in_lds) {
        __builtin_amdgcn_s_waitcnt(0);  // the async copies above have landed
        S = run_plan(tvals, ops_s, lev_s, nt, m.nlev, m.result, lane);
    } else {
        S = run_plan(tg, P.lib.ops + m.op_base, P.lib.lvl_end + m.lvl_base, nt, m.nlev, m.result, lane);
    }
    if (lane == 0) RT_STAMP(e, 7);
    int cnt = 0;
    float dl = 0.0f;
    if (P.incremental) {
        // maintained by k_beam: exact count, f64 sum rounded once
        cnt = P.st.lung_cnt[e];
        dl = (float)P.st.lung_sum[e];
    } else {
        if constexpr (PF) {
            cnt = pf_cnt;
        } else {
#pragma unroll
            for (int k = 0; k < kPartPF; ++k)
                if (64 * k + lane < P.n_chunk) pv[k] = P.part_sum[(size_t)e * P.n_chunk + 64 * k + lane];
            for (int j = lane; j < P.n_chunk; j += 64) cnt += P.part_cnt[(size_t)e * P.n_chunk + j];
        }
        cnt = wave_sum_i(cnt);
        dl = chunk_fold(pv, P, e, lane);
    }
    if (lane == 0) {
        const long long c = (long long)cnt - ctum;  // lungs * (1 - tumours)
        const float ratio = S / m.T;
        const float r_tum = ratio * P.C.tum_reward;
        const double r_lung = (double)c / m.lung_total * P.C.lung_reward;
        const int ix = (int)((bc >> 20) & 1023u), iy = (int)((bc >> 10) & 1023u), iz = (int)(bc & 1023u);
        const double dn = ddot_norm3((double)ix - px, (double)iy - py, (double)iz - pz);
        const double r_dist = dn / P.G.normS * P.C.dist_reward;
        const double total = ((double)r_tum + r_lung) + r_dist;
        const int t = PF ? pf_t : P.st.t[e];
        const bool done = (ratio >= P.C.tum_thr) || (t >= P.C.max_t);
        if (!P.vision) write_obs9(P.obs, P.G, e, pose, m);
        P.reward[e] = (float)total;
        P.terminated[e] = done ? 1 : 0;
        const double ret = (PF ? pf_ret : P.st.ep_return[e]) + total;
        const int len = (PF ? pf_len : P.st.ep_len[e]) + 1;
        P.st.ep_return[e] = ret;
        P.st.ep_len[e] = len;
        if (done) P.st.flags[e] |= FLAG_NEEDS_RESET;
        if (P.info) {
            float* inf = P.info + (size_t)e * RT_INFO_W;
            inf[RT_INFO_TOTAL] = (float)total;
            inf[RT_INFO_TUMOUR] = r_tum;
            inf[RT_INFO_LUNG] = (float)r_lung;
            inf[RT_INFO_DISTANCE] = (float)r_dist;
            inf[RT_INFO_DOSE_TUMOUR] = S;
            inf[RT_INFO_DOSE_LUNG] = dl;
            for (int i = 0; i < 3; ++i) {
                inf[RT_INFO_OVERSHOOT_T + i] = s.os_t[i];
                inf[RT_INFO_POS + i] = (float)pose[i];
                inf[RT_INFO_DIR + i] = (float)pose[3 + i];
            }
            inf[RT_INFO_OVERSHOOT_R] = s.os_r;
            inf[RT_INFO_STEPPED] = 1.0f;
            inf[RT_INFO_EP_DONE] = done ? 1.0f : 0.0f;
            inf[RT_INFO_EP_RETURN] = (float)ret;
            inf[RT_INFO_EP_LENGTH] = (float)len;
        }
        RT_STAMP(e, 8);
    }
    if (P.vision) vision_scatter(P, e, lane, pose, m, wave_lds);
}

// k_finish: one wave per env.  The tail's scalars are loaded before the
// tumour gather (finish_env<true>).  Measured and not kept: 4 or 8
// tumour voxels per lane in flight (VGPRs 78 -> 106, the pipelined step
// slower) and wave issue priority for the latency chain (s_setprio 3: the
// co-running dose stream loses issue slots).
__global__ __launch_bounds__(256) void k_finish(FinishParams P) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int e = P.e_begin + blockIdx.x * P.wpb + w;
    if (e >= P.N) return;
    extern __shared__ __attribute__((aligned(16))) unsigned char fsm_raw[];
    finish_env<true>(P, e, lane, fsm_raw + (size_t)w * P.wave_lds);
}

// ---------------------------------------------------------------------------
// k_step_policy: the rollout step of the visionless agent fused with the env
// step (train.py:143-158): one wave per env, `wpb` envs per block.  The block
// stages the policy parameters in LDS, each wave samples its env's action
// (policy_core.h: the same arithmetic as k_policy_sample, so the same bits),
// writes the step's rollout storage, then runs the env's pose update + beam
// march (beam_env) on that action from registers.  FINISH (incremental step
// mode, no dense pass in between): the same wave then finishes the env
// (finish_env), so the whole step is one launch.  The finish reuses the LDS
// of the parameters after a block barrier.
// ---------------------------------------------------------------------------
struct PolicyStepParams {
    rtpol::Weights w;
    const float* obs_in;       // [N][9]  the observation the policy acts on
    const uint8_t* done_in;    // [N]     next_done or null
    float* obs_store;          // [N][9]  storage obs[step]
    float* done_store;         // [N]
    float* act_store;          // [N][6]
    float* logp_store;         // [N]
    float* value_store;        // [N]
    uint64_t seed;
    uint64_t counter;
    int64_t id_base;
    int32_t wpb;
};

template <bool FINISH>
__global__ __launch_bounds__(1024) void k_step_policy(BeamParams B, FinishParams F, PolicyStepParams Q) {
    extern __shared__ __attribute__((aligned(16))) unsigned char psm[];
    rtpol::Lds& L = *reinterpret_cast<rtpol::Lds*>(psm);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int e = B.e_begin + blockIdx.x * Q.wpb + w;
    const bool live = e < B.N;
    if (lane == 0) RT_STAMP(e, 0);
    rtpol::stage(L, Q.w, tid, (int)blockDim.x);
    __syncthreads();
    float act = 0.0f;
    if (live) {
        if (lane == 0) RT_STAMP(e, 9);
        float* h1 = reinterpret_cast<float*>(psm + sizeof(rtpol::Lds)) + w * rtpol::H;
        float x[rtpol::NOBS];
#pragma unroll
        for (int i = 0; i < rtpol::NOBS; ++i) x[i] = Q.obs_in[(size_t)e * rtpol::NOBS + i];
        const rtpol::Sample smp = rtpol::policy_env(L, h1, x, lane, Q.seed, Q.counter, (uint64_t)(Q.id_base + e));
        if (lane < rtpol::NOBS) {
            float xi = x[0];
#pragma unroll
            for (int i = 1; i < rtpol::NOBS; ++i) xi = lane == i ? x[i] : xi;
            Q.obs_store[(size_t)e * rtpol::NOBS + lane] = xi;
        }
        if (lane == rtpol::NOBS) Q.done_store[e] = Q.done_in ? (float)Q.done_in[e] : 0.0f;
        if (lane < rtpol::NACT) Q.act_store[(size_t)e * rtpol::NACT + lane] = smp.action;
        if (lane == 0) {
            Q.logp_store[e] = smp.logp;
            Q.value_store[e] = smp.value;
            RT_STAMP(e, 1);
        }
        act = smp.action;
    }
    if (FINISH) __syncthreads();  // every wave is done with the parameters' LDS
    if (!live) return;
    float a6[rtpol::NACT];
#pragma unroll
    for (int i = 0; i < rtpol::NACT; ++i) a6[i] = rtpol::lane_f(act, i);
    beam_env(B, e, lane, a6);
    if (FINISH) {
        // this wave's dose stores are visible to its own lanes' loads below
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        finish_env(F, e, lane, psm + (size_t)w * F.wave_lds);
    }
}

// ---------------------------------------------------------------------------
// k_rollout_policy: n_steps rollout steps of the visionless agent in ONE
// persistent launch (incremental step mode).  Envs never interact, so a wave
// can run its env's whole step chain -- policy sample, pose update, march,
// finish -- n_steps times back to back without any grid- or block-wide
// synchronisation after the one-time parameter staging: the waves of a CU
// drift into different phases (f64 pose ALU, random-line dose RMW, LDS sum
// plan) and hide each other's latency, and the per-launch costs of the
// stepwise path (launch, parameter staging, the tail of the slowest env) are
// paid once per rollout.  LDS: the parameters (once per block) and one region
// per wave, 16 waves per block so a CU holds 16 envs: the wave's h1 during
// its policy, its finish scratch after it.  A tumour whose sum plan exceeds
// the region keeps its plan slots in a global scratch row.  The step body is
// k_step_policy<true>'s, so the bits are the same.
// ---------------------------------------------------------------------------
struct RolloutParams {
    PolicyStepParams q;  // storage rows of the first step, its Philox counter
    float* reward_store; // [n][N]
    float* info_store;   // [n][N][RT_INFO_W] or null
    int32_t n_steps;
    int32_t fin_off;     // byte offset of the finish scratch in dynamic LDS
};

struct RolloutArgs {
    BeamParams B;
    FinishParams F;
    RolloutParams R;
};

__global__ __launch_bounds__(1024) void k_rollout_policy(RolloutArgs A) {
    extern __shared__ __attribute__((aligned(16))) unsigned char rsm[];
    rtpol::Lds& L = *reinterpret_cast<rtpol::Lds*>(rsm);
    const int tid = threadIdx.x, lane0 = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int e0 = blockIdx.x * A.R.q.wpb + w;
    rtpol::stage(L, A.R.q.w, tid, (int)blockDim.x);
    __syncthreads();
    if (e0 >= A.B.N) return;  // wave-uniform; no block barrier follows
    // the wave's region: h1 during the policy, the finish scratch after it
    unsigned char* const fin_0 = rsm + A.R.fin_off + (size_t)w * A.F.wave_lds;
    float* const h1_0 = reinterpret_cast<float*>(fin_0);
    const int n_steps = A.R.n_steps;
    if (lane0 == 0) RT_STAMP(e0, 13);
    for (int t = 0; t < n_steps; ++t) {
        // Issue priority rotated over the 4 waves each SIMD holds (waves w,
        // w + 4, w + 8, w + 12 of the block share one): with the hardware's
        // oldest-first pick the youngest wave of a SIMD fell 27 % behind the
        // oldest over a rollout, and the launch ended on it with its SIMD
        // mostly idle (tools/trace_env.py --persistent --dump: life 675 /
        // 720 / 783 / 859 us by age rank, 24 steps)
        switch (((w >> 2) + t) & 3) {
            case 0: __builtin_amdgcn_s_setprio(0); break;
            case 1: __builtin_amdgcn_s_setprio(1); break;
            case 2: __builtin_amdgcn_s_setprio(2); break;
            default: __builtin_amdgcn_s_setprio(3); break;
        }
        // Re-derive the loop-invariant inputs (kernel arguments through a
        // laundered kernarg pointer, lane, env, LDS bases) every step: hoisted
        // out of the loop they stay live across the whole step body and push
        // it past 128 VGPRs into scratch.  Scalar loads from the kernarg
        // segment are cheap.
        typedef const __attribute__((address_space(4))) RolloutArgs* KPtr;
        KPtr ap = (KPtr)(__builtin_amdgcn_kernarg_segment_ptr());
        asm volatile("" : "+s"(ap));
        const RolloutArgs& K = *(const RolloutArgs*)ap;
        const BeamParams& B = K.B;
        const FinishParams& F = K.F;
        const RolloutParams& R = K.R;
        const PolicyStepParams& Q = R.q;
        int lane = lane0, e = e0;
        asm volatile("" : "+v"(lane));
        asm volatile("" : "+s"(e));
        float* h1 = h1_0;
        unsigned char* fin = fin_0;
        asm volatile("" : "+s"(h1));
        asm volatile("" : "+s"(fin));
        const size_t N = (size_t)B.N;
        const float* obs_in = t == 0 ? Q.obs_in : F.obs;
        const uint8_t* done_in = t == 0 ? Q.done_in : F.terminated;
        if (lane == 0) {
            RT_STAMP(e, 0);
            RT_STAMP(e, 9);
        }
        float x[rtpol::NOBS];
#pragma unroll
        for (int i = 0; i < rtpol::NOBS; ++i) x[i] = obs_in[(size_t)e * rtpol::NOBS + i];
        const rtpol::Sample smp =
            rtpol::policy_env(L, h1, x, lane, Q.seed, Q.counter + (uint64_t)t, (uint64_t)(Q.id_base + e));
        if (lane == 0) RT_STAMP(e, 1);
        const size_t r9 = (size_t)t * N * rtpol::NOBS + (size_t)e * rtpol::NOBS;
        const size_t r6 = (size_t)t * N * rtpol::NACT + (size_t)e * rtpol::NACT;
        const size_t r1 = (size_t)t * N + (size_t)e;
        if (lane < rtpol::NOBS) {
            float xi = x[0];
#pragma unroll
            for (int i = 1; i < rtpol::NOBS; ++i) xi = lane == i ? x[i] : xi;
            Q.obs_store[r9 + lane] = xi;
        }
        if (lane == rtpol::NOBS) Q.done_store[r1] = done_in ? (float)done_in[e] : 0.0f;
        if (lane < rtpol::NACT) Q.act_store[r6 + lane] = smp.action;
        if (lane == 0) {
            Q.logp_store[r1] = smp.logp;
            Q.value_store[r1] = smp.value;
        }
        float a6[rtpol::NACT];
#pragma unroll
        for (int i = 0; i < rtpol::NACT; ++i) a6[i] = rtpol::lane_f(smp.action, i);
        beam_env(B, e, lane, a6);
        // this wave's dose stores are visible to its own lanes' loads below
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        FinishParams Ft = F;
        Ft.reward = R.reward_store + (size_t)t * N;
        Ft.info = R.info_store ? R.info_store + (size_t)t * N * RT_INFO_W : nullptr;
        finish_env(Ft, e, lane, fin);
        // obs / terminated / dose of this step -> every lane of the next
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
    }
    if (lane0 == 0) RT_STAMP(e0, 14);
}

// ---------------------------------------------------------------------------
// Parity hooks
// ---------------------------------------------------------------------------
// Random-line read-modify-write probe: the access shape of the incremental
// step's march (each lane read-modify-writes dose floats of its own 128-B
// line, lines scattered over a multi-GiB dose array).  Every lane RMWs
// `lines_per_lane` random lines of buf (one float each, 4 in flight); bench.py
// divides lines by time for the random-line ceiling the incremental step's
// transaction model is priced against.
__device__ __forceinline__ uint64_t probe_hash(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

__global__ __launch_bounds__(256) void k_probe_rmw(float* buf, int64_t n_lines, int lines_per_lane, uint64_t seed) {
    const uint64_t lane = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    for (int i = 0; i < lines_per_lane; i += 4) {
        float* p[4];
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint64_t h = probe_hash(seed ^ (lane * 0x9E3779B97F4A7C15ull + (uint64_t)(i + u)));
            p[u] = buf + (h % (uint64_t)n_lines) * 32 + (h >> 59);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = *p[u];
#pragma unroll
        for (int u = 0; u < 4; ++u) *p[u] = v[u] + 1.0f;
    }
}

// HBM stream ceilings (measurement hook, bench.py): a grid-stride sweep of
// non-temporal 16-B loads -- k_dense's access shape -- either reduced to one
// value per block (READ) or stored to a second buffer (COPY), 8 loads in
// flight per lane.
template <bool COPY>
__global__ __launch_bounds__(256) void k_probe_stream(const float4* __restrict__ src, float4* __restrict__ dst,
                                                      int64_t n4, float* __restrict__ sink) {
    typedef float nf4 __attribute__((ext_vector_type(4)));
    constexpr int U = 8;
    const int64_t stride = (int64_t)gridDim.x * 256;
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    float acc = 0.0f;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
        nf4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(src + i + u * stride));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if constexpr (COPY)
                *reinterpret_cast<nf4*>(dst + i + u * stride) = v[u];
            else
                acc += (v[u].x + v[u].y) + (v[u].z + v[u].w);
        }
    }
    for (; i < n4; i += stride) {
        const nf4 v = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(src + i));
        if constexpr (COPY)
            *reinterpret_cast<nf4*>(dst + i) = v;
        else
            acc += (v.x + v.y) + (v.z + v.w);
    }
    if constexpr (!COPY) {
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if ((threadIdx.x & 63) == 0) sink[blockIdx.x * 4 + (threadIdx.x >> 6)] = acc;
    }
}

// beam_voxels (draw_line.py:4-102) as raw splats in march order; -1 for the
// reference's ValueError (direction norm < eps).
__device__ int emit_beam_list(const Geom& G, const double p[3], const double d[3], int cap, int32_t* idx_row,
                              float* w_row) {
    BeamSetup s{};
    if (beam_setup(G.g, p, d, s) < 0) return -1;
    int n = 0;
    float y = s.intery0, z = s.interz0;
    for (int k = 0; k < s.niter; ++k) {
        int32_t ii[4];
        float ww[4];
        march_splats(G.g, s, k, y, z, ii, ww);
        for (int i = 0; i < 4; ++i) {
            if (ii[i] < 0) continue;
            if (n < cap) {
                idx_row[n] = ii[i];
                w_row[n] = ww[i];
            }
            ++n;
        }
        y = y + s.sgy;
        z = z + s.sgz;
    }
    return n;
}

__global__ void k_debug_beam(Geom G, int m, const double* pos, const double* dir, int cap,
                             int32_t* idx_out, float* w_out, int32_t* count) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= m) return;
    double p[3] = {pos[c * 3], pos[c * 3 + 1], pos[c * 3 + 2]};
    double d[3] = {dir[c * 3], dir[c * 3 + 1], dir[c * 3 + 2]};
    count[c] = emit_beam_list(G, p, d, cap, idx_out + (size_t)c * cap, w_out + (size_t)c * cap);
}

// The beam each env applied on its last step (environment.py:107-110 adds
// beam_voxels(pos, dir) of the post-update pose, which is the pose the env
// holds now); an env whose last call was a reset (t = 0) applied none.
__global__ void k_env_beam_list(Geom G, int n_env, const double* pose, const int32_t* t, int cap,
                                int32_t* idx_out, float* w_out, int32_t* count) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n_env) return;
    if (t[e] == 0) {
        count[e] = 0;
        return;
    }
    const double* q = pose + (size_t)e * 6;
    double p[3] = {q[0], q[1], q[2]};
    double d[3] = {q[3], q[4], q[5]};
    count[e] = emit_beam_list(G, p, d, cap, idx_out + (size_t)e * cap, w_out + (size_t)e * cap);
}

__global__ void k_debug_pose(Geom G, Consts C, int m, const double* pos, const double* dir,
                             const float* act, double* out) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= m) return;
    double p[3] = {pos[c * 3], pos[c * 3 + 1], pos[c * 3 + 2]};
    double d[3] = {dir[c * 3], dir[c * 3 + 1], dir[c * 3 + 2]};
    float a[6];
    for (int i = 0; i < 6; ++i) a[i] = act[c * 6 + i];
    PoseOut o;
    pose_update(G, C, p, d, a, o);
    double* r = out + (size_t)c * 10;
    for (int i = 0; i < 3; ++i) {
        r[i] = o.pos[i];
        r[3 + i] = o.dir[i];
        r[6 + i] = o.os_t[i];
    }
    r[9] = o.os_r;
}

__global__ void k_set_next(EnvState st, int N, const int32_t* ids) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < N) st.next_tumour[e] = ids[e];
}

__global__ void k_set_tumours(EnvState st, int N, int K, const int32_t* ids) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < N && ids[e] >= 0 && ids[e] < K) st.tumour[e] = ids[e];
}

__global__ void k_get_state(EnvState st, int N, double* pose, int32_t* t, int32_t* tum) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    if (pose)
        for (int i = 0; i < 6; ++i) pose[(size_t)e * 6 + i] = st.pose[(size_t)e * 6 + i];
    if (t) t[e] = st.t[e];
    if (tum) tum[e] = st.tumour[e];
}

__global__ void k_set_pose(EnvState st, int N, const double* pose) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    for (int i = 0; i < 6; ++i) st.pose[(size_t)e * 6 + i] = pose[(size_t)e * 6 + i];
}

// train.py:163-181, one lane per env; same operation order as the torch loop
// (gamma and gamma*lambda are applied as f32 scalars, as torch does).
__global__ void k_gae(int T, int N, const float* __restrict__ rew, const float* __restrict__ val,
                      const float* __restrict__ dones, const float* __restrict__ next_value,
                      const float* __restrict__ next_done, float gamma, float gl,
                      float* __restrict__ adv, float* __restrict__ ret) {
    int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= N) return;
    float last = 0.0f;
    float nv = next_value[n];
    float nnt = 1.0f - next_done[n];
    // the scan is serial in t, its loads are not: each chunk of kGaeChunk
    // steps loads all its rewards / values / dones before the dependent chain
    // (one memory round trip per chunk instead of per step: 35 -> ~8 us for
    // T = 64, N = 4096)
    constexpr int kGaeChunk = 16;
    for (int hi = T; hi > 0; hi -= kGaeChunk) {
        const int lo = hi - kGaeChunk > 0 ? hi - kGaeChunk : 0;
        float r[kGaeChunk], v[kGaeChunk], d[kGaeChunk];
#pragma unroll
        for (int k = 0; k < kGaeChunk; ++k) {
            const int t = hi - 1 - k;
            const size_t i = (size_t)(t >= lo ? t : lo) * N + n;
            r[k] = rew[i];
            v[k] = val[i];
            d[k] = dones[i];
        }
#pragma unroll
        for (int k = 0; k < kGaeChunk; ++k) {
            const int t = hi - 1 - k;
            if (t >= lo) {  // (no break: the loop stays unrolled, r / v / d in registers)
                const size_t i = (size_t)t * N + n;
                const float delta = (r[k] + (gamma * nv) * nnt) - v[k];
                last = delta + ((gl * nnt) * last);
                adv[i] = last;
                ret[i] = last + v[k];
                nv = v[k];
                nnt = 1.0f - d[k];
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Host: exact-sum plan for one tumour.
// np.sum over the dense f32 volume adds 8192-element buffers, each summed by
// numpy's pairwise routine (8-way unrolled leaves of <=128 elements), into an
// accumulator.  Zeros are exact identities, so restricted to the tumour voxels
// the sum is a fixed binary tree over those voxels; the plan lists its adds in
// dependency levels (slot = leaf index for i < n, n + op index otherwise).
// ---------------------------------------------------------------------------
struct PlanBuilder {
    const int32_t* idx;
    int n;
    int64_t V;
    int p = 0;
    std::vector<int> opa, opb, lvl;

    int level(int s) const { return s < n ? 0 : lvl[s - n]; }
    int add(int x, int y) {
        if (x < 0) return y;
        if (y < 0) return x;
        int s = n + (int)opa.size();
        opa.push_back(x);
        opb.push_back(y);
        lvl.push_back(std::max(level(x), level(y)) + 1);
        return s;
    }
    int pairwise(int64_t start, int64_t len) {
        const int64_t stop = start + len;
        if (p >= n || idx[p] >= stop) return -1;
        if (len < 8) {
            int r = -1;
            while (p < n && idx[p] < stop) r = add(r, p++);
            return r;
        }
        if (len <= 128) {
            const int64_t cut = stop - len % 8;
            int r[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
            while (p < n && idx[p] < cut) {
                int j = (int)((idx[p] - start) & 7);
                r[j] = add(r[j], p++);
            }
            int res = add(add(add(r[0], r[1]), add(r[2], r[3])), add(add(r[4], r[5]), add(r[6], r[7])));
            while (p < n && idx[p] < stop) res = add(res, p++);
            return res;
        }
        int64_t n2 = len / 2;
        n2 -= n2 % 8;
        int a = pairwise(start, n2);
        int b = pairwise(start + n2, len - n2);
        return add(a, b);
    }
    int build() {
        int acc = -1;
        while (p < n) {
            int64_t c = idx[p] / 8192;
            int64_t len = std::min<int64_t>(8192, V - c * 8192);
            acc = add(acc, pairwise(c * 8192, len));
        }
        return acc;
    }
};

// Host side of the lung sum plan (see LChunk): numpy's leaves of one buffer
// [start, start + len) in order, and its tree as PlanBuilder-style ops.
struct LeafTree {
    std::vector<std::pair<int64_t, int64_t>> leaves;
    std::vector<int> opa, opb, lvl;
    int n_leaf = 0;
    int level(int s) const { return s < n_leaf ? 0 : lvl[s - n_leaf]; }
    void split(int64_t start, int64_t len) {
        if (len <= 128) {
            leaves.push_back({start, len});
            return;
        }
        int64_t n2 = len / 2;
        n2 -= n2 % 8;
        split(start, n2);
        split(start + n2, len - n2);
    }
    int tree(int64_t len, int& next_leaf) {  // same recursion, emitting the adds
        if (len <= 128) return next_leaf++;
        int64_t n2 = len / 2;
        n2 -= n2 % 8;
        const int a = tree(n2, next_leaf);
        const int b = tree(len - n2, next_leaf);
        opa.push_back(a);
        opb.push_back(b);
        lvl.push_back(std::max(level(a), level(b)) + 1);
        return n_leaf + (int)opa.size() - 1;
    }
};

struct LungPlanHost {
    int64_t V = 0;
    int32_t n_seg = 0;            // segment slots: the lung voxels and the rows' pad slots
    std::vector<int32_t> pos_of;  // [V] voxel -> segment position (-1: not lung)
    std::vector<int32_t> lpos;    // [n_seg + 256] segment position -> voxel (-1: pad)
    std::vector<LChunk> chunk;
    std::vector<LGroup> grp;
    std::vector<uint64_t> slot;
    std::vector<LGeneric> gen;
    std::vector<uint32_t> ops;
    std::vector<int32_t> lvl_end, tail_off, tail_pos;
};

// Lays out the lung segment by numpy buffer, then by chain (LChunk comment):
// chains of a buffer sorted by length (longest first, ties in slot order),
// 256 per group (4 per lane), ragged rows padded to a multiple of 4 slots.
// lpos: segment position -> voxel, -1 for a pad slot, plus 4 * 64 trailing
// -1 entries (the gather reads a whole wave's float4 of a row's last lanes).
int build_lung_plan(const uint8_t* lungs, int64_t V, LungPlanHost& P) {
    P.V = V;
    P.pos_of.assign((size_t)V, -1);
    P.lpos.clear();
    int32_t seg = 0;
    struct Chain {
        uint16_t slot;
        std::vector<int32_t> vox;
    };
    for (int64_t c0 = 0; c0 < V; c0 += kLungChunk) {
        const int64_t len = std::min<int64_t>(kLungChunk, V - c0);
        bool any = false;
        for (int64_t v = c0; v < c0 + len && !any; ++v) any = lungs[v] != 0;
        if (!any) continue;
        LeafTree lt;
        lt.split(c0, len);
        const int nl = (int)lt.leaves.size();
        if (nl > kLungLeafMax) return fail(RT_ELIMIT, "lung sum plan: more leaves per buffer than expected");
        std::vector<Chain> chains;
        std::vector<std::vector<int32_t>> tails(nl);
        for (int li = 0; li < nl; ++li) {
            const int64_t s = lt.leaves[li].first, n = lt.leaves[li].second;
            const int64_t m = n < 8 ? 0 : n - n % 8;
            for (int j = 0; j < 8; ++j) {
                Chain ch{(uint16_t)(li * 8 + j), {}};
                for (int64_t v = s + j; v < s + m; v += 8)
                    if (lungs[v]) ch.vox.push_back((int32_t)v);
                if (!ch.vox.empty()) chains.push_back(std::move(ch));
            }
            for (int64_t v = s + m; v < s + n; ++v)
                if (lungs[v]) {
                    tails[li].push_back((int32_t)v);
                    chains.push_back(Chain{kNoSlot, {(int32_t)v}});
                }
        }
        std::stable_sort(chains.begin(), chains.end(),
                         [](const Chain& a, const Chain& b) { return a.vox.size() > b.vox.size(); });
        LChunk ch{};
        ch.seg_base = seg;
        ch.grp_base = (int32_t)P.grp.size();
        for (size_t g0 = 0; g0 < chains.size(); g0 += kLungGroup) {
            const size_t g1 = std::min(chains.size(), g0 + kLungGroup);
            LGroup G{};
            const int rows = (int)chains[g0].vox.size();
            if (rows > 16) return fail(RT_ELIMIT, "lung sum plan: chain longer than 16");
            for (int k = 0; k < rows; ++k) {
                int nk = 0;
                for (size_t l = g0; l < g1; ++l) nk += (int)chains[l].vox.size() > k ? 1 : 0;
                // a row: its float4 (ceil(nk / 4) lanes), padded to a whole number of
                // 64-B sectors (rows meeting inside a sector made the non-temporal
                // loads fetch it twice: +15 % HBM bytes; padded to 128-B lines the
                // pads cost 6 %, to 64-B sectors 3.5 %, and the 16-row stream ran
                // 2.6 % faster: profiles/r06/r06_s27_row_pad_64.txt)
                const int nk4 = (nk + 3) / 4 * 4, span = (nk + kLungRowAlign - 1) / kLungRowAlign * kLungRowAlign;
                if (seg - ch.seg_base + span > 0xffff) return fail(RT_ELIMIT, "lung sum plan: chunk too large");
                G.row[k] = (uint32_t)(seg - ch.seg_base) | (uint32_t)(nk4 / 4) << 16;
                for (int l = 0; l < span; ++l) {
                    const int32_t v = l < nk ? chains[g0 + l].vox[k] : -1;
                    if (v >= 0) P.pos_of[v] = seg + l;
                    P.lpos.push_back(v);
                }
                seg += span;
            }
            P.grp.push_back(G);
            for (size_t l = g0; l < g0 + kLungGroup; l += 4) {
                uint64_t w = 0;
                for (int i = 0; i < 4; ++i)
                    w |= (uint64_t)(l + i < g1 ? chains[l + i].slot : kNoSlot) << (16 * i);
                P.slot.push_back(w);
            }
        }
        ch.n_grp = (int32_t)P.grp.size() - ch.grp_base;
        ch.gen = -1;
        if (len != kLungChunk) {
            LGeneric q{};
            q.n_leaf = nl;
            lt.n_leaf = nl;
            int next = 0;
            const int res = lt.tree(len, next);
            const int nops = (int)lt.opa.size();
            std::vector<int> ord(nops), remap(nops);
            for (int o = 0; o < nops; ++o) ord[o] = o;
            std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return lt.lvl[x] < lt.lvl[y]; });
            for (int o = 0; o < nops; ++o) remap[ord[o]] = o;
            auto slot = [&](int s) { return s < nl ? s : nl + remap[s - nl]; };
            q.op_base = (int32_t)P.ops.size();
            q.lvl_base = (int32_t)P.lvl_end.size();
            for (int o = 0; o < nops; ++o) {
                const int src = ord[o];
                P.ops.push_back((uint32_t)slot(lt.opa[src]) | ((uint32_t)slot(lt.opb[src]) << 16));
                if (o + 1 == nops || lt.lvl[ord[o + 1]] != lt.lvl[src]) {
                    P.lvl_end.push_back(o + 1);
                    ++q.nlev;
                }
            }
            q.result = slot(res);
            q.tail_base = (int32_t)P.tail_off.size();
            for (int li = 0; li < nl; ++li) {
                P.tail_off.push_back((int32_t)P.tail_pos.size());
                for (int32_t v : tails[li]) P.tail_pos.push_back(P.pos_of[v]);
            }
            P.tail_off.push_back((int32_t)P.tail_pos.size());
            ch.gen = (int32_t)P.gen.size();
            P.gen.push_back(q);
        }
        P.chunk.push_back(ch);
    }
    P.n_seg = seg;
    P.lpos.insert(P.lpos.end(), 4 * 64, -1);
    return RT_OK;
}

// The plan evaluated on the host exactly as k_dense + k_finish evaluate it
// (chains, LDS slots, leaf formula, butterfly or level plan, chunk fold):
// np.sum(dose * lungs) of a C-order f32 volume (parity hook).
float eval_lung_plan(const LungPlanHost& P, const float* dose) {
    float acc = 0.0f;
    for (size_t j = 0; j < P.chunk.size(); ++j) {
        const LChunk& c = P.chunk[j];
        float slots[kLungSlotFloats] = {};
        for (int g = c.grp_base; g < c.grp_base + c.n_grp; ++g) {
            const LGroup& G = P.grp[g];
            float chain[kLungGroup] = {};
            for (int k = 0; k < 16; ++k) {
                const int pos = c.seg_base + (int)(G.row[k] & 0xffffu), n4 = 4 * (int)(G.row[k] >> 16);
                for (int l = 0; l < n4; ++l) {
                    const int32_t v = P.lpos[pos + l];
                    chain[l] = chain[l] + (v >= 0 ? dose[v] : 0.0f);
                }
            }
            for (int l = 0; l < kLungGroup; ++l) {
                const uint32_t sl = (uint32_t)(P.slot[(size_t)g * 64 + l / 4] >> (16 * (l % 4))) & 0xffffu;
                if (sl != kNoSlot) slots[sl] = chain[l];
            }
        }
        auto leaf = [&](int L) {
            const float* r = slots + 8 * L;
            return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        };
        float v;
        if (c.gen < 0) {
            float lv[64];
            for (int L = 0; L < 64; ++L) lv[L] = leaf(L);
            for (int off = 1; off < 64; off <<= 1) {
                float nx[64];
                for (int L = 0; L < 64; ++L) nx[L] = lv[L] + lv[L ^ off];
                std::copy(nx, nx + 64, lv);
            }
            v = lv[0];
        } else {
            const LGeneric& q = P.gen[c.gen];
            std::vector<float> tv((size_t)2 * q.n_leaf);
            for (int L = 0; L < q.n_leaf; ++L) {
                float t = leaf(L);
                for (int i = P.tail_off[q.tail_base + L]; i < P.tail_off[q.tail_base + L + 1]; ++i)
                    t = t + dose[P.lpos[P.tail_pos[i]]];
                tv[L] = t;
            }
            int lo = 0;
            for (int l = 0; l < q.nlev; ++l) {
                const int hi = P.lvl_end[q.lvl_base + l];
                for (int o = lo; o < hi; ++o) {
                    const uint32_t ab = P.ops[q.op_base + o];
                    tv[q.n_leaf + o] = tv[ab & 0xffffu] + tv[ab >> 16];
                }
                lo = hi;
            }
            v = tv[q.result];
        }
        acc = acc + v;
    }
    return acc;
}

}  // namespace

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
struct rt_env {
    int device = 0;
    int N = 0;
    Geom G{};
    Consts C{};
    uint64_t seed = 0;
    int64_t env_id_base = 0;
    int visionless = 1;
    int incremental = 0;
    EnvState st{};
    Library lib{};
    int max_tvox = 0;
    int slices = 0;          // k_dense slices per env
    int vec_per_slice = 0;   // float4 per slice
    int lung_first = 0;      // dose rows lung-first (dense visionless), else C order
    int lung_n = 0;          // lung voxels (the lung-first segment)
    int n_chunk = 0;         // numpy buffers holding lung voxels (k_dense items per env)
    int dense_bpc = 0;       // k_dense blocks resident per CU (occupancy query, first launch)
    LungParams lplan{};      // the lung sum plan (device copies)
    int32_t* dose_pos_d = nullptr;  // voxel -> row position (lung_first)
    size_t finish_smem = 0;  // k_finish dynamic LDS (4 waves)
    int finish_wave_lds = 0; // bytes per wave
    int finish_wpb = 4;      // k_finish envs per block
    int fused_wpb = 16;      // k_step_policy envs (waves) per block
    int pipe_wpb = 8;        // ... in the pipelined dense rollout
    int pipe_dense_bpc = RT_PIPE_DENSE_BPC;  // its k_dense: persistent, blocks per CU
    int num_cu = 256;        // compute units of the device
    size_t pipe_smem = 0;
    size_t fused_smem = 0;   // k_step_policy dynamic LDS
    int rollout_wpb = 0;     // k_rollout_policy envs per block (0: does not fit LDS)
    size_t rollout_smem = 0; // k_rollout_policy dynamic LDS
    int rollout_fin_off = 0; // offset of its per-wave regions
    int rollout_wave_lds = 0;// bytes per wave region
    int rollout_cap = 0;     // largest tumour whose sum plan fits a region
    float* gscratch = nullptr;  // [N][2 * max_tvox] plan slots of tumours above a kernel's LDS capacity
    uint32_t view_hash_mask = 0;
    int32_t* part_cnt = nullptr;
    float* part_sum = nullptr;
    // optional live kernel timing: 4 events per step (before k_beam, k_dense,
    // k_finish, after k_finish) in a ring of `timing_cap` steps
    std::vector<hipEvent_t> tev;
    int timing_cap = 0;
    int timing_n = 0;
    // pipelined dense rollout (rt_env_rollout_policy in dense step mode): env
    // groups on two library streams; events fork, hand the k_dense turn from
    // one group to the other, join
    int rollout_groups = 2;  // DESIGN.md §3 "Pipelined dense rollout"
    // rt_env_set_render_source: read by the next reset's k_dense_vis, then cleared
    const float* render_src = nullptr;
    const int64_t* render_rows = nullptr;
    int64_t render_stride = 0;
    int32_t render_n = 0;
    hipStream_t pipe[kMaxRolloutGroups] = {};
    hipEvent_t pev[1 + 2 * kMaxRolloutGroups] = {};  // fork, dense[G], join[G]
    std::vector<void*> allocs;
};

namespace {

template <typename T>
int dev_alloc(rt_env* env, T** p, size_t count) {
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, std::max<size_t>(count, 1) * sizeof(T));
    if (e != hipSuccess) return fail(RT_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    env->allocs.push_back(q);
    *p = static_cast<T*>(q);
    return RT_OK;
}

template <typename T>
int dev_upload(rt_env* env, const T** p, const std::vector<T>& h) {
    T* d = nullptr;
    if (int rc = dev_alloc(env, &d, h.size())) return rc;
    if (!h.empty() && hipMemcpy(d, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
        return fail(RT_EDEVICE, "lung sum plan upload failed");
    *p = d;
    return RT_OK;
}

int upload_lung_plan(rt_env* env, const LungPlanHost& lp) {
    LungParams& L = env->lplan;
    int rc;
    if ((rc = dev_upload(env, &L.chunk, lp.chunk)) || (rc = dev_upload(env, &L.grp, lp.grp)) ||
        (rc = dev_upload(env, &L.slot, lp.slot)) || (rc = dev_upload(env, &L.gen, lp.gen)) ||
        (rc = dev_upload(env, &L.ops, lp.ops)) || (rc = dev_upload(env, &L.lvl_end, lp.lvl_end)) ||
        (rc = dev_upload(env, &L.tail_off, lp.tail_off)) || (rc = dev_upload(env, &L.tail_pos, lp.tail_pos)))
        return rc;
    L.lpos = nullptr;
    if (!env->lung_first && (rc = dev_upload(env, &L.lpos, lp.lpos))) return rc;
    L.n_chunk = (int32_t)lp.chunk.size();
    return RT_OK;
}

uint32_t next_pow2(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

void free_env(rt_env* env) {
    if (!env) return;
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(env->device);
    for (hipEvent_t e : env->tev) (void)hipEventDestroy(e);
    for (hipEvent_t e : env->pev)
        if (e) (void)hipEventDestroy(e);
    for (hipStream_t q : env->pipe)
        if (q) (void)hipStreamDestroy(q);
    for (void* p : env->allocs) (void)hipFree(p);
    (void)hipSetDevice(cur);
    delete env;
}

int fill_geom(const int32_t grid[3], Geom& G) {
    for (int i = 0; i < 3; ++i)
        if (grid[i] < 1 || grid[i] > kMaxGridDim) return fail(RT_ELIMIT, "grid dimension out of range [1,1024]");
    int64_t V = (int64_t)grid[0] * grid[1] * grid[2];
    if (V > (int64_t)1 << 30) return fail(RT_ELIMIT, "grid too large");
    for (int i = 0; i < 3; ++i) {
        G.g[i] = grid[i];
        G.S[i] = (double)grid[i];
    }
    G.V = (int32_t)V;
    G.Vpad = (int32_t)((V + 1023) / 1024 * 1024);
    G.normS = std::sqrt(std::fma(G.S[2], G.S[2], std::fma(G.S[1], G.S[1], G.S[0] * G.S[0])));
    return RT_OK;
}

Consts make_consts(const rt_env_config& c) {
    Consts C{};
    C.max_t = c.max_time_steps;
    C.beam_dose = c.beam_dose;
    C.lung_thr = c.lung_dose_threshold;
    C.tum_thr = c.tumour_dose_threshold;
    C.min_angle = c.min_angle_z;
    C.cos_min_angle = std::cos(c.min_angle_z);
    C.move_speed = c.movement_speed;
    C.rot_speed = c.rotation_speed;
    C.tum_reward = c.tumour_dose_reward;
    C.lung_reward = c.lung_dose_reward;
    C.dist_reward = c.distance_reward;
    C.pi_f = (float)M_PI;
    return C;
}

}  // namespace

RT_TRACE_READ_FN(rt_trace_read_env)

extern "C" {

int rt_abi_version(void) { return RTENV_ABI_VERSION; }

// shared error reporting for the other translation units of the library
int rt_internal_fail(int code, const char* msg) { return fail(code, msg); }

int rt_host_tumour_sum(int64_t V, int32_t n, const int32_t* idx_h, const float* vals_h, float* out_h) {
    if (V < 1 || n < 0 || !out_h || (n && (!idx_h || !vals_h))) return fail(RT_EINVAL, "bad argument");
    for (int32_t i = 0; i < n; ++i)
        if (idx_h[i] < 0 || idx_h[i] >= V || (i && idx_h[i] <= idx_h[i - 1]))
            return fail(RT_EINVAL, "indices must be sorted, unique and < V");
    PlanBuilder pb{idx_h, n, V};
    int res = pb.build();
    // evaluate in level order exactly as k_finish does
    int nops = (int)pb.opa.size();
    std::vector<int> order(nops);
    for (int i = 0; i < nops; ++i) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return pb.lvl[x] < pb.lvl[y]; });
    std::vector<float> slot((size_t)n + nops);
    for (int i = 0; i < n; ++i) slot[i] = vals_h[i];
    for (int o = 0; o < nops; ++o) {
        int src = order[o];
        slot[(size_t)n + src] = slot[pb.opa[src]] + slot[pb.opb[src]];
    }
    *out_h = res < 0 ? 0.0f : slot[res];
    return RT_OK;
}

int rt_host_lung_sum(const int32_t grid[3], const uint8_t* lungs_h, const float* dose_h, float* out_h) {
    if (!grid || !lungs_h || !dose_h || !out_h) return fail(RT_EINVAL, "NULL argument");
    Geom G{};
    if (int rc = fill_geom(grid, G)) return rc;
    LungPlanHost lp;
    if (int rc = build_lung_plan(lungs_h, G.V, lp)) return rc;
    *out_h = eval_lung_plan(lp, dose_h);
    return RT_OK;
}

int rt_host_sincos(int32_t n, const double* x_h, double* sin_h, double* cos_h) {
    if (n < 0 || (n && (!x_h || !sin_h || !cos_h))) return fail(RT_EINVAL, "bad argument");
    for (int32_t i = 0; i < n; ++i) {
        if (x_h[i] <= 1.6) {
            rtdd::sincos_cr(x_h[i], &sin_h[i], &cos_h[i]);
        } else {
            sin_h[i] = std::sin(x_h[i]);
            cos_h[i] = std::cos(x_h[i]);
        }
    }
    return RT_OK;
}

const char* rt_last_error(void) { return g_last_error.c_str(); }

static int check_config_size(const rt_env_config* cfg) {
    if (cfg->struct_size != sizeof(rt_env_config))
        return fail(RT_EINVAL, "rt_env_config.struct_size is " + std::to_string(cfg->struct_size) + ", expected " +
                                   std::to_string(sizeof(rt_env_config)) +
                                   " (set it to sizeof(rt_env_config); the binding's declaration may be stale)");
    return RT_OK;
}

int rt_env_config_default(rt_env_config* cfg) {
    if (!cfg) return fail(RT_EINVAL, "cfg is NULL");
    if (int rc = check_config_size(cfg)) return rc;
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->struct_size = sizeof(rt_env_config);
    cfg->grid[0] = 67;
    cfg->grid[1] = 43;
    cfg->grid[2] = 70;
    cfg->num_envs = 1;
    cfg->visionless = 1;
    cfg->max_time_steps = 100;
    cfg->beam_dose = 0.1f;
    cfg->lung_dose_threshold = 0.2f;
    cfg->tumour_dose_threshold = 0.9f;
    cfg->min_angle_z = M_PI / 4.0;
    cfg->movement_speed = 0.2;
    cfg->rotation_speed = 0.5f;
    cfg->lung_dose_reward = -1.0;
    cfg->tumour_dose_reward = 10.0f;
    cfg->distance_reward = -1.0;
    return RT_OK;
}

int rt_env_create(const rt_env_config* cfg, int device, rt_env** out) {
    if (!cfg || !out) return fail(RT_EINVAL, "NULL argument");
    *out = nullptr;
    if (int rc = check_config_size(cfg)) return rc;
    if (cfg->num_envs < 1) return fail(RT_EINVAL, "num_envs must be >= 1");
    if (!cfg->lungs_h || !cfg->tumour_voxels_h || !cfg->tumour_offsets_h || cfg->n_tumours < 1)
        return fail(RT_EINVAL, "lungs / tumour library missing");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RT_EDEVICE, "no HIP device");
    if (device < 0 || device >= ndev) return fail(RT_EDEVICE, "bad device id");
    RT_HIP(hipSetDevice(device));

    rt_env* env = new rt_env();
    env->device = device;
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
            env->num_cu = prop.multiProcessorCount;
    }
    env->N = cfg->num_envs;
    env->seed = cfg->seed;
    env->env_id_base = cfg->env_id_base;
    env->visionless = cfg->visionless;
    if (cfg->step_mode != RT_STEP_DENSE && cfg->step_mode != RT_STEP_INCREMENTAL) {
        delete env;
        return fail(RT_EINVAL, "unknown step_mode");
    }
    env->incremental = (cfg->step_mode == RT_STEP_INCREMENTAL && cfg->visionless) ? 1 : 0;
    int rc = fill_geom(cfg->grid, env->G);
    if (rc) { free_env(env); return rc; }
    env->C = make_consts(*cfg);
    const Geom& G = env->G;
    const int K = cfg->n_tumours;

    // ---- library (host build) ----
    std::vector<uint32_t> lbits(G.Vpad / 32, 0u);
    int64_t lung_count = 0;
    for (int64_t v = 0; v < G.V; ++v) {
        if (cfg->lungs_h[v]) {
            lbits[v >> 5] |= 1u << (v & 31);
            ++lung_count;
        }
    }
    // dense handles: the lung sum plan (k_dense); dense visionless handles keep
    // their rows lung-first in the plan's segment order (k_dense streams the
    // lung segment), vision handles C order (k_dense<true> gathers)
    env->lung_first = env->visionless && !env->incremental;
    env->lung_n = (int)lung_count;
    LungPlanHost lp;
    if (!env->incremental)
        if (int rc_plan = build_lung_plan(cfg->lungs_h, G.V, lp)) {
            free_env(env);
            return rc_plan;
        }
    std::vector<int32_t> dpos;
    if (env->lung_first) {
        // rows: the lung segment (chains + pad slots), then the other voxels
        const int64_t need = (int64_t)lp.n_seg + (G.V - lung_count);
        env->G.Vpad = std::max<int32_t>(G.Vpad, (int32_t)((need + 1023) / 1024 * 1024));
        dpos.resize(G.V);
        int64_t b = lp.n_seg;
        for (int64_t v = 0; v < G.V; ++v) dpos[v] = lp.pos_of[v] >= 0 ? lp.pos_of[v] : (int32_t)b++;
    }
    env->n_chunk = (int)lp.chunk.size();
    std::vector<TumourMeta> meta(K);
    std::vector<int32_t> vox, vpos;
    std::vector<uint32_t> coord;
    std::vector<uint32_t> ops;
    std::vector<int32_t> lvl_end;
    int max_n = 0;
    for (int k = 0; k < K; ++k) {
        int64_t a = cfg->tumour_offsets_h[k], b = cfg->tumour_offsets_h[k + 1];
        int n = (int)(b - a);
        if (n < 1) { free_env(env); return fail(RT_EINVAL, "empty tumour in library"); }
        if (n > kMaxTumourVoxels) { free_env(env); return fail(RT_ELIMIT, "tumour larger than 16384 voxels"); }
        const int32_t* iv = cfg->tumour_voxels_h + a;
        int64_t in_lung = 0;
        double csum[3] = {0, 0, 0};
        for (int i = 0; i < n; ++i) {
            if (iv[i] < 0 || iv[i] >= G.V || (i && iv[i] <= iv[i - 1])) {
                free_env(env);
                return fail(RT_EINVAL, "tumour voxels must be sorted, unique and inside the grid");
            }
            if (cfg->lungs_h[iv[i]]) ++in_lung;
            int64_t v = iv[i];
            csum[0] += (double)(v / ((int64_t)G.g[1] * G.g[2]));
            csum[1] += (double)((v / G.g[2]) % G.g[1]);
            csum[2] += (double)(v % G.g[2]);
        }
        max_n = std::max(max_n, n);
        TumourMeta& m = meta[k];
        m.vox_base = (int32_t)vox.size();
        m.n = n;
        m.T = (float)n;
        m.lung_total = (double)(lung_count - in_lung);
        for (int i = 0; i < 3; ++i) {
            double c = csum[i] / (double)n;  // np.mean of exact integer sums
            m.obs_c[i] = (float)(c / G.S[i] * 2.0 - 1.0);
        }
        vox.insert(vox.end(), iv, iv + n);
        for (int i = 0; i < n; ++i) vpos.push_back(env->lung_first ? dpos[iv[i]] : iv[i]);
        for (int i = 0; i < n; ++i) {
            const int64_t v = iv[i];
            coord.push_back((cfg->lungs_h[v] ? 1u << 31 : 0u) | (uint32_t)(v / ((int64_t)G.g[1] * G.g[2])) << 20 |
                            (uint32_t)((v / G.g[2]) % G.g[1]) << 10 | (uint32_t)(v % G.g[2]));
        }
        PlanBuilder pb{iv, n, (int64_t)G.V};
        int res = pb.build();
        // order ops by level; op at sorted position o writes slot n + o
        int nops = (int)pb.opa.size();
        std::vector<int> order(nops);
        for (int i = 0; i < nops; ++i) order[i] = i;
        std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return pb.lvl[x] < pb.lvl[y]; });
        std::vector<int> remap(nops);
        for (int o = 0; o < nops; ++o) remap[order[o]] = o;
        auto slot = [&](int s) { return s < n ? s : n + remap[s - n]; };
        m.op_base = (int32_t)ops.size();
        m.lvl_base = (int32_t)lvl_end.size();
        int nlev = 0;
        for (int o = 0; o < nops; ++o) {
            int src = order[o];
            ops.push_back((uint32_t)slot(pb.opa[src]) | ((uint32_t)slot(pb.opb[src]) << 16));
            int L = pb.lvl[src];
            if (o + 1 == nops || pb.lvl[order[o + 1]] != L) {
                lvl_end.push_back(o + 1);
                ++nlev;
            }
        }
        if (nops != n - 1 || nlev > kMaxPlanLevels) {
            free_env(env);
            return fail(RT_ELIMIT, "tumour sum plan: unexpected shape");
        }
        m.nlev = nlev;
        m.result = res < 0 ? -1 : slot(res);
    }
    env->lib.K = K;
    env->max_tvox = max_n;
    const int nvec = G.Vpad / 4;
    // k_dense_vis: whole rows in slices
    env->vec_per_slice = std::min(nvec, kSliceVec);
    env->slices = (nvec + env->vec_per_slice - 1) / env->vec_per_slice;
    const int maxdim = std::max(G.g[0], std::max(G.g[1], G.g[2]));
    env->view_hash_mask = env->visionless ? 0u : next_pow2((uint32_t)(8 * (maxdim + 2))) - 1;
    // per wave: plan slots (2 n floats), then either the plan's operands and
    // level ends (STEP) or the vision beam-view hash (used after the plan)
    size_t plan_bytes = (size_t)max_n * sizeof(uint32_t) + kMaxPlanLevels * sizeof(int32_t);
    size_t hash_bytes = env->visionless ? 0 : (size_t)(env->view_hash_mask + 1) * 8;
    size_t wave_bytes = (size_t)2 * max_n * sizeof(float) + std::max(plan_bytes, hash_bytes);
    wave_bytes = (wave_bytes + 15) / 16 * 16;
    env->finish_wave_lds = (int)wave_bytes;
    env->finish_wpb = 4;  // 1 / 2 waves per block measured 4 % slower
    while (env->finish_wpb > 1 && (size_t)env->finish_wpb * wave_bytes > 160 * 1024) env->finish_wpb /= 2;
    env->finish_smem = (size_t)env->finish_wpb * wave_bytes;
    if (env->finish_smem > 160 * 1024) { free_env(env); return fail(RT_ELIMIT, "LDS budget exceeded"); }
    // k_step_policy: parameters + per-wave h1, or (incremental, after the
    // barrier) the per-wave finish scratch in the same bytes
    auto fused_bytes = [&](int wpb) {
        size_t pol = sizeof(rtpol::Lds) + (size_t)wpb * rtpol::H * sizeof(float);
        size_t fin = env->incremental ? (size_t)wpb * wave_bytes : 0;
        return std::max(pol, fin);
    };
    env->fused_wpb = 16;
    while (env->fused_wpb > 1 && fused_bytes(env->fused_wpb) > 160 * 1024) env->fused_wpb /= 2;
    env->fused_smem = fused_bytes(env->fused_wpb);
    // pipelined dense rollout: small policy blocks, so that they find room on
    // CUs beside the other env group's k_dense blocks (a 16-wave block needs a
    // whole CU's registers)
    env->pipe_wpb = std::min(8, env->fused_wpb);
    env->pipe_smem = fused_bytes(env->pipe_wpb);
    // k_rollout_policy: the parameters once per block, then 16 per-wave
    // regions (h1 during the policy, the finish scratch after it); tumours
    // above the region's plan capacity keep their plan slots in gscratch
    {
        const size_t off = (sizeof(rtpol::Lds) + 15) / 16 * 16;
        const int wpb = 16;
        const size_t per_wave = (160 * 1024 - off) / wpb / 16 * 16;
        const int cap = (int)((per_wave - kMaxPlanLevels * sizeof(int32_t)) / (3 * sizeof(float)));
        if (env->visionless && per_wave >= rtpol::H * sizeof(float) && cap >= 1) {
            env->rollout_wpb = wpb;
            env->rollout_fin_off = (int)off;
            env->rollout_wave_lds = (int)per_wave;
            env->rollout_cap = std::min(cap, max_n);
            env->rollout_smem = off + (size_t)wpb * per_wave;
        }
    }

    // ---- device allocations ----
    const int N = env->N;
    uint32_t* d_lbits;
    uint32_t* d_coord;
    int32_t *d_vox, *d_lvl, *d_vpos = nullptr;
    uint32_t* d_ops;
    TumourMeta* d_meta;
    EnvState& st = env->st;
    if ((rc = dev_alloc(env, &d_lbits, lbits.size())) || (rc = dev_alloc(env, &d_vox, vox.size())) ||
        (env->lung_first && ((rc = dev_alloc(env, &d_vpos, vpos.size())) ||
                              (rc = dev_alloc(env, &env->dose_pos_d, dpos.size())))) ||
        (rc = dev_alloc(env, &d_coord, coord.size())) ||
        (rc = dev_alloc(env, &d_ops, ops.size())) || (rc = dev_alloc(env, &d_lvl, lvl_end.size())) ||
        (rc = dev_alloc(env, &d_meta, meta.size())) ||
        (rc = dev_alloc(env, &st.dose, (size_t)N * G.Vpad)) || (rc = dev_alloc(env, &st.pose, (size_t)N * 6)) ||
        (rc = dev_alloc(env, &st.t, N)) || (rc = dev_alloc(env, &st.tumour, N)) ||
        (rc = dev_alloc(env, &st.flags, N)) || (rc = dev_alloc(env, &st.episode, N)) ||
        (rc = dev_alloc(env, &st.ep_return, N)) || (rc = dev_alloc(env, &st.ep_len, N)) ||
        (rc = dev_alloc(env, &st.next_tumour, N)) || (rc = dev_alloc(env, &st.setup, N)) ||
        (rc = dev_alloc(env, &st.mode_b, N)) ||
        (rc = dev_alloc(env, &env->part_cnt, (size_t)N * env->n_chunk)) ||
        (rc = dev_alloc(env, &env->part_sum, (size_t)N * env->n_chunk)) ||
        (!env->incremental && (rc = upload_lung_plan(env, lp))) ||
        (rc = dev_alloc(env, &st.lung_cnt, N)) || (rc = dev_alloc(env, &st.lung_sum, N)) ||
        // the persistent rollout's plan slots for tumours above its LDS share
        (env->incremental && env->rollout_wpb && env->rollout_cap < max_n &&
         (rc = dev_alloc(env, &env->gscratch, (size_t)N * 2 * max_n)))) {
        free_env(env);
        return rc;
    }
    auto h2d = [&](void* d, const void* h, size_t bytes) { return hipMemcpy(d, h, bytes, hipMemcpyHostToDevice); };
    std::vector<int32_t> ones(N, FLAG_NEEDS_RESET), neg(N, -1);
    std::vector<double> pose0((size_t)N * 6, 0.0);
    for (int e = 0; e < N; ++e) {
        for (int i = 0; i < 3; ++i) pose0[(size_t)e * 6 + i] = G.S[i] / 2.0;
        pose0[(size_t)e * 6 + 4] = 1.0;
    }
    if (h2d(d_lbits, lbits.data(), lbits.size() * 4) || h2d(d_vox, vox.data(), vox.size() * 4) ||
        (env->lung_first && (h2d(d_vpos, vpos.data(), vpos.size() * 4) ||
                             h2d(env->dose_pos_d, dpos.data(), dpos.size() * 4))) ||
        h2d(d_coord, coord.data(), coord.size() * 4) ||
        (ops.size() && h2d(d_ops, ops.data(), ops.size() * 4)) ||
        (lvl_end.size() && h2d(d_lvl, lvl_end.data(), lvl_end.size() * 4)) ||
        h2d(d_meta, meta.data(), meta.size() * sizeof(TumourMeta)) ||
        h2d(st.flags, ones.data(), N * 4) || h2d(st.next_tumour, neg.data(), N * 4) ||
        h2d(st.pose, pose0.data(), pose0.size() * 8) ||
        hipMemset(st.dose, 0, (size_t)N * G.Vpad * 4) || hipMemset(st.t, 0, N * 4) ||
        hipMemset(st.tumour, 0, N * 4) || hipMemset(st.episode, 0, N * 4) || hipMemset(st.mode_b, 0, N) ||
        hipMemset(st.ep_return, 0, N * 8) || hipMemset(st.ep_len, 0, N * 4) ||
        hipMemset(st.lung_cnt, 0, N * 4) || hipMemset(st.lung_sum, 0, N * 8) ||
        hipMemset(st.setup, 0, (size_t)N * sizeof(BeamSetup)) || hipDeviceSynchronize()) {
        free_env(env);
        return fail(RT_EDEVICE, "initial upload failed");
    }
    env->lib.lung_bits = d_lbits;
    env->lib.dose_pos = env->dose_pos_d;
    env->lib.vox = d_vox;
    env->lib.vpos = env->lung_first ? d_vpos : d_vox;
    env->lib.coord = d_coord;
    env->lib.ops = d_ops;
    env->lib.lvl_end = d_lvl;
    env->lib.meta = d_meta;
    if (env->lung_first) {
        for (hipStream_t& q : env->pipe)
            if (hipStreamCreateWithFlags(&q, hipStreamNonBlocking) != hipSuccess) {
                free_env(env);
                return fail(RT_EDEVICE, "hipStreamCreateWithFlags failed");
            }
        for (hipEvent_t& ev : env->pev)
            if (hipEventCreateWithFlags(&ev, hipEventDisableTiming | kEventNoSysFence) != hipSuccess) {
                free_env(env);
                return fail(RT_EDEVICE, "hipEventCreateWithFlags failed");
            }
    }
    *out = env;
    return RT_OK;
}

void rt_env_destroy(rt_env* env) { free_env(env); }

int rt_env_num_envs(const rt_env* env) { return env ? env->N : 0; }

const int32_t* rt_env_dose_index(rt_env* env) { return env ? env->dose_pos_d : nullptr; }

float* rt_env_dose(rt_env* env, int64_t* stride) {
    if (!env) return nullptr;
    if (stride) *stride = env->G.Vpad;
    return env->st.dose;
}

BeamParams beam_params(const rt_env* env, bool reset_call, const float* actions, const uint8_t* mask,
                       const int32_t* ids) {
    BeamParams bp{};
    bp.G = env->G;
    bp.C = env->C;
    bp.st = env->st;
    bp.lib = env->lib;
    bp.actions = actions;
    bp.reset_mask = mask;
    bp.reset_ids = ids;
    bp.N = env->N;
    bp.is_reset_call = reset_call ? 1 : 0;
    bp.incremental = env->incremental;
    bp.seed = env->seed;
    bp.env_id_base = env->env_id_base;
    return bp;
}

FinishParams finish_params(const rt_env* env, float* obs, float* reward, uint8_t* term, float* info) {
    FinishParams fp{};
    fp.G = env->G;
    fp.C = env->C;
    fp.st = env->st;
    fp.lib = env->lib;
    fp.obs = obs;
    fp.reward = reward;
    fp.terminated = term;
    fp.info = info;
    fp.part_cnt = env->part_cnt;
    fp.part_sum = env->part_sum;
    fp.n_chunk = env->n_chunk;
    fp.max_tvox = env->max_tvox;
    fp.gscratch = nullptr;
    fp.gscratch_stride = 0;
    fp.N = env->N;
    fp.vision = env->visionless ? 0 : 1;
    fp.incremental = env->incremental;
    fp.hash_mask = env->view_hash_mask;
    fp.wave_lds = env->finish_wave_lds;
    fp.wpb = env->finish_wpb;
    return fp;
}

// Raise a kernel's dynamic-LDS limit to the full 160 KiB on its first launch
// in the process, whatever that launch needs: the limit is per kernel, not per
// handle, and a later handle (bigger tumour library, vision hash) may need more
// than 64 KiB.  The limit does not reserve LDS; occupancy follows each launch's
// actual request.
int allow_lds(const void* kernel, bool& raised) {
    if (raised) return RT_OK;
    hipFuncAttributes fa{};  // the kernel's static LDS counts against the same 160 KiB
    if (hipFuncGetAttributes(&fa, kernel) != hipSuccess) return fail(RT_EDEVICE, "hipFuncGetAttributes");
    const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                             160 * 1024 - (int)fa.sharedSizeBytes);
    if (e != hipSuccess) return fail(RT_EDEVICE, std::string("hipFuncSetAttribute(LDS): ") + hipGetErrorString(e));
    raised = true;
    return RT_OK;
}

// k_finish of envs [e0, e1)
int launch_finish(rt_env* env, float* obs, float* reward, uint8_t* term, float* info, hipStream_t stream, int e0,
                  int e1) {
    FinishParams fp = finish_params(env, obs, reward, term, info);
    fp.e_begin = e0;
    fp.N = e1;
    static bool big_lds = false;
    if (const int rc_lds = allow_lds(reinterpret_cast<const void*>(&k_finish), big_lds)) return rc_lds;
    hipLaunchKernelGGL(k_finish, dim3((e1 - e0 + fp.wpb - 1) / fp.wpb), dim3(64 * fp.wpb), env->finish_smem, stream,
                       fp);
    RT_LAUNCH_CHECK("k_finish");
    return RT_OK;
}

DenseParams dense_params(const rt_env* env, int e0) {
    DenseParams dp{};
    dp.G = env->G;
    dp.lung_thr = env->C.lung_thr;
    dp.st = env->st;
    dp.lung_bits = env->lib.lung_bits;
    dp.part_cnt = env->part_cnt;
    dp.part_sum = env->part_sum;
    dp.L = env->lplan;
    dp.slices = env->slices;
    dp.vec_per_slice = env->vec_per_slice;
    dp.e_begin = e0;
    return dp;
}

// k_dense / k_dense_vis of envs [e0, e0 + n) (nothing in incremental mode);
// persist_bpc > 0: the persistent k_dense with that many blocks per CU
int launch_dense(rt_env* env, int e0, int n, float* obs, int persist_bpc, hipStream_t stream) {
    const DenseParams dp = dense_params(env, e0);
    if (env->incremental) {
        // no dense pass: k_beam maintains the lung count and sum
    } else {
        if (!env->visionless) {
            DenseVisParams dv{dp, obs, env->render_src, env->render_rows, env->render_stride, env->render_n};
            hipLaunchKernelGGL(k_dense_vis, dim3(env->slices, n), dim3(kStepThreads), 0, stream, dv);
            RT_LAUNCH_CHECK("k_dense_vis");
        }
        // persist_bpc blocks per CU (the pipelined rollout), else as many as are
        // resident at once (a strided wave's items all run in one round)
        if (env->dense_bpc == 0) {
            int bpc = 0;
            const void* kf = env->visionless ? reinterpret_cast<const void*>(&k_dense<false>)
                                             : reinterpret_cast<const void*>(&k_dense<true>);
            if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bpc, kf, kStepThreads, 0) != hipSuccess || bpc < 1)
                bpc = 4;
            env->dense_bpc = bpc;
        }
        const int bpc = persist_bpc > 0 ? persist_bpc : env->dense_bpc;
        const int64_t items = (int64_t)n * env->n_chunk;
        const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)bpc * env->num_cu, (items + 3) / 4));
        if (env->visionless) {
            hipLaunchKernelGGL(k_dense<false>, dim3(std::max(blocks, persist_bpc > 0 ? blocks : kZeroBlocks)),
                               dim3(kStepThreads), 0, stream, dp, n);
            RT_LAUNCH_CHECK("k_dense");
        } else if (items > 0) {
            hipLaunchKernelGGL(k_dense<true>, dim3(blocks), dim3(kStepThreads), 0, stream, dp, n);
            RT_LAUNCH_CHECK("k_dense<gather>");
        }
    }
    return RT_OK;
}

// k_dense / k_dense_vis (skipped in incremental mode) then k_finish of envs
// [e0, e1) (e1 < 0: all) on one stream
int launch_dense_finish(rt_env* env, float* obs, float* reward, uint8_t* term, float* info, hipStream_t stream,
                        hipEvent_t* ev, int e0 = 0, int e1 = -1) {
    if (e1 < 0) e1 = env->N;
    if (ev) (void)hipEventRecord(ev[1], stream);
    if (const int rc = launch_dense(env, e0, e1 - e0, obs, 0, stream)) return rc;
    if (ev) (void)hipEventRecord(ev[2], stream);
    if (const int rc = launch_finish(env, obs, reward, term, info, stream, e0, e1)) return rc;
    if (ev) (void)hipEventRecord(ev[3], stream);
    return RT_OK;
}

hipEvent_t* next_timing_slot(rt_env* env) {
    if (env->timing_cap > 0 && env->timing_n < env->timing_cap) return &env->tev[(size_t)4 * env->timing_n++];
    return nullptr;
}

static int launch_step(rt_env* env, bool reset_call, const float* actions, const uint8_t* mask,
                       const int32_t* ids, float* obs, float* reward, uint8_t* term, float* info,
                       hipStream_t stream) {
    hipEvent_t* ev = next_timing_slot(env);
    if (ev) (void)hipEventRecord(ev[0], stream);
    BeamParams bp = beam_params(env, reset_call, actions, mask, ids);
    hipLaunchKernelGGL(k_beam, dim3((env->N + 3) / 4), dim3(256), 0, stream, bp);
    RT_LAUNCH_CHECK("k_beam");
    return launch_dense_finish(env, obs, reward, term, info, stream, ev);
}

int rt_env_reset(rt_env* env, const uint8_t* mask_d, const int32_t* tumour_ids_d, float* obs_d,
                 void* stream) {
    if (!env || !obs_d) return fail(RT_EINVAL, "NULL argument");
    const int rc = launch_step(env, true, nullptr, mask_d, tumour_ids_d, obs_d, nullptr, nullptr, nullptr,
                               as_stream(stream));
    env->render_src = nullptr;  // one reset only
    env->render_rows = nullptr;
    env->render_n = 0;
    return rc;
}

int rt_env_set_render_source(rt_env* env, const float* dose_store_d, int64_t store_stride, const int64_t* rows_d,
                             int32_t n_rows) {
    if (!env) return fail(RT_EINVAL, "NULL argument");
    if (env->visionless) return fail(RT_EINVAL, "rt_env_set_render_source: vision handles only");
    if (n_rows < 0 || n_rows > env->N) return fail(RT_EINVAL, "rt_env_set_render_source: n_rows outside [0, N]");
    if (n_rows > 0 && (!dose_store_d || !rows_d)) return fail(RT_EINVAL, "NULL argument");
    if (store_stride < env->G.Vpad || store_stride % 4 || (reinterpret_cast<uintptr_t>(dose_store_d) & 15))
        return fail(RT_EINVAL, "rt_env_set_render_source: rows must be >= the padded volume, 16-B aligned");
    env->render_src = dose_store_d;
    env->render_rows = rows_d;
    env->render_stride = store_stride;
    env->render_n = n_rows;
    return RT_OK;
}

int rt_env_step(rt_env* env, const float* actions_d, float* obs_d, float* reward_d,
                uint8_t* terminated_d, float* info_d, void* stream) {
    if (!env || !actions_d || !obs_d || !reward_d || !terminated_d) return fail(RT_EINVAL, "NULL argument");
    return launch_step(env, false, actions_d, nullptr, nullptr, obs_d, reward_d, terminated_d, info_d,
                       as_stream(stream));
}

int rt_env_step_policy(rt_env* env, const rt_policy_step* ps, float* obs_d, float* reward_d,
                       uint8_t* terminated_d, float* info_d, void* stream) {
    if (!env || !ps || !ps->params || !ps->obs_in || !ps->obs_store || !ps->done_store || !ps->act_store ||
        !ps->logp_store || !ps->value_store || !obs_d || !reward_d || !terminated_d)
        return fail(RT_EINVAL, "NULL argument");
    if (!env->visionless) return fail(RT_EINVAL, "rt_env_step_policy: the fused policy is the visionless MLP");
    if (ps->n_params != rtpol::kTensors) return fail(RT_EINVAL, "rt_env_step_policy: expected 13 parameter tensors");
    PolicyStepParams Q{};
    for (int i = 0; i < rtpol::kTensors; ++i) {
        if (!ps->params[i]) return fail(RT_EINVAL, "rt_env_step_policy: NULL parameter");
        Q.w.p[i] = ps->params[i];
    }
    Q.obs_in = ps->obs_in;
    Q.done_in = ps->done_in;
    Q.obs_store = ps->obs_store;
    Q.done_store = ps->done_store;
    Q.act_store = ps->act_store;
    Q.logp_store = ps->logp_store;
    Q.value_store = ps->value_store;
    Q.seed = ps->seed;
    Q.counter = ps->counter;
    Q.id_base = ps->env_id_base;
    Q.wpb = env->fused_wpb;
    hipStream_t s = as_stream(stream);
    hipEvent_t* ev = next_timing_slot(env);
    if (ev) (void)hipEventRecord(ev[0], s);
    BeamParams bp = beam_params(env, false, Q.act_store, nullptr, nullptr);
    FinishParams fp = finish_params(env, obs_d, reward_d, terminated_d, info_d);
    const dim3 grid((env->N + Q.wpb - 1) / Q.wpb), block(64 * Q.wpb);
    if (env->incremental) {
        static bool big = false;
        if (const int rc_lds = allow_lds(reinterpret_cast<const void*>(&k_step_policy<true>), big)) return rc_lds;
        hipLaunchKernelGGL(k_step_policy<true>, grid, block, env->fused_smem, s, bp, fp, Q);
        RT_LAUNCH_CHECK("k_step_policy");
        if (ev)
            for (int k = 1; k < 4; ++k) (void)hipEventRecord(ev[k], s);
        return RT_OK;
    }
    static bool big = false;
    if (const int rc_lds = allow_lds(reinterpret_cast<const void*>(&k_step_policy<false>), big)) return rc_lds;
    hipLaunchKernelGGL(k_step_policy<false>, grid, block, env->fused_smem, s, bp, fp, Q);
    RT_LAUNCH_CHECK("k_step_policy");
    return launch_dense_finish(env, obs_d, reward_d, terminated_d, info_d, s, ev);
}

// ---------------------------------------------------------------------------
// Dense step mode rollout: per step k_step_policy -> k_dense -> k_finish (the
// launches of rt_env_step_policy, same bits), with the envs split in two
// groups on two library streams.  k_dense is HBM-bound and needs the whole
// chip; the policy/pose/march kernel and k_finish are latency-bound one wave
// per env.  The groups take turns on k_dense (each group's k_dense waits for
// the other's previous one), so while one group streams its dose rows the
// other runs its latency-bound kernels beside it; only the first policy
// kernel and the last finish are not hidden.  Group 0 runs on the caller's
// stream, the others fork and join by events; nothing synchronises the host.
// ---------------------------------------------------------------------------
static int rollout_dense(rt_env* env, const rt_policy_rollout* r, float* obs_d, uint8_t* terminated_d,
                         hipStream_t s) {
    const rt_policy_step* ps = &r->step;
    const int N = env->N;
    int G = env->pipe[0] ? env->rollout_groups : 1;
    while (G > 1 && N < 16 * G) --G;
    const bool piped = G > 1;
    const int wpb = piped ? env->pipe_wpb : env->fused_wpb;
    const size_t smem = piped ? env->pipe_smem : env->fused_smem;
    // group boundaries on block boundaries
    int bounds[kMaxRolloutGroups + 1];
    for (int g = 0; g <= G; ++g) bounds[g] = g == G ? N : (int)((int64_t)N * g / G / wpb * wpb);
    hipStream_t S[kMaxRolloutGroups];
    hipEvent_t* dense_ev = env->pev + 1;
    hipEvent_t* join_ev = env->pev + 1 + kMaxRolloutGroups;
    // group 0 runs on the caller's stream itself (ordered after the caller's
    // work without a fork, so the call's first kernel is its first packet);
    // the other groups fork from it onto library streams and join back
    for (int g = 0; g < G; ++g) S[g] = s;
    if (piped) {
        RT_HIP(hipEventRecord(env->pev[0], s));
        for (int g = 1; g < G; ++g) {
            S[g] = env->pipe[g];
            RT_HIP(hipStreamWaitEvent(S[g], env->pev[0], 0));
        }
    }
    static bool big = false;
    if (const int rc_lds = allow_lds(reinterpret_cast<const void*>(&k_step_policy<false>), big)) return rc_lds;
    PolicyStepParams Q{};
    for (int i = 0; i < rtpol::kTensors; ++i) {
        if (!ps->params[i]) return fail(RT_EINVAL, "rt_env_rollout_policy: NULL parameter");
        Q.w.p[i] = ps->params[i];
    }
    Q.seed = ps->seed;
    Q.id_base = ps->env_id_base;
    Q.wpb = wpb;
    const size_t Nn = (size_t)N;
    for (int t = 0; t < r->n_steps; ++t) {
        Q.obs_in = t == 0 ? ps->obs_in : obs_d;
        Q.done_in = t == 0 ? ps->done_in : terminated_d;
        Q.obs_store = ps->obs_store + (size_t)t * Nn * rtpol::NOBS;
        Q.done_store = ps->done_store + (size_t)t * Nn;
        Q.act_store = ps->act_store + (size_t)t * Nn * rtpol::NACT;
        Q.logp_store = ps->logp_store + (size_t)t * Nn;
        Q.value_store = ps->value_store + (size_t)t * Nn;
        Q.counter = ps->counter + (uint64_t)t;
        float* rew = r->reward_store + (size_t)t * Nn;
        float* info = r->info_store ? r->info_store + (size_t)t * Nn * RT_INFO_W : nullptr;
        for (int g = 0; g < G; ++g) {
            const int e0 = bounds[g], e1 = bounds[g + 1];
            hipEvent_t* ev = next_timing_slot(env);
            if (ev) (void)hipEventRecord(ev[0], S[g]);
            BeamParams bp = beam_params(env, false, Q.act_store, nullptr, nullptr);
            FinishParams fp = finish_params(env, obs_d, rew, terminated_d, info);
            bp.e_begin = e0;
            bp.N = e1;
            hipLaunchKernelGGL(k_step_policy<false>, dim3((e1 - e0 + wpb - 1) / wpb), dim3(64 * wpb), smem,
                               S[g], bp, fp, Q);
            RT_LAUNCH_CHECK("k_step_policy");
            if (!piped) {
                if (const int rc = launch_dense_finish(env, obs_d, rew, terminated_d, info, s, ev, e0, e1)) return rc;
                continue;
            }
            // k_dense turns in a ring: group g of step t after group g-1 of step t
            // (group 0 after group G-1 of step t-1), each on its group's stream
            // (one cross-stream wait per turn; a dedicated dose stream, two
            // waits per turn, measured 18 % slower: DESIGN §10)
            if (t > 0 || g > 0) RT_HIP(hipStreamWaitEvent(S[g], dense_ev[(g + G - 1) % G], 0));
            if (ev) (void)hipEventRecord(ev[1], S[g]);
            if (const int rc = launch_dense(env, e0, e1 - e0, obs_d, env->pipe_dense_bpc, S[g])) return rc;
            RT_HIP(hipEventRecord(dense_ev[g], S[g]));
            if (ev) (void)hipEventRecord(ev[2], S[g]);
            if (const int rc = launch_finish(env, obs_d, rew, terminated_d, info, S[g], e0, e1)) return rc;
            if (ev) (void)hipEventRecord(ev[3], S[g]);
        }
    }
    if (piped) {
        for (int g = 1; g < G; ++g) {
            RT_HIP(hipEventRecord(join_ev[g], S[g]));
            RT_HIP(hipStreamWaitEvent(s, join_ev[g], 0));
        }
    }
    return RT_OK;
}

int rt_env_set_rollout_groups(rt_env* env, int32_t groups) {
    if (!env || groups < 0 || groups > kMaxRolloutGroups)
        return fail(RT_EINVAL, "rt_env_set_rollout_groups: groups must be 0 (persistent) or 1..4");
    if (groups == 0 && !env->incremental)
        return fail(RT_EINVAL, "rt_env_set_rollout_groups: groups 0 (one persistent launch) is the incremental "
                               "step mode's rollout; dense handles take 1..4");
    if (groups > 0 && env->incremental)
        return fail(RT_EINVAL, "rt_env_set_rollout_groups: incremental handles roll out in one persistent launch "
                               "(groups 0)");
    env->rollout_groups = groups;
    return RT_OK;
}

// Incremental step mode: one persistent launch for the whole rollout
// (k_rollout_policy).
static int rollout_persistent(rt_env* env, const rt_policy_rollout* r, float* obs_d, uint8_t* terminated_d,
                              hipStream_t s) {
    const rt_policy_step* ps = &r->step;
    RolloutParams R{};
    PolicyStepParams& Q = R.q;
    for (int i = 0; i < rtpol::kTensors; ++i) {
        if (!ps->params[i]) return fail(RT_EINVAL, "rt_env_rollout_policy: NULL parameter");
        Q.w.p[i] = ps->params[i];
    }
    Q.obs_in = ps->obs_in;
    Q.done_in = ps->done_in;
    Q.obs_store = ps->obs_store;
    Q.done_store = ps->done_store;
    Q.act_store = ps->act_store;
    Q.logp_store = ps->logp_store;
    Q.value_store = ps->value_store;
    Q.seed = ps->seed;
    Q.counter = ps->counter;
    Q.id_base = ps->env_id_base;
    Q.wpb = env->rollout_wpb;
    R.reward_store = r->reward_store;
    R.info_store = r->info_store;
    R.n_steps = r->n_steps;
    R.fin_off = env->rollout_fin_off;
    hipEvent_t* ev = next_timing_slot(env);
    if (ev) (void)hipEventRecord(ev[0], s);
    BeamParams bp = beam_params(env, false, nullptr, nullptr, nullptr);
    FinishParams fp = finish_params(env, obs_d, nullptr, terminated_d, nullptr);
    fp.max_tvox = env->rollout_cap;
    fp.wave_lds = env->rollout_wave_lds;
    if (env->rollout_cap < env->max_tvox && !env->gscratch)
        return fail(RT_EINVAL, "rt_env_rollout_policy: persistent rollout scratch missing");
    fp.gscratch = env->gscratch;
    fp.gscratch_stride = 2 * (int64_t)env->max_tvox;
    const dim3 grid((env->N + Q.wpb - 1) / Q.wpb), block(64 * Q.wpb);
    RolloutArgs A{bp, fp, R};
    static bool big = false;
    if (const int rc_lds = allow_lds(reinterpret_cast<const void*>(&k_rollout_policy), big)) return rc_lds;
    hipLaunchKernelGGL(k_rollout_policy, grid, block, env->rollout_smem, s, A);
    RT_LAUNCH_CHECK("k_rollout_policy");
    if (ev)
        for (int k = 1; k < 4; ++k) (void)hipEventRecord(ev[k], s);
    return RT_OK;
}

int rt_env_rollout_policy(rt_env* env, const rt_policy_rollout* r, float* obs_d, uint8_t* terminated_d,
                          void* stream) {
    if (!env || !r || !obs_d || !terminated_d || !r->reward_store) return fail(RT_EINVAL, "NULL argument");
    const rt_policy_step* ps = &r->step;
    if (!ps->params || !ps->obs_in || !ps->obs_store || !ps->done_store || !ps->act_store || !ps->logp_store ||
        !ps->value_store)
        return fail(RT_EINVAL, "NULL argument");
    if (!env->visionless) return fail(RT_EINVAL, "rt_env_rollout_policy: the fused policy is the visionless MLP");
    if (ps->n_params != rtpol::kTensors) return fail(RT_EINVAL, "rt_env_rollout_policy: expected 13 parameter tensors");
    if (r->n_steps < 1) return fail(RT_EINVAL, "rt_env_rollout_policy: n_steps < 1");
    if (!env->incremental) return rollout_dense(env, r, obs_d, terminated_d, as_stream(stream));
    if (env->rollout_wpb == 0)
        return fail(RT_ELIMIT, "rt_env_rollout_policy: policy + finish scratch exceed LDS (largest tumour too big)");
    return rollout_persistent(env, r, obs_d, terminated_d, as_stream(stream));
}

int rt_env_kernel_timing(rt_env* env, int32_t capacity) {
    if (!env || capacity < 0) return fail(RT_EINVAL, "bad argument");
    for (hipEvent_t e : env->tev) (void)hipEventDestroy(e);
    env->tev.clear();
    env->timing_cap = 0;
    env->timing_n = 0;
    if (capacity == 0) return RT_OK;
    env->tev.resize((size_t)4 * capacity);
    for (auto& e : env->tev) RT_HIP(hipEventCreateWithFlags(&e, kEventNoSysFence));
    env->timing_cap = capacity;
    return RT_OK;
}

int rt_env_kernel_timing_read(rt_env* env, double* ms_out, int32_t* steps) {
    if (!env || !ms_out || !steps) return fail(RT_EINVAL, "bad argument");
    double acc[3] = {0.0, 0.0, 0.0};
    for (int i = 0; i < env->timing_n; ++i) {
        hipEvent_t* ev = &env->tev[(size_t)4 * i];
        RT_HIP(hipEventSynchronize(ev[3]));
        for (int k = 0; k < 3; ++k) {
            float ms = 0.0f;
            RT_HIP(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
            acc[k] += ms;
        }
    }
    for (int k = 0; k < 3; ++k) ms_out[k] = acc[k];
    *steps = env->timing_n;
    env->timing_n = 0;
    return RT_OK;
}

int rt_env_set_next_tumours(rt_env* env, const int32_t* ids_d, void* stream) {
    if (!env || !ids_d) return fail(RT_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_set_next, dim3((env->N + 255) / 256), dim3(256), 0, as_stream(stream), env->st,
                       env->N, ids_d);
    RT_LAUNCH_CHECK("k_set_next");
    return RT_OK;
}

int rt_env_reseed(rt_env* env, uint64_t seed, void* stream) {
    if (!env) return fail(RT_EINVAL, "NULL argument");
    // launches already queued captured the old key in their parameters; the
    // counters restart on the caller's stream, in order with them
    RT_HIP(hipMemsetAsync(env->st.episode, 0, (size_t)env->N * sizeof(uint32_t), as_stream(stream)));
    env->seed = seed;
    return RT_OK;
}

int rt_env_get_state(rt_env* env, double* pose_d, int32_t* t_d, int32_t* tumour_d, void* stream) {
    if (!env) return fail(RT_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_get_state, dim3((env->N + 255) / 256), dim3(256), 0, as_stream(stream), env->st,
                       env->N, pose_d, t_d, tumour_d);
    RT_LAUNCH_CHECK("k_get_state");
    return RT_OK;
}

int rt_env_set_tumours(rt_env* env, const int32_t* tumour_d, void* stream) {
    if (!env || !tumour_d) return fail(RT_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_set_tumours, dim3((env->N + 255) / 256), dim3(256), 0, as_stream(stream), env->st,
                       env->N, env->lib.K, tumour_d);
    RT_LAUNCH_CHECK("k_set_tumours");
    return RT_OK;
}

int rt_env_set_pose(rt_env* env, const double* pose_d, void* stream) {
    if (!env || !pose_d) return fail(RT_EINVAL, "NULL argument");
    hipLaunchKernelGGL(k_set_pose, dim3((env->N + 255) / 256), dim3(256), 0, as_stream(stream), env->st,
                       env->N, pose_d);
    RT_LAUNCH_CHECK("k_set_pose");
    return RT_OK;
}

int rt_debug_beam(const int32_t grid[3], int32_t m, const double* pos_d, const double* dir_d,
                  int32_t cap, int32_t* idx_d, float* w_d, int32_t* count_d, void* stream) {
    Geom G{};
    int rc = fill_geom(grid, G);
    if (rc) return rc;
    if (m < 0 || cap < 0 || !pos_d || !dir_d || !count_d) return fail(RT_EINVAL, "bad argument");
    if (m == 0) return RT_OK;
    hipLaunchKernelGGL(k_debug_beam, dim3((m + 63) / 64), dim3(64), 0, as_stream(stream), G, m, pos_d, dir_d,
                       cap, idx_d, w_d, count_d);
    RT_LAUNCH_CHECK("k_debug_beam");
    return RT_OK;
}

int rt_probe_random_rmw(float* buf_d, int64_t n_floats, int32_t lanes, int32_t lines_per_lane, uint64_t seed,
                        void* stream) {
    if (!buf_d || n_floats < 32 || lanes < 256 || lanes % 256 || lines_per_lane < 4 || lines_per_lane % 4)
        return fail(RT_EINVAL, "bad argument");
    hipLaunchKernelGGL(k_probe_rmw, dim3(lanes / 256), dim3(256), 0, as_stream(stream), buf_d, n_floats / 32,
                       lines_per_lane, seed);
    RT_LAUNCH_CHECK("k_probe_rmw");
    return RT_OK;
}

int rt_probe_stream(const float* src_d, float* dst_d, int64_t n_floats, int32_t mode, int32_t blocks, void* stream) {
    if (!src_d || !dst_d || n_floats < 4 || n_floats % 4 || (mode != 0 && mode != 1) || blocks < 1 ||
        (reinterpret_cast<uintptr_t>(src_d) & 15) || (reinterpret_cast<uintptr_t>(dst_d) & 15))
        return fail(RT_EINVAL, "rt_probe_stream: bad argument");
    if (mode == 0 && n_floats < (int64_t)blocks * 4)
        return fail(RT_EINVAL, "rt_probe_stream: READ needs dst_d of >= 4 * blocks floats");
    const float4* s4 = reinterpret_cast<const float4*>(src_d);
    if (mode == 1)
        hipLaunchKernelGGL(k_probe_stream<true>, dim3(blocks), dim3(256), 0, as_stream(stream), s4,
                           reinterpret_cast<float4*>(dst_d), n_floats / 4, nullptr);
    else
        hipLaunchKernelGGL(k_probe_stream<false>, dim3(blocks), dim3(256), 0, as_stream(stream), s4, nullptr,
                           n_floats / 4, dst_d);
    RT_LAUNCH_CHECK("k_probe_stream");
    return RT_OK;
}

int rt_env_beam_list(rt_env* env, int32_t cap, int32_t* idx_d, float* w_d, int32_t* count_d, void* stream) {
    if (!env || cap < 0 || !count_d || (cap > 0 && (!idx_d || !w_d))) return fail(RT_EINVAL, "bad argument");
    hipLaunchKernelGGL(k_env_beam_list, dim3((env->N + 63) / 64), dim3(64), 0, as_stream(stream), env->G, env->N,
                       env->st.pose, env->st.t, cap, idx_d, w_d, count_d);
    RT_LAUNCH_CHECK("k_env_beam_list");
    return RT_OK;
}

int rt_debug_pose(const int32_t grid[3], int32_t m, const double* pos_d, const double* dir_d,
                  const float* action_d, double* out_d, void* stream) {
    Geom G{};
    int rc = fill_geom(grid, G);
    if (rc) return rc;
    if (m < 0 || !pos_d || !dir_d || !action_d || !out_d) return fail(RT_EINVAL, "bad argument");
    if (m == 0) return RT_OK;
    rt_env_config cfg;
    cfg.struct_size = sizeof(cfg);
    rt_env_config_default(&cfg);
    Consts C = make_consts(cfg);
    hipLaunchKernelGGL(k_debug_pose, dim3((m + 63) / 64), dim3(64), 0, as_stream(stream), G, C, m, pos_d,
                       dir_d, action_d, out_d);
    RT_LAUNCH_CHECK("k_debug_pose");
    return RT_OK;
}

int rt_gae(int32_t T, int32_t N, const float* rewards_d, const float* values_d, const float* dones_d,
           const float* next_value_d, const float* next_done_d, double gamma, double gae_lambda, float* adv_d,
           float* ret_d, void* stream) {
    if (T < 1 || N < 1 || !rewards_d || !values_d || !dones_d || !next_value_d || !next_done_d || !adv_d || !ret_d)
        return fail(RT_EINVAL, "bad argument");
    // torch applies python-float scalars in f32: gamma, and gamma*lambda (a python product)
    float gl = (float)(gamma * gae_lambda);
    hipLaunchKernelGGL(k_gae, dim3((N + 255) / 256), dim3(256), 0, as_stream(stream), T, N, rewards_d,
                       values_d, dones_d, next_value_d, next_done_d, (float)gamma, gl, adv_d, ret_d);
    RT_LAUNCH_CHECK("k_gae");
    return RT_OK;
}

}  // extern "C"
