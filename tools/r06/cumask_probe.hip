// Probe: where do the blocks of a CU-masked stream land (hipExtStreamCreateWithCUMask),
// and what read bandwidth does a non-temporal 16-B stream reach on a masked
// subset of the CUs?  Decides the CU split of the pipelined dense rollout
// (chain kernels on a few CUs per XCD, the lung stream on the rest).
// Build: hipcc --offload-arch=gfx950 -O3 cumask_probe.hip -o cumask_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

__global__ void k_where(unsigned* out) {
    if (threadIdx.x == 0) out[blockIdx.x] = __smid();
    // keep the block alive a little so the dispatcher spreads blocks
    long t0 = clock64();
    while (clock64() - t0 < 20000) {
    }
}

__global__ __launch_bounds__(256) void k_read(const float4* __restrict__ p, size_t n4, float* out) {
    typedef float nf4 __attribute__((ext_vector_type(4)));
    float acc = 0.f;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 7 * stride < n4; i += 8 * stride) {
        nf4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p + i + k * stride));
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
    }
    for (; i < n4; i += stride) acc += p[i].x;
    if (acc == 12345.f) out[0] = acc;
}

static std::vector<uint32_t> mask_of(int ncu, bool (*in)(int)) {
    std::vector<uint32_t> m((ncu + 31) / 32, 0u);
    for (int i = 0; i < ncu; ++i)
        if (in(i)) m[i / 32] |= 1u << (i % 32);
    return m;
}

static bool s_chain64(int i) {
    const int r = i % 32;
    return r == 0 || r == 4 || r == 9 || r == 13 || r == 18 || r == 22 || r == 27 || r == 31;
}
static bool s_chain32(int i) {
    const int r = i % 32;
    return r == 0 || r == 9 || r == 18 || r == 27;
}
static bool s_dense192(int i) { return !s_chain64(i); }
static bool s_dense224(int i) { return !s_chain32(i); }
static bool s_low64(int i) { return i < 64; }
static bool s_mod4(int i) { return i % 4 == 0; }
static bool s_all(int) { return true; }

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    std::printf("device %s, %d CUs\n", prop.name, ncu);
    struct M {
        const char* name;
        bool (*f)(int);
    } masks[] = {{"all", s_all},       {"chain64", s_chain64}, {"chain32", s_chain32}, {"dense192", s_dense192},
                 {"dense224", s_dense224}, {"low64", s_low64},   {"mod4", s_mod4}};
    const int nb = 8192;
    unsigned* d_out;
    CK(hipMalloc(&d_out, nb * 4));
    std::vector<unsigned> h(nb);
    for (auto& mk : masks) {
        auto m = mask_of(ncu, mk.f);
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
        std::vector<uint32_t> back(m.size());
        CK(hipExtStreamGetCUMask(s, (uint32_t)back.size(), back.data()));
        hipLaunchKernelGGL(k_where, dim3(nb), dim3(64), 0, s, d_out);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), d_out, nb * 4, hipMemcpyDeviceToHost));
        std::set<unsigned> uniq(h.begin(), h.end());
        std::map<unsigned, std::set<unsigned>> per_xcc, per_se;
        for (unsigned v : uniq) {
            per_xcc[v >> 7].insert(v);
            per_se[v >> 4].insert(v);
        }
        std::printf("mask %-9s bits %3d  distinct CUs %3zu  per XCC:", mk.name,
                    [&] { int c = 0; for (int i = 0; i < ncu; ++i) c += mk.f(i); return c; }(), uniq.size());
        for (auto& kv : per_xcc) std::printf(" %u:%zu", kv.first, kv.second.size());
        std::printf("  per (XCC,SE):");
        for (auto& kv : per_se) std::printf(" %u.%u:%zu", kv.first >> 3, kv.first & 7, kv.second.size());
        std::printf("  getmask[0]=%08x\n", back[0]);
        CK(hipStreamDestroy(s));
    }
    // bandwidth on masked subsets
    const size_t bytes = (size_t)4 << 30;
    float4* buf;
    float* d_acc;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&d_acc, 4));
    CK(hipMemset(buf, 0, bytes));
    for (auto& mk : masks) {
        if (mk.f == s_low64 || mk.f == s_mod4) continue;
        auto m = mask_of(ncu, mk.f);
        int k = 0;
        for (int i = 0; i < ncu; ++i) k += mk.f(i);
        hipStream_t s;
        CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        for (int bpc : {4, 8}) {
            const int blocks = bpc * k;
            for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, s, buf, bytes / 16, d_acc);
            CK(hipEventRecord(a, s));
            const int reps = 10;
            for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_read, dim3(blocks), dim3(256), 0, s, buf, bytes / 16, d_acc);
            CK(hipEventRecord(b, s));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            std::printf("read  mask %-9s CUs %3d  blocks/CU %d  %.1f GB/s\n", mk.name, k, bpc,
                        bytes * (double)reps / (ms * 1e-3) / 1e9);
        }
        CK(hipStreamDestroy(s));
    }
    std::printf("PROBE_DONE\n");
    return 0;
}
