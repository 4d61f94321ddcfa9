// Probe of the HIP stream memory operations the device hand-off relies on
// (hipStreamWaitValue64 / hipStreamWriteValue64) on gfx950 / ROCm 7.2:
//   1. a WaitValue64 on stream A must hold A's next kernel until a kernel on
//      stream B (launched later, delayed ~20 ms) bumps the word -- for a
//      hipMalloc word and for hipMallocSignalMemory;
//   2. a WriteValue64 queued on A behind a delayed kernel must become visible
//      to a kernel already running on a CU-masked stream D that polls it
//      (bounded poll: the probe reports a timeout instead of hanging).
// Build: hipcc --offload-arch=gfx950 -O2 tools/probe_streamops.cpp -o tools/_probe_streamops
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::printf("FAIL %s: %s\n", #x, hipGetErrorString(e_));                       \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

__global__ void k_delay_add(uint64_t* w, uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
    __hip_atomic_fetch_add(w, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_delay(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}

__global__ void k_read(const uint64_t* w, uint64_t* out) {
    out[0] = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// poll until *w >= want or timeout; out = {seen value, waited ticks, timed out}
__global__ void k_poll(uint64_t* w, uint64_t want, uint64_t timeout, uint64_t* out) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t v = 0;
    int to = 0;
    while ((v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < want) {
        __builtin_amdgcn_s_sleep(4);
        if (__builtin_amdgcn_s_memrealtime() - t0 > timeout) {
            to = 1;
            break;
        }
    }
    out[0] = v;
    out[1] = __builtin_amdgcn_s_memrealtime() - t0;
    out[2] = to;
}

__global__ void k_stamp(uint64_t* out) {
    if (threadIdx.x == 0) __hip_atomic_store(out, (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void k_delay_stamp_add(uint64_t* w, uint64_t ticks, uint64_t* out) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
    if (threadIdx.x == 0) {
        __hip_atomic_store(out, (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(w, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ void k_poll_stamp(uint64_t* w, uint64_t want, uint64_t* out) {
    if (threadIdx.x != 0) return;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000) break;
    }
    __hip_atomic_store(out, (uint64_t)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static int wait_case(const char* name, uint64_t* w, hipStream_t a, hipStream_t b, uint64_t* out) {
    CK(hipMemset(out, 0xff, 8));
    CK(hipDeviceSynchronize());
    CK(hipStreamWaitValue64(a, w, 1, hipStreamWaitValueGte, ~0ull));
    hipLaunchKernelGGL(k_read, dim3(1), dim3(1), 0, a, w, out);
    hipLaunchKernelGGL(k_delay_add, dim3(1), dim3(1), 0, b, w, (uint64_t)2000000);  // 20 ms
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    uint64_t h = 0;
    CK(hipMemcpy(&h, out, 8, hipMemcpyDeviceToHost));
    std::printf("%s: reader after WaitValue64 saw %llu (1 = the wait held it)\n", name, (unsigned long long)h);
    return 0;
}

int main() {
    int ok = 0;
    CK(hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, 0));
    std::printf("hipDeviceAttributeCanUseStreamWaitValue = %d\n", ok);
    hipStream_t a, b, d;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    std::vector<uint32_t> mask((prop.multiProcessorCount + 31) / 32, 0u);
    for (int c = 0; c < prop.multiProcessorCount; ++c) mask[c / 32] |= 1u << (c % 32);
    CK(hipExtStreamCreateWithCUMask(&d, (uint32_t)mask.size(), mask.data()));
    uint64_t *w, *out, *sig = nullptr;
    CK(hipMalloc(&w, 256));
    CK(hipMalloc(&out, 256));
    CK(hipMemset(w, 0, 256));
    if (wait_case("hipMalloc word", w, a, b, out)) return 1;
    hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&sig), 8, hipMallocSignalMemory);
    std::printf("hipExtMallocWithFlags(hipMallocSignalMemory): %s\n", hipGetErrorString(e));
    if (e == hipSuccess) {
        CK(hipMemset(sig, 0, 8));
        if (wait_case("signal word", sig, a, b, out)) return 1;
    }
    // 2: WriteValue64 behind a delayed kernel on a, poller on the CU-masked d
    CK(hipMemset(w, 0, 256));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_poll, dim3(1), dim3(64), 0, d, w, (uint64_t)5, (uint64_t)100000000, out);
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(1), 0, a, (uint64_t)2000000);
    CK(hipStreamWriteValue64(a, w, 5, 0));
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    uint64_t h[3];
    CK(hipMemcpy(h, out, 24, hipMemcpyDeviceToHost));
    std::printf("WriteValue64 -> poller on CU-masked stream: saw %llu after %.2f ms, timeout %llu\n",
                (unsigned long long)h[0], h[1] / 1e5, (unsigned long long)h[2]);
    // 3: the same with the poller on an ordinary stream created BEFORE a and b
    CK(hipMemset(w, 0, 256));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_poll, dim3(1), dim3(64), 0, b, w, (uint64_t)5, (uint64_t)100000000, out);
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(1), 0, a, (uint64_t)2000000);
    CK(hipStreamWriteValue64(a, w, 5, 0));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h, out, 24, hipMemcpyDeviceToHost));
    std::printf("WriteValue64 -> poller on stream b: saw %llu after %.2f ms, timeout %llu\n",
                (unsigned long long)h[0], h[1] / 1e5, (unsigned long long)h[2]);
    // 4: latencies (s_memrealtime, 10 ns ticks), 5 repetitions each
    {
        uint64_t *st, *w2, *sig2 = sig;
        CK(hipMalloc(&st, 4096));
        CK(hipMalloc(&w2, 256));
        auto lat = [&](const char* name, int kind) -> int {
            double acc = 0, mx = 0;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipMemset(st, 0, 4096));
                CK(hipMemset(w2, 0, 256));
                if (sig2) CK(hipMemset(sig2, 0, 8));
                CK(hipDeviceSynchronize());
                uint64_t* word = kind == 1 && sig2 ? sig2 : w2;
                if (kind == 0 || kind == 1) {  // WaitValue wake-up: bump (stamp st[1]) -> reader start (st[0])
                    CK(hipStreamWaitValue64(a, word, 1, hipStreamWaitValueGte, ~0ull));
                    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, a, st + 0);
                    hipLaunchKernelGGL(k_delay_stamp_add, dim3(1), dim3(64), 0, b, word, (uint64_t)1000000, st + 1);
                } else if (kind == 2) {  // WriteValue: delayed kernel end (st[1]) -> poller sees (st[0])
                    hipLaunchKernelGGL(k_poll_stamp, dim3(1), dim3(64), 0, d, w2, (uint64_t)5, st + 0);
                    hipLaunchKernelGGL(k_delay_stamp_add, dim3(1), dim3(64), 0, a, st + 8, (uint64_t)1000000, st + 1);
                    CK(hipStreamWriteValue64(a, w2, 5, 0));
                } else if (kind == 3) {  // event across streams: kernel end (st[1]) -> next kernel start (st[0])
                    hipEvent_t ev;
                    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
                    hipLaunchKernelGGL(k_delay_stamp_add, dim3(1), dim3(64), 0, a, st + 8, (uint64_t)1000000, st + 1);
                    CK(hipEventRecord(ev, a));
                    CK(hipStreamWaitEvent(b, ev, 0));
                    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, b, st + 0);
                    CK(hipDeviceSynchronize());
                    CK(hipEventDestroy(ev));
                } else {  // same stream kernel boundary
                    hipLaunchKernelGGL(k_delay_stamp_add, dim3(1), dim3(64), 0, a, st + 8, (uint64_t)1000000, st + 1);
                    hipLaunchKernelGGL(k_stamp, dim3(1), dim3(64), 0, a, st + 0);
                }
                CK(hipDeviceSynchronize());
                uint64_t h2[2];
                CK(hipMemcpy(h2, st, 16, hipMemcpyDeviceToHost));
                const double us = ((double)h2[0] - (double)h2[1]) / 100.0;
                acc += us;
                mx = us > mx ? us : mx;
            }
            std::printf("latency %-44s mean %8.2f us  max %8.2f us\n", name, acc / 5, mx);
            return 0;
        };
        if (lat("WaitValue64 wake-up, hipMalloc word", 0)) return 1;
        if (sig2 && lat("WaitValue64 wake-up, signal word", 1)) return 1;
        if (lat("WriteValue64 after kernel -> poller", 2)) return 1;
        if (lat("event record/wait across streams", 3)) return 1;
        if (lat("same-stream kernel boundary", 4)) return 1;
    }
    std::printf("PROBE DONE\n");
    return 0;
}
