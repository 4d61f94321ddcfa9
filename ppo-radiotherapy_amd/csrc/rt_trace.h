// rt_trace.h -- per-env phase timestamps for latency analysis (profiling aid).
//
// Compiled out unless -DRT_TRACE (tools/trace_env.py builds a separate traced
// library); the product library carries none of it.  Each translation unit
// has its own table: kTraceSlots 64-bit s_memrealtime stamps (100 MHz, one
// clock for every CU) per env, read back with rt_trace_read_<unit>.
#pragma once

#ifdef RT_TRACE
#include <cstdint>
constexpr int kTraceEnvs = 8192;
constexpr int kTraceSlots = 16;
__device__ uint64_t g_rt_trace[kTraceEnvs * kTraceSlots];
#define RT_STAMP(e, slot)                                                                        \
    do {                                                                                         \
        if ((e) < kTraceEnvs) g_rt_trace[(size_t)(e) * kTraceSlots + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#define RT_TRACE_READ_FN(name)                                                                   \
    extern "C" int name(uint64_t* out) {                                                         \
        return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_trace), sizeof(g_rt_trace)) == hipSuccess ? 0 : -1; \
    }
#else
#define RT_STAMP(e, slot) \
    do {                  \
    } while (0)
#define RT_TRACE_READ_FN(name)
#endif
