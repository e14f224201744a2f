// flrl_common.hip — library plumbing (error strings, device query) and the
// device-side synthetic input generator of SURVEY.md §8(d).
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "flrl.h"
#include "flrl_device.hpp"
#include "flrl_internal.hpp"

namespace flrl {

static thread_local char g_err[512];

int set_error(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

void clear_error() { g_err[0] = 0; }

// Pending kernel-timing events of this thread (flrl_time_next_kernel).
static thread_local hipEvent_t g_ev_start = nullptr, g_ev_stop = nullptr;

void kernel_timing_begin(hipStream_t s)
{
    if (g_ev_start)
        (void)hipEventRecord(g_ev_start, s);
}

void kernel_timing_end(hipStream_t s)
{
    if (g_ev_stop)
        (void)hipEventRecord(g_ev_stop, s);
    g_ev_start = g_ev_stop = nullptr;
}

// Scratch resets. A kernel rather than hipMemsetAsync: captured into a HIP
// graph (torch.cuda.graph around encode/decode), hipMemsetAsync resets did not
// take effect on re-launch here (the second replay of an encode + decode step
// saw the previous launch's ticket: scripts/graph_probe.py), while a kernel
// node is stream-ordered like the kernels around it.
__global__ __launch_bounds__(kThreads) void zero_kernel(uint8_t *p, uint64_t bytes)
{
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    const uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(p) & 15u) == 0) {
        for (uint64_t c = i; c * 16 < bytes; c += stride) {
            if (c * 16 + 16 <= bytes)
                *reinterpret_cast<u32x4 *>(p + c * 16) = u32x4{0u, 0u, 0u, 0u};
            else
                for (uint64_t b = c * 16; b < bytes; ++b)
                    p[b] = 0;
        }
    } else {
        for (uint64_t b = i; b < bytes; b += stride)
            p[b] = 0;
    }
}

hipError_t zero_async(void *p, size_t bytes, hipStream_t s)
{
    if (bytes == 0)
        return hipSuccess;
    const size_t blocks = div_up(div_up(bytes, 16), (size_t)kThreads);
    hipLaunchKernelGGL(zero_kernel, dim3((uint32_t)(blocks < 1024 ? blocks : 1024)), dim3(kThreads), 0, s,
                       static_cast<uint8_t *>(p), (uint64_t)bytes);
    return hipGetLastError();
}

// [p, p + 16 head16) and the 8-byte words at p + 16 head16 + k stride (k <
// count): a Ctrl plus look-back status words that sit one per cache line
// (only the words are ever read, so the lines' other bytes stay as they are)
__global__ __launch_bounds__(kThreads) void zero_strided_kernel(uint8_t *p, uint32_t head16, uint64_t count,
                                                                 uint32_t stride)
{
    const uint64_t total = head16 + count;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < total;
         i += (uint64_t)gridDim.x * kThreads) {
        if (i < head16)
            *reinterpret_cast<u32x4 *>(p + 16 * i) = u32x4{0u, 0u, 0u, 0u};
        else
            *reinterpret_cast<uint64_t *>(p + 16ull * head16 + (i - head16) * stride) = 0;
    }
}

__global__ void raise_error_kernel(Ctrl *ctrl, uint32_t code)
{
    raise_error(ctrl, code);
}

hipError_t raise_error_async(void *scratch, int code, hipStream_t s)
{
    hipLaunchKernelGGL(raise_error_kernel, dim3(1), dim3(1), 0, s, static_cast<Ctrl *>(scratch), (uint32_t)code);
    return hipGetLastError();
}

static thread_local int g_skip_resets = 0;

hipError_t scratch_reset(void *p, size_t bytes, hipStream_t s)
{
    if (g_skip_resets > 0) {
        --g_skip_resets;
        return hipSuccess;
    }
    return zero_async(p, bytes, s);
}

hipError_t scratch_reset_strided(void *p, size_t head_bytes, size_t count, size_t stride, hipStream_t s)
{
    if (g_skip_resets > 0) {
        --g_skip_resets;
        return hipSuccess;
    }
    const size_t total = head_bytes / 16 + count;
    const size_t blocks = div_up(total, (size_t)kThreads);
    hipLaunchKernelGGL(zero_strided_kernel, dim3((uint32_t)(blocks < 1024 ? blocks : 1024)), dim3(kThreads), 0, s,
                       static_cast<uint8_t *>(p), (uint32_t)(head_bytes / 16), (uint64_t)count, (uint32_t)stride);
    return hipGetLastError();
}

// splitmix64 draw number w+1 from `seed` (counter form of SURVEY.md §8(d)).
__device__ __forceinline__ uint64_t splitmix_at(uint64_t seed, uint64_t w)
{
    uint64_t z = seed + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Each thread writes 16 bytes = two 8-byte words per grid-stride step.
__global__ __launch_bounds__(kThreads) void gen_kernel(uint32_t mask8, uint64_t seed,
                                                       uint64_t word_offset, uint8_t *out,
                                                       uint64_t n)
{
    const uint64_t mask = (uint64_t)mask8 * 0x0101010101010101ull;
    const uint64_t stride = (uint64_t)gridDim.x * kThreads;
    for (uint64_t t = (uint64_t)blockIdx.x * kThreads + threadIdx.x; t * 16 < n; t += stride) {
        const uint64_t a = splitmix_at(seed, word_offset + 2 * t) & mask;
        const uint64_t b = splitmix_at(seed, word_offset + 2 * t + 1) & mask;
        const u32x4 v = u32x4{(uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32)};
        store16_tail(out, t * 16, n, v);
    }
}

}  // namespace flrl

using namespace flrl;

extern "C" const char *flrl_last_error(void) { return g_err; }

extern "C" const char *flrl_version(void) { return "flrl 0.1.0 (gfx950)"; }

extern "C" int flrl_time_next_kernel(void *start_event, void *stop_event)
{
    if ((start_event == nullptr) != (stop_event == nullptr))
        return set_error(FLRL_E_ARG, "flrl_time_next_kernel: pass both events or neither");
    g_ev_start = static_cast<hipEvent_t>(start_event);
    g_ev_stop = static_cast<hipEvent_t>(stop_event);
    return FLRL_OK;
}

static std::atomic<long long> g_fail_chunk{-1};

bool flrl::debug_fail_chunk(size_t c) { return (long long)c == g_fail_chunk.load(std::memory_order_relaxed); }

extern "C" int flrl_debug_fail_chunk(long long chunk)
{
    g_fail_chunk.store(chunk < 0 ? -1 : chunk);
    return FLRL_OK;
}

static thread_local int g_fail_rank_step = 0;

bool flrl::debug_fail_rank_step(int step)
{
    if (g_fail_rank_step != step)
        return false;
    g_fail_rank_step = 0;
    return true;
}

extern "C" int flrl_debug_fail_rank_step(int step)
{
    if (step < 0 || step > FLRL_DEBUG_RANK_READ_SUM)
        return set_error(FLRL_E_ARG, "flrl_debug_fail_rank_step: step %d", step);
    g_fail_rank_step = step;
    return FLRL_OK;
}

// flrl_debug_lookback_help_us: the decoupled-fallback threshold of this
// thread's look-back launches in s_memrealtime ticks (-1: each kernel's default)
static thread_local int64_t g_help_ticks = -1;

uint64_t flrl::lookback_help_ticks(uint64_t dflt) { return g_help_ticks < 0 ? dflt : (uint64_t)g_help_ticks; }

extern "C" int flrl_debug_lookback_help_us(int microseconds)
{
    if (microseconds < -1)
        return set_error(FLRL_E_ARG, "flrl_debug_lookback_help_us: %d < -1", microseconds);
    g_help_ticks = microseconds < 0 ? -1 : (int64_t)microseconds * 100;  // 100 MHz ticks
    return FLRL_OK;
}

extern "C" int flrl_debug_skip_scratch_resets(int calls)
{
    if (calls < 0)
        return set_error(FLRL_E_ARG, "flrl_debug_skip_scratch_resets: negative count");
    g_skip_resets = calls;
    return FLRL_OK;
}

extern "C" int flrl_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

extern "C" int flrl_gen_device(int kind, uint64_t seed, uint64_t word_offset, uint8_t *d_out,
                               size_t n, void *stream)
{
    if (kind < 0 || kind > 2)
        return set_error(FLRL_E_ARG, "flrl_gen_device: kind %d is not counter-based (0-2)", kind);
    if (n == 0)
        return FLRL_OK;
    if (!d_out || !aligned16(d_out))
        return set_error(FLRL_E_ARG, "flrl_gen_device: output must be non-null, 16-B aligned");
    const uint32_t mask8 = kind == 0 ? 0xFFu : (kind == 1 ? 0x0Fu : 0u);
    const size_t threads_needed = div_up(n, 16);
    const size_t blocks = threads_needed / kThreads + 1;
    const uint32_t grid = (uint32_t)(blocks < 8192 ? blocks : 8192);
    hipLaunchKernelGGL(gen_kernel, dim3(grid), dim3(kThreads), 0,
                       static_cast<hipStream_t>(stream), mask8, seed, word_offset, d_out,
                       (uint64_t)n);
    FLRL_HIP(hipGetLastError());
    return FLRL_OK;
}

static uint64_t splitmix_next(uint64_t *state)
{
    uint64_t z = (*state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

extern "C" int flrl_gen_host(int kind, uint64_t seed, uint64_t word_offset, uint8_t *out, size_t n)
{
    if (n && !out)
        return set_error(FLRL_E_ARG, "flrl_gen_host: null output");
    if (kind >= 0 && kind <= 2) {
        const uint8_t mask = kind == 0 ? 0xFF : (kind == 1 ? 0x0F : 0x00);
        for (size_t w = 0; w * 8 < n; ++w) {
            uint64_t st = seed + (word_offset + w) * 0x9E3779B97F4A7C15ull;
            const uint64_t word = splitmix_next(&st);
            for (size_t j = 0; j < 8 && w * 8 + j < n; ++j)
                out[w * 8 + j] = (uint8_t)((word >> (8 * j)) & mask);
        }
        return FLRL_OK;
    }
    if (kind == 3 || kind == 4) {
        if (word_offset != 0)
            return set_error(FLRL_E_ARG, "flrl_gen_host: run kinds are sequential (word_offset 0)");
        const uint64_t mod = kind == 3 ? 63 : 1023;
        uint64_t st = seed;
        size_t i = 0;
        uint8_t prev = 0;
        while (i < n) {
            const uint64_t r = splitmix_next(&st);
            size_t len = (size_t)(1 + r % mod);
            uint8_t val = (uint8_t)((r >> 32) & 0xFF);
            if (i > 0 && val == prev)
                val ^= 0x80;
            if (len > n - i)
                len = n - i;
            memset(out + i, val, len);
            i += len;
            prev = val;
        }
        return FLRL_OK;
    }
    return set_error(FLRL_E_ARG, "flrl_gen_host: unknown kind %d", kind);
}

// Error word of a device call (Ctrl::error in the scratch area; FL and RL).
extern "C" int flrl_scratch_error(const void *d_scratch, void *stream)
{
    if (!d_scratch)
        return set_error(FLRL_E_ARG, "flrl_scratch_error: null scratch");
    Ctrl c;
    FLRL_HIP(hipMemcpyAsync(&c, d_scratch, sizeof(c), hipMemcpyDeviceToHost,
                            static_cast<hipStream_t>(stream)));
    FLRL_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return (int)c.error;
}
