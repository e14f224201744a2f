// flrl_internal.hpp — host-side plumbing shared by the C-ABI translation units:
// thread-local last-error string and HIP status checking that preserves the
// message (the reference re-throws a sliced std::exception and loses it,
// src/fl/fl_gpu.cu:296,401,419).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <atomic>

#include "flrl.h"

namespace flrl {

int set_error(int code, const char *fmt, ...);
void clear_error();

// flrl_time_next_kernel: record this thread's pending start/stop events on `s`
// tightly around a device call's main kernel (no-ops when none are pending).
// Zero `bytes` at device pointer p on stream s (a kernel, also inside graphs).
hipError_t zero_async(void *p, size_t bytes, hipStream_t s);
// The per-call scratch reset (ticket, error word, status granules) of a device
// call: zero_async unless flrl_debug_skip_scratch_resets asked this thread to
// skip it (tests of the kernels' stale-ticket checks).
hipError_t scratch_reset(void *p, size_t bytes, hipStream_t s);
// As scratch_reset for a Ctrl area of head_bytes (a multiple of 16) followed by
// `count` 8-byte status words `stride` bytes apart: only those words are zeroed.
hipError_t scratch_reset_strided(void *p, size_t head_bytes, size_t count, size_t stride, hipStream_t s);
// Raise FLRL_E_* `code` in the scratch's error word from stream s (stream
// ordered, no host sync): errors a device call finds on the host side but
// reports, like the kernels' own, through flrl_scratch_error.
hipError_t raise_error_async(void *scratch, int code, hipStream_t s);

// The decoupled-fallback threshold for a look-back launch: `dflt` ticks
// (s_memrealtime, 100 MHz) unless flrl_debug_lookback_help_us set this thread's.
uint64_t lookback_help_ticks(uint64_t dflt);
// flrl_debug_fail_chunk: true when the streamed file paths should fail chunk c.
bool debug_fail_chunk(size_t c);
// flrl_debug_fail_rank_step: true (once) when this thread's next per-rank call
// should fail at `step` (FLRL_DEBUG_RANK_*).
bool debug_fail_rank_step(int step);

// Host-buffer FL through the pinned chunk pipelines (flrl_stream.hip).
int fl_compress_host(const uint8_t *data, size_t size, flrl_fl_buf *out);
int fl_decompress_host(size_t n, const uint8_t *bits, size_t F, const uint8_t *values, size_t V, uint8_t **out);

void kernel_timing_begin(hipStream_t s);
void kernel_timing_end(hipStream_t s);

inline size_t div_up(size_t a, size_t b) { return (a + b - 1) / b; }
inline size_t round_up(size_t a, size_t b) { return div_up(a, b) * b; }

inline bool aligned16(const void *p) { return ((uintptr_t)p & 15u) == 0; }

#define FLRL_HIP(expr)                                                                         \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return ::flrl::set_error(FLRL_E_HIP, "%s failed: %s (%s:%d)", #expr,               \
                                     hipGetErrorString(e_), __FILE__, __LINE__);                \
    } while (0)

// RAII device allocation for the synchronous host-buffer entry points.
struct DevBuf {
    void *p = nullptr;
    ~DevBuf()
    {
        if (p)
            (void)hipFree(p);
    }
    hipError_t alloc(size_t bytes) { return hipMalloc(&p, bytes ? bytes : 16); }
    template <typename T>
    T *as(size_t byte_off = 0) const
    {
        return reinterpret_cast<T *>(static_cast<uint8_t *>(p) + byte_off);
    }
};

// Compute units of the current device (cached per device): persistent grids.
inline int cu_count()
{
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        dev = 0;
    if (dev >= 0 && dev < 64) {
        const int c = cache[dev].load(std::memory_order_relaxed);
        if (c > 0)
            return c;
    }
    int c = 0;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
        c = 256;
    if (dev >= 0 && dev < 64)
        cache[dev].store(c, std::memory_order_relaxed);
    return c;
}

}  // namespace flrl
