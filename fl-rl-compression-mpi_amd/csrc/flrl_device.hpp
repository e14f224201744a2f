// flrl_device.hpp — gfx950 device helpers shared by the FL and RL kernels:
// dynamic tile tickets, decoupled look-back over 8-byte status granules, wave /
// block scans, tail-guarded 16-byte loads and stores.
//
// Cross-workgroup hand-off follows MI355X_MICROARCH.md "Valid forms", R2: every
// status word is ONE naturally aligned 8-byte granule that carries its own flag
// and payload, stored and loaded with agent-scope relaxed atomics (sc1, L1
// bypass), so no release/acquire fence is needed. Status words are zeroed by a
// hipMemsetAsync before every launch (Guideline 16, "Re-initialise every call").
// Tiles are numbered by an atomic ticket in launch order, so the look-back only
// ever waits on tiles that already hold a ticket (forward progress does not
// depend on dispatch order); every spin is bounded and reports FLRL_E_TIMEOUT.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flrl.h"

namespace flrl {

// Native 16-byte vector (HIP's uint4 is a struct; the nontemporal builtins and
// dwordx4 codegen want a real vector type).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;
constexpr int kThreads = 256;            // 4 waves per workgroup
constexpr int kWaves = kThreads / kWave;
constexpr int kFrame = FLRL_FRAME_LENGTH;

// status granule: bits 63..62 = flag, 61..0 = payload
constexpr uint64_t kFlagA = 1ull << 62;  // tile aggregate published
constexpr uint64_t kFlagP = 2ull << 62;  // inclusive prefix published
constexpr uint64_t kPayload = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 22;

// 16-byte control header at the start of every scratch area.
struct Ctrl {
    uint32_t ticket;   // next tile number
    uint32_t error;    // first FLRL_E_* raised by any workgroup
    uint64_t aux;
};

__device__ __forceinline__ void granule_store(uint64_t *p, uint64_t v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t granule_load(uint64_t *p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void raise_error(Ctrl *c, uint32_t code)
{
    atomicCAS(&c->error, 0u, code);
}

// Take the next tile number; must be called by every thread of the block.
__device__ __forceinline__ uint32_t take_ticket(Ctrl *c, uint32_t *s_slot)
{
    if (threadIdx.x == 0)
        *s_slot = atomicAdd(&c->ticket, 1u);
    __syncthreads();
    return *s_slot;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        v += __shfl_xor(v, o, kWave);
    return v;
}

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v)
{
    const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t t = __shfl_up(v, o, kWave);
        if (lane >= o)
            v += t;
    }
    return v;
}

// Exclusive scan of N small counts held in LDS (s_in, any integer type) into
// s_out. Returns the total to every thread. Requires N % 256 == 0 or N < 256.
// Caller must __syncthreads() before reading s_out and before reusing s_wave.
template <int N, typename TIn>
__device__ __forceinline__ uint32_t block_excl_scan(const TIn *s_in, uint32_t *s_out,
                                                    uint32_t *s_wave)
{
    constexpr int E = N >= kThreads ? N / kThreads : 1;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const bool active = tid * E < N;
    uint32_t vals[E];
    uint32_t sum = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        vals[e] = active ? (uint32_t)s_in[tid * E + e] : 0u;
        sum += vals[e];
    }
    const uint32_t inc = wave_incl_scan_u32(sum);
    if (lane == kWave - 1)
        s_wave[wave] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
        const uint32_t t = s_wave[w];
        before += w < wave ? t : 0u;
        total += t;
    }
    uint32_t run = before + inc - sum;
    if (active) {
#pragma unroll
        for (int e = 0; e < E; ++e) {
            s_out[tid * E + e] = run;
            run += vals[e];
        }
    }
    return total;
}

// Decoupled look-back for an additive u64 scan (payload < 2^62), split in two
// so a caller can publish its aggregate early and resolve its prefix later.
// publish_aggregate: ONE lane stores the tile's aggregate (tile 0 publishes its
// inclusive prefix directly).
__device__ __forceinline__ void publish_aggregate(uint64_t *status, uint32_t tile, uint64_t agg)
{
    granule_store(&status[tile], (tile == 0 ? kFlagP : kFlagA) | agg);
}

// lookback_resolve: called by ONE full wave after publish_aggregate. Sums
// predecessors 64 at a time until it meets an inclusive prefix, publishes the
// tile's inclusive prefix and returns the exclusive prefix (to every lane).
__device__ __noinline__ uint64_t lookback_resolve(uint64_t *status, uint32_t tile, uint64_t agg,
                                                  Ctrl *ctrl)
{
    const int lane = threadIdx.x & (kWave - 1);
    if (tile == 0)
        return 0;
    uint64_t excl = 0;
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0;
    for (;;) {
        const int64_t idx = j - lane;
        uint64_t s;
        for (;;) {
            s = idx >= 0 ? granule_load(&status[idx]) : kFlagP;
            if (!__any((s >> 62) == 0))
                break;
            if (++spins > kSpinLimit) {
                if (lane == 0)
                    raise_error(ctrl, FLRL_E_TIMEOUT);
                return excl;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const unsigned long long pm = __ballot((s >> 62) == 2);
        const int first_p = pm ? __ffsll(pm) - 1 : kWave;
        excl += wave_sum_u64(lane <= first_p ? (s & kPayload) : 0ull);
        if (pm)
            break;
        j -= kWave;
    }
    if (lane == 0)
        granule_store(&status[tile], kFlagP | (excl + agg));
    return excl;
}

// Both halves in one call (ONE full wave).
__device__ __forceinline__ uint64_t lookback_sum(uint64_t *status, uint32_t tile, uint64_t agg,
                                                 Ctrl *ctrl)
{
    if ((threadIdx.x & (kWave - 1)) == 0)
        publish_aggregate(status, tile, agg);
    return lookback_resolve(status, tile, agg, ctrl);
}

// 16-byte load of bytes [o, o+16) of p, zero-filling past n.
__device__ __forceinline__ u32x4 load16_tail(const uint8_t *p, uint64_t o, uint64_t n)
{
    if (o + 16 <= n)
        return *reinterpret_cast<const u32x4 *>(p + o);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (o + i < n)
            w[i >> 2] |= (uint32_t)p[o + i] << (8 * (i & 3));
    return u32x4{w[0], w[1], w[2], w[3]};
}

// 16-byte store of v to bytes [o, o+16) of p, dropping bytes at or past n.
__device__ __forceinline__ void store16_tail(uint8_t *p, uint64_t o, uint64_t n, u32x4 v)
{
    if (o + 16 <= n) {
        *reinterpret_cast<u32x4 *>(p + o) = v;
        return;
    }
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (o + i < n)
            p[o + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

}  // namespace flrl
