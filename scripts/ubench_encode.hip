// ubench_encode.hip — tuning harness (not product code): times FL-encode kernel
// variants and plain copy kernels on one 1 GiB u8 buffer, interleaved in one
// process (cdna_hip_programming.md §5.4 rule 24), with ablation switches to
// find what bounds the encode:
//   MODE & 1  no look-back (base = tile * TB/16: exact for u8 input, all b = 8)
//   MODE & 2  no value stores
//   MODE & 4  no packing (LDS staging not written)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include -I <pkg>/csrc \
//          scripts/ubench_encode.hip -o /tmp/ubench_encode
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "flrl_device.hpp"

using namespace flrl;

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                      \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

__device__ __forceinline__ uint64_t pack8(uint64_t x, uint32_t b)
{
    const uint64_t y = (x & 0x00FF00FF00FF00FFull) | ((x & 0xFF00FF00FF00FF00ull) >> (8 - b));
    const uint64_t z = (y & 0x0000FFFF0000FFFFull) | ((y & 0xFFFF0000FFFF0000ull) >> (16 - 2 * b));
    return (z & 0xFFFFFFFFull) | ((z >> 32) << (4 * b));
}

__device__ __forceinline__ void stage_packed(uint8_t *s, uint32_t off, uint32_t b, uint64_t lo,
                                             uint64_t hi)
{
    if (b == 8) {
        *reinterpret_cast<u32x4 *>(s + off) =
            u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
    } else if (b == 4) {
        *reinterpret_cast<uint64_t *>(s + off) = lo;
    } else {
        uint16_t *d = reinterpret_cast<uint16_t *>(s + off);
#pragma unroll
        for (int i = 0; i < 7; ++i)
            if (i < (int)b)
                d[i] = (uint16_t)((i < 4 ? lo >> (16 * i) : hi >> (16 * (i - 4))) & 0xFFFFu);
    }
}

__device__ unsigned long long g_steps, g_spins, g_calls;

// lookback_resolve with counters (diagnostic build only)
__device__ __forceinline__ uint64_t lookback_counted(uint64_t *status, uint32_t tile, uint64_t agg,
                                                     Ctrl *ctrl)
{
    const int lane = threadIdx.x & (kWave - 1);
    if (tile == 0)
        return 0;
    uint64_t excl = 0;
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0, steps = 0;
    for (;;) {
        const int64_t idx = j - lane;
        uint64_t s;
        for (;;) {
            s = idx >= 0 ? granule_load(&status[idx]) : kFlagP;
            if (window_ready(s))
                break;
            ++spins;
            __builtin_amdgcn_s_sleep(1);
        }
        ++steps;
        const unsigned long long pm = __ballot((s >> 62) == 2);
        const int first_p = pm ? __ffsll(pm) - 1 : kWave;
        excl += wave_sum_u64(lane <= first_p ? (s & kPayload) : 0ull);
        if (pm)
            break;
        j -= kWave;
    }
    if (lane == 0) {
        granule_store(&status[tile], kFlagP | (excl + agg));
        atomicAdd(&g_steps, steps);
        atomicAdd(&g_spins, spins);
        atomicAdd(&g_calls, 1ull);
    }
    return excl;
}

template <int ITEMS, int MODE, int BPC>
__global__ __launch_bounds__(kThreads, BPC) void enc_block(const uint8_t *__restrict__ in,
                                                           uint64_t n, uint32_t ntiles,
                                                           uint8_t *__restrict__ bits,
                                                           uint8_t *__restrict__ values,
                                                           Ctrl *ctrl, uint64_t *status)
{
    constexpr int TB = kThreads * 16 * ITEMS;
    constexpr int TF = TB / 128;
    __shared__ u32x4 s_out[TB / 16];
    __shared__ u32x4 s_w4[TF / 16];
    __shared__ uint32_t s_pref[TF];
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_next;
    __shared__ uint64_t s_base;
    uint8_t *s_w = reinterpret_cast<uint8_t *>(s_w4);
    uint8_t *s_out_b = reinterpret_cast<uint8_t *>(s_out);
    const int tid = threadIdx.x;
    const int wave = tid / kWave;
    if (tid == 0)
        s_next = atomicAdd(&ctrl->ticket, 1u);
    __syncthreads();
    uint32_t tile = s_next;
    if (tile >= ntiles)
        return;
    u32x4 a[ITEMS];
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)tile * TB);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            a[k] = __builtin_nontemporal_load(src + k * kThreads + tid);
    }
    for (;;) {
        __syncthreads();
        if (tid == 0)
            s_next = atomicAdd(&ctrl->ticket, 1u);
        const uint64_t frame0 = (uint64_t)tile * TF;
        uint32_t bw[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t o = a[k].x | a[k].y | a[k].z | a[k].w;
            o |= o >> 16;
            o |= o >> 8;
            o = or_8lanes(o & 0xFFu);
            const uint32_t b = o ? 32u - __clz(o) : 1u;
            bw[k] = b;
            if ((tid & 7) == 0)
                s_w[k * (kThreads / 8) + (tid >> 3)] = (uint8_t)b;
        }
        __syncthreads();
        const uint32_t nxt = s_next;
        const uint32_t agg = block_excl_scan<TF>(s_w, s_pref, s_wave);
        __syncthreads();
        if (!(MODE & 1) && tid == 0)
            publish_aggregate(status, tile, agg);
        // MODE & 8: issue the first look-back probe now, before the pack and the
        // prefetch, so its result does not queue behind the prefetch loads
        uint64_t probe = 0;
        if ((MODE & 8) && wave == 0 && tile > 0) {
            const int64_t idx = (int64_t)tile - 1 - (tid & 63);
            probe = idx >= 0 ? granule_load(&status[idx]) : kFlagP;
        }
        for (int i = tid; i < TF / 16; i += kThreads)
            reinterpret_cast<u32x4 *>(bits + frame0)[i] = s_w4[i];
        if (!(MODE & 4)) {
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                const uint32_t b = bw[k];
                const int ft = k * (kThreads / 8) + (tid >> 3);
                const uint32_t off = 16u * s_pref[ft] + 2u * b * (uint32_t)(tid & 7);
                const uint64_t x0 = ((uint64_t)a[k].y << 32) | a[k].x;
                const uint64_t x1 = ((uint64_t)a[k].w << 32) | a[k].z;
                uint64_t lo = x0, hi = x1;
                if (b != 8) {
                    const uint64_t p0 = pack8(x0, b), p1 = pack8(x1, b);
                    lo = p0 | (p1 << (8 * b));
                    hi = p1 >> (64 - 8 * b);
                }
                stage_packed(s_out_b, off, b, lo, hi);
            }
        } else {
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < ITEMS; ++k)
                acc ^= a[k].x ^ a[k].w;
            if (acc == 0x12345678u)
                s_out[tid] = a[0];
        }
        const bool more = nxt < ntiles;
        if (more) {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)nxt * TB);
#pragma unroll
            for (int k = 0; k < ITEMS; ++k)
                a[k] = __builtin_nontemporal_load(src + k * kThreads + tid);
        }
        if (wave == 0) {
            uint64_t excl;
            if (MODE & 1)
                excl = (uint64_t)tile * (TB / 16);
            else if (MODE & 8)
                excl = lookback_resolve_probed(status, tile, agg, ctrl, probe);
            else if (MODE & 16)
                excl = lookback_counted(status, tile, agg, ctrl);
            else
                excl = lookback_resolve(status, tile, agg, ctrl);
            if (tid == 0)
                s_base = excl;
        }
        __syncthreads();
        if (!(MODE & 2)) {
            u32x4 *dst = reinterpret_cast<u32x4 *>(values) + s_base;
            for (uint32_t c = tid; c < agg; c += kThreads)
                __builtin_nontemporal_store(s_out[c], dst + c);
        }
        if (!more)
            break;
        tile = nxt;
    }
}


// Lag-1 variant: tile t's look-back is resolved and its packed bytes stored at
// the START of the next iteration, one full iteration after its aggregate was
// published (predecessors have long published by then).
template <int ITEMS, int MODE, int BPC>
__global__ __launch_bounds__(kThreads, BPC) void enc_lag(const uint8_t *__restrict__ in,
                                                         uint64_t n, uint32_t ntiles,
                                                         uint8_t *__restrict__ bits,
                                                         uint8_t *__restrict__ values,
                                                         Ctrl *ctrl, uint64_t *status)
{
    constexpr int TB = kThreads * 16 * ITEMS;
    constexpr int TF = TB / 128;
    __shared__ u32x4 s_out[TB / 16];
    __shared__ u32x4 s_w4[TF / 16];
    __shared__ uint32_t s_pref[TF];
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_next;
    __shared__ uint64_t s_base;
    uint8_t *s_w = reinterpret_cast<uint8_t *>(s_w4);
    uint8_t *s_out_b = reinterpret_cast<uint8_t *>(s_out);
    const int tid = threadIdx.x;
    const int wave = tid / kWave;
    if (tid == 0)
        s_next = atomicAdd(&ctrl->ticket, 1u);
    __syncthreads();
    uint32_t tile = s_next;
    if (tile >= ntiles)
        return;
    u32x4 a[ITEMS];
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)tile * TB);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            a[k] = __builtin_nontemporal_load(src + k * kThreads + tid);
    }
    uint32_t prev = 0xFFFFFFFFu, agg_prev = 0;
    for (;;) {
        __syncthreads();
        if (tid == 0)
            s_next = atomicAdd(&ctrl->ticket, 1u);
        // ---- finish the previous tile: resolve its offset, store it
        if (prev != 0xFFFFFFFFu) {
            if (wave == 0) {
                const uint64_t e = (MODE & 1) ? (uint64_t)prev * (TB / 16)
                                              : lookback_resolve(status, prev, agg_prev, ctrl);
                if (tid == 0)
                    s_base = e;
            }
            __syncthreads();
            if (!(MODE & 2)) {
                u32x4 *dst = reinterpret_cast<u32x4 *>(values) + s_base;
                for (uint32_t c = tid; c < agg_prev; c += kThreads)
                    __builtin_nontemporal_store(s_out[c], dst + c);
            }
            __syncthreads();
        }
        // ---- this tile: widths, scan, publish, pack
        const uint64_t frame0 = (uint64_t)tile * TF;
        uint32_t bw[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t o = a[k].x | a[k].y | a[k].z | a[k].w;
            o |= o >> 16;
            o |= o >> 8;
            o = or_8lanes(o & 0xFFu);
            const uint32_t b = o ? 32u - __clz(o) : 1u;
            bw[k] = b;
            if ((tid & 7) == 0)
                s_w[k * (kThreads / 8) + (tid >> 3)] = (uint8_t)b;
        }
        __syncthreads();
        const uint32_t nxt = s_next;
        const uint32_t agg = block_excl_scan<TF>(s_w, s_pref, s_wave);
        __syncthreads();
        if (!(MODE & 1) && tid == 0)
            publish_aggregate(status, tile, agg);
        for (int i = tid; i < TF / 16; i += kThreads)
            reinterpret_cast<u32x4 *>(bits + frame0)[i] = s_w4[i];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t b = bw[k];
            const int ft = k * (kThreads / 8) + (tid >> 3);
            const uint32_t off = 16u * s_pref[ft] + 2u * b * (uint32_t)(tid & 7);
            const uint64_t x0 = ((uint64_t)a[k].y << 32) | a[k].x;
            const uint64_t x1 = ((uint64_t)a[k].w << 32) | a[k].z;
            uint64_t lo = x0, hi = x1;
            if (b != 8) {
                const uint64_t p0 = pack8(x0, b), p1 = pack8(x1, b);
                lo = p0 | (p1 << (8 * b));
                hi = p1 >> (64 - 8 * b);
            }
            stage_packed(s_out_b, off, b, lo, hi);
        }
        prev = tile;
        agg_prev = agg;
        if (nxt >= ntiles)
            break;
        {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)nxt * TB);
#pragma unroll
            for (int k = 0; k < ITEMS; ++k)
                a[k] = __builtin_nontemporal_load(src + k * kThreads + tid);
        }
        tile = nxt;
    }
    // drain the last tile
    __syncthreads();
    if (wave == 0) {
        const uint64_t e = (MODE & 1) ? (uint64_t)prev * (TB / 16)
                                      : lookback_resolve(status, prev, agg_prev, ctrl);
        if (tid == 0)
            s_base = e;
    }
    __syncthreads();
    if (!(MODE & 2)) {
        u32x4 *dst = reinterpret_cast<u32x4 *>(values) + s_base;
        for (uint32_t c = tid; c < agg_prev; c += kThreads)
            __builtin_nontemporal_store(s_out[c], dst + c);
    }
}


// Direct-store variant: no LDS output staging. Each lane stores its 2b packed
// bytes straight from registers at 16*(base+pref) + 2b*j with the widest store
// its alignment allows; LDS holds only widths/prefixes, so BPC workgroups fit.
__device__ __forceinline__ void store_packed(uint8_t *dst, uint32_t b, uint64_t lo, uint64_t hi)
{
    if (b == 8) {
        __builtin_nontemporal_store(
            u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)},
            reinterpret_cast<u32x4 *>(dst));
    } else if (b == 4) {
        __builtin_nontemporal_store(lo, reinterpret_cast<uint64_t *>(dst));
    } else if ((b & 1) == 0) {
        uint32_t *d = reinterpret_cast<uint32_t *>(dst);
        d[0] = (uint32_t)lo;
        if (b == 6) {
            d[1] = (uint32_t)(lo >> 32);
            d[2] = (uint32_t)hi;
        }
    } else {
        uint16_t *d = reinterpret_cast<uint16_t *>(dst);
#pragma unroll
        for (int i = 0; i < 7; ++i)
            if (i < (int)b)
                d[i] = (uint16_t)((i < 4 ? lo >> (16 * i) : hi >> (16 * (i - 4))) & 0xFFFFu);
    }
}

template <int ITEMS, int MODE, int BPC>
__global__ __launch_bounds__(kThreads, BPC) void enc_direct(const uint8_t *__restrict__ in,
                                                            uint64_t n, uint32_t ntiles,
                                                            uint8_t *__restrict__ bits,
                                                            uint8_t *__restrict__ values,
                                                            Ctrl *ctrl, uint64_t *status)
{
    constexpr int TB = kThreads * 16 * ITEMS;
    constexpr int TF = TB / 128;
    __shared__ u32x4 s_w4[TF / 16];
    __shared__ uint32_t s_pref[TF];
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_base;
    uint8_t *s_w = reinterpret_cast<uint8_t *>(s_w4);
    const int tid = threadIdx.x;
    const int wave = tid / kWave;
    for (;;) {
        if (tid == 0)
            s_tile = atomicAdd(&ctrl->ticket, 1u);
        __syncthreads();
        const uint32_t tile = s_tile;
        if (tile >= ntiles)
            return;
        u32x4 a[ITEMS];
        const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)tile * TB);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            a[k] = __builtin_nontemporal_load(src + k * kThreads + tid);
        const uint64_t frame0 = (uint64_t)tile * TF;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t o = a[k].x | a[k].y | a[k].z | a[k].w;
            o |= o >> 16;
            o |= o >> 8;
            o = or_8lanes(o & 0xFFu);
            const uint32_t b = o ? 32u - __clz(o) : 1u;
            if ((tid & 7) == 0)
                s_w[k * (kThreads / 8) + (tid >> 3)] = (uint8_t)b;
        }
        __syncthreads();
        const uint32_t agg = block_excl_scan<TF>(s_w, s_pref, s_wave);
        __syncthreads();
        if (wave == 0) {
            uint64_t e;
            if (MODE & 1) {
                e = (uint64_t)tile * (TB / 16);
            } else {
                if (tid == 0)
                    publish_aggregate(status, tile, agg);
                e = lookback_resolve(status, tile, agg, ctrl);
            }
            if (tid == 0)
                s_base = e;
        }
        for (int i = tid; i < TF / 16; i += kThreads)
            reinterpret_cast<u32x4 *>(bits + frame0)[i] = s_w4[i];
        __syncthreads();
        const uint64_t base = s_base;
        if (!(MODE & 2)) {
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                const int ft = k * (kThreads / 8) + (tid >> 3);
                const uint32_t b = s_w[ft];
                const uint64_t x0 = ((uint64_t)a[k].y << 32) | a[k].x;
                const uint64_t x1 = ((uint64_t)a[k].w << 32) | a[k].z;
                uint64_t lo = x0, hi = x1;
                if (b != 8) {
                    const uint64_t p0 = pack8(x0, b), p1 = pack8(x1, b);
                    lo = p0 | (p1 << (8 * b));
                    hi = p1 >> (64 - 8 * b);
                }
                store_packed(values + 16ull * (base + s_pref[ft]) + 2u * b * (tid & 7), b, lo, hi);
            }
        }
        __syncthreads();  // s_tile / LDS reuse
    }
}


template <int N, int T>
__device__ __forceinline__ uint32_t blk_scan(const uint8_t *s_in, uint32_t *s_out, uint32_t *s_wave)
{
    constexpr int E = N / T;
    constexpr int W = T / kWave;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid / 64;
    uint32_t vals[E], sum = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        vals[e] = s_in[tid * E + e];
        sum += vals[e];
    }
    const uint32_t inc = wave_incl_scan_u32(sum);
    if (lane == 63)
        s_wave[wave] = inc;
    __syncthreads();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        const uint32_t t = s_wave[w];
        before += w < wave ? t : 0u;
        total += t;
    }
    uint32_t run = before + inc - sum;
#pragma unroll
    for (int e = 0; e < E; ++e) {
        s_out[tid * E + e] = run;
        run += vals[e];
    }
    return total;
}

// enc_block generalised to T threads per workgroup (LDS-staged, prefetching)
__device__ unsigned long long g_ph[8];

__device__ __forceinline__ uint64_t stamp()
{
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}

template <int T, int ITEMS, int MODE, int BPC>
__global__ __launch_bounds__(T, BPC) void enc_blockT(const uint8_t *__restrict__ in, uint64_t n,
                                                     uint32_t ntiles, uint8_t *__restrict__ bits,
                                                     uint8_t *__restrict__ values, Ctrl *ctrl,
                                                     uint64_t *status)
{
    constexpr int TB = T * 16 * ITEMS;
    constexpr int TF = TB / 128;
    __shared__ u32x4 s_out[TB / 16];
    __shared__ u32x4 s_w4[TF / 16];
    __shared__ uint32_t s_pref[TF];
    __shared__ uint32_t s_wave[T / 64];
    __shared__ uint32_t s_next;
    __shared__ uint64_t s_base;
    uint8_t *s_w = reinterpret_cast<uint8_t *>(s_w4);
    uint8_t *s_out_b = reinterpret_cast<uint8_t *>(s_out);
    const int tid = threadIdx.x;
    const int wave = tid / kWave;
    if (tid == 0)
        s_next = atomicAdd(&ctrl->ticket, 1u);
    __syncthreads();
    uint32_t tile = s_next;
    if (tile >= ntiles)
        return;
    u32x4 a[ITEMS];
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)tile * TB);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            a[k] = __builtin_nontemporal_load(src + k * T + tid);
    }
    uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
    uint64_t t0 = 0, t1;
    for (;;) {
        __syncthreads();
        if (MODE & 64) { __builtin_amdgcn_sched_barrier(0); t1 = stamp(); if (t0) ph[5] += t1 - t0; t0 = t1; __builtin_amdgcn_sched_barrier(0); }
        if (tid == 0)
            s_next = atomicAdd(&ctrl->ticket, 1u);
        const uint64_t frame0 = (uint64_t)tile * TF;
        uint32_t bw[ITEMS];
        if (MODE & 64) {
            uint32_t acc = 0;
#pragma unroll
            for (int k = 0; k < ITEMS; ++k)
                acc |= a[k].x;
            asm volatile("" ::"v"(acc));
            __builtin_amdgcn_sched_barrier(0); t1 = stamp(); ph[0] += t1 - t0; t0 = t1; __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t o = a[k].x | a[k].y | a[k].z | a[k].w;
            o |= o >> 16;
            o |= o >> 8;
            o = or_8lanes(o & 0xFFu);
            const uint32_t b = o ? 32u - __clz(o) : 1u;
            bw[k] = b;
            if ((tid & 7) == 0)
                s_w[k * (T / 8) + (tid >> 3)] = (uint8_t)b;
        }
        __syncthreads();
        const uint32_t nxt = s_next;
        const uint32_t agg = blk_scan<TF, T>(s_w, s_pref, s_wave);
        __syncthreads();
        if (MODE & 64) { __builtin_amdgcn_sched_barrier(0); t1 = stamp(); ph[1] += t1 - t0; t0 = t1; __builtin_amdgcn_sched_barrier(0); }
        if (!(MODE & 1) && tid == 0)
            publish_aggregate(status, tile, agg);
        for (int i = tid; i < TF / 16; i += T)
            reinterpret_cast<u32x4 *>(bits + frame0)[i] = s_w4[i];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t b = bw[k];
            const int ft = k * (T / 8) + (tid >> 3);
            const uint32_t off = 16u * s_pref[ft] + 2u * b * (uint32_t)(tid & 7);
            const uint64_t x0 = ((uint64_t)a[k].y << 32) | a[k].x;
            const uint64_t x1 = ((uint64_t)a[k].w << 32) | a[k].z;
            uint64_t lo = x0, hi = x1;
            if (b != 8) {
                const uint64_t p0 = pack8(x0, b), p1 = pack8(x1, b);
                lo = p0 | (p1 << (8 * b));
                hi = p1 >> (64 - 8 * b);
            }
            stage_packed(s_out_b, off, b, lo, hi);
        }
        if (MODE & 64) { __builtin_amdgcn_sched_barrier(0); t1 = stamp(); ph[2] += t1 - t0; t0 = t1; __builtin_amdgcn_sched_barrier(0); }
        const bool more = nxt < ntiles;
        // MODE & 32: the look-back wave (wave 0) issues its prefetch only after
        // resolving, so its status loads never queue behind its own bulk loads
        const bool late = (MODE & 32) && wave == 0;
        if (more && !late) {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)nxt * TB);
#pragma unroll
            for (int k = 0; k < ITEMS; ++k)
                a[k] = __builtin_nontemporal_load(src + k * T + tid);
        }
        if (wave == 0) {
            const uint64_t excl = (MODE & 1) ? (uint64_t)tile * (TB / 16)
                                             : lookback_resolve(status, tile, agg, ctrl);
            if (tid == 0)
                s_base = excl;
            if (more && late) {
                const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)nxt * TB);
#pragma unroll
                for (int k = 0; k < ITEMS; ++k)
                    a[k] = __builtin_nontemporal_load(src + k * T + tid);
            }
        }
        __syncthreads();
        if (MODE & 64) { __builtin_amdgcn_sched_barrier(0); t1 = stamp(); ph[3] += t1 - t0; t0 = t1; __builtin_amdgcn_sched_barrier(0); }
        u32x4 *dst = reinterpret_cast<u32x4 *>(values) + s_base;
        if (MODE & 128) {  // static trip count: LDS reads hoisted, stores predicated
            u32x4 o[ITEMS];
#pragma unroll
            for (int k = 0; k < ITEMS; ++k)
                o[k] = s_out[k * T + tid];
#pragma unroll
            for (int k = 0; k < ITEMS; ++k)
                if ((uint32_t)(k * T + tid) < agg)
                    __builtin_nontemporal_store(o[k], dst + k * T + tid);
        } else {
            for (uint32_t c = tid; c < agg; c += T)
                __builtin_nontemporal_store(s_out[c], dst + c);
        }
        if (MODE & 64) { __builtin_amdgcn_sched_barrier(0); t1 = stamp(); ph[4] += t1 - t0; t0 = t1; __builtin_amdgcn_sched_barrier(0); }
        if (!more)
            break;
        tile = nxt;
    }
    if ((MODE & 64) && (tid == 0 || tid == 64)) {
        const int o = tid == 0 ? 0 : 0;
        (void)o;
        if (tid == 0)
            for (int i = 0; i < 6; ++i)
                atomicAdd(&g_ph[i], ph[i]);
    }
}


// 256-tile look-back window: lane l, slot q holds the status of tile j - (64q + l).
struct Win4 {
    uint64_t s[4];
};

__device__ __forceinline__ Win4 probe4(uint64_t *status, int64_t j)
{
    const int lane = threadIdx.x & 63;
    Win4 w;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int64_t idx = j - (64 * q + lane);
        w.s[q] = idx >= 0 ? granule_load(&status[idx]) : kFlagP;
    }
    return w;
}

// Resolve an exclusive prefix from a 256-wide window; returns true when done.
__device__ __forceinline__ bool consume4(const Win4 &w, uint64_t &excl)
{
    const int lane = threadIdx.x & 63;
    unsigned long long xm[4], pm[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        xm[q] = __ballot((w.s[q] >> 62) == 0);
        pm[q] = __ballot((w.s[q] >> 62) == 2);
    }
    int qp = 4;
#pragma unroll
    for (int q = 3; q >= 0; --q)
        if (pm[q])
            qp = q;
    // readiness: no X before the nearest P (or anywhere if no P)
    for (int q = 0; q < 4; ++q) {
        if (q < qp && xm[q])
            return false;
        if (q == qp) {
            const unsigned long long upto = pm[q] & (~pm[q] + 1);
            if (xm[q] & ((upto << 1) - 1))
                return false;
        }
    }
    uint64_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if (q < qp)
            v += w.s[q] & kPayload;
        else if (q == qp) {
            const int fp = __ffsll(pm[q]) - 1;
            v += lane <= fp ? (w.s[q] & kPayload) : 0ull;
        }
    }
    excl += wave_sum_u64(v);
    return qp < 4;
}

template <int T, int ITEMS, int MODE>
__global__ __launch_bounds__(T, 1) void enc_lag2(const uint8_t *__restrict__ in, uint64_t n,
                                                 uint32_t ntiles, uint8_t *__restrict__ bits,
                                                 uint8_t *__restrict__ values, Ctrl *ctrl,
                                                 uint64_t *status)
{
    constexpr int TB = T * 16 * ITEMS;
    constexpr int TF = TB / 128;
    __shared__ u32x4 s_out[2][TB / 16];
    __shared__ u32x4 s_w4[TF / 16];
    __shared__ uint32_t s_pref[TF];
    __shared__ uint32_t s_wave[T / 64];
    __shared__ uint32_t s_t[3];
    __shared__ uint64_t s_base;
    uint8_t *s_w = reinterpret_cast<uint8_t *>(s_w4);
    const int tid = threadIdx.x;
    const int wave = tid / kWave;
    if (tid == 0) {
        s_t[0] = atomicAdd(&ctrl->ticket, 1u);
        s_t[1] = atomicAdd(&ctrl->ticket, 1u);
    }
    __syncthreads();
    uint32_t cur = s_t[0], nxt = s_t[1];
    if (cur >= ntiles)
        return;
    u32x4 a[ITEMS];
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)cur * TB);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            a[k] = __builtin_nontemporal_load(src + k * T + tid);
    }
    uint32_t prev = 0xFFFFFFFFu, agg_prev = 0, last_buf = 0;
    Win4 w{};
    for (uint32_t it = 0;; ++it) {
        // (a) probe for the previous tile, before any bulk load of this iteration
        if (wave == 0 && prev != 0xFFFFFFFFu && prev > 0)
            w = probe4(status, (int64_t)prev - 1);
        if (tid == 0)
            s_t[(it + 2) % 3] = nxt < ntiles ? atomicAdd(&ctrl->ticket, 1u) : 0xFFFFFFFFu;
        // (b) widths, scan, publish this tile
        const uint64_t frame0 = (uint64_t)cur * TF;
        uint32_t bw[ITEMS];
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t o = a[k].x | a[k].y | a[k].z | a[k].w;
            o |= o >> 16;
            o |= o >> 8;
            o = or_8lanes(o & 0xFFu);
            const uint32_t b = o ? 32u - __clz(o) : 1u;
            bw[k] = b;
            if ((tid & 7) == 0)
                s_w[k * (T / 8) + (tid >> 3)] = (uint8_t)b;
        }
        __syncthreads();
        const uint32_t agg = blk_scan<TF, T>(s_w, s_pref, s_wave);
        __syncthreads();
        if (tid == 0)
            publish_aggregate(status, cur, agg);
        for (int i = tid; i < TF / 16; i += T)
            reinterpret_cast<u32x4 *>(bits + frame0)[i] = s_w4[i];
        // (c) pack into this iteration's staging buffer
        uint8_t *ob = reinterpret_cast<uint8_t *>(s_out[it & 1]);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t b = bw[k];
            const int ft = k * (T / 8) + (tid >> 3);
            const uint32_t off = 16u * s_pref[ft] + 2u * b * (uint32_t)(tid & 7);
            const uint64_t x0 = ((uint64_t)a[k].y << 32) | a[k].x;
            const uint64_t x1 = ((uint64_t)a[k].w << 32) | a[k].z;
            uint64_t lo = x0, hi = x1;
            if (b != 8) {
                const uint64_t p0 = pack8(x0, b), p1 = pack8(x1, b);
                lo = p0 | (p1 << (8 * b));
                hi = p1 >> (64 - 8 * b);
            }
            stage_packed(ob, off, b, lo, hi);
        }
        // (d) prefetch the next tile (wave 0 after its look-back)
        const bool more = nxt < ntiles;
        if (more && wave != 0) {
            const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)nxt * TB);
#pragma unroll
            for (int k = 0; k < ITEMS; ++k)
                a[k] = __builtin_nontemporal_load(src + k * T + tid);
        }
        // (e) resolve + store the previous tile
        if (wave == 0) {
            if (prev != 0xFFFFFFFFu) {
                uint64_t excl = 0;
                if (prev > 0) {
                    int64_t j = (int64_t)prev - 1;
                    uint32_t spins = 0;
                    for (;;) {
                        uint64_t part = 0;
                        if (consume4(w, part)) {
                            excl += part;
                            break;
                        }
                        // not ready or no P in 256: if ready-without-P, advance the window
                        bool ready_nop = true;
                        for (int q = 0; q < 4; ++q)
                            ready_nop &= __ballot((w.s[q] >> 62) == 0) == 0;
                        if (ready_nop) {
                            excl += part;
                            j -= 256;
                        } else if (++spins > kSpinLimit) {
                            raise_error(ctrl, FLRL_E_TIMEOUT);
                            break;
                        } else {
                            __builtin_amdgcn_s_sleep(1);
                        }
                        w = probe4(status, j);
                    }
                }
                if (tid == 0) {
                    granule_store(&status[prev], kFlagP | (excl + agg_prev));
                    s_base = excl;
                }
            }
            if (more) {
                const u32x4 *src = reinterpret_cast<const u32x4 *>(in + (uint64_t)nxt * TB);
#pragma unroll
                for (int k = 0; k < ITEMS; ++k)
                    a[k] = __builtin_nontemporal_load(src + k * T + tid);
            }
        }
        __syncthreads();
        if (prev != 0xFFFFFFFFu) {
            u32x4 *dst = reinterpret_cast<u32x4 *>(values) + s_base;
            const u32x4 *sb = s_out[(it + 1) & 1];
            for (uint32_t c = tid; c < agg_prev; c += T)
                __builtin_nontemporal_store(sb[c], dst + c);
        }
        prev = cur;
        agg_prev = agg;
        last_buf = it & 1;
        if (!more)
            break;
        __syncthreads();
        cur = nxt;
        nxt = s_t[(it + 2) % 3];
    }
    // drain: resolve + store the last tile
    if (wave == 0) {
        uint64_t excl = 0;
        if (prev > 0)
            excl = lookback_resolve(status, prev, agg_prev, ctrl);
        else if (tid == 0)
            granule_store(&status[0], kFlagP | agg_prev);
        if (tid == 0)
            s_base = excl;
    }
    __syncthreads();
    {
        u32x4 *dst = reinterpret_cast<u32x4 *>(values) + s_base;
        const u32x4 *sb = s_out[last_buf];
        for (uint32_t c = tid; c < agg_prev; c += T)
            __builtin_nontemporal_store(sb[c], dst + c);
    }
}

// Plain streaming copy: U 16-B chunks per lane per step, grid-stride.
template <int U, bool NT>
__global__ __launch_bounds__(kThreads) void copy_kernel(const u32x4 *__restrict__ in,
                                                        u32x4 *__restrict__ out, uint64_t nchunks)
{
    const uint64_t stride = (uint64_t)gridDim.x * kThreads * U;
    for (uint64_t base = (uint64_t)blockIdx.x * kThreads * U; base < nchunks; base += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c = base + (uint64_t)u * kThreads + threadIdx.x;
            if (c < nchunks)
                v[u] = NT ? __builtin_nontemporal_load(in + c) : in[c];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t c = base + (uint64_t)u * kThreads + threadIdx.x;
            if (c < nchunks) {
                if (NT)
                    __builtin_nontemporal_store(v[u], out + c);
                else
                    out[c] = v[u];
            }
        }
    }
}

__global__ void gen_u8(uint8_t *out, uint64_t n)
{
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t * 8 < n;
         t += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = 42 + (t + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        *reinterpret_cast<uint64_t *>(out + 8 * t) = z ^ (z >> 31);
    }
}

struct Var {
    const char *name;
    void (*run)(hipStream_t);
    double bytes;
    std::vector<float> ms;
};

static uint8_t *g_in, *g_bits, *g_vals, *g_out, *g_scr;
static uint64_t g_n;
static int g_cus;

template <int ITEMS, int MODE, int BPC>
static void run_enc(hipStream_t s)
{
    constexpr uint64_t TB = kThreads * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)(g_n / TB);
    CK(hipMemsetAsync(g_scr, 0, 16 + 8ull * ntiles, s));
    const uint32_t grid = std::min<uint32_t>(ntiles, BPC * g_cus);
    hipLaunchKernelGGL((enc_block<ITEMS, MODE, BPC>), dim3(grid), dim3(kThreads), 0, s, g_in, g_n,
                       ntiles, g_bits, g_vals, (Ctrl *)g_scr, (uint64_t *)(g_scr + 16));
}

template <int ITEMS, int MODE, int BPC>
static void run_lag(hipStream_t s)
{
    constexpr uint64_t TB = kThreads * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)(g_n / TB);
    CK(hipMemsetAsync(g_scr, 0, 16 + 8ull * ntiles, s));
    const uint32_t grid = std::min<uint32_t>(ntiles, BPC * g_cus);
    hipLaunchKernelGGL((enc_lag<ITEMS, MODE, BPC>), dim3(grid), dim3(kThreads), 0, s, g_in, g_n,
                       ntiles, g_bits, g_vals, (Ctrl *)g_scr, (uint64_t *)(g_scr + 16));
}

template <int ITEMS, int MODE, int BPC>
static void run_direct(hipStream_t s)
{
    constexpr uint64_t TB = kThreads * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)(g_n / TB);
    CK(hipMemsetAsync(g_scr, 0, 16 + 8ull * ntiles, s));
    const uint32_t grid = std::min<uint32_t>(ntiles, BPC * g_cus);
    hipLaunchKernelGGL((enc_direct<ITEMS, MODE, BPC>), dim3(grid), dim3(kThreads), 0, s, g_in,
                       g_n, ntiles, g_bits, g_vals, (Ctrl *)g_scr, (uint64_t *)(g_scr + 16));
}

template <int T, int ITEMS, int MODE, int BPC>
static void run_blockT(hipStream_t s)
{
    constexpr uint64_t TB = T * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)(g_n / TB);
    CK(hipMemsetAsync(g_scr, 0, 16 + 8ull * ntiles, s));
    const uint32_t grid = std::min<uint32_t>(ntiles, BPC * g_cus);
    hipLaunchKernelGGL((enc_blockT<T, ITEMS, MODE, BPC>), dim3(grid), dim3(T), 0, s, g_in, g_n,
                       ntiles, g_bits, g_vals, (Ctrl *)g_scr, (uint64_t *)(g_scr + 16));
}

template <int T, int ITEMS, int MODE>
static void run_lag2(hipStream_t s)
{
    constexpr uint64_t TB = T * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)(g_n / TB);
    CK(hipMemsetAsync(g_scr, 0, 16 + 8ull * ntiles, s));
    const uint32_t grid = std::min<uint32_t>(ntiles, g_cus);
    hipLaunchKernelGGL((enc_lag2<T, ITEMS, MODE>), dim3(grid), dim3(T), 0, s, g_in, g_n, ntiles,
                       g_bits, g_vals, (Ctrl *)g_scr, (uint64_t *)(g_scr + 16));
}

// reference output for correctness checks of the variants
static uint8_t *g_ref;

template <int U, bool NT, int BPC>
static void run_copy(hipStream_t s)
{
    const uint64_t nch = g_n / 16;
    hipLaunchKernelGGL((copy_kernel<U, NT>), dim3(BPC * g_cus), dim3(kThreads), 0, s,
                       (const u32x4 *)g_in, (u32x4 *)g_out, nch);
}

int main(int argc, char **argv)
{
    g_n = 1ull << 30;
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    CK(hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, 0));
    CK(hipMalloc(&g_in, g_n));
    CK(hipMalloc(&g_out, g_n));
    CK(hipMalloc(&g_vals, g_n));
    CK(hipMalloc(&g_bits, g_n / 128));
    CK(hipMalloc(&g_scr, 16 + 8 * (g_n / 8192) + 64));
    hipLaunchKernelGGL(gen_u8, dim3(8192), dim3(256), 0, 0, g_in, g_n);
    CK(hipDeviceSynchronize());
    const double enc_bytes = g_n + g_n / 128 + g_n;  // N + F + V (u8: V = N)
    std::vector<Var> vars = {
        {"copy U4 nt bpc8", run_copy<4, true, 8>, 2.0 * g_n},
        {"copy U4 plain bpc8", run_copy<4, false, 8>, 2.0 * g_n},
        {"copy U8 nt bpc4", run_copy<8, true, 4>, 2.0 * g_n},
        {"copy U16 nt bpc2", run_copy<16, true, 2>, 2.0 * g_n},
        {"enc16 full", run_enc<16, 0, 2>, enc_bytes},
        {"enc16 nolookback", run_enc<16, 1, 2>, enc_bytes},
        {"enc16 nostore", run_enc<16, 2, 2>, enc_bytes},
        {"enc16 nopack", run_enc<16, 4, 2>, enc_bytes},
        {"enc16 nolb+nopack", run_enc<16, 5, 2>, enc_bytes},
        {"enc16 loads only", run_enc<16, 7, 2>, enc_bytes},
        {"blk512x16 bpc1", run_blockT<512, 16, 0, 1>, enc_bytes},
        {"blk512x16 bpc1 late", run_blockT<512, 16, 32, 1>, enc_bytes},
        {"blk512x16 late static", run_blockT<512, 16, 32 + 128, 1>, enc_bytes},

        {"blk256x16 bpc2 static", run_blockT<256, 16, 128, 2>, enc_bytes},
        {"blk512x16 STAMPED static", run_blockT<512, 16, 64 + 32 + 128, 1>, enc_bytes},
        {"blk512x16 static nolb", run_blockT<512, 16, 1 + 128, 1>, enc_bytes},
        
        {"blk512x16 bpc1 nolb", run_blockT<512, 16, 1, 1>, enc_bytes},
        {"blk256x16 bpc2", run_blockT<256, 16, 0, 2>, enc_bytes},
        {"blk256x16 bpc2 late", run_blockT<256, 16, 32, 2>, enc_bytes},
        {"direct32 bpc3", run_direct<32, 0, 3>, enc_bytes},
        {"enc16 counted", run_enc<16, 16, 2>, enc_bytes},
        {"lag2 512x8", run_lag2<512, 8, 0>, enc_bytes},
    };
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < reps + 2; ++r)
        for (auto &v : vars) {
            CK(hipEventRecord(e0, s));
            v.run(s);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2)
                v.ms.push_back(ms);
        }
    CK(hipGetLastError());
    unsigned long long st = 0, sp = 0, ca = 0;
    CK(hipMemcpyFromSymbol(&st, HIP_SYMBOL(g_steps), 8));
    CK(hipMemcpyFromSymbol(&sp, HIP_SYMBOL(g_spins), 8));
    CK(hipMemcpyFromSymbol(&ca, HIP_SYMBOL(g_calls), 8));
    {
        // u8 input: every b = 8, so the packed values must equal the input bytes
        std::vector<uint8_t> h1(1 << 20), h2(1 << 20);
        bool ok = true;
        for (uint64_t off = 0; off < g_n && ok; off += (g_n / 7) & ~((1ull << 20) - 1)) {
            CK(hipMemcpy(h1.data(), g_in + off, 1 << 20, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), g_vals + off, 1 << 20, hipMemcpyDeviceToHost));
            ok = h1 == h2;
        }
        printf("last variant values == input (sampled): %s\n", ok ? "yes" : "NO");
    }
    unsigned long long ph[8];
    CK(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_ph), sizeof(ph)));
    double tot = 0;
    for (int i = 0; i < 6; ++i) tot += ph[i];
    printf("phases (wave 0, %% of cycles; both stamped variants summed): wait-data %.1f  widths+scan %.1f  pack %.1f  prefetch+lookback+barrier %.1f  stores %.1f  loop-top barrier %.1f\n",
           100 * ph[0] / tot, 100 * ph[1] / tot, 100 * ph[2] / tot, 100 * ph[3] / tot, 100 * ph[4] / tot, 100 * ph[5] / tot);
    printf("look-back: calls %llu, window steps/call %.3f, spins/call %.3f\n", ca,
           ca ? (double)st / ca : 0.0, ca ? (double)sp / ca : 0.0);
    for (auto &v : vars) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2];
        printf("%-24s min %.4f med %.4f ms  -> %.0f GB/s (med)\n", v.name, v.ms[0], med,
               v.bytes / (med * 1e-3) / 1e9);
    }
    return 0;
}
