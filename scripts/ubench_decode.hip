// ubench_decode.hip — tuning harness (not product code): FL decode variants on
// the 1 GiB u8 (or lo4) bench input, interleaved in one process with the
// library's decode (memset + fl_offsets_kernel + fl_decode_kernel) and a copy.
//   variant P<T,ITEMS,BPC>: persistent grid-stride workgroups over 16*T*ITEMS-byte
//   output tiles; the tile's packed bytes are prefetched into registers one tile
//   ahead, staged in LDS, unpacked by lane groups that own ITEMS consecutive
//   frames (prefix = register running sum after one wave scan) and stored
//   straight from registers.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include \
//   -I fl-rl-compression-mpi_amd/csrc scripts/ubench_decode.hip \
//   -L fl-rl-compression-mpi_amd/lib -lflrl -Wl,-rpath,$PWD/fl-rl-compression-mpi_amd/lib \
//   -o scripts/ubench_decode.bin
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "flrl.h"
#include "flrl_device.hpp"

using namespace flrl;

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

__device__ __forceinline__ uint64_t unpack8(uint64_t w, uint32_t b)
{
    const uint64_t m4 = (b >= 8) ? 0xFFFFFFFFull : ((1ull << (4 * b)) - 1);
    const uint64_t z = (w & m4) | (((w >> (4 * b)) & m4) << 32);
    const uint64_t m2 = (1ull << (2 * b)) - 1;
    const uint64_t M2 = m2 | (m2 << 32);
    const uint64_t y = (z & M2) | (((z >> (2 * b)) & M2) << 16);
    const uint64_t M1 = ((1ull << b) - 1) * 0x0001000100010001ull;
    return (y & M1) | (((y >> b) & M1) << 8);
}

__device__ __forceinline__ uint32_t clamp_width(uint32_t b) { return b < 1 ? 1u : (b > 8 ? 8u : b); }

template <int ITEMS>
struct WVec;
template <>
struct WVec<16> {
    typedef u32x4 T;
};
template <>
struct WVec<8> {
    typedef uint64_t T;
};
template <>
struct WVec<4> {
    typedef uint32_t T;
};

template <int T, int ITEMS, int NTL = 1>
__device__ __forceinline__ void load_vals(u32x4 (&a)[ITEMS], const uint8_t *values, uint64_t base,
                                          uint32_t agg, uint64_t vsize)
{
    const int tid = threadIdx.x;
    const u32x4 *src = reinterpret_cast<const u32x4 *>(values) + base;
    if (16ull * (base + agg) <= vsize) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            if ((uint32_t)(k * T + tid) < agg)
                a[k] = NTL ? __builtin_nontemporal_load(src + k * T + tid) : src[k * T + tid];
    } else {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            if ((uint32_t)(k * T + tid) < agg)
                a[k] = load16_tail(values, 16ull * (base + k * T + tid), vsize);
    }
}

// widths of a lane group's ITEMS frames (group = tid/8), zero past nframes
template <int ITEMS>
__device__ __forceinline__ typename WVec<ITEMS>::T load_w(const uint8_t *bits, uint64_t f0,
                                                          uint64_t nframes)
{
    typedef typename WVec<ITEMS>::T V;
    if (f0 + ITEMS <= nframes)
        return *reinterpret_cast<const V *>(bits + f0);
    V v{};
    uint8_t *p = reinterpret_cast<uint8_t *>(&v);
    for (int i = 0; i < ITEMS; ++i)
        p[i] = f0 + i < nframes ? bits[f0 + i] : 0;
    return v;
}

template <int ITEMS>
__device__ __forceinline__ uint32_t wbyte(const typename WVec<ITEMS>::T &v, int k)
{
    if constexpr (ITEMS == 16)
        return (v[k >> 2] >> (8 * (k & 3))) & 0xFFu;
    else
        return (uint32_t)((uint64_t)v >> (8 * k)) & 0xFFu;
}

template <int T, int ITEMS, int BPC>
__global__ __launch_bounds__(T, BPC) void dec_p(const uint8_t *__restrict__ bits, uint64_t nframes,
                                                const uint8_t *__restrict__ values, uint64_t vsize,
                                                uint8_t *__restrict__ out, uint64_t n,
                                                const uint64_t *__restrict__ tb, uint32_t stride,
                                                uint32_t ntb, uint32_t ntiles)
{
    constexpr int TB = T * 16 * ITEMS;
    constexpr int TF = TB / kFrame;
    __shared__ u32x4 s_in[TB / 16 + 2];
    __shared__ uint32_t s_wave[T / kWave];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles)
        return;
    auto tbase = [&](uint32_t t) { return tb[(uint64_t)t * stride < ntb ? (uint64_t)t * stride : ntb]; };
    uint64_t base = tbase(tile);
    uint32_t agg = (uint32_t)(tbase(tile + 1) - base);
    u32x4 a[ITEMS];
    load_vals<T, ITEMS>(a, values, base, agg, vsize);
    typename WVec<ITEMS>::T wv = load_w<ITEMS>(bits, (uint64_t)tile * TF + (tid >> 3) * ITEMS, nframes);
    for (;;) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            if ((uint32_t)(k * T + tid) < agg)
                s_in[k * T + tid] = a[k];
        if (tid < 2)
            s_in[agg + tid] = u32x4{0u, 0u, 0u, 0u};
        uint32_t bw[ITEMS];
        uint32_t gtot = 0;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t b = wbyte<ITEMS>(wv, k);
            const uint64_t f = (uint64_t)tile * TF + (tid >> 3) * ITEMS + k;
            b = f < nframes ? clamp_width(b) : 0u;
            bw[k] = b;
            gtot += b;
        }
        const uint32_t gincl = wave_incl_scan_u32((lane & 7) == 0 ? gtot : 0u);
        if (lane == kWave - 1)
            s_wave[wave] = gincl;
        __syncthreads();
        uint32_t wbase = 0;
#pragma unroll
        for (int v = 0; v < T / kWave; ++v)
            wbase += v < wave ? s_wave[v] : 0u;
        // prefetch the next tile
        const uint32_t nxt = tile + gridDim.x;
        const bool more = nxt < ntiles;
        const uint64_t tile_off = (uint64_t)tile * TB;
        if (more) {
            base = tbase(nxt);
            agg = (uint32_t)(tbase(nxt + 1) - base);
            load_vals<T, ITEMS>(a, values, base, agg, vsize);
            wv = load_w<ITEMS>(bits, (uint64_t)nxt * TF + (tid >> 3) * ITEMS, nframes);
        }
        // unpack + store
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s_in);
        const bool full = tile_off + TB <= n;
        uint32_t run = wbase + gincl - gtot;
        uint8_t *dst = out + tile_off + (uint32_t)(tid >> 3) * ITEMS * kFrame + (tid & 7) * 16;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t b = bw[k];
            const uint32_t off = 16u * run + 2u * b * (uint32_t)(tid & 7);
            run += b;
            if (b == 0)
                continue;
            const uint32_t ad = off >> 2;
            const uint64_t w01 = ((uint64_t)s32[ad + 1] << 32) | s32[ad];
            const uint64_t w23 = ((uint64_t)s32[ad + 3] << 32) | s32[ad + 2];
            uint64_t lo = w01, hi = w23;
            if (off & 2) {
                const uint64_t w4 = s32[ad + 4];
                lo = (w01 >> 16) | (w23 << 48);
                hi = (w23 >> 16) | (w4 << 48);
            }
            const uint64_t p1 = b == 8 ? hi : ((lo >> (8 * b)) | (hi << (64 - 8 * b)));
            const uint64_t x0 = unpack8(lo, b);
            const uint64_t x1 = unpack8(p1, b);
            const u32x4 r = u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
            if (full)
                __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(dst + k * kFrame));
            else
                store16_tail(out, (uint64_t)(dst - out) + k * kFrame, n, r);
        }
        if (!more)
            break;
        tile = nxt;
        __syncthreads();  // LDS reuse
    }
}

// PT: P with tiles taken by ticket (in-order progress across workgroups)
template <int T, int ITEMS, int BPC, int NTS = 1, int NTL = 1>
__global__ __launch_bounds__(T, BPC) void dec_pt(const uint8_t *__restrict__ bits, uint64_t nframes,
                                                const uint8_t *__restrict__ values, uint64_t vsize,
                                                uint8_t *__restrict__ out, uint64_t n,
                                                const uint64_t *__restrict__ tb, uint32_t stride,
                                                uint32_t ntb, uint32_t ntiles, Ctrl *ctrl)
{
    constexpr int TB = T * 16 * ITEMS;
    constexpr int TF = TB / kFrame;
    __shared__ u32x4 s_in[TB / 16 + 2];
    __shared__ uint32_t s_wave[T / kWave];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    __shared__ uint32_t s_next;
    if (tid == 0)
        s_next = atomicAdd(&ctrl->ticket, 1u);
    __syncthreads();
    uint32_t tile = s_next;
    if (tile >= ntiles)
        return;
    auto tbase = [&](uint32_t t) { return tb[(uint64_t)t * stride < ntb ? (uint64_t)t * stride : ntb]; };
    uint64_t base = tbase(tile);
    uint32_t agg = (uint32_t)(tbase(tile + 1) - base);
    u32x4 a[ITEMS];
    load_vals<T, ITEMS, NTL>(a, values, base, agg, vsize);
    typename WVec<ITEMS>::T wv = load_w<ITEMS>(bits, (uint64_t)tile * TF + (tid >> 3) * ITEMS, nframes);
    for (;;) {
        if (tid == 0)
            s_next = atomicAdd(&ctrl->ticket, 1u);  // read after the scan barrier
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            if ((uint32_t)(k * T + tid) < agg)
                s_in[k * T + tid] = a[k];
        if (tid < 2)
            s_in[agg + tid] = u32x4{0u, 0u, 0u, 0u};
        uint32_t bw[ITEMS];
        uint32_t gtot = 0;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t b = wbyte<ITEMS>(wv, k);
            const uint64_t f = (uint64_t)tile * TF + (tid >> 3) * ITEMS + k;
            b = f < nframes ? clamp_width(b) : 0u;
            bw[k] = b;
            gtot += b;
        }
        const uint32_t gincl = wave_incl_scan_u32((lane & 7) == 0 ? gtot : 0u);
        if (lane == kWave - 1)
            s_wave[wave] = gincl;
        __syncthreads();
        uint32_t wbase = 0;
#pragma unroll
        for (int v = 0; v < T / kWave; ++v)
            wbase += v < wave ? s_wave[v] : 0u;
        // prefetch the next tile
        const uint32_t nxt = s_next;
        const bool more = nxt < ntiles;
        const uint64_t tile_off = (uint64_t)tile * TB;
        if (more) {
            base = tbase(nxt);
            agg = (uint32_t)(tbase(nxt + 1) - base);
            load_vals<T, ITEMS, NTL>(a, values, base, agg, vsize);
            wv = load_w<ITEMS>(bits, (uint64_t)nxt * TF + (tid >> 3) * ITEMS, nframes);
        }
        // unpack + store
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s_in);
        const bool full = tile_off + TB <= n;
        uint32_t run = wbase + gincl - gtot;
        uint8_t *dst = out + tile_off + (uint32_t)(tid >> 3) * ITEMS * kFrame + (tid & 7) * 16;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t b = bw[k];
            const uint32_t off = 16u * run + 2u * b * (uint32_t)(tid & 7);
            run += b;
            if (b == 0)
                continue;
            const uint32_t ad = off >> 2;
            const uint64_t w01 = ((uint64_t)s32[ad + 1] << 32) | s32[ad];
            const uint64_t w23 = ((uint64_t)s32[ad + 3] << 32) | s32[ad + 2];
            uint64_t lo = w01, hi = w23;
            if (off & 2) {
                const uint64_t w4 = s32[ad + 4];
                lo = (w01 >> 16) | (w23 << 48);
                hi = (w23 >> 16) | (w4 << 48);
            }
            const uint64_t p1 = b == 8 ? hi : ((lo >> (8 * b)) | (hi << (64 - 8 * b)));
            const uint64_t x0 = unpack8(lo, b);
            const uint64_t x1 = unpack8(p1, b);
            const u32x4 r = u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
            if (full)
                if (NTS)
                    __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(dst + k * kFrame));
                else
                    *reinterpret_cast<u32x4 *>(dst + k * kFrame) = r;
            else
                store16_tail(out, (uint64_t)(dst - out) + k * kFrame, n, r);
        }
        if (!more)
            break;
        tile = nxt;
        __syncthreads();  // LDS reuse
    }
}

template <int T, int ITEMS, int BPC, int NTS = 1, int NTL = 1>
// PAIR: one ticket = two consecutive tiles (half the atomics)
__global__ __launch_bounds__(T, BPC) void dec_pt2(const uint8_t *__restrict__ bits, uint64_t nframes,
                                                const uint8_t *__restrict__ values, uint64_t vsize,
                                                uint8_t *__restrict__ out, uint64_t n,
                                                const uint64_t *__restrict__ tb, uint32_t stride,
                                                uint32_t ntb, uint32_t ntiles, Ctrl *ctrl)
{
    constexpr int TB = T * 16 * ITEMS;
    constexpr int TF = TB / kFrame;
    __shared__ u32x4 s_in[TB / 16 + 2];
    __shared__ uint32_t s_wave[T / kWave];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    __shared__ uint32_t s_next;
    if (tid == 0)
        s_next = 2u * atomicAdd(&ctrl->ticket, 1u);
    __syncthreads();
    uint32_t tile = s_next;
    uint32_t pending = tile + 1;
    bool have = true;
    if (tile >= ntiles)
        return;
    auto tbase = [&](uint32_t t) { return tb[(uint64_t)t * stride < ntb ? (uint64_t)t * stride : ntb]; };
    uint64_t base = tbase(tile);
    uint32_t agg = (uint32_t)(tbase(tile + 1) - base);
    u32x4 a[ITEMS];
    load_vals<T, ITEMS, NTL>(a, values, base, agg, vsize);
    typename WVec<ITEMS>::T wv = load_w<ITEMS>(bits, (uint64_t)tile * TF + (tid >> 3) * ITEMS, nframes);
    for (;;) {
        if (tid == 0)
            if (!have)
                s_next = 2u * atomicAdd(&ctrl->ticket, 1u);  // read after the scan barrier
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            if ((uint32_t)(k * T + tid) < agg)
                s_in[k * T + tid] = a[k];
        if (tid < 2)
            s_in[agg + tid] = u32x4{0u, 0u, 0u, 0u};
        uint32_t bw[ITEMS];
        uint32_t gtot = 0;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t b = wbyte<ITEMS>(wv, k);
            const uint64_t f = (uint64_t)tile * TF + (tid >> 3) * ITEMS + k;
            b = f < nframes ? clamp_width(b) : 0u;
            bw[k] = b;
            gtot += b;
        }
        const uint32_t gincl = wave_incl_scan_u32((lane & 7) == 0 ? gtot : 0u);
        if (lane == kWave - 1)
            s_wave[wave] = gincl;
        __syncthreads();
        uint32_t wbase = 0;
#pragma unroll
        for (int v = 0; v < T / kWave; ++v)
            wbase += v < wave ? s_wave[v] : 0u;
        // prefetch the next tile
        const uint32_t nxt = have ? pending : s_next;
        if (!have)
            pending = nxt + 1;
        have = !have;
        const bool more = nxt < ntiles;
        const uint64_t tile_off = (uint64_t)tile * TB;
        if (more) {
            base = tbase(nxt);
            agg = (uint32_t)(tbase(nxt + 1) - base);
            load_vals<T, ITEMS, NTL>(a, values, base, agg, vsize);
            wv = load_w<ITEMS>(bits, (uint64_t)nxt * TF + (tid >> 3) * ITEMS, nframes);
        }
        // unpack + store
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s_in);
        const bool full = tile_off + TB <= n;
        uint32_t run = wbase + gincl - gtot;
        uint8_t *dst = out + tile_off + (uint32_t)(tid >> 3) * ITEMS * kFrame + (tid & 7) * 16;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t b = bw[k];
            const uint32_t off = 16u * run + 2u * b * (uint32_t)(tid & 7);
            run += b;
            if (b == 0)
                continue;
            const uint32_t ad = off >> 2;
            const uint64_t w01 = ((uint64_t)s32[ad + 1] << 32) | s32[ad];
            const uint64_t w23 = ((uint64_t)s32[ad + 3] << 32) | s32[ad + 2];
            uint64_t lo = w01, hi = w23;
            if (off & 2) {
                const uint64_t w4 = s32[ad + 4];
                lo = (w01 >> 16) | (w23 << 48);
                hi = (w23 >> 16) | (w4 << 48);
            }
            const uint64_t p1 = b == 8 ? hi : ((lo >> (8 * b)) | (hi << (64 - 8 * b)));
            const uint64_t x0 = unpack8(lo, b);
            const uint64_t x1 = unpack8(p1, b);
            const u32x4 r = u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
            if (full)
                if (NTS)
                    __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(dst + k * kFrame));
                else
                    *reinterpret_cast<u32x4 *>(dst + k * kFrame) = r;
            else
                store16_tail(out, (uint64_t)(dst - out) + k * kFrame, n, r);
        }
        if (!more)
            break;
        tile = nxt;
        __syncthreads();  // LDS reuse
    }
}

// Non-persistent (the library's shape): one 256-thread workgroup per
// 16*256*ITEMS-byte output tile; DMA = packed bytes by LDS-DMA instead of
// load -> VGPR -> ds_write.
template <int ITEMS, int DMA>
__global__ __launch_bounds__(256) void dec_np(const uint8_t *__restrict__ bits, uint64_t nframes,
                                              const uint8_t *__restrict__ values, uint64_t vsize,
                                              uint8_t *__restrict__ out, uint64_t n,
                                              const uint64_t *__restrict__ tb, uint32_t stride, uint32_t ntb)
{
    constexpr int T = 256;
    constexpr int TB = T * 16 * ITEMS;
    constexpr int TF = TB / kFrame;
    __shared__ u32x4 s_in[TB / 16 + 2];
    __shared__ u32x4 s_w4[(TF + 15) / 16];
    __shared__ uint32_t s_pref[TF];
    __shared__ uint32_t s_wave[kWaves];
    uint8_t *s_w = reinterpret_cast<uint8_t *>(s_w4);
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const uint64_t tile = blockIdx.x;
    const uint64_t tile_off = tile * TB;
    const uint64_t frame0 = tile * TF;
    const uint64_t i0 = tile * stride, i1 = (tile + 1) * stride;
    const uint64_t base = tb[i0 < ntb ? i0 : ntb];
    const uint32_t agg = (uint32_t)(tb[i1 < ntb ? i1 : ntb] - base);
    if (tid < TF / 16) {
        u32x4 w = load16_tail(bits, frame0 + 16 * tid, nframes);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t raw = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            const uint32_t b = frame0 + 16 * tid + i < nframes ? clamp_width(raw) : 0u;
            w[i >> 2] = (w[i >> 2] & ~(0xFFu << (8 * (i & 3)))) | (b << (8 * (i & 3)));
        }
        s_w4[tid] = w;
    }
    const u32x4 *src = reinterpret_cast<const u32x4 *>(values) + base;
    if (16ull * (base + agg) <= vsize) {
        if (DMA) {
#pragma unroll
            for (int k = 0; k < ITEMS; ++k) {
                const uint32_t c = k * T + tid;
                if (c < agg)
                    __builtin_amdgcn_global_load_lds(
                        (const __attribute__((address_space(1))) void *)(src + c),
                        (__attribute__((address_space(3))) void *)(s_in + k * T + wave * 64), 16, 0, 0);
            }
        } else {
            for (uint32_t c = tid; c < agg; c += T)
                s_in[c] = __builtin_nontemporal_load(src + c);
        }
    } else {
        for (uint32_t c = tid; c < agg; c += T)
            s_in[c] = load16_tail(values, 16ull * (base + c), vsize);
    }
    if (tid < 2)
        s_in[agg + tid] = u32x4{0u, 0u, 0u, 0u};
    __syncthreads();
    block_excl_scan<TF>(s_w, s_pref, s_wave);
    __syncthreads();
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s_in);
    const bool full = tile_off + TB <= n;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const int c = k * T + tid;
        const int ft = c >> 3;
        const uint32_t b = s_w[ft];
        if (b == 0)
            continue;
        const uint32_t off = 16u * s_pref[ft] + 2u * b * (uint32_t)(tid & 7);
        const uint32_t a = off >> 2;
        const uint64_t w01 = ((uint64_t)s32[a + 1] << 32) | s32[a];
        const uint64_t w23 = ((uint64_t)s32[a + 3] << 32) | s32[a + 2];
        uint64_t lo = w01, hi = w23;
        if (off & 2) {
            const uint64_t w4 = s32[a + 4];
            lo = (w01 >> 16) | (w23 << 48);
            hi = (w23 >> 16) | (w4 << 48);
        }
        const uint64_t p1 = b == 8 ? hi : ((lo >> (8 * b)) | (hi << (64 - 8 * b)));
        const uint64_t x0 = unpack8(lo, b);
        const uint64_t x1 = unpack8(p1, b);
        const u32x4 r = u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
        if (full)
            __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(out + tile_off) + c);
        else
            store16_tail(out, tile_off + (uint64_t)c * 16, n, r);
    }
}

// Q: P with branch-free loads (no tail paths whose join makes the compiler wait
// for the prefetch): values index clamped to [base, base+agg-1] and to the last
// unit below vsize (bytes past vsize only feed outputs past n); widths loaded
// ITEMS bytes at min(f0, F - ITEMS) and realigned (requires F >= ITEMS).
template <int T, int ITEMS, int BPC>
__global__ __launch_bounds__(T, BPC) void dec_q(const uint8_t *__restrict__ bits, uint64_t nframes,
                                                const uint8_t *__restrict__ values, uint64_t vsize,
                                                uint8_t *__restrict__ out, uint64_t n,
                                                const uint64_t *__restrict__ tb, uint32_t stride,
                                                uint32_t ntb, uint32_t ntiles)
{
    constexpr int TB = T * 16 * ITEMS;
    constexpr int TF = TB / kFrame;
    typedef typename WVec<ITEMS>::T WV;
    __shared__ u32x4 s_in[TB / 16 + 2];
    __shared__ uint32_t s_wave[T / kWave];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    uint32_t tile = blockIdx.x;
    if (tile >= ntiles)
        return;
    if (tid < 2)
        s_in[TB / 16 + tid] = u32x4{0u, 0u, 0u, 0u};
    const u32x4 *v16 = reinterpret_cast<const u32x4 *>(values);
    const uint64_t lastu = (vsize - 1) / 16;
    auto tbase = [&](uint32_t t) { return tb[(uint64_t)t * stride < ntb ? (uint64_t)t * stride : ntb]; };
    auto load = [&](uint32_t t, u32x4 (&a)[ITEMS], WV &wv, uint32_t &agg) {
        const uint64_t base = tbase(t);
        agg = (uint32_t)(tbase(t + 1) - base);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t c = k * T + tid;
            uint64_t u = base + (c < agg ? c : agg - 1);
            u = u < lastu ? u : lastu;
            a[k] = __builtin_nontemporal_load(v16 + u);
        }
        const uint64_t f0 = (uint64_t)t * TF + (tid >> 3) * ITEMS;
        const uint64_t fc = f0 + ITEMS <= nframes ? f0 : nframes - ITEMS;
        wv = *reinterpret_cast<const WV *>(bits + fc);
        if constexpr (ITEMS == 16) {
            // realign is rare (last group only): done in the width loop via index shift
        }
        return (uint32_t)(f0 - fc);
    };
    u32x4 a[ITEMS];
    WV wv;
    uint32_t agg;
    uint32_t sh = load(tile, a, wv, agg);
    for (;;) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t c = k * T + tid;
            s_in[c] = c < agg ? a[k] : u32x4{0u, 0u, 0u, 0u};
        }
        uint32_t bw[ITEMS];
        uint32_t gtot = 0;
        const uint64_t f0 = (uint64_t)tile * TF + (tid >> 3) * ITEMS;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t kk = k + sh < ITEMS ? k + sh : 0;
            uint32_t b = wbyte<ITEMS>(wv, kk);
            b = f0 + k < nframes ? clamp_width(b) : 0u;
            bw[k] = b;
            gtot += b;
        }
        const uint32_t gincl = wave_incl_scan_u32((lane & 7) == 0 ? gtot : 0u);
        if (lane == kWave - 1)
            s_wave[wave] = gincl;
        __syncthreads();
        uint32_t wbase = 0;
#pragma unroll
        for (int v = 0; v < T / kWave; ++v)
            wbase += v < wave ? s_wave[v] : 0u;
        const uint32_t nxt = tile + gridDim.x;
        const bool more = nxt < ntiles;
        const uint64_t tile_off = (uint64_t)tile * TB;
        if (more)
            sh = load(nxt, a, wv, agg);
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s_in);
        const bool full = tile_off + TB <= n;
        uint32_t run = wbase + gincl - gtot;
        uint8_t *dst = out + tile_off + (uint32_t)(tid >> 3) * ITEMS * kFrame + (tid & 7) * 16;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t b = bw[k] ? bw[k] : 1u;
            const uint32_t off = 16u * run + 2u * b * (uint32_t)(tid & 7);
            run += bw[k];
            const uint32_t ad = off >> 2;
            const uint64_t w01 = ((uint64_t)s32[ad + 1] << 32) | s32[ad];
            const uint64_t w23 = ((uint64_t)s32[ad + 3] << 32) | s32[ad + 2];
            const uint64_t w4 = s32[ad + 4];
            const bool h = off & 2;
            const uint64_t lo = h ? (w01 >> 16) | (w23 << 48) : w01;
            const uint64_t hi = h ? (w23 >> 16) | (w4 << 48) : w23;
            const uint64_t p1 = b == 8 ? hi : ((lo >> (8 * b)) | (hi << (64 - 8 * b)));
            const uint64_t x0 = unpack8(lo, b);
            const uint64_t x1 = unpack8(p1, b);
            const u32x4 r = u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
            if (full)
                __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(dst + k * kFrame));
            else if (bw[k])
                store16_tail(out, (uint64_t)(dst - out) + k * kFrame, n, r);
        }
        if (!more)
            break;
        tile = nxt;
        __syncthreads();  // LDS reuse
    }
}

// F: offsets pre-pass fused into P. Workgroup = ticket g owns output tiles
// [g*per, (g+1)*per): phase 1 scans their widths (tile-local bases into tbl[],
// validation), block_prefix_all gives the range's base; phase 2 = P over the
// range (values of tile t+1 prefetched while tile t is unpacked).
template <int T, int ITEMS, int BPC>
__global__ __launch_bounds__(T, BPC) void dec_f(const uint8_t *__restrict__ bits, uint64_t nframes,
                                                const uint8_t *__restrict__ values, uint64_t vsize,
                                                uint8_t *__restrict__ out, uint64_t n, uint32_t ntiles,
                                                uint32_t per, uint32_t *__restrict__ tbl, Ctrl *ctrl,
                                                uint64_t *status)
{
    constexpr int TB = T * 16 * ITEMS;
    constexpr int TF = TB / kFrame;
    constexpr int FPT = 64;            // phase 1: frames per thread per round
    constexpr int LPT = TF / FPT;      // lanes per tile in phase 1
    constexpr int TPR = T / LPT;       // tiles per round
    static_assert(TF % FPT == 0 && (LPT & (LPT - 1)) == 0, "phase-1 layout");
    __shared__ u32x4 s_in[TB / 16 + 2];
    __shared__ uint32_t s_wave[T / kWave];
    __shared__ uint64_t s_red[T / kWave];
    __shared__ uint32_t s_ticket;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const uint32_t blk = take_ticket(ctrl, &s_ticket);
    const uint32_t t0 = blk * per;
    const uint32_t t1 = t0 + per < ntiles ? t0 + per : ntiles;
    // ---- phase 1: widths of tiles [t0, t1)
    uint32_t local = 0;
    bool bad = false;
    for (uint32_t r = t0; r < t1; r += TPR) {
        const uint32_t tile = r + tid / LPT;
        const uint64_t f0 = (uint64_t)tile * TF + (uint64_t)(tid % LPT) * FPT;
        uint32_t sum = 0;
        if (tile < t1) {
#pragma unroll
            for (int q = 0; q < FPT / 16; ++q) {
                const uint64_t fq = f0 + 16 * q;
                if (fq + 16 <= nframes) {
                    const u32x4 w = *reinterpret_cast<const u32x4 *>(bits + fq);
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        const uint32_t x = w[d];
                        const uint32_t zero = (x - 0x01010101u) & ~x & 0x80808080u;
                        const uint32_t big = (((x & 0x7F7F7F7Fu) + 0x77777777u) | x) & 0x80808080u;
                        if (zero | big) {
                            bad = true;
                            for (int i = 0; i < 4; ++i)
                                sum += clamp_width((x >> (8 * i)) & 0xFFu);
                        } else {
                            const uint32_t h = (x & 0x00FF00FFu) + ((x >> 8) & 0x00FF00FFu);
                            sum += (h & 0xFFFFu) + (h >> 16);
                        }
                    }
                } else {
                    for (int i = 0; i < 16 && fq + i < nframes; ++i) {
                        const uint32_t raw = bits[fq + i];
                        bad |= raw < 1 || raw > 8;
                        sum += clamp_width(raw);
                    }
                }
            }
        }
        const uint32_t inc = wave_incl_scan_u32(sum);
        if (r > t0)
            __syncthreads();
        if (lane == kWave - 1)
            s_wave[wave] = inc;
        __syncthreads();
        uint32_t before = 0, agg = 0;
#pragma unroll
        for (int w = 0; w < T / kWave; ++w) {
            before += w < wave ? s_wave[w] : 0u;
            agg += s_wave[w];
        }
        if (tid % LPT == 0 && tile < t1)
            tbl[tile] = local + before + inc - sum;
        local += agg;
    }
    if (bad)
        raise_error(ctrl, FLRL_E_FORMAT);
    const uint64_t rbase = block_prefix_all<T>(status, blk, local, ctrl, s_red);
    // ---- phase 2
    const u32x4 *v16 = reinterpret_cast<const u32x4 *>(values);
    (void)v16;
    uint32_t tile = t0;
    if (tile >= t1)
        return;
    auto tloc = [&](uint32_t t) { return t < t1 ? tbl[t] : local; };
    uint64_t base = rbase + tloc(tile);
    uint32_t agg = tloc(tile + 1) - tloc(tile);
    u32x4 a[ITEMS];
    load_vals<T, ITEMS>(a, values, base, agg, vsize);
    typename WVec<ITEMS>::T wv = load_w<ITEMS>(bits, (uint64_t)tile * TF + (tid >> 3) * ITEMS, nframes);
    for (;;) {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            if ((uint32_t)(k * T + tid) < agg)
                s_in[k * T + tid] = a[k];
        if (tid < 2)
            s_in[agg + tid] = u32x4{0u, 0u, 0u, 0u};
        uint32_t bw[ITEMS];
        uint32_t gtot = 0;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            uint32_t b = wbyte<ITEMS>(wv, k);
            const uint64_t f = (uint64_t)tile * TF + (tid >> 3) * ITEMS + k;
            b = f < nframes ? clamp_width(b) : 0u;
            bw[k] = b;
            gtot += b;
        }
        const uint32_t gincl = wave_incl_scan_u32((lane & 7) == 0 ? gtot : 0u);
        if (lane == kWave - 1)
            s_wave[wave] = gincl;
        __syncthreads();
        uint32_t wbase = 0;
#pragma unroll
        for (int v = 0; v < T / kWave; ++v)
            wbase += v < wave ? s_wave[v] : 0u;
        const uint32_t nxt = tile + 1;
        const bool more = nxt < t1;
        const uint64_t tile_off = (uint64_t)tile * TB;
        if (more) {
            base += agg;
            agg = tloc(nxt + 1) - tloc(nxt);
            load_vals<T, ITEMS>(a, values, base, agg, vsize);
            wv = load_w<ITEMS>(bits, (uint64_t)nxt * TF + (tid >> 3) * ITEMS, nframes);
        }
        const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s_in);
        const bool full = tile_off + TB <= n;
        uint32_t run = wbase + gincl - gtot;
        uint8_t *dst = out + tile_off + (uint32_t)(tid >> 3) * ITEMS * kFrame + (tid & 7) * 16;
#pragma unroll
        for (int k = 0; k < ITEMS; ++k) {
            const uint32_t b = bw[k];
            const uint32_t off = 16u * run + 2u * b * (uint32_t)(tid & 7);
            run += b;
            if (b == 0)
                continue;
            const uint32_t ad = off >> 2;
            const uint64_t w01 = ((uint64_t)s32[ad + 1] << 32) | s32[ad];
            const uint64_t w23 = ((uint64_t)s32[ad + 3] << 32) | s32[ad + 2];
            uint64_t lo = w01, hi = w23;
            if (off & 2) {
                const uint64_t w4 = s32[ad + 4];
                lo = (w01 >> 16) | (w23 << 48);
                hi = (w23 >> 16) | (w4 << 48);
            }
            const uint64_t p1 = b == 8 ? hi : ((lo >> (8 * b)) | (hi << (64 - 8 * b)));
            const uint64_t x0 = unpack8(lo, b);
            const uint64_t x1 = unpack8(p1, b);
            const u32x4 rr = u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1, (uint32_t)(x1 >> 32)};
            if (full)
                __builtin_nontemporal_store(rr, reinterpret_cast<u32x4 *>(dst + k * kFrame));
            else
                store16_tail(out, (uint64_t)(dst - out) + k * kFrame, n, rr);
        }
        if (!more)
            break;
        tile = nxt;
        __syncthreads();
    }
}

template <int U>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4 *__restrict__ in, u32x4 *__restrict__ out,
                                                   uint64_t n16)
{
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n16)
                v[u] = __builtin_nontemporal_load(in + i + u * 256);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n16)
                __builtin_nontemporal_store(v[u], out + i + u * 256);
    }
}

struct Ctx {
    uint8_t *d_in, *d_bits, *d_vals, *d_out;
    uint64_t *d_vsize;
    void *d_scr;
    size_t n, frames, vsize, scr_b;
    const uint64_t *tb32;  // library's per-32 KiB tile offsets (after one decode)
    uint32_t ntb32;
};

template <int T, int ITEMS, int BPC>
static void run_p(const Ctx &c, hipStream_t s, int cus)
{
    constexpr int TB = T * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)((c.n + TB - 1) / TB);
    const uint32_t grid = std::min<uint32_t>(ntiles, (uint32_t)cus * BPC);
    hipLaunchKernelGGL((dec_p<T, ITEMS, BPC>), dim3(grid), dim3(T), 0, s, c.d_bits, (uint64_t)c.frames,
                       c.d_vals, (uint64_t)c.vsize, c.d_out, (uint64_t)c.n, c.tb32, (uint32_t)(TB / 16384),
                       c.ntb32, ntiles);
}

template <int ITEMS, int DMA>
static void run_np(const Ctx &c, hipStream_t s, int)
{
    constexpr int TB = 256 * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)((c.n + TB - 1) / TB);
    const uint32_t stride = TB / 16384;
    hipLaunchKernelGGL((dec_np<ITEMS, DMA>), dim3(ntiles), dim3(256), 0, s, c.d_bits, (uint64_t)c.frames,
                       c.d_vals, (uint64_t)c.vsize, c.d_out, (uint64_t)c.n, c.tb32, stride, c.ntb32);
}

template <int U, int G>
static void run_copy(const Ctx &c, hipStream_t s, int cus)
{
    hipLaunchKernelGGL(copy_kernel<U>, dim3(cus * G), dim3(256), 0, s, reinterpret_cast<const u32x4 *>(c.d_in),
                       reinterpret_cast<u32x4 *>(c.d_out), (uint64_t)(c.n / 16));
}

template <int T, int ITEMS, int BPC>
static void run_q(const Ctx &c, hipStream_t s, int cus)
{
    constexpr int TB = T * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)((c.n + TB - 1) / TB);
    const uint32_t grid = std::min<uint32_t>(ntiles, (uint32_t)cus * BPC);
    hipLaunchKernelGGL((dec_q<T, ITEMS, BPC>), dim3(grid), dim3(T), 0, s, c.d_bits, (uint64_t)c.frames,
                       c.d_vals, (uint64_t)c.vsize, c.d_out, (uint64_t)c.n, c.tb32, (uint32_t)(TB / 16384),
                       c.ntb32, ntiles);
}

struct FScr {
    uint8_t *p = nullptr;
    size_t bytes = 0;
};
static FScr g_fscr;

template <int T, int ITEMS, int BPC>
static void run_f(const Ctx &c, hipStream_t s, int cus)
{
    constexpr int TB = T * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)((c.n + TB - 1) / TB);
    uint32_t g = std::min<uint32_t>(ntiles, (uint32_t)cus * BPC);
    const uint32_t per = (ntiles + g - 1) / g;
    g = (ntiles + per - 1) / per;
    const size_t zero = 16 + ((size_t)g * 8 + 15) / 16 * 16;
    const size_t need = zero + ((size_t)ntiles + 1) * 4;
    if (g_fscr.bytes < need) {
        if (g_fscr.p)
            CK(hipFree(g_fscr.p));
        CK(hipMalloc(&g_fscr.p, need));
        g_fscr.bytes = need;
    }
    CK(hipMemsetAsync(g_fscr.p, 0, zero, s));
    hipLaunchKernelGGL((dec_f<T, ITEMS, BPC>), dim3(g), dim3(T), 0, s, c.d_bits, (uint64_t)c.frames, c.d_vals,
                       (uint64_t)c.vsize, c.d_out, (uint64_t)c.n, ntiles, per,
                       reinterpret_cast<uint32_t *>(g_fscr.p + zero), reinterpret_cast<Ctrl *>(g_fscr.p),
                       reinterpret_cast<uint64_t *>(g_fscr.p + 16));
}

template <int T, int ITEMS, int BPC, int PAIR = 0>
static void run_pt2(const Ctx &c, hipStream_t s, int cus)
{
    constexpr int TB = T * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)((c.n + TB - 1) / TB);
    const uint32_t grid = std::min<uint32_t>((ntiles + 1) / 2, (uint32_t)cus * BPC);
    if (!g_fscr.p) {
        CK(hipMalloc(&g_fscr.p, 1 << 20));
        g_fscr.bytes = 1 << 20;
    }
    CK(hipMemsetAsync(g_fscr.p, 0, 16, s));
    hipLaunchKernelGGL((dec_pt2<T, ITEMS, BPC>), dim3(grid), dim3(T), 0, s, c.d_bits, (uint64_t)c.frames,
                       c.d_vals, (uint64_t)c.vsize, c.d_out, (uint64_t)c.n, c.tb32, (uint32_t)(TB / 16384),
                       c.ntb32, ntiles, reinterpret_cast<Ctrl *>(g_fscr.p));
}

template <int T, int ITEMS, int BPC, int NTS = 1, int NTL = 1>
static void run_pt(const Ctx &c, hipStream_t s, int cus)
{
    constexpr int TB = T * 16 * ITEMS;
    const uint32_t ntiles = (uint32_t)((c.n + TB - 1) / TB);
    const uint32_t grid = std::min<uint32_t>(ntiles, (uint32_t)cus * BPC);
    if (!g_fscr.p) {
        CK(hipMalloc(&g_fscr.p, 1 << 20));
        g_fscr.bytes = 1 << 20;
    }
    CK(hipMemsetAsync(g_fscr.p, 0, 16, s));
    hipLaunchKernelGGL((dec_pt<T, ITEMS, BPC, NTS, NTL>), dim3(grid), dim3(T), 0, s, c.d_bits, (uint64_t)c.frames,
                       c.d_vals, (uint64_t)c.vsize, c.d_out, (uint64_t)c.n, c.tb32, (uint32_t)(TB / 16384),
                       c.ntb32, ntiles, reinterpret_cast<Ctrl *>(g_fscr.p));
}

static int check(const Ctx &c, const char *name)
{
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> a(c.n), b(c.n);
    CK(hipMemcpy(a.data(), c.d_in, c.n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), c.d_out, c.n, hipMemcpyDeviceToHost));
    if (memcmp(a.data(), b.data(), c.n)) {
        size_t i = 0;
        while (a[i] == b[i])
            ++i;
        printf("MISMATCH %s at %zu\n", name, i);
        return 1;
    }
    printf("ok %s\n", name);
    return 0;
}

int main(int argc, char **argv)
{
    const size_t n = argc > 1 ? strtoull(argv[1], 0, 0) : (1ull << 30);
    const int kind = argc > 2 ? atoi(argv[2]) : 0;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    Ctx c{};
    c.n = n;
    c.frames = (n + 127) / 128;
    c.scr_b = flrl_fl_scratch_bytes(n);
    CK(hipMalloc(&c.d_in, n + 16));
    CK(hipMalloc(&c.d_bits, c.frames + 16));
    CK(hipMalloc(&c.d_vals, flrl_fl_values_capacity(n) + 16));
    CK(hipMalloc(&c.d_out, n + 16));
    CK(hipMalloc(&c.d_vsize, 16));
    CK(hipMalloc(&c.d_scr, c.scr_b));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (flrl_gen_device(kind, 42, 0, c.d_in, n, s) || flrl_fl_encode_device(c.d_in, n, c.d_bits, c.d_vals,
                                                                            c.d_vsize, c.d_scr, c.scr_b, s))
        return printf("lib error %s\n", flrl_last_error()), 1;
    CK(hipMemcpyAsync(&c.vsize, c.d_vsize, 8, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    if (flrl_fl_decode_device(c.d_bits, c.frames, c.d_vals, c.vsize, c.d_out, n, c.d_scr, c.scr_b, s))
        return 1;
    if (check(c, "lib"))
        return 1;
    // tile_base table of the library decode: [Ctrl][status[off_blocks] 16-B padded][tile_base]
    const size_t off_frames = 256 * 64;
    size_t off_iters = ((c.frames + off_frames - 1) / off_frames + 1023) / 1024;
    off_iters = off_iters ? off_iters : 1;
    const size_t off_blocks = (c.frames + off_frames * off_iters - 1) / (off_frames * off_iters);
    c.tb32 = reinterpret_cast<const uint64_t *>(static_cast<uint8_t *>(c.d_scr) + 16 +
                                                ((off_blocks * 8 + 15) / 16) * 16);
    c.ntb32 = (uint32_t)((n + 32767) / 32768);
    {  // host-built 16 KiB-granular table (128 frames per entry) for all variants
        std::vector<uint8_t> hb(c.frames);
        CK(hipMemcpy(hb.data(), c.d_bits, c.frames, hipMemcpyDeviceToHost));
        const size_t nt = (n + 16383) / 16384;
        std::vector<uint64_t> t(nt + 1);
        uint64_t acc = 0;
        for (size_t i = 0; i < nt; ++i) {
            t[i] = acc;
            for (size_t f = i * 128; f < std::min(c.frames, (i + 1) * 128); ++f)
                acc += hb[f];
        }
        t[nt] = acc;
        uint64_t *d;
        CK(hipMalloc(&d, (nt + 1) * 8));
        CK(hipMemcpy(d, t.data(), (nt + 1) * 8, hipMemcpyHostToDevice));
        c.tb32 = d;
        c.ntb32 = (uint32_t)nt;
    }

    struct V {
        const char *name;
        void (*fn)(const Ctx &, hipStream_t, int);
    };
    static const V vars[] = {
        {"lib decode (memset+offsets+decode)",
         [](const Ctx &c, hipStream_t s, int) {
             flrl_fl_decode_device(c.d_bits, c.frames, c.d_vals, c.vsize, c.d_out, c.n, c.d_scr, c.scr_b, s);
         }},
        {"NP<8,0> 32K (lib kernel)", run_np<8, 0>},
        {"PT2<512,8,2> pair tickets", run_pt2<512, 8, 2>},
        {"PT2<256,8,4> 32K pair tickets", run_pt2<256, 8, 4>},
        {"PT<512,8,2> 64K ticket", run_pt<512, 8, 2>},
        {"copy U4 x8", run_copy<4, 8>},
        {"copy U8 x4", run_copy<8, 4>},
        {"copy U16 x1", run_copy<16, 1>},
    };
    const int nv = sizeof(vars) / sizeof(vars[0]);
    for (int v = 1; v + 3 < nv; ++v) {
        CK(hipMemsetAsync(c.d_out, 0xA5, n, s));
        vars[v].fn(c, s, cus);
        if (check(c, vars[v].name))
            return 1;
    }
    std::vector<double> tot(nv, 0.0);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < reps; ++r)
        for (int v = 0; v < nv; ++v) {
            CK(hipEventRecord(e0, s));
            vars[v].fn(c, s, cus);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0)
                tot[v] += ms;
        }
    const double alg = (double)c.frames + (double)c.vsize + (double)n;
    for (int v = 0; v < nv; ++v) {
        const double ms = tot[v] / (reps - 1);
        printf("%-40s %8.4f ms  %7.1f GB/s alg\n", vars[v].name, ms, alg / ms / 1e6);
    }
    return 0;
}
