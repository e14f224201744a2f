// flrl_device.hpp — gfx950 device helpers shared by the FL and RL kernels:
// dynamic tile tickets, decoupled look-back over 8-byte status granules, wave /
// block scans, tail-guarded 16-byte loads and stores.
//
// Cross-workgroup hand-off follows MI355X_MICROARCH.md "Valid forms", R2: every
// status word is ONE naturally aligned 8-byte granule that carries its own flag
// and payload, stored and loaded with agent-scope relaxed atomics (sc1, L1
// bypass), so no release/acquire fence is needed. Status words are zeroed by a
// zero-fill kernel before every launch (Guideline 16, "Re-initialise every call").
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

// u64 moves between lanes without the LDS crossbar: DPP from a higher (row_shl)
// or lower (row_shr) lane within 16-lane rows (lanes without a source read 0),
// and a wave-uniform read of one lane.
template <int CTRL>
__device__ __forceinline__ uint64_t dpp64_0(uint64_t v)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xF, 0xF, true);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, true);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l) << 32) |
           (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
}

// Sum over the wave (wave-uniform result): four DPP row_shr steps leave each
// 16-lane row's sum in its lane 15, then the four row sums are added. (Six
// xor-butterfly shuffles were twelve dependent LDS-crossbar round trips.)
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
    v += dpp64_0<0x111>(v);
    v += dpp64_0<0x112>(v);
    v += dpp64_0<0x114>(v);
    v += dpp64_0<0x118>(v);
    return readlane64(v, 15) + readlane64(v, 31) + readlane64(v, 47) + readlane64(v, 63);
}

// OR across each aligned group of 8 lanes with DPP (no LDS crossbar):
// quad_perm [1,0,3,2], quad_perm [2,3,0,1], then row_half_mirror (lane i <-> 7-i).
__device__ __forceinline__ uint32_t or_8lanes(uint32_t o)
{
    o |= (uint32_t)__builtin_amdgcn_mov_dpp((int)o, 0xB1, 0xF, 0xF, false);
    o |= (uint32_t)__builtin_amdgcn_mov_dpp((int)o, 0x4E, 0xF, 0xF, false);
    o |= (uint32_t)__builtin_amdgcn_mov_dpp((int)o, 0x141, 0xF, 0xF, false);
    return o;
}

// DPP move from a lower lane (row_shr:k within 16-lane rows; row_bcast:15 /
// row_bcast:31 across rows); lanes without a source (and rows outside RM) read 0.
template <int CTRL, int RM>
__device__ __forceinline__ uint32_t dpp_up0(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, RM, 0xF, true);
}

// The value of lane i-1 (lane 0: 0), by DPP wave_shr:1 instead of an LDS
// crossbar round trip (ds_bpermute).
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, false);
}

__device__ __forceinline__ uint64_t wave_shr1_64(uint64_t v)
{
    return ((uint64_t)wave_shr1((uint32_t)(v >> 32)) << 32) | wave_shr1((uint32_t)v);
}

// Inclusive wave scan in six DPP steps (no LDS crossbar round trips):
// row_shr 1/2/4/8 scan each row, row_bcast:15 and :31 carry row totals up.
// Each step folds into one v_add_u32_dpp -- unless a caller's arithmetic on
// the result (e.g. incl - own) lets the compiler reuse the shifted partial
// sums, which then stay separate v_mov_b32_dpp + v_add pairs with wait
// states between them (seen in the RL encode's scan loop): the empty asm
// makes the result opaque, so the six steps stay six instructions.
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v)
{
    v += dpp_up0<0x111, 0xF>(v);
    v += dpp_up0<0x112, 0xF>(v);
    v += dpp_up0<0x114, 0xF>(v);
    v += dpp_up0<0x118, 0xF>(v);
    v += dpp_up0<0x142, 0xA>(v);
    v += dpp_up0<0x143, 0xC>(v);
    asm volatile("" : "+v"(v));
    return v;
}

// Exclusive scan of N small counts held in LDS (s_in, any integer type) into
// s_out by a T-thread block. Returns the total to every thread. Requires
// N % T == 0 or N < T. Caller must __syncthreads() before reading s_out and
// before reusing s_wave (T/64 words).
template <int N, typename TIn, int T = kThreads>
__device__ __forceinline__ uint32_t block_excl_scan(const TIn *s_in, uint32_t *s_out,
                                                    uint32_t *s_wave)
{
    constexpr int E = N >= T ? N / T : 1;
    constexpr int kWaves = T / kWave;
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
template <int S = 1>
__device__ __forceinline__ void publish_aggregate(uint64_t *status, uint32_t tile, uint64_t agg)
{
    granule_store(&status[(size_t)tile * S], (tile == 0 ? kFlagP : kFlagA) | agg);
}

// lookback_resolve: called by ONE full wave after publish_aggregate. Sums
// predecessors 64 G at a time (lane i holds tiles j-iG .. j-iG-G+1) until it
// meets an inclusive prefix (P), publishes the tile's inclusive prefix and
// returns the exclusive prefix (to every lane). A window is usable once every
// slot up to and including the nearest P is published; slots beyond that P are
// not needed, so a straggler further back never stalls us. A wider window (G >
// 1) resolves the first round of a launch -- every tile's predecessors are
// aggregates back to tile 0 -- in fewer round trips.
// Must stay inlined: a call makes the callee open with s_waitcnt vmcnt(0),
// which would drain the caller's in-flight prefetch loads before the look-back.
template <int G, int L = kWave, int S = 1>
__device__ __forceinline__ uint64_t lookback_resolve(uint64_t *status, uint32_t tile, uint64_t agg,
                                                  Ctrl *ctrl)
{
    static_assert(L >= 1 && L <= kWave && (G == 1 || L == kWave), "window of L lanes x G granules");
    const int lane = threadIdx.x & (kWave - 1);
    if (tile == 0)
        return 0;
    uint64_t excl = 0;
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0;
    for (;;) {
        const int64_t idx = j - (int64_t)lane * G;
        uint64_t part;
        bool has_p;
        for (;;) {
            uint64_t s[G];
#pragma unroll
            for (int k = 0; k < G; ++k)
                s[k] = lane >= L     ? kFlagA
                       : idx - k >= 0 ? granule_load(&status[(idx - k) * S])
                                      : kFlagP;
            // lane-local: sum from the lane's newest slot back to its nearest P
            has_p = false;
            bool ok = true;
            part = 0;
#pragma unroll
            for (int k = 0; k < G; ++k) {
                if (!has_p) {
                    const uint32_t f = (uint32_t)(s[k] >> 62);
                    ok = ok && f != 0;
                    has_p = f == 2;
                    part += s[k] & kPayload;
                }
            }
            const unsigned long long pm = __ballot(has_p);
            const unsigned long long bad = __ballot(!ok);
            const unsigned long long upto = pm ? ((pm & (~pm + 1)) << 1) - 1 : ~0ull;
            if ((bad & upto) == 0)
                break;
            if (++spins > kSpinLimit) {
                if (lane == 0)
                    raise_error(ctrl, FLRL_E_TIMEOUT);
                return excl;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const unsigned long long pm = __ballot(has_p);
        const int first_p = pm ? __ffsll(pm) - 1 : kWave;
        excl += wave_sum_u64(lane <= first_p ? part : 0ull);
        if (pm)
            break;
        j -= (int64_t)L * G;
    }
    if (lane == 0)
        granule_store(&status[(size_t)tile * S], kFlagP | (excl + agg));
    return excl;
}

// Exclusive prefix of per-workgroup aggregates for the pre-pass scans: the
// whole T-thread workgroup publishes its aggregate and then reads EVERY
// predecessor's (4 per thread per round, all loads in flight together), so the
// prefix costs one round trip once they are published instead of a chain of
// look-back windows, each waiting for an inclusive prefix further back. For
// grids of at most kMaxPrefixBlocks workgroups, taken in ticket order (so each
// predecessor is running or done). s_red: T/64 words of LDS.
constexpr uint32_t kMaxPrefixBlocks = 1024;
template <int T>
__device__ __forceinline__ uint64_t block_prefix_all(uint64_t *status, uint32_t blk, uint64_t agg,
                                                     Ctrl *ctrl, uint64_t *s_red)
{
    const int tid = threadIdx.x;
    if (tid == 0)
        granule_store(&status[blk], kFlagA | agg);
    uint64_t sum = 0;
    for (uint32_t j0 = 0; j0 < blk; j0 += 4 * T) {
        uint64_t g[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = j0 + (uint32_t)tid + (uint32_t)k * T;
            g[k] = j < blk ? granule_load(&status[j]) : kFlagA;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = j0 + (uint32_t)tid + (uint32_t)k * T;
            uint32_t spins = 0;
            while ((g[k] >> 62) == 0) {
                if (++spins > kSpinLimit) {
                    raise_error(ctrl, FLRL_E_TIMEOUT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                g[k] = granule_load(&status[j]);
            }
            sum += g[k] & kPayload;
        }
    }
    sum = wave_sum_u64(sum);
    if ((tid & (kWave - 1)) == 0)
        s_red[tid / kWave] = sum;
    __syncthreads();
    uint64_t excl = 0;
#pragma unroll
    for (int v = 0; v < T / kWave; ++v)
        excl += s_red[v];
    return excl;
}

// 16-byte load of bytes [o, o+16) of p (o and p 16-byte aligned), zero-filling
// past n. A straddling chunk is read whole: a 16-byte-aligned block never
// crosses a page, so this cannot fault; the bytes at or past n are masked off.
__device__ __forceinline__ u32x4 load16_tail(const uint8_t *p, uint64_t o, uint64_t n)
{
    if (o >= n)
        return u32x4{0u, 0u, 0u, 0u};
    u32x4 v = *reinterpret_cast<const u32x4 *>(p + o);
    if (o + 16 > n) {
        const uint32_t r = (uint32_t)(n - o);  // 1..15 valid bytes
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t keep = r >= 4u * (d + 1) ? 4u : (r > 4u * d ? r - 4u * d : 0u);
            v[d] &= keep >= 4 ? 0xFFFFFFFFu : ((1u << (8 * keep)) - 1u);
        }
    }
    return v;
}

// Branch-free pieces of load16_tail for software pipelines: the load itself
// with its address clamped to the last 16-byte block of [0, n) (n >= 1; every
// lane issues exactly one load and no wait, so the compiler can count the
// loads in flight across it), and the masking, applied when the data is used:
// bytes at or past n read as zero.
__device__ __forceinline__ u32x4 load16_clamped(const uint8_t *p, uint64_t o, uint64_t n)
{
    const uint64_t last = (n - 1) & ~15ull;
    return *reinterpret_cast<const u32x4 *>(p + (o < last ? o : last));
}
__device__ __forceinline__ uint32_t valid16(uint64_t o, uint64_t n)
{
    return o >= n ? 0u : (n - o >= 16 ? 16u : (uint32_t)(n - o));
}
__device__ __forceinline__ uint32_t mask_dword(uint32_t x, uint32_t valid, int d)
{
    const uint32_t vb = valid > 4u * d ? valid - 4u * d : 0u;
    return vb >= 4 ? x : x & ((1u << (8 * vb)) - 1u);
}

// 16-byte store of v to bytes [o, o+16) of p, dropping bytes at or past n.
__device__ __forceinline__ void store16_tail(uint8_t *p, uint64_t o, uint64_t n, u32x4 v)
{
    if (o + 16 <= n) {
        *reinterpret_cast<u32x4 *>(p + o) = v;
        return;
    }
    const uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
#pragma unroll 1
    for (uint32_t i = 0; i < 16 && o + i < n; ++i)
        p[o + i] = (uint8_t)(i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8)));
}

}  // namespace flrl
