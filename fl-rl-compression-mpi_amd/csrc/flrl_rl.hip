// flrl_rl.hip — run-length (RL) encode / decode for MI355X (gfx950).
//
// Semantics (IMPLEMENTATION-PLAN.md:81-179; the reference fork has no RL code,
// SURVEY.md §0 item 2): maximal runs of equal bytes become (count, value)
// pairs; a run longer than 255 is split into 255-byte chunks counted from the
// run start (:125-147). Output: counts[R], values[R].
//
// Encode formulation. A byte is a natural head if it differs from its
// predecessor (or is byte 0). The state c before a byte is the number of bytes
// of the current chunk so far (1..254, with 255 written as 0); byte i is a head
// iff it is natural or c == 0, and then c becomes 1, else c = (c+1) mod 255.
// A segment of L bytes acts on c as a PhaseMap: a constant (if it contains a
// natural head: c after it depends only on its last natural head) or
// "+L mod 255" — maps compose associatively, so the chunk state at every byte
// comes from an exclusive scan of maps (lanes -> waves -> tiles, the last by a
// decoupled look-back). With c known, head counts are local; a second,
// additive look-back gives each tile its first output index. Each head h
// emits the run that ENDS at h-1 (count = c before h, value = x[h-1]); the
// tile holding byte n-1 emits the final run. So no tile ever needs bytes of
// its successor.
//
// Decode: rl_offsets_kernel scans the counts (R bytes) into per-tile output
// offsets (and validates them); rl_decode_kernel then expands each tile of
// 4096 runs independently, in 32 KiB LDS output windows: the runs overlapping
// a window memset their bytes into it with aligned dword stores, and the window
// leaves in 16-byte stores (the two chunks a tile shares with its neighbours
// byte by byte).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "flrl.h"
#include "flrl_device.hpp"
#include "flrl_internal.hpp"

namespace flrl {

constexpr int kRlThreads = 512;                      // encode workgroup: 8 waves
constexpr int kRlItems = 16;                         // 16 x 16 B per lane
constexpr int kRlWaveBytes = kWave * 16 * kRlItems;  // 16 KiB per wave (contiguous)
constexpr int kRlTileBytes = kRlWaveBytes * (kRlThreads / kWave);  // 128 KiB

constexpr int kRdRuns = 4096;        // runs per decode tile
constexpr int kRdThreads = 256;
constexpr int kRdWindow = 32768;     // LDS output window (bytes)
constexpr int kRoRunsPerThread = 256;
constexpr int kRoRuns = kRoRunsPerThread * kThreads;  // runs per offsets workgroup
static_assert(kRdRuns % kRoRunsPerThread == 0, "whole offsets lanes per decode tile");

// ---- PhaseMap packed in a u32: bit 8 = constant, bits 0-7 = value (< 255) ----
constexpr uint32_t kMapIdent = 0;
__device__ __forceinline__ uint32_t pm_make(bool constant, uint32_t v)
{
    return (constant ? 0x100u : 0u) | v;
}
// a then b
__device__ __forceinline__ uint32_t pm_compose(uint32_t a, uint32_t b)
{
    if (b & 0x100u)
        return b;
    uint32_t v = (a & 0xFFu) + (b & 0xFFu);
    v = v >= 255u ? v - 255u : v;
    return (a & 0x100u) | v;
}
__device__ __forceinline__ uint32_t pm_apply(uint32_t m, uint32_t c)
{
    if (m & 0x100u)
        return m & 0xFFu;
    const uint32_t v = c + (m & 0xFFu);
    return v >= 255u ? v - 255u : v;
}
__device__ __forceinline__ uint32_t wave_incl_scan_map(uint32_t m)
{
    const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t t = __shfl_up(m, o, kWave);
        if (lane >= o)
            m = pm_compose(t, m);
    }
    return m;
}

// Look-back over PhaseMaps: status granule payload = map (9 bits). A published
// constant map (A with a natural head) or an inclusive P stops the walk.
// Returns the chunk state c at the tile start; publishes the tile's P.
__device__ __forceinline__ uint32_t lookback_phase(uint64_t *status, uint32_t tile, uint32_t map,
                                                   Ctrl *ctrl)
{
    const int lane = threadIdx.x & (kWave - 1);
    if (tile == 0) {
        if (lane == 0)
            granule_store(&status[0], kFlagP | pm_apply(map, 0) | 0x100u);
        return 0;
    }
    uint32_t acc = kMapIdent;  // composition of the maps walked so far (nearest last)
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0;
    uint32_t c_in = 0;
    for (;;) {
        const int64_t idx = j - lane;
        uint64_t s;
        bool done = false;
        for (;;) {
            s = idx >= 0 ? granule_load(&status[idx]) : (kFlagP | 0x100u);
            const unsigned long long xm = __ballot((s >> 62) == 0);
            const unsigned long long stop = __ballot((s >> 62) == 2 || (s & 0x100u));
            const unsigned long long upto = stop ? (stop & (~stop + 1)) : 0;
            if (stop ? (xm & ((upto << 1) - 1)) == 0 : xm == 0)
                break;
            if (++spins > kSpinLimit) {
                if (lane == 0)
                    raise_error(ctrl, FLRL_E_TIMEOUT);
                return 0;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const unsigned long long stop = __ballot((s >> 62) == 2 || (s & 0x100u));
        const int first = stop ? __ffsll(stop) - 1 : kWave;
        // compose lanes first..0 (oldest first) onto acc (which is newer)
        uint32_t m = lane <= first ? (uint32_t)(s & 0x1FFu) : kMapIdent;
        // lane order is newest (0) to oldest (63): inclusive scan from high lanes
        // down = compose(older, newer). Do it serially in lane 0 for clarity.
        uint32_t win = kMapIdent;
        for (int l = (first < kWave ? first : kWave - 1); l >= 0; --l)
            win = pm_compose(win, __shfl(m, l, kWave));
        acc = pm_compose(win, acc);
        if (stop) {
            c_in = pm_apply(acc, 0);  // acc starts with a constant map
            done = true;
        }
        if (done)
            break;
        j -= kWave;
    }
    if (lane == 0)
        granule_store(&status[tile], kFlagP | 0x100u | pm_apply(map, c_in));
    return c_in;
}

// 16-bit mask of bytes of x that differ from their predecessor (p = byte before).
__device__ __forceinline__ uint32_t nat_mask(u32x4 x, uint32_t p)
{
    const uint32_t y0 = (x.x << 8) | (p & 0xFFu), y1 = (x.y << 8) | (x.x >> 24);
    const uint32_t y2 = (x.z << 8) | (x.y >> 24), y3 = (x.w << 8) | (x.z >> 24);
    const uint32_t d[4] = {x.x ^ y0, x.y ^ y1, x.z ^ y2, x.w ^ y3};
    uint32_t m = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t nz = (((d[q] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d[q]) & 0x80808080u;
        const uint32_t b4 = ((nz >> 7) & 1u) | ((nz >> 14) & 2u) | ((nz >> 21) & 4u) | ((nz >> 28) & 8u);
        m |= b4 << (4 * q);
    }
    return m;
}

__device__ __forceinline__ uint32_t byte_at(u32x4 x, uint32_t i)
{
    const uint64_t lo = ((uint64_t)x.y << 32) | x.x, hi = ((uint64_t)x.w << 32) | x.z;
    return (uint32_t)((i < 8 ? lo >> (8 * i) : hi >> (8 * (i - 8))) & 0xFFu);
}

template <int T, int ITEMS>
__global__ __launch_bounds__(T) void rl_encode_kernel(
    const uint8_t *__restrict__ in, uint64_t n, uint32_t ntiles, uint8_t *__restrict__ counts,
    uint8_t *__restrict__ values, uint64_t *__restrict__ runs_out, Ctrl *ctrl,
    uint64_t *st_phase, uint64_t *st_heads)
{
    constexpr int W = T / kWave;
    constexpr int WB = kWave * 16 * ITEMS;
    constexpr int TB = WB * W;
    __shared__ uint32_t s_wmap[W];
    __shared__ uint32_t s_whead[W];
    __shared__ uint8_t s_stc[W][kWave * 16];
    __shared__ uint8_t s_stv[W][kWave * 16];
    __shared__ uint32_t s_ticket, s_cin;
    __shared__ uint64_t s_hin;

    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int w = tid / kWave;
    const uint32_t tile = take_ticket(ctrl, &s_ticket);
    const uint64_t tile_off = (uint64_t)tile * TB;
    const uint64_t wave_off = tile_off + (uint64_t)w * WB;

    // ---- load this wave's contiguous 16 KiB (lane: chunk k*64 + lane) -----
    u32x4 a[ITEMS];
    if (wave_off + WB <= n) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(in + wave_off);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            a[k] = __builtin_nontemporal_load(src + k * kWave + lane);
    } else {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            a[k] = load16_tail(in, wave_off + (uint64_t)(k * kWave + lane) * 16, n);
    }
    const uint32_t pwave = (wave_off > 0 && wave_off <= n) ? in[wave_off - 1] : 0u;

    // ---- natural heads and the lane -> wave exclusive scan of phase maps --
    uint32_t nat[ITEMS], rel[ITEMS], prevb[ITEMS];
    uint32_t carry = kMapIdent;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const uint32_t up = __shfl_up(a[k].w, 1, kWave) >> 24;
        const uint32_t last_prev_item =
            k > 0 ? (uint32_t)__builtin_amdgcn_readlane((int)a[k > 0 ? k - 1 : 0].w, kWave - 1) >> 24
                  : pwave;
        const uint32_t p = lane > 0 ? up : last_prev_item;
        prevb[k] = p;
        const uint64_t gpos = wave_off + (uint64_t)(k * kWave + lane) * 16;
        const uint32_t vb = gpos >= n ? 0u : (n - gpos >= 16 ? 16u : (uint32_t)(n - gpos));
        uint32_t m = nat_mask(a[k], p);
        if (gpos == 0)
            m |= 1u;
        m &= vb >= 16 ? 0xFFFFu : ((1u << vb) - 1u);
        nat[k] = m;
        const uint32_t lmap = m ? pm_make(true, vb - (31u - __clz(m))) : pm_make(false, vb);
        const uint32_t incl = wave_incl_scan_map(lmap);
        const uint32_t excl = __shfl_up(incl, 1, kWave);
        rel[k] = pm_compose(carry, lane > 0 ? excl : kMapIdent);
        carry = pm_compose(carry, (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1));
    }
    if (lane == 0)
        s_wmap[w] = carry;
    __syncthreads();
    uint32_t tile_map = kMapIdent, wave_pre = kMapIdent;
#pragma unroll
    for (int v = 0; v < W; ++v) {
        if (v == w)
            wave_pre = tile_map;
        tile_map = pm_compose(tile_map, s_wmap[v]);
    }

    // ---- look-back 1: chunk state at the tile start ----------------------
    if (w == 0) {
        if (lane == 0 && tile > 0)
            granule_store(&st_phase[tile], kFlagA | tile_map);
        const uint32_t c = lookback_phase(st_phase, tile, tile_map, ctrl);
        if (lane == 0)
            s_cin = c;
    }
    __syncthreads();
    const uint32_t c_wave = pm_apply(wave_pre, s_cin);

    // ---- heads (natural, or chunk full) and their counts per lane-item ----
    uint32_t head[ITEMS], cst[ITEMS];
    uint32_t wheads = 0;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const uint32_t c0 = pm_apply(rel[k], c_wave);
        cst[k] = c0;
        uint32_t h = nat[k];
        if (c0 == 0 || c0 >= 240) {  // a split can only fall inside this lane then
            const uint64_t gpos = wave_off + (uint64_t)(k * kWave + lane) * 16;
            const uint32_t vb = gpos >= n ? 0u : (n - gpos >= 16 ? 16u : (uint32_t)(n - gpos));
            uint32_t c = c0;
            h = 0;
            for (uint32_t i = 0; i < vb; ++i) {
                if (((nat[k] >> i) & 1u) || c == 0) {
                    h |= 1u << i;
                    c = 1;
                } else {
                    c = c + 1 == 255u ? 0u : c + 1;
                }
            }
        }
        head[k] = h;
        wheads += __popc(h);
    }
    wheads = (uint32_t)wave_sum_u64(wheads);
    if (lane == 0)
        s_whead[w] = wheads;
    __syncthreads();
    uint32_t tile_heads = 0, wave_hpre = 0;
#pragma unroll
    for (int v = 0; v < W; ++v) {
        wave_hpre += v < w ? s_whead[v] : 0u;
        tile_heads += s_whead[v];
    }

    // ---- look-back 2: index of the tile's first head -----------------------
    if (w == 0) {
        const uint64_t e = lookback_sum(st_heads, tile, tile_heads, ctrl);
        if (lane == 0)
            s_hin = e;
    }
    __syncthreads();
    const uint64_t h_in = s_hin;

    // ---- emit: head g writes run g-1 (count = chunk state before it, value =
    // the byte before it), staged per wave-item in LDS, then stored as bytes
    uint64_t g_item = h_in + wave_hpre;  // global index of the item's first head
    uint8_t *stc = s_stc[w];
    uint8_t *stv = s_stv[w];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const uint32_t h = head[k];
        const uint32_t cnt = __popc(h);
        const uint32_t inc = wave_incl_scan_u32(cnt);
        const uint32_t item_total = (uint32_t)__builtin_amdgcn_readlane((int)inc, kWave - 1);
        if (h) {
            uint32_t slot = inc - cnt;
            // chunk state before the first head at byte i: no head in between,
            // so c0 just advanced i bytes; before a later head: distance (< 16)
            uint32_t prev_i = 0;
            bool seen = false;
            uint32_t hm = h;
            while (hm) {
                const uint32_t i = __ffs(hm) - 1;
                hm &= hm - 1;
                uint32_t cb = seen ? i - prev_i : cst[k] + i;
                cb = cb >= 255u ? cb - 255u : cb;
                seen = true;
                prev_i = i;
                stc[slot] = (uint8_t)(cb == 0 ? 255u : cb);
                stv[slot] = (uint8_t)(i == 0 ? prevb[k] : byte_at(a[k], i - 1));
                ++slot;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t j = lane; j < item_total; j += kWave) {
            const uint64_t gi = g_item + j;
            if (gi > 0) {
                counts[gi - 1] = stc[j];
                values[gi - 1] = stv[j];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        g_item += item_total;
    }

    // ---- the final run (ends at byte n-1) ----------------------------------
    if (tile + 1 == ntiles && tid == 0) {
        const uint64_t R = h_in + tile_heads;
        const uint32_t c_end = pm_apply(tile_map, s_cin);
        counts[R - 1] = (uint8_t)(c_end == 0 ? 255u : c_end);
        values[R - 1] = in[n - 1];
        *runs_out = R;
    }
}

// ---- decode pre-pass: output offsets of each decode tile ------------------
__global__ __launch_bounds__(kThreads) void rl_offsets_kernel(
    const uint8_t *__restrict__ counts, uint64_t runs, uint64_t n, uint64_t *__restrict__ tile_base,
    uint32_t ntiles, uint32_t nblocks, Ctrl *ctrl, uint64_t *status)
{
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_ticket;
    __shared__ uint64_t s_base;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const uint32_t blk = take_ticket(ctrl, &s_ticket);
    const uint64_t r0 = (uint64_t)blk * kRoRuns + (uint64_t)tid * kRoRunsPerThread;

    uint32_t sum = 0;
    bool bad = false;
#pragma unroll 4
    for (int q = 0; q < kRoRunsPerThread / 16; ++q) {
        const uint64_t rq = r0 + 16 * q;
        const u32x4 v = load16_tail(counts, rq, runs);
#pragma unroll
        for (int d = 0; d < 4; ++d) {
            const uint32_t x = v[d];
            const uint32_t h = (x & 0x00FF00FFu) + ((x >> 8) & 0x00FF00FFu);
            sum += (h & 0xFFFFu) + (h >> 16);
            // a zero count inside [0, runs) is malformed
            const uint32_t zero = (x - 0x01010101u) & ~x & 0x80808080u;
            if (zero) {
                for (int i = 0; i < 4; ++i)
                    bad |= rq + 4 * d + i < runs && ((x >> (8 * i)) & 0xFFu) == 0;
            }
        }
    }
    if (bad)
        raise_error(ctrl, FLRL_E_FORMAT);
    const uint32_t inc = wave_incl_scan_u32(sum);
    if (lane == kWave - 1)
        s_wave[wave] = inc;
    __syncthreads();
    uint32_t before = 0, agg = 0;
#pragma unroll
    for (int v = 0; v < kWaves; ++v) {
        before += v < wave ? s_wave[v] : 0u;
        agg += s_wave[v];
    }
    const uint32_t excl = before + inc - sum;
    if (wave == 0) {
        const uint64_t e = lookback_sum(status, blk, agg, ctrl);
        if (tid == 0)
            s_base = e;
    }
    __syncthreads();
    const uint64_t base = s_base;
    constexpr int kLanesPerTile = kRdRuns / kRoRunsPerThread;
    const uint64_t tile = r0 / kRdRuns;
    if (tid % kLanesPerTile == 0 && tile < ntiles)
        tile_base[tile] = base + excl;
    if (blk + 1 == nblocks && tid == 0) {
        tile_base[ntiles] = base + agg;
        if (base + agg != n)
            raise_error(ctrl, FLRL_E_FORMAT);
    }
}

// ---- decode: expand one tile of kRdRuns runs ------------------------------
// The tile's output [base, end) is produced in kRdWindow-byte windows aligned to
// global 16-byte boundaries: the runs overlapping a window (one binary search
// of the count prefix per window) memset their bytes into an LDS window with
// aligned dword stores, then the window leaves in 16-byte stores (the two
// chunks a tile shares with its neighbours byte by byte).
__device__ __forceinline__ uint32_t run_lower(const uint32_t *pre, uint32_t nr, uint32_t x)
{
    // last j in [0, nr) with pre[j] <= x (pre[0] = 0 <= x)
    uint32_t a = 0, b = nr;
    while (b - a > 1) {
        const uint32_t m = (a + b) >> 1;
        if (pre[m] <= x)
            a = m;
        else
            b = m;
    }
    return a;
}

__global__ __launch_bounds__(kRdThreads) void rl_decode_kernel(
    const uint8_t *__restrict__ counts, const uint8_t *__restrict__ values, uint64_t runs,
    uint8_t *__restrict__ out, uint64_t n, const uint64_t *__restrict__ tile_base)
{
    __shared__ uint32_t s_pre[kRdRuns + 1];  // local output offset of each run
    __shared__ u32x4 s_val4[kRdRuns / 16];
    __shared__ u32x4 s_win4[kRdWindow / 16];
    __shared__ uint32_t s_wave[kRdThreads / kWave];
    uint8_t *s_val = reinterpret_cast<uint8_t *>(s_val4);
    uint8_t *s_win = reinterpret_cast<uint8_t *>(s_win4);
    uint32_t *s_win32 = reinterpret_cast<uint32_t *>(s_win4);
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const uint64_t tile = blockIdx.x;
    const uint64_t r0 = tile * kRdRuns;
    const uint64_t base = tile_base[tile];
    const uint64_t end = tile_base[tile + 1];
    if (end > n || base >= end)
        return;  // empty, or malformed (flagged by rl_offsets_kernel)
    const uint32_t nr = (uint32_t)(runs - r0 < (uint64_t)kRdRuns ? runs - r0 : kRdRuns);

    // ---- counts -> block scan -> s_pre; values -> LDS ------------------------
    constexpr int RPT = kRdRuns / kRdThreads;
    static_assert(RPT % 16 == 0, "whole 16-byte count vectors per thread");
    uint32_t c[RPT];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < RPT / 16; ++q) {
        const u32x4 v = load16_tail(counts, r0 + tid * RPT + 16 * q, runs);
        s_val4[(tid * RPT) / 16 + q] = load16_tail(values, r0 + tid * RPT + 16 * q, runs);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            c[16 * q + i] = (v[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            sum += c[16 * q + i];
        }
    }
    const uint32_t inc = wave_incl_scan_u32(sum);
    if (lane == kWave - 1)
        s_wave[wave] = inc;
    __syncthreads();
    uint32_t before = 0;
#pragma unroll
    for (int v = 0; v < kRdThreads / kWave; ++v)
        before += v < wave ? s_wave[v] : 0u;
    uint32_t run = before + inc - sum;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
        s_pre[tid * RPT + i] = run;
        run += c[i];
    }
    if (tid == 0)
        s_pre[kRdRuns] = (uint32_t)(end - base);
    __syncthreads();

    // ---- windows ---------------------------------------------------------------
    const uint64_t g0 = base & ~15ull;
    for (uint64_t gw = g0; gw < end; gw += kRdWindow) {
        const uint32_t lo = (uint32_t)((gw > base ? gw : base) - base);  // owned, tile-local
        const uint32_t hi = (uint32_t)((gw + kRdWindow < end ? gw + kRdWindow : end) - base);
        const uint32_t shift = (uint32_t)(gw < base ? base - gw : 0);    // window pos of local lo
        const uint32_t ja = run_lower(s_pre, nr, lo);
        const uint32_t jb = run_lower(s_pre, nr, hi - 1) + 1;
        for (uint32_t j = ja + tid; j < jb; j += kRdThreads) {
            uint32_t x = s_pre[j], y = j + 1 < nr ? s_pre[j + 1] : hi;
            x = x < lo ? lo : x;
            y = y > hi ? hi : y;
            if (x >= y)
                continue;
            // window positions [x - lo + shift, y - lo + shift)
            uint32_t p = x - lo + shift, q = y - lo + shift;
            const uint32_t v = s_val[j];
            while (p < q && (p & 3)) s_win[p++] = (uint8_t)v;
            const uint32_t v4 = v * 0x01010101u;
            while (p + 4 <= q) {
                s_win32[p >> 2] = v4;
                p += 4;
            }
            while (p < q) s_win[p++] = (uint8_t)v;
        }
        __syncthreads();
        const uint32_t wlen = (uint32_t)(end - gw < (uint64_t)kRdWindow ? end - gw : kRdWindow);
        for (uint32_t ch = tid; ch * 16 < wlen; ch += kRdThreads) {
            const uint64_t gp = gw + 16ull * ch;
            if (gp >= base && gp + 16 <= end) {
                __builtin_nontemporal_store(s_win4[ch], reinterpret_cast<u32x4 *>(out + gp));
            } else {
                for (uint32_t f = 0; f < 16; ++f)
                    if (gp + f >= base && gp + f < end)
                        out[gp + f] = s_win[16 * ch + f];
            }
        }
        __syncthreads();
    }
}

struct RlEncLayout {
    size_t tiles, bytes;
    explicit RlEncLayout(size_t n)
    {
        tiles = div_up(n, (size_t)kRlTileBytes);
        bytes = sizeof(Ctrl) + 2 * round_up(tiles * 8, 16);
    }
};

struct RlDecLayout {
    size_t tiles, blocks, zero, bytes;
    explicit RlDecLayout(size_t runs)
    {
        tiles = div_up(runs, (size_t)kRdRuns);
        blocks = div_up(runs, (size_t)kRoRuns);
        zero = sizeof(Ctrl) + round_up(blocks * 8, 16);
        bytes = zero + round_up((tiles + 1) * 8, 16);
    }
};

}  // namespace flrl

using namespace flrl;

extern "C" size_t flrl_rl_scratch_bytes(size_t n) { return RlEncLayout(n).bytes; }
extern "C" size_t flrl_rl_decode_scratch_bytes(size_t runs) { return RlDecLayout(runs).bytes; }

extern "C" int flrl_rl_encode_device(const uint8_t *d_in, size_t n, uint8_t *d_counts,
                                     uint8_t *d_values, uint64_t *d_runs, void *d_scratch,
                                     size_t scratch_bytes, void *stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    const RlEncLayout L(n);
    if (!d_runs || !d_scratch)
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: null runs/scratch");
    if (scratch_bytes < L.bytes)
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: scratch %zu < required %zu",
                         scratch_bytes, L.bytes);
    if (!aligned16(d_scratch))
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: scratch not 16-byte aligned");
    FLRL_HIP(hipMemsetAsync(d_scratch, 0, L.bytes, s));
    if (n == 0) {
        FLRL_HIP(hipMemsetAsync(d_runs, 0, sizeof(uint64_t), s));
        return FLRL_OK;
    }
    if (!d_in || !d_counts || !d_values)
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: null buffer");
    if (!aligned16(d_in))
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: input must be 16-byte aligned");
    if (L.tiles > 0xFFFFFFFFull)
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: input too large");
    Ctrl *ctrl = static_cast<Ctrl *>(d_scratch);
    uint64_t *st_phase = reinterpret_cast<uint64_t *>(ctrl + 1);
    uint64_t *st_heads = st_phase + round_up(L.tiles * 8, 16) / 8;
    hipLaunchKernelGGL((rl_encode_kernel<kRlThreads, kRlItems>), dim3((uint32_t)L.tiles),
                       dim3(kRlThreads), 0, s, d_in, (uint64_t)n, (uint32_t)L.tiles, d_counts,
                       d_values, d_runs, ctrl, st_phase, st_heads);
    FLRL_HIP(hipGetLastError());
    return FLRL_OK;
}

extern "C" int flrl_rl_decode_device(const uint8_t *d_counts, const uint8_t *d_values, size_t runs,
                                     uint8_t *d_out, size_t n, void *d_scratch,
                                     size_t scratch_bytes, void *stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    const RlDecLayout L(runs);
    if (!d_scratch)
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: null scratch");
    if (scratch_bytes < L.bytes)
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: scratch %zu < required %zu",
                         scratch_bytes, L.bytes);
    if (!aligned16(d_scratch))
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: scratch not 16-byte aligned");
    FLRL_HIP(hipMemsetAsync(d_scratch, 0, L.zero, s));
    if (runs == 0) {
        if (n != 0) {
            const uint32_t e = FLRL_E_FORMAT;
            FLRL_HIP(hipMemcpyAsync(static_cast<uint8_t *>(d_scratch) + 4, &e, 4,
                                    hipMemcpyHostToDevice, s));
            FLRL_HIP(hipStreamSynchronize(s));
        }
        return FLRL_OK;
    }
    if (!d_counts || !d_values || !d_out)
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: null buffer");
    if (!aligned16(d_counts) || !aligned16(d_values) || !aligned16(d_out))
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: buffers must be 16-byte aligned");
    if (L.tiles > 0x7FFFFFFFull)
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: too many runs");
    Ctrl *ctrl = static_cast<Ctrl *>(d_scratch);
    uint64_t *status = reinterpret_cast<uint64_t *>(ctrl + 1);
    uint64_t *tile_base =
        reinterpret_cast<uint64_t *>(static_cast<uint8_t *>(d_scratch) + L.zero);
    hipLaunchKernelGGL(rl_offsets_kernel, dim3((uint32_t)L.blocks), dim3(kThreads), 0, s, d_counts,
                       (uint64_t)runs, (uint64_t)n, tile_base, (uint32_t)L.tiles,
                       (uint32_t)L.blocks, ctrl, status);
    FLRL_HIP(hipGetLastError());
    hipLaunchKernelGGL(rl_decode_kernel, dim3((uint32_t)L.tiles), dim3(kRdThreads), 0, s, d_counts,
                       d_values, (uint64_t)runs, d_out, (uint64_t)n, tile_base);
    FLRL_HIP(hipGetLastError());
    return FLRL_OK;
}

// ---------------------------------------------------------------------------
// Host-buffer entry points (synchronous).
// ---------------------------------------------------------------------------

extern "C" int flrl_rl_compress(const uint8_t *data, size_t size, flrl_rl_buf *out)
{
    clear_error();
    if (!out || (!data && size))
        return set_error(FLRL_E_ARG, "flrl_rl_compress: null argument");
    memset(out, 0, sizeof(*out));
    out->input_size = size;
    if (size == 0)
        return FLRL_OK;
    if (flrl_device_count() <= 0)
        return set_error(FLRL_E_NODEV, "flrl_rl_compress: no HIP device visible");
    const size_t in_b = round_up(size, 16), scr_b = flrl_rl_scratch_bytes(size);
    DevBuf dev;
    if (dev.alloc(3 * in_b + 16 + scr_b) != hipSuccess)
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory (device, %zu bytes)",
                         3 * in_b + 16 + scr_b);
    uint8_t *d_in = dev.as<uint8_t>(0);
    uint8_t *d_counts = dev.as<uint8_t>(in_b);
    uint8_t *d_vals = dev.as<uint8_t>(2 * in_b);
    uint64_t *d_runs = dev.as<uint64_t>(3 * in_b);
    void *d_scr = dev.as<void>(3 * in_b + 16);
    FLRL_HIP(hipMemcpy(d_in, data, size, hipMemcpyHostToDevice));
    int rc = flrl_rl_encode_device(d_in, size, d_counts, d_vals, d_runs, d_scr, scr_b, nullptr);
    if (rc)
        return rc;
    uint64_t runs = 0;
    FLRL_HIP(hipMemcpy(&runs, d_runs, sizeof(runs), hipMemcpyDeviceToHost));
    const int kerr = flrl_scratch_error(d_scr, nullptr);
    if (kerr)
        return set_error(kerr, "flrl_rl_compress: device error %d", kerr);
    uint8_t *hc = static_cast<uint8_t *>(malloc(runs ? runs : 1));
    uint8_t *hv = static_cast<uint8_t *>(malloc(runs ? runs : 1));
    if (!hc || !hv) {
        free(hc);
        free(hv);
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory");
    }
    hipError_t e1 = hipMemcpy(hc, d_counts, runs, hipMemcpyDeviceToHost);
    hipError_t e2 = hipMemcpy(hv, d_vals, runs, hipMemcpyDeviceToHost);
    if (e1 != hipSuccess || e2 != hipSuccess) {
        free(hc);
        free(hv);
        return set_error(FLRL_E_HIP, "flrl_rl_compress: copy-out failed");
    }
    out->counts = hc;
    out->values = hv;
    out->runs = runs;
    return FLRL_OK;
}

extern "C" int flrl_rl_decompress(size_t output_size, const uint8_t *counts, const uint8_t *values,
                                  size_t runs, uint8_t **out, size_t *out_size)
{
    clear_error();
    if (!out || !out_size)
        return set_error(FLRL_E_ARG, "flrl_rl_decompress: null output pointer");
    *out = nullptr;
    *out_size = 0;
    if (runs && (!counts || !values))
        return set_error(FLRL_E_ARG, "flrl_rl_decompress: null input");
    if (runs == 0) {
        if (output_size != 0)
            return set_error(FLRL_E_FORMAT, "RL: 0 runs but inputSize %zu", output_size);
        return FLRL_OK;
    }
    if (flrl_device_count() <= 0)
        return set_error(FLRL_E_NODEV, "flrl_rl_decompress: no HIP device visible");
    const size_t r_b = round_up(runs, 16), o_b = round_up(output_size ? output_size : 1, 16);
    const size_t scr_b = flrl_rl_decode_scratch_bytes(runs);
    DevBuf dev;
    if (dev.alloc(2 * r_b + o_b + scr_b) != hipSuccess)
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory (device)");
    uint8_t *d_c = dev.as<uint8_t>(0);
    uint8_t *d_v = dev.as<uint8_t>(r_b);
    uint8_t *d_o = dev.as<uint8_t>(2 * r_b);
    void *d_scr = dev.as<void>(2 * r_b + o_b);
    FLRL_HIP(hipMemcpy(d_c, counts, runs, hipMemcpyHostToDevice));
    FLRL_HIP(hipMemcpy(d_v, values, runs, hipMemcpyHostToDevice));
    int rc = flrl_rl_decode_device(d_c, d_v, runs, d_o, output_size, d_scr, scr_b, nullptr);
    if (rc)
        return rc;
    const int kerr = flrl_scratch_error(d_scr, nullptr);
    if (kerr)
        return set_error(kerr, "flrl_rl_decompress: malformed runs (device error %d)", kerr);
    uint8_t *h = static_cast<uint8_t *>(malloc(output_size ? output_size : 1));
    if (!h)
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory");
    if (output_size && hipMemcpy(h, d_o, output_size, hipMemcpyDeviceToHost) != hipSuccess) {
        free(h);
        return set_error(FLRL_E_HIP, "flrl_rl_decompress: copy-out failed");
    }
    *out = h;
    *out_size = output_size;
    return FLRL_OK;
}
