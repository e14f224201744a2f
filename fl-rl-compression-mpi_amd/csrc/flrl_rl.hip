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
// Each head h emits the run that ENDS at h-1 (count = c before h, value =
// x[h-1]); the tile holding byte n-1 emits the final run, so no tile needs
// bytes of its successor. A tile is four 32 KiB sub-tiles that pass through LDS
// one after the other (LDS-DMA); each lane owns 128 contiguous bytes of a
// sub-tile, so a lane holds at most one split head (before its first natural
// head). Within a sub-tile two 32-bit scans suffice: a PhaseMap scan of lane
// states (constant after a natural head, else "+L mod 255") and a sum of the
// heads that do not depend on the tile's incoming state (those from its first
// natural head on), whose runs are staged in LDS as the sub-tiles go by.
// Across tiles ONE decoupled look-back per tile composes segment maps {bytes
// before the first natural head, heads from it on, state after} into (heads
// before the tile, state at its start); then only the split heads before the
// first natural head are written and the staged runs leave contiguously.
//
// Decode: rl_offsets_kernel scans the counts (R bytes) into per-tile output
// offsets (and validates them); rl_decode_kernel (4 workgroups per CU,
// grid-stride, the next tile's counts and values prefetched into registers)
// then expands each tile of 4096 runs independently. Output-driven: per 64 KiB
// window the runs starting in it set bits in an LDS bitmap, a popcount scan
// ranks every 16-byte chunk, and each lane assembles whole chunks (byte
// permutes over the 16 values from the chunk's first run on) and stores them
// coalesced from registers. Dense tiles (<= 32 KiB of output) memset their runs
// into an LDS byte window instead. Chunks a tile shares with its neighbours are
// written byte by byte.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "flrl.h"
#include "flrl_device.hpp"
#include "flrl_internal.hpp"
#include "flrl_tuning.hpp"


namespace flrl {

constexpr int kRlThreads = FLRL_RL_THREADS;         // encode workgroup: 4 waves (LB 64: 94 VGPRs, < 32 KiB LDS, 5 per CU)
constexpr int kRlLaneBytes = 64;                    // contiguous bytes per lane (a u64 head mask)
constexpr int kRlSub = FLRL_RL_SUB;                 // sub-chunks of 4 KiB per wave chunk (one look-back per tile)
constexpr int kRlTileBytes = kRlLaneBytes * kRlThreads * kRlSub;  // 128 KiB: 4 waves x 32 KiB
constexpr int kRlLookG = FLRL_RL_LOOKG;  // look-back granules per lane (window 64 G tiles)
constexpr int kRlLookL = FLRL_RL_LOOKL;  // look-back lanes polled per window
constexpr int kRlStatusStride = FLRL_RL_STATUS_STRIDE;  // status granules per tile
constexpr size_t kRlStatusOff = FLRL_RL_STATUS_OFF;    // status array offset in the scratch
constexpr int kRlStageBytes = FLRL_RL_STAGE;  // LDS run staging per workgroup
// 5 workgroups of 4 waves per CU (LDS-bound: < 32 KiB each): 5 waves per SIMD,
// so at most 96 VGPRs
constexpr int kRlWavesPerSimd = FLRL_RL_WPS;

// Block decode workgroups: 512 threads over 8192-run tiles, 2 per CU, unless the
// mean run is at least kRdNarrowMean bytes (runs near the 255 maximum: little
// assembly per chunk), then 256 threads over 4096-run tiles, 4 per CU. 1 GiB,
// 512 vs 256 threads: runs32 -7 %, runs of 1..48 -5 %, 1..256 -8 %, long runs
// (1..1023 bytes, split) -4 %; all-zero +10 %.
constexpr int kRdThreads = 256;
constexpr int kRdThreadsWide = 512;
constexpr uint64_t kRdNarrowMean = FLRL_RD_NARROW_MEAN;
template <int T>
constexpr int rd_per_cu() { return T == 512 ? 2 : 4; }  // LDS-bound: 59 / 31 KB per workgroup

// ---- PhaseMap packed in a u32: bit 31 = constant, bits 0-30 = value --------
// The value is kept unreduced (a byte count within one tile, < 2^31) and taken
// mod 255 only when the map is applied, so composing is one add and a select
// (the reduced form needed a compare, a subtract and two masks per step).
constexpr uint32_t kMapIdent = 0;
constexpr uint32_t kMapConst = 0x80000000u;
__device__ __forceinline__ uint32_t pm_make(bool constant, uint32_t v)
{
    return (constant ? kMapConst : 0u) | v;
}
// a then b
__device__ __forceinline__ uint32_t pm_compose(uint32_t a, uint32_t b)
{
    return (b & kMapConst) ? b : a + b;
}
// x mod 255 without the quarter-rate multiplies of a division: 256 = 1 (mod
// 255), so x's byte sum (one dot product, <= 1020) keeps its residue; a second
// fold leaves <= 258 and one subtract finishes
__device__ __forceinline__ uint32_t mod255(uint32_t x)
{
    uint32_t s = __builtin_amdgcn_udot4(x, 0x01010101u, 0u, false);
    s = (s & 0xFFu) + (s >> 8);
    return s >= 255u ? s - 255u : s;
}
__device__ __forceinline__ uint32_t pm_apply(uint32_t m, uint32_t c)
{
    return mod255((m & kMapConst) ? (m & ~kMapConst) : c + m);
}
// inclusive PhaseMap scan, DPP steps as wave_incl_scan_u32 (0 = identity map)
__device__ __forceinline__ uint32_t wave_incl_scan_map(uint32_t m)
{
    m = pm_compose(dpp_up0<0x111, 0xF>(m), m);
    m = pm_compose(dpp_up0<0x112, 0xF>(m), m);
    m = pm_compose(dpp_up0<0x114, 0xF>(m), m);
    m = pm_compose(dpp_up0<0x118, 0xF>(m), m);
    m = pm_compose(dpp_up0<0x142, 0xA>(m), m);
    m = pm_compose(dpp_up0<0x143, 0xC>(m), m);
    return m;
}

// 16-bit mask of bytes of x that differ from their predecessor (p = byte before):
// SWAR non-zero test of x ^ (x shifted by a byte) leaves 0x80 in each differing
// byte, and byte dot products with 2^k weights gather those top bits in order.
__device__ __forceinline__ uint32_t nat_mask(u32x4 x, uint32_t p)
{
    const uint32_t y0 = (x.x << 8) | (p & 0xFFu), y1 = (x.y << 8) | (x.x >> 24);
    const uint32_t y2 = (x.z << 8) | (x.y >> 24), y3 = (x.w << 8) | (x.z >> 24);
    const uint32_t d[4] = {x.x ^ y0, x.y ^ y1, x.z ^ y2, x.w ^ y3};
    uint32_t nz[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        nz[q] = (((d[q] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | d[q]) & 0x80808080u;
    const uint32_t lo = __builtin_amdgcn_udot4(nz[1], 0x80402010u, __builtin_amdgcn_udot4(nz[0], 0x08040201u, 0u, false), false);
    const uint32_t hi = __builtin_amdgcn_udot4(nz[3], 0x80402010u, __builtin_amdgcn_udot4(nz[2], 0x08040201u, 0u, false), false);
    return (lo >> 7) | (hi << 1);  // each sum is 128 x (8-bit mask)
}

// ---- composite segment map for the single tile look-back -------------------
// Acting on the state (H = heads before, c = chunk state) at a segment start:
//   kind NoNat (L):       H += splits(c, L);        c = (c + L) mod 255
//   kind Nat (pre, K, ca): H += splits(c, pre) + K;  c = ca
//   kind Const (H, c):    the state itself (an inclusive prefix)
// splits(c, m) = #{j < m : (c + j) mod 255 == 0}. Packed in the 62 payload bits
// of a status granule: c in 0-7, pre/L in 8-33, K in 34-59, kind in 60-61;
// Const keeps H in bits 8-59.
constexpr uint64_t kSmNat = 1ull << 60, kSmConst = 2ull << 60, kSmKind = 3ull << 60;
constexpr uint32_t kSmField = (1u << 26) - 1;
__device__ __forceinline__ uint64_t sm_nonat(uint32_t L) { return (uint64_t)L << 8; }
__device__ __forceinline__ uint64_t sm_nat(uint32_t pre, uint32_t K, uint32_t c)
{
    return kSmNat | ((uint64_t)K << 34) | ((uint64_t)pre << 8) | c;
}
__device__ __forceinline__ uint64_t sm_const(uint64_t H, uint32_t c) { return kSmConst | (H << 8) | c; }
__device__ __forceinline__ uint32_t sm_c(uint64_t m) { return (uint32_t)(m & 0xFFu); }
__device__ __forceinline__ uint32_t sm_a(uint64_t m) { return (uint32_t)(m >> 8) & kSmField; }
__device__ __forceinline__ uint32_t sm_b(uint64_t m) { return (uint32_t)(m >> 34) & kSmField; }
__device__ __forceinline__ uint64_t sm_h(uint64_t m) { return (m >> 8) & ((1ull << 52) - 1); }
// 32-bit forms for packed (< 2^26) lengths; the 64-bit ones only for the
// cross-window accumulator of the look-back
__device__ __forceinline__ uint32_t splits(uint32_t c, uint32_t m)
{
    const uint32_t j0 = c == 0 ? 0 : 255 - c;
    return m > j0 ? 1 + (m - 1 - j0) / 255 : 0;
}
__device__ __forceinline__ uint32_t add_c(uint32_t c, uint32_t L) { return (c + L) % 255; }
__device__ __forceinline__ uint64_t splits64(uint32_t c, uint64_t m)
{
    const uint64_t j0 = c == 0 ? 0 : 255 - c;
    return m > j0 ? 1 + (m - 1 - j0) / 255 : 0;
}
__device__ __forceinline__ uint32_t add_c64(uint32_t c, uint64_t L) { return (uint32_t)((c + L) % 255); }
// a then b. Const appears only as the oldest operand.
__device__ __forceinline__ uint64_t sm_compose(uint64_t a, uint64_t b)
{
    const uint64_t kb = b & kSmKind, ka = a & kSmKind;
    if (kb == kSmConst)
        return b;
    if (ka == kSmConst) {
        const uint64_t H = sm_h(a);
        const uint32_t c = sm_c(a);
        if (kb == kSmNat)
            return sm_const(H + splits(c, sm_a(b)) + sm_b(b), sm_c(b));
        return sm_const(H + splits(c, sm_a(b)), add_c(c, sm_a(b)));
    }
    if (kb == kSmNat) {
        if (ka == kSmNat)
            return sm_nat(sm_a(a), sm_b(a) + splits(sm_c(a), sm_a(b)) + sm_b(b), sm_c(b));
        return sm_nat(sm_a(a) + sm_a(b), sm_b(b), sm_c(b));
    }
    if (ka == kSmNat)
        return sm_nat(sm_a(a), sm_b(a) + splits(sm_c(a), sm_a(b)), add_c(sm_c(a), sm_a(b)));
    return sm_nonat(sm_a(a) + sm_a(b));
}

// Look-back for (H, c), run by ONE wave after the tile published its composite
// map (A; tile 0 publishes its inclusive prefix P instead). Each lane loads G
// granules at once (tiles j-G*lane .. j-G*lane-G+1), so one round trip covers
// 64*G predecessors: a persistent grid of one workgroup per CU has about that
// many tiles in flight, all at the same stage, and a 64-wide window would need
// several dependent round trips to reach the last inclusive prefix (P). The
// window is composed from its nearest P forward (per lane, then a 6-level
// shuffle tree), this tile's P is published and the Const state at the tile
// start returned. Composed window maps span <= 64*G tiles of <= 128 KiB, within
// the 26-bit packed fields; across windows the accumulator is kept unpacked.
template <int S>
__device__ __forceinline__ void publish_seg(uint64_t *status, uint32_t tile, uint64_t map)
{
    if ((threadIdx.x & (kWave - 1)) == 0)
        granule_store(&status[(size_t)tile * S], tile == 0 ? (kFlagP | sm_compose(sm_const(0, 0), map))
                                               : (kFlagA | map));
}

// help(t): tile t's map computed by this wave from the input (decoupled
// fallback). Tiles are numbered by workgroup index, not by a ticket: a ticket
// per workgroup start cost 10-23 % (its atomic round trip on one counter heads
// every tile's life). Within one launch the dispatcher starts workgroups in
// index order on each XCD, so a predecessor that has not published is running
// or about to start; but with other work on the GPU (another look-back kernel
// on a second stream holding the CUs) it may not start for a long time, so a
// slot unpublished for help_ticks (s_memrealtime, 100 MHz; kRlHelpTicks unless
// flrl_debug_lookback_help_us sets it) is computed here instead of waited for.
constexpr uint64_t kRlHelpTicks = 20000;  // 200 us
template <int G, int L, int S, class Help>
__device__ __forceinline__ uint64_t lookback_seg(uint64_t *status, uint32_t tile, uint64_t map,
                                                 Ctrl *ctrl, uint64_t help_ticks, Help &&help)
{
    static_assert(L >= 1 && L <= kWave && (G == 1 || L == kWave), "window of L lanes x G granules");
    static_assert((uint64_t)kWave * G * kRlTileBytes < (1ull << 26), "window maps within the 26-bit fields");
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t kPay = (1ull << 62) - 1;
    if (tile == 0)
        return sm_const(0, 0);
    // accumulator for windows without an inclusive prefix (newest part), unpacked
    uint32_t acc_kind = 0;  // 0 no-nat, 1 nat
    uint64_t acc_a = 0, acc_b = 0;
    uint32_t acc_c = 0;
    int64_t j = (int64_t)tile - 1;
    uint32_t spins = 0, rounds = 0;
    for (;;) {
        ++rounds;
        const int64_t idx = j - (int64_t)lane * G;  // the lane's newest slot; k = 0..G-1 older
        uint64_t ov[G];  // this lane's slots as computed by help (0: none)
#pragma unroll
        for (int k = 0; k < G; ++k)
            ov[k] = 0;
        uint64_t t0 = 0;
        bool helping = false;
        uint64_t m;
        bool has_p;
        for (;;) {
            uint64_t sv[G];
#pragma unroll
            for (int k = 0; k < G; ++k) {
                sv[k] = lane >= L       ? (kFlagA | sm_nonat(0))
                        : idx - k >= 0 ? granule_load(&status[(idx - k) * S])
                                       : (kFlagP | sm_const(0, 0));
                if ((sv[k] >> 62) == 0 && ov[k] != 0)
                    sv[k] = ov[k];
            }
            // lane-local, newest slot first: ready if nothing up to the lane's
            // nearest P is unpublished; kp = that P (G - 1: none), kbad = the
            // newest unpublished slot before it
            has_p = false;
            bool ok = true;
            int kp = G - 1, kbad = 0;
#pragma unroll
            for (int k = 0; k < G; ++k) {
                if (!has_p) {
                    const uint32_t f = (uint32_t)(sv[k] >> 62);
                    if (f == 0 && ok) {
                        ok = false;
                        kbad = k;
                    }
                    if (f == 2) {
                        has_p = true;
                        kp = k;
                    }
                }
            }
            // the lane's map, oldest needed slot first (identity: no-nat L 0)
            m = sm_nonat(0);
#pragma unroll
            for (int k = G - 1; k >= 0; --k)
                if (k <= kp)
                    m = sm_compose(m, (sv[k] >> 62) == 2 ? sm_const(sm_h(sv[k]), sm_c(sv[k])) : (sv[k] & kPay));
            const unsigned long long pm = __ballot(has_p);
            const unsigned long long bad = __ballot(!ok);
            const unsigned long long upto = pm ? ((pm & (~pm + 1)) << 1) - 1 : ~0ull;
            if ((bad & upto) == 0)
                break;
            if (++spins > kSpinLimit) {
                if (lane == 0)
                    raise_error(ctrl, FLRL_E_TIMEOUT);
                return sm_const(0, 0);
            }
            const uint64_t now = __builtin_amdgcn_s_memrealtime();
            if (!helping) {  // the clock starts at the first unpublished poll (help_ticks 0: help at once)
                if (t0 == 0)
                    t0 = now;
                if (now - t0 >= help_ticks)
                    helping = true;
            }
            if (helping) {  // an unpublished slot the window needs (uniform: lane l, slot kl)
                const int l = __ffsll(bad & upto) - 1;
                const int kl = __builtin_amdgcn_readlane(kbad, l);
                const uint64_t hm = help((uint32_t)(j - (int64_t)l * G - kl));
#pragma unroll
                for (int k = 0; k < G; ++k)
                    if (lane == l && k == kl)
                        ov[k] = kFlagA | hm;
                continue;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const unsigned long long pm = __ballot(has_p);
        const int first = pm ? __ffsll(pm) - 1 : kWave;
        if (lane > first)
            m = sm_nonat(0);
        // composition of the window, oldest first (identity: no-nat L 0 = 0):
        // four DPP row_shl steps compose each 16-lane row into its lane 0 (lanes
        // past a row read 0), then the four row results are composed
        m = sm_compose(dpp64_0<0x101>(m), m);
        m = sm_compose(dpp64_0<0x102>(m), m);
        m = sm_compose(dpp64_0<0x104>(m), m);
        m = sm_compose(dpp64_0<0x108>(m), m);
        const uint64_t win = sm_compose(sm_compose(sm_compose(readlane64(m, 48), readlane64(m, 32)),
                                                   readlane64(m, 16)),
                                        readlane64(m, 0));
        // combine with the newer accumulator: win then acc
        uint64_t res;
        if ((win & kSmKind) == kSmConst) {
            uint64_t H = sm_h(win);
            uint32_t c = sm_c(win);
            if (acc_kind == 1) {
                H += splits64(c, acc_a) + acc_b;
                c = acc_c;
            } else {
                H += splits64(c, acc_a);
                c = add_c64(c, acc_a);
            }
            res = sm_const(H, c);
            if (lane == 0)
                granule_store(&status[(size_t)tile * S], kFlagP | sm_compose(res, map));
            FLRL_RL_LB_STAT(tile, spins, rounds);
            return res;
        }
        // no inclusive prefix in this window: fold it into the accumulator
        if ((win & kSmKind) == kSmNat) {
            if (acc_kind == 1) {
                acc_b = sm_b(win) + splits64(sm_c(win), acc_a) + acc_b;
                acc_a = sm_a(win);
            } else {
                acc_b = sm_b(win) + splits64(sm_c(win), acc_a);
                acc_c = add_c64(sm_c(win), acc_a);
                acc_a = sm_a(win);
                acc_kind = 1;
            }
        } else {
            acc_a = sm_a(win) + acc_a;
        }
        j -= (int64_t)L * G;
    }
}

// Bytes [lo, hi) of the 16-byte chunk v (0 <= lo < hi <= 16) stored at dst (16-byte
// aligned) as naturally aligned pieces: 1, 2, 4, 8 bytes up to a 16-byte
// boundary, then 8, 4, 2, 1 while they fit.
__device__ __forceinline__ void store_chunk_part(uint8_t *dst, u32x4 v, uint32_t lo, uint32_t hi)
{
    auto dw = [&](uint32_t a) { return a < 8 ? (a < 4 ? v[0] : v[1]) : (a < 12 ? v[2] : v[3]); };
    auto qw = [&](uint32_t a) {
        return a < 8 ? ((uint64_t)v[1] << 32) | v[0] : ((uint64_t)v[3] << 32) | v[2];
    };
    uint32_t a = lo;
    if ((a & 1u) && a + 1 <= hi) {
        dst[a] = (uint8_t)(dw(a) >> (8 * (a & 3)));
        a += 1;
    }
    if ((a & 2u) && a + 2 <= hi) {
        *reinterpret_cast<uint16_t *>(dst + a) = (uint16_t)(dw(a) >> (8 * (a & 3)));
        a += 2;
    }
    if ((a & 4u) && a + 4 <= hi) {
        *reinterpret_cast<uint32_t *>(dst + a) = dw(a);
        a += 4;
    }
    if ((a & 8u) && a + 8 <= hi) {
        *reinterpret_cast<uint64_t *>(dst + a) = qw(a);
        a += 8;
    }
    if (a + 8 <= hi) {
        *reinterpret_cast<uint64_t *>(dst + a) = qw(a);
        a += 8;
    }
    if (a + 4 <= hi) {
        *reinterpret_cast<uint32_t *>(dst + a) = dw(a);
        a += 4;
    }
    if (a + 2 <= hi) {
        *reinterpret_cast<uint16_t *>(dst + a) = (uint16_t)(dw(a) >> (8 * (a & 3)));
        a += 2;
    }
    if (a + 1 <= hi)
        dst[a] = (uint8_t)(dw(a) >> (8 * (a & 3)));
}

// Wave-uniform values held in scalar registers (the compiler cannot prove
// that values read from LDS or derived from the wave index are uniform).
__device__ __forceinline__ uint32_t uniform32(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v)
{
    return ((uint64_t)uniform32((uint32_t)(v >> 32)) << 32) | uniform32((uint32_t)v);
}

// LDS operations of one wave complete in order; the fences keep the compiler
// from moving this wave's LDS accesses across this point.
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// RL encode, per wave. A tile is 128 KiB; wave w of its workgroup owns the w-th
// contiguous 32 KiB chunk and streams it as SUB sub-chunks of 64*LB bytes
// through its OWN slice of LDS (registers -> ds_write -> each lane reads its LB
// contiguous bytes; LDS ops of one wave are in order, so no barrier), with the
// next sub-chunk's loads in flight during each scan. The image is swizzled so
// that those lane reads are bank-conflict free: row r keeps its 16-byte chunk c
// at r*LB + ((c ^ swz(r)) * 16). LB < 255, so a lane holds at most one split
// head, before its first natural head. All scans are wave scans with the
// carries (PhaseMap, first natural head, state-independent head count) in
// uniform registers, and each wave stages its own state-independent runs. The
// wave maps compose (sm_compose) into the tile's map for the one look-back; the
// resolved state is then advanced wave by wave, and every wave emits its own
// prefix (split heads before its first natural head), staged runs and, past a
// staging overflow, re-read sub-chunks: sparse ones through the staging area,
// dense ones one lane row at a time (contiguous stores).
template <int LB, int SUB, int W, int STG = kRlStageBytes, int PFD = FLRL_RL_PF>
struct RlWave {
    static constexpr int CH = LB / 16;      // 16-byte chunks per lane
    static constexpr int WB = kWave * LB;   // sub-chunk bytes
    static constexpr int CB = WB * SUB;     // wave chunk bytes
    static constexpr int TBT = CB * W;      // tile bytes
    static constexpr int SW = STG / W / 2;  // staged records per wave
    static constexpr int NJ = WB / 1024;    // 1 KiB wave-loads per sub-chunk
    static constexpr int RPL = 1024 / LB;   // image rows per wave-load
    static constexpr uint32_t kNone = 0xFFFFFFFFu;
    // LDS per workgroup: W images and the run staging
    static constexpr int kLdsBytes = W * WB + STG;
    static_assert(LB == 64, "one u64 head mask per lane (piece emission: 4 x 16 positions)");
    static_assert(TBT == kRlTileBytes, "tile geometry shared with the layout");
    static_assert(SW >= 16 * LB + 15, "a piece part (16 rows) and the carried records fit the staging");
    static constexpr uint32_t kPieceSink = 1152;  // piece_part's sink bytes (4 per lane) in stc/stv
    static_assert(kPieceSink >= 16 * LB + 16 && kPieceSink + 4 * kWave <= SW, "sink past the part's records");

    struct Sub {
        uint32_t nat[CH / 2];  // 16-bit natural-head masks, two per word
        uint32_t ncnt, fpos, lpos, vbl, p0;
        uint32_t lrel;    // lane start state from the sub-chunk's start (PhaseMap)
        uint32_t smap;    // the sub-chunk's PhaseMap
        uint32_t sfirst;  // first natural head in the sub-chunk (kNone: none)
    };
    // A wave chunk after the staging pass (wave-uniform values).
    struct Chunk {
        uint64_t off;     // first byte
        uint32_t len;     // bytes (0: past the input)
        int ns;           // sub-chunks
        int nst;          // sub-chunks whose runs are all staged
        uint32_t first;   // first natural head (chunk-relative; kNone: none)
        uint32_t K;       // state-independent heads (runs ended by the heads from `first` on)
        uint32_t Kst;     // of them staged
        uint32_t rel_in;  // PhaseMap over the whole chunk
        uint32_t rel_st;  // PhaseMap over the staged sub-chunks
        uint32_t v0;      // the chunk's first byte
        __device__ uint32_t pre() const { return first != kNone ? first : len; }
        __device__ uint64_t map() const { return first != kNone ? sm_nat(first, K, pm_apply(rel_in, 0)) : sm_nonat(len); }
    };

    const uint8_t *in;
    uint64_t n;
    uint8_t *img, *stc, *stv;
    const uint8_t *my;
    int lane, wi;
    uint32_t row, o, sw, swz_c;

    // this wave's staging slice of a W-wave staging area at `st` (STG bytes)
    __device__ void stage_at(uint8_t *st)
    {
        stc = st + wi * 2 * SW;
        stv = stc + SW;
    }

    // The lane-derived members again, from a lane index the compiler cannot
    // see through: called at the top of each tile of a persistent loop, it
    // keeps the per-lane addresses derived from them inside the iteration
    // (hoisted out of the loop, they stayed live across it and the loop
    // spilled).
    __device__ void relane()
    {
        int l = (int)(threadIdx.x & (kWave - 1));
        asm volatile("" : "+v"(l));
        lane = l;
        row = (uint32_t)l;
        o = row * LB;
        my = img + o;
        sw = swz(row);
        swz_c = ((uint32_t)l % CH) ^ swz((uint32_t)l / CH);
    }

    // swizzle of row r: its chunk c sits at position c ^ swz(r); 16 lanes of a
    // ds_read_b128 (rows r..r+15, one chunk each) then cover all 64 banks
    __device__ static uint32_t swz(uint32_t r) { return LB == 128 ? (r & 7u) : ((r >> 2) & 3u); }

    __device__ RlWave(const uint8_t *in_, uint64_t n_, uint8_t *lds, int w_) : in(in_), n(n_)
    {
        const int w = (int)uniform32((uint32_t)w_);
        wi = w;
        lane = threadIdx.x & (kWave - 1);
        img = lds + w * WB;
        stage_at(lds + W * WB);
        row = (uint32_t)lane;
        o = row * LB;
        my = img + o;
        sw = swz(row);
        // LDS slot (j, lane) = byte j*1024 + lane*16 = row j*RPL + lane/CH, position
        // lane % CH; swz(row) depends on lane/CH only, as RPL is a multiple of 8
        // (LB 128) or 16 (LB 64)
        swz_c = ((uint32_t)lane % CH) ^ swz((uint32_t)lane / CH);
    }

    // sub-chunk s of the chunk at `off` into registers, placed as the LDS image
    // wants it, each wave-load 1 KiB of LDS
    __device__ void load_sub(uint64_t off, int s, u32x4 (&pf)[NJ]) const
    {
        const uint64_t so = off + (uint64_t)s * WB;
        if (so + WB <= n) {
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                pf[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(
                    in + so + (uint32_t)(j * RPL + lane / CH) * LB + swz_c * 16));
        } else {
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                pf[j] = load16_tail(in, so + (uint32_t)(j * RPL + lane / CH) * LB + swz_c * 16, n);
        }
    }

    // sub-chunk s (in pf) through the wave's LDS image; p_sub = the byte before
    // it; s_next >= 0: load sub-chunk s_next into pf once this one is in LDS.
    // Returns the sub-chunk's last byte (uniform).
    __device__ uint32_t scan_sub(uint64_t off, int s, Sub &L, u32x4 (&pf)[NJ], uint32_t p_sub, int s_next) const
    {
        const uint64_t so = off + (uint64_t)s * WB;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
            *reinterpret_cast<u32x4 *>(img + j * 1024 + lane * 16) = pf[j];
        if (s_next >= 0)
            load_sub(off, s_next, pf);  // lands while this sub-chunk (and, PF = 2, the next) is scanned
        const uint64_t lane_off = so + o;
        L.vbl = lane_off >= n ? 0u : (n - lane_off >= LB ? (uint32_t)LB : (uint32_t)(n - lane_off));
        u32x4 x[CH];
#pragma unroll
        for (int c = 0; c < CH; ++c)
            x[c] = *reinterpret_cast<const u32x4 *>(my + ((c ^ sw) * 16));
        const uint32_t mylast = x[CH - 1].w >> 24;
        const uint32_t up = wave_shr1(mylast);
        L.p0 = lane == 0 ? p_sub : up;
        {
            uint32_t p = L.p0;
            const bool full = so + WB <= n;  // wave-uniform: no per-chunk length masks
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                uint32_t m = nat_mask(x[c], p);
                if (!full) {
                    const uint32_t vb = L.vbl > 16u * c ? (L.vbl - 16u * c >= 16 ? 16u : L.vbl - 16u * c) : 0u;
                    m &= vb >= 16 ? 0xFFFFu : ((1u << vb) - 1u);
                }
                if (c & 1)
                    L.nat[c / 2] |= m << 16;
                else
                    L.nat[c / 2] = m;
                p = x[c].w >> 24;
            }
            if (lane_off == 0)
                L.nat[0] |= 1u;  // byte 0 is a head
            const uint64_t a = ((uint64_t)L.nat[1] << 32) | L.nat[0];
            uint64_t b = 0;
            if constexpr (CH == 8)
                b = ((uint64_t)L.nat[3] << 32) | L.nat[2];
            L.ncnt = (uint32_t)(__popcll(a) + __popcll(b));
            L.fpos = a ? (uint32_t)__builtin_ctzll(a) : (b ? 64u + (uint32_t)__builtin_ctzll(b) : (uint32_t)LB);
            L.lpos = b ? 127u - (uint32_t)__builtin_clzll(b) : (a ? 63u - (uint32_t)__builtin_clzll(a) : 0u);
        }
        const bool has = L.ncnt != 0;
        const uint32_t lmap = has ? pm_make(true, L.vbl - L.lpos) : pm_make(false, L.vbl);
        const uint32_t incl = wave_incl_scan_map(lmap);
        uint32_t lexcl = wave_shr1(incl);
        L.lrel = lane == 0 ? kMapIdent : lexcl;
        L.smap = (uint32_t)__builtin_amdgcn_readlane((int)incl, kWave - 1);
        const unsigned long long hb = __ballot(has);
        const int fl = hb ? __ffsll(hb) - 1 : 0;
        const uint32_t ff = (uint32_t)__builtin_amdgcn_readlane((int)L.fpos, fl);  // fl is uniform
        L.sfirst = hb ? (uint32_t)fl * LB + ff : kNone;
        return (uint32_t)__builtin_amdgcn_readlane((int)mylast, kWave - 1);
    }

    __device__ void head_masks(const Sub &L, uint32_t c0, bool with_split, uint64_t &h0, uint64_t &h1) const
    {
        const uint32_t j0 = c0 == 0 ? 0u : 255u - c0;
        const bool split = with_split && j0 < L.fpos && j0 < L.vbl;
        if constexpr (CH == 4) {  // one u64: the natural heads and the split bit
            h0 = (((uint64_t)L.nat[1] << 32) | L.nat[0]) | (split ? 1ull << j0 : 0ull);
            h1 = 0;
            return;
        }
        h0 = h1 = 0;
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            uint32_t h = (L.nat[c / 2] >> (16 * (c & 1))) & 0xFFFFu;
            if (split && (j0 >> 4) == (uint32_t)c)
                h |= 1u << (j0 & 15u);
            if (c < 4)
                h0 |= (uint64_t)h << (16 * c);
            else
                h1 |= (uint64_t)h << (16 * (c - 4));
        }
    }

    // a lane's runs from its head masks: head h ends the run before it (count =
    // h - previous head, or c_first + h for the lane's first head, 255 for 0;
    // value = the byte before h), records at slot, slot + 1, ...
    __device__ void lane_runs(const Sub &L, uint64_t h0, uint64_t h1, uint32_t c_first, uint32_t slot) const
    {
        // before the lane's first head prev = -c_first: c_first + pos <= 255
        // (a longer chunk would have a split head first), so every count is
        // pos - prev in [1, 255] with no modulo and no branch in the loop; the
        // state 0 stands for 255 bytes (a head at pos 0 then ends a 255-run).
        // (The chunk's first natural head gets a count here that emit()
        // replaces: it depends on the tile's incoming state.)
        int prev = c_first == 0 ? -255 : -(int)c_first;
        uint32_t val = L.p0;
        const uint32_t sw16 = sw << 4;  // image byte of lane position q: (((q >> 4) ^ sw) << 4) | (q & 15)
        while (h0 | h1) {
            int pos;
            if (h0) {
                pos = __builtin_ctzll(h0);
                h0 &= h0 - 1;
            } else {
                pos = 64 + __builtin_ctzll(h1);
                h1 &= h1 - 1;
            }
            const uint32_t cnt = (uint32_t)(pos - prev);
            const uint32_t nval = my[(uint32_t)pos ^ sw16];
            stc[slot] = (uint8_t)cnt;
            stv[slot] = (uint8_t)val;
            val = nval;
            ++slot;
            prev = pos;
        }
    }

    // Dense emission (a sub-chunk with more records than the staging holds),
    // part p: rows 16p .. 16p+15 of the image (row r = lane r's 64 bytes, head
    // mask hm, state c_lane before it, first record at `slot`, byte before it
    // p0 -- all held by lane r). Lane t takes piece k = t mod 4 (positions 16k
    // .. 16k+15) of row 16p + t / 4, so every lane is busy whatever the density,
    // and walks its 16 positions unrolled: values from the piece's bytes in
    // registers, counts from the previous head's position (or the row's state
    // before its first head); non-heads store to a sink byte of their own lane
    // (round 3's single sink address for all lanes was 12 % slower than a
    // branch per position; one per lane is 1 % faster). Record j of the part
    // (j = record - base + carry < 1024 + 15) goes to
    // stc/stv[pswz(j)]: the swizzle spreads the 64 lanes' stores, 16 rows x 4
    // pieces about 64 records apart, over all 64 banks. (Replaced one-row-at-
    // a-time emission, whose readlane/rank work per row made dense inputs 3.7x
    // slower than without it.)
    __device__ static uint32_t pswz(uint32_t j) { return j ^ (((j >> 8) & 3u) << 2); }
    __device__ void piece_part(int p, uint64_t hm, uint32_t c_lane, uint32_t slot, uint32_t p0, uint32_t base) const
    {
        const int k = lane & 3;
        const int r = 16 * p + (lane >> 2);
        const int src = r * 4;  // ds_bpermute address of lane r
        const uint32_t mlo = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)hm);
        const uint32_t mhi = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)(uint32_t)(hm >> 32));
        const uint32_t sr = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)slot);
        const uint32_t cr = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)c_lane);
        const uint32_t pr = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)p0);
        const uint64_t m = ((uint64_t)mhi << 32) | mlo;
        const u32x4 x = *reinterpret_cast<const u32x4 *>(img + (uint32_t)r * LB + (((uint32_t)k ^ swz((uint32_t)r)) * 16));
        const uint32_t up = wave_shr1(x.w >> 24);  // lane t-1 holds piece k-1 of the same row when k > 0
        const uint32_t pb = k == 0 ? pr : up;      // the byte before the piece
        const uint64_t below = k == 0 ? 0ull : m & ((1ull << (16 * k)) - 1);
        const uint32_t rank0 = sr + (uint32_t)__popcll(below) - base;
        // count of a head at pos = pos - prev; before the row's first head prev
        // is -c (the state before the row): c + pos <= 255 by the 255-split
        // rule, and the state 0 (255 bytes) has its head at pos 0, so every
        // count is in [1, 255]
        // (prev relative to the piece: the positions are then immediates, not
        // sixteen registers of 16k + i)
        int32_t prev = (below ? 63 - __builtin_clzll(below) : (cr == 0 ? -255 : -(int32_t)cr)) - 16 * k;
        const uint32_t m16 = (uint32_t)(m >> (16 * k)) & 0xFFFFu;
        uint32_t rank = rank0;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            // heads at positions <= i (bits 0..i moved to the top): position
            // i is a head iff it raises the rank
            // (v_bcnt with the add folded in: written as a sum, the compiler
            // compares the two popcounts and adds rank0 again under the head)
            uint32_t rnext;
            asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(rnext) : "v"(m16 << (31 - i)), "v"(rank0));
            const int32_t pos = i;
            const uint32_t val = i == 0 ? pb : (x[(i - 1) >> 2] >> (8 * ((i - 1) & 3))) & 0xFFu;
            // (non-heads to a per-lane sink byte past the part's records
            // instead of a branch per position: random bytes -1 %)
            const bool h = rnext != rank;
            const uint32_t at = h ? pswz(rank) : kPieceSink + 4u * (uint32_t)lane;
            stc[at] = (uint8_t)(pos - prev);
            stv[at] = (uint8_t)val;
            prev = h ? pos : prev;
            rank = rnext;
        }
    }

    // 16 bytes of records o .. o+15 of a piece-staged array (pswz layout; o may
    // be negative: those bytes read as 0 and are never stored)
    __device__ static u32x4 piece_gather(const uint8_t *st, int32_t o)
    {
        const int32_t d = o >> 2;  // arithmetic: floor
        const uint32_t sh = (uint32_t)o & 3u;
        uint32_t w[5];
#pragma unroll
        for (int i = 0; i < 5; ++i)
            w[i] = d + i < 0 ? 0u : *reinterpret_cast<const uint32_t *>(st + pswz(4u * (uint32_t)(d + i)));
        return u32x4{__builtin_amdgcn_alignbyte(w[1], w[0], sh), __builtin_amdgcn_alignbyte(w[2], w[1], sh),
                     __builtin_amdgcn_alignbyte(w[3], w[2], sh), __builtin_amdgcn_alignbyte(w[4], w[3], sh)};
    }

    // Records [0, nrec) of a piece-staged part to counts/values at global record
    // index g0 + j, i.e. byte g0 + j - 1 (the input's first head, g0 + j == 0,
    // ends no run): one 16-byte store per lane and array for every aligned
    // chunk inside the range, 1/2/4/8-byte pieces for a chunk the range shares.
    // Unless `last`, the records of a trailing partial chunk are not stored but
    // moved to staging [0, keep) (returned) and go out with the next part: a
    // dense run of parts then stores whole chunks only, one instruction per
    // lane and array (a part is <= 1024 records + the carry, <= 64 chunks
    // after the first), apart from its first and last chunk.
    __device__ uint32_t piece_flush(uint32_t nrec, uint64_t g0, bool last, uint8_t *__restrict__ counts,
                                    uint8_t *__restrict__ values) const
    {
        const uint32_t j0 = g0 == 0 ? 1u : 0u;
        if (nrec <= j0)
            return last ? 0u : nrec;
        // destination bytes [A, E) = [g0 + j0 - 1, g0 + nrec - 1), in 16-byte
        // chunks from the one holding A; chunk q starts at record (q - h) * 16 - a
        const uint64_t A = g0 + j0 - 1;
        const uint32_t a = (uint32_t)(A & 15u);  // A's offset in its chunk
        const uint32_t span = a + (nrec - j0);   // bytes from the chunk start to E
        // kept: the records of the chunk holding E - 1 when it is partial (all
        // of them when that chunk is also A's)
        const uint32_t keep = last || (span & 15u) == 0 ? 0u : (span < 16 ? nrec : (span & 15u));
        const uint32_t stop = span - ((span & 15u) && !last ? (span & 15u) : 0u);
        uint8_t *const pc = counts + (A - a), *const pv = values + (A - a);
        if (a == 0 && j0 == 0) {
            // chunk q = staged records 16q .. 16q+15, one aligned 16-byte group
            // whose dwords pswz permutes by t = bits 8-9 of 16q: dword i at i ^ t
            for (uint32_t q = (uint32_t)lane; 16 * q < stop; q += kWave) {
                const uint32_t t = (q >> 4) & 3u;
                const uint32_t hi = span - 16 * q < 16 ? span - 16 * q : 16u;
#pragma unroll
                for (int arr = 0; arr < 2; ++arr) {
                    const u32x4 r = *reinterpret_cast<const u32x4 *>((arr ? stv : stc) + 16 * q);
                    const u32x4 s = (t & 1u) ? u32x4{r.y, r.x, r.w, r.z} : r;
                    const u32x4 v = (t & 2u) ? u32x4{s.z, s.w, s.x, s.y} : s;
                    uint8_t *const d = (arr ? pv : pc) + 16 * q;
                    if (hi == 16)
                        *reinterpret_cast<u32x4 *>(d) = v;
                    else
                        store_chunk_part(d, v, 0u, hi);
                }
            }
        } else {
            for (uint32_t q = (uint32_t)lane; 16 * q < stop; q += kWave) {
                const int32_t o = (int32_t)(16 * q) - (int32_t)a + (int32_t)j0;  // record of the chunk's first byte
                const uint32_t lo = q == 0 ? a : 0u;
                const uint32_t hi = span - 16 * q < 16 ? span - 16 * q : 16u;
#pragma unroll
                for (int arr = 0; arr < 2; ++arr) {
                    const u32x4 v = piece_gather(arr ? stv : stc, o);
                    uint8_t *const d = (arr ? pv : pc) + 16 * q;
                    if (lo == 0 && hi == 16) {
                        *reinterpret_cast<u32x4 *>(d) = v;  // (non-temporal: +-0.2 %)
                    } else {
                        store_chunk_part(d, v, lo, hi);
                    }
                }
            }
        }
        if (keep != 0 && keep != nrec) {  // wave-uniform; the wave's reads all precede its writes
            const uint32_t j = (uint32_t)lane;
            uint32_t c = 0, v = 0;
            if (j < keep) {
                const uint32_t from = pswz(nrec - keep + j);
                c = stc[from];
                v = stv[from];
            }
            if (j < keep) {
                const uint32_t to = pswz(j);
                stc[to] = (uint8_t)c;
                stv[to] = (uint8_t)v;
            }
        }
        return keep;
    }

    // The staging pass over the chunk at `off` (`len` bytes): every sub-chunk's
    // PhaseMap and natural heads; the runs of the state-independent heads are
    // staged in LDS (stc/stv) at their chunk-local index until the staging area
    // is full (nst: the sub-chunks staged completely).
    __device__ void scan_chunk(uint64_t off, uint32_t len, Chunk &C) const
    {
        C.off = off;
        C.len = len;
        C.ns = (int)((len + WB - 1) / WB);
        // PF sub-chunks in flight per wave (register sets used in turn)
        constexpr int PF = PFD;
        static_assert(PF >= 1 && PF <= SUB && SUB % PF == 0, "prefetch depth");
        u32x4 pf[PF][NJ];
        uint32_t p_sub = 0;
        C.v0 = 0;
        if (C.ns > 0) {
            load_sub(off, 0, pf[0]);
#pragma unroll
            for (int k = 1; k < PF; ++k)
                if (k < C.ns)
                    load_sub(off, k, pf[k]);
            p_sub = off > 0 ? (uint32_t)in[off - 1] : 0u;
        }
        uint32_t rel_in = kMapIdent;  // PhaseMap from the chunk start to this sub-chunk
        uint32_t first = kNone;
        uint32_t K = 0;
        int nst = SUB;
        uint32_t Kst = 0, rel_st = kMapIdent;
        auto step = [&](int s, u32x4 (&buf)[NJ]) {
            Sub L;
            const uint32_t last = scan_sub(off, s, L, buf, p_sub, s + PF < C.ns ? s + PF : -1);
            if (s == 0)
                C.v0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)img[0]);
            p_sub = last;
            const bool seen = first != kNone;
            const uint32_t lrel = pm_compose(rel_in, L.lrel);
            bool lane_indep = false, after = false;
            if (seen) {
                lane_indep = after = true;
            } else if (L.sfirst != kNone && o + LB > L.sfirst) {
                lane_indep = true;
                after = o > L.sfirst;
            }
            const uint32_t cr = after ? pm_apply(lrel, 1) : 0u;  // constant after the first head
            uint64_t h0 = 0, h1 = 0;
            uint32_t indep = 0;
            if (lane_indep) {
                head_masks(L, cr, after, h0, h1);
                indep = (uint32_t)(__popcll(h0) + __popcll(h1));
            }
            const uint32_t hincl = wave_incl_scan_u32(indep);
            const uint32_t ks = (uint32_t)__builtin_amdgcn_readlane((int)hincl, kWave - 1);
            if (nst == SUB && K + ks > (uint32_t)SW) {  // wave-uniform
                nst = s;
                Kst = K;
                rel_st = rel_in;
            }
            const uint32_t slot = K + (hincl - indep);
            if (!seen && L.sfirst != kNone)
                first = (uint32_t)s * WB + L.sfirst;
            K += ks;
            rel_in = pm_compose(rel_in, L.smap);
            if (nst == SUB && indep)
                lane_runs(L, h0, h1, cr, slot);
        };
        for (int s = 0; s < C.ns; s += PF) {
            step(s, pf[0]);
#pragma unroll
            for (int k = 1; k < PF; ++k)
                if (s + k < C.ns)
                    step(s + k, pf[k]);
        }
        if (nst >= C.ns) {
            nst = C.ns;
            Kst = K;
            rel_st = rel_in;
        }
        C.nst = nst;
        C.first = first;
        C.K = K;
        C.Kst = Kst;
        C.rel_in = rel_in;
        C.rel_st = rel_st;
    }

    // Sub-chunks [s0, ns) of the chunk at `off`, re-read and emitted with the
    // true states: hb = the global index of sub-chunk s0's first record, rel =
    // the PhaseMap from the chunk start to s0, c_in = the chunk's incoming state.
    __device__ void reread(uint64_t off, int s0, int ns, uint64_t hb, uint32_t rel, uint32_t c_in,
                           uint8_t *__restrict__ counts, uint8_t *__restrict__ values) const
    {
        off = uniform64(off);
        hb = uniform64(hb);
        rel = uniform32(rel);
        c_in = uniform32(c_in);
        const uint64_t re_off = off + (uint64_t)s0 * WB;
        uint32_t pb = uniform32(re_off > 0 ? (uint32_t)in[re_off - 1] : 0u);
        u32x4 pf[NJ];
        load_sub(off, s0, pf);
        // records of the piece parts not yet stored (a partial last chunk),
        // staged at [0, carry): global record indices hb - carry .. hb - 1
        uint32_t carry = 0;
        for (int s = s0; s < ns; ++s) {
            // the previous sub-chunk's reads of the staging and the image are
            // this wave's own LDS ops: in order
            Sub L;
            pb = scan_sub(off, s, L, pf, pb, -1);
#pragma unroll
            for (int j = 0; j < NJ; ++j)
                pf[j] = u32x4{0u, 0u, 0u, 0u};  // consumed: not live until the next load
            const uint32_t c_lane = pm_apply(pm_compose(rel, L.lrel), c_in);
            uint64_t hm0, hm1;
            head_masks(L, c_lane, true, hm0, hm1);
            const uint32_t hl = (uint32_t)(__popcll(hm0) + __popcll(hm1));
            const uint32_t hincl = wave_incl_scan_u32(hl);
            const uint32_t hs = (uint32_t)__builtin_amdgcn_readlane((int)hincl, kWave - 1);
            const uint64_t g = hb + (hincl - hl);
            if (hs <= (uint32_t)SW) {
                // stage at (g - hb), store contiguously
                if (s + 1 < ns)
                    load_sub(off, s + 1, pf);
                if (carry) {  // the pieces' last records first: the staging is reused
                    piece_flush(carry, hb - carry, true, counts, values);
                    carry = 0;
                    wave_lds_sync();
                }
                lane_runs(L, hm0, hm1, c_lane, (uint32_t)(g - hb));
                wave_lds_sync();
                for (uint32_t j = lane; j < hs; j += kWave) {
                    const uint64_t gi = hb + j;
                    if (gi > 0) {
                        counts[gi - 1] = stc[j];
                        values[gi - 1] = stv[j];
                    }
                }
                wave_lds_sync();
            } else {
                // four parts of 16 rows (<= 1024 records each + the carry, within
                // the staging), each staged by piece_part after the carried records
                // and stored with 16-byte stores
                const uint32_t sl = (uint32_t)(g - hb);
                // the next sub-chunk's loads before the pieces, older than their
                // stores (round 6: random bytes -0.5 %, runs of 1..2 -2.2 %, 1..3
                // -2.8 %, runs32 equal; in round 5, before the carry, within noise)
                if (s + 1 < ns)
                    load_sub(off, s + 1, pf);
#pragma unroll 1
                for (int p = 0; p < kWave / 16; ++p) {
                    const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)sl, 16 * p);
                    const uint32_t b1 = p + 1 < kWave / 16 ? (uint32_t)__builtin_amdgcn_readlane((int)sl, 16 * (p + 1)) : hs;
                    piece_part(p, hm0, c_lane, sl, L.p0, b0 - carry);
                    wave_lds_sync();
                    carry = uniform32(piece_flush(carry + (b1 - b0), hb + b0 - carry, false, counts, values));
                    wave_lds_sync();
                }
            }
            hb += hs;
            rel = pm_compose(rel, L.smap);
        }
        if (carry)
            piece_flush(carry, hb - carry, true, counts, values);
    }

    // Emission of chunk C with the state (heads before it, chunk state) at its
    // start; its staged records are in stc/stv. The wave whose chunk ends the
    // input also writes the final run and R.
    __device__ void emit(const Chunk &C, uint64_t h_in, uint32_t c_in, uint8_t *__restrict__ counts,
                         uint8_t *__restrict__ values, uint64_t *__restrict__ runs_out) const
    {
        if (C.ns == 0)
            return;
        h_in = uniform64(h_in);
        c_in = uniform32(c_in);
        const uint32_t pre = C.pre();
        {
            // staged sub-chunks [0, nst): split heads h_in + j end full 255-byte
            // chunks of the chunk's first byte, then the staged records
            const uint32_t st_len = (uint32_t)C.nst * WB;
            const uint32_t S_st = splits(c_in, pre < st_len ? pre : st_len);
            for (uint32_t j = (uint32_t)lane; j < S_st; j += kWave) {
                const uint64_t gi = h_in + j;
                if (gi > 0) {
                    counts[gi - 1] = 255;
                    values[gi - 1] = (uint8_t)C.v0;
                }
            }
            const uint64_t g0 = h_in + S_st;  // global index of the first natural head
            if (C.Kst) {
                if (lane == 0 && g0 > 0) {
                    const uint32_t c = add_c(c_in, C.first);
                    counts[g0 - 1] = (uint8_t)(c == 0 ? 255u : c);
                    values[g0 - 1] = stv[0];
                }
                for (uint32_t j = 1 + (uint32_t)lane; j < C.Kst; j += kWave) {
                    counts[g0 + j - 1] = stc[j];
                    values[g0 + j - 1] = stv[j];
                }
            }
        }
        if (C.nst < C.ns) {
            // sub-chunks [nst, ns) overflowed the staging: re-read and emitted
            // with the true states (the tile was read a few microseconds ago:
            // the re-read mostly hits the caches; deferring it to a second
            // kernel, which re-reads from HBM, was 1.4-1.9x slower on dense inputs)
            const uint64_t hb = h_in + splits(c_in, pre < (uint32_t)C.nst * WB ? pre : (uint32_t)C.nst * WB) + C.Kst;
            reread(C.off, C.nst, C.ns, hb, C.rel_st, c_in, counts, values);
        }
        // the final run (ends at byte n-1): the wave whose chunk holds it
        if (C.off + C.len == n && lane == 0) {
            const uint64_t R = h_in + splits(c_in, pre) + C.K;
            const uint32_t c_end = pm_apply(C.rel_in, c_in);
            counts[R - 1] = (uint8_t)(c_end == 0 ? 255u : c_end);
            values[R - 1] = in[n - 1];
            *runs_out = R;
        }
    }
};

__device__ __forceinline__ uint64_t dpp64_up(uint64_t v, int step)
{
    switch (step) {
    case 0: return ((uint64_t)dpp_up0<0x111, 0xF>((uint32_t)(v >> 32)) << 32) | dpp_up0<0x111, 0xF>((uint32_t)v);
    case 1: return ((uint64_t)dpp_up0<0x112, 0xF>((uint32_t)(v >> 32)) << 32) | dpp_up0<0x112, 0xF>((uint32_t)v);
    case 2: return ((uint64_t)dpp_up0<0x114, 0xF>((uint32_t)(v >> 32)) << 32) | dpp_up0<0x114, 0xF>((uint32_t)v);
    case 3: return ((uint64_t)dpp_up0<0x118, 0xF>((uint32_t)(v >> 32)) << 32) | dpp_up0<0x118, 0xF>((uint32_t)v);
    case 4: return ((uint64_t)dpp_up0<0x142, 0xA>((uint32_t)(v >> 32)) << 32) | dpp_up0<0x142, 0xA>((uint32_t)v);
    default: return ((uint64_t)dpp_up0<0x143, 0xC>((uint32_t)(v >> 32)) << 32) | dpp_up0<0x143, 0xC>((uint32_t)v);
    }
}
__device__ __forceinline__ uint64_t wave_incl_scan_sm(uint64_t m)
{
#pragma unroll
    for (int k = 0; k < 6; ++k)
        m = sm_compose(dpp64_up(m, k), m);
    return m;
}

// The map of tile t from its input, for the look-back's fallback (help): each
// lane walks its 1/64 of the tile byte by byte with the encoder's state rule
// (a byte is a head iff it is natural or c == 0; then c = 1, else c = c + 1
// mod 255) and the lanes' maps are composed across the wave. Few registers, so
// the hot path keeps its allocation; slow (~tens of microseconds), which the
// fallback can afford.
template <int TBT>
__device__ uint64_t rl_tile_map_slow(const uint8_t *__restrict__ in, uint64_t n, uint32_t t)
{
    constexpr uint32_t PER = TBT / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    const uint64_t a = (uint64_t)t * TBT + (uint64_t)lane * PER;  // 4-byte aligned
    const uint64_t b = a + PER < n ? a + PER : n;
    const uint32_t cnt = a < b ? (uint32_t)(b - a) : 0u;
    const uint8_t *const p = in + a;
    uint32_t pre = 0, K = 0, c = 0, prev = a > 0 && a < n ? p[-1] : 0u;
    bool seen = false;
    auto step = [&](uint32_t x, bool first_of_input) {
        const bool nat = first_of_input || x != prev;
        if (!seen) {
            if (nat) {
                seen = true;
                K = 1;
                c = 1;
            } else {
                ++pre;
            }
        } else if (nat || c == 0) {
            ++K;
            c = 1;
        } else {
            c = c + 1 == 255 ? 0u : c + 1;
        }
        prev = x;
    };
    // whole words with the next one in flight (few registers: the hot path
    // keeps its allocation), then the last bytes
    const uint32_t nw = cnt / 4;
    const uint32_t *const p32 = reinterpret_cast<const uint32_t *>(p);
    uint32_t w = nw ? p32[0] : 0u;
#pragma unroll 1
    for (uint32_t i = 0; i < nw; ++i) {
        const uint32_t cur = w;
        if (i + 1 < nw)
            w = p32[i + 1];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            step((cur >> (8 * k)) & 0xFFu, a == 0 && i == 0 && k == 0);
    }
#pragma unroll 1
    for (uint32_t i = 4 * nw; i < cnt; ++i)
        step(p[i], a == 0 && i == 0);
    const uint64_t m = seen ? sm_nat(pre, K, c) : sm_nonat(cnt);
    return readlane64(wave_incl_scan_sm(m), kWave - 1);
}

// One tile per workgroup (grid = tiles, tile = workgroup index): stage,
// publish the tile map, ONE look-back by wave 0 while waves 1-3 wait, emit.
// Two block barriers per tile (wave maps, state).
template <int T, int LB, int SUB>
__global__ __launch_bounds__(T, kRlWavesPerSimd) void rl_encode_wave_kernel(  // (2nd: waves per SIMD)
    const uint8_t *__restrict__ in, uint64_t n, uint32_t ntiles, uint8_t *__restrict__ counts,
    uint8_t *__restrict__ values, uint64_t *__restrict__ runs_out, Ctrl *ctrl, uint64_t *status,
    uint64_t help_ticks)
{
    constexpr int W = T / kWave;
    using Wv = RlWave<LB, SUB, W>;
    __shared__ __attribute__((aligned(16))) uint8_t s_lds[Wv::kLdsBytes];
    __shared__ uint64_t s_map[W];
    __shared__ uint64_t s_st[W];

    const int tid = threadIdx.x;
    // the wave index in a scalar register: every chunk offset, length and
    // "whole sub-chunk" test below is then wave-uniform, so the compiler emits
    // scalar branches instead of executing masked tail paths (which it did,
    // at ~40 VALU instructions per sub-chunk)
    const int w = __builtin_amdgcn_readfirstlane(tid / kWave);
    const Wv V(in, n, s_lds, w);
    const uint32_t tile = blockIdx.x;  // (lookback_seg: why not a ticket)
    if (tile >= ntiles)
        return;
    FLRL_RL_TRACE(tile, 0);
    typename Wv::Chunk C;
    {
        const uint64_t off = (uint64_t)tile * Wv::TBT + (uint64_t)w * Wv::CB;
        const uint32_t len = off >= n ? 0u : (n - off < (uint64_t)Wv::CB ? (uint32_t)(n - off) : (uint32_t)Wv::CB);
        V.scan_chunk(off, len, C);
    }
    // ---- the wave maps -> the tile's map -> ONE look-back -> each wave's state
    if (V.lane == 0)
        s_map[w] = C.map();
    __syncthreads();
    FLRL_RL_TRACE(tile, 1);
    if (w == 0) {
        uint64_t tmap = s_map[0];
#pragma unroll
        for (int v = 1; v < W; ++v)
            tmap = sm_compose(tmap, s_map[v]);
        publish_seg<kRlStatusStride>(status, tile, tmap);
        FLRL_RL_TRACE(tile, 2);
        // decoupled fallback: a predecessor tile's map from its input
        auto help = [&](uint32_t t) -> uint64_t { return rl_tile_map_slow<Wv::TBT>(in, n, t); };
#if FLRL_RL_PMC_NOLB  // PMC builds only (output wrong): no status traffic, every tile at state (0, 0)
        uint64_t st = sm_const(0, 0);
        (void)help;
#else
        uint64_t st = lookback_seg<kRlLookG, kRlLookL, kRlStatusStride>(status, tile, tmap, ctrl, help_ticks, help);
#endif
        FLRL_RL_TRACE(tile, 3);
        if (V.lane == 0) {
#pragma unroll
            for (int v = 0; v < W; ++v) {
                s_st[v] = st;
                st = sm_compose(st, s_map[v]);
            }
        }
    }
    __syncthreads();
    V.emit(C, sm_h(s_st[w]), sm_c(s_st[w]), counts, values, runs_out);
    FLRL_RL_TRACE(tile, 4);
    // a launch counts exactly ntiles: more means the scratch was not reset for
    // it (its status words were stale too, so the output is not trusted)
    if (tid == 0 && atomicAdd(&ctrl->ticket, 1u) >= ntiles)
        raise_error(ctrl, FLRL_E_ARG);
}

// ---- decode pre-pass: output offsets of each decode tile ------------------
// A workgroup (4 waves) takes a contiguous span of iters x kRoRuns counts by
// ticket; wave w owns the w-th quarter of it and walks it in steps of 16384
// counts with no block barrier (waves overlap each other's loads), each step
// loaded coalesced (one load instruction = 1 KiB of consecutive counts: lane
// l, vector q holds counts 16 (64 q + l) .. + 15) and summed into TR-run tile
// sums by wave reductions; tile entries are written wave-relative. Then one
// block scan of the wave totals, the workgroup's base from all predecessors
// (block_prefix_all), and each wave adds its base to its own entries.
// (Lane-contiguous 128- or 256-byte segments with a block barrier per round
// ran at ~4 TB/s.)
constexpr int kRoThreads = 256;
constexpr int kRoWaves = kRoThreads / kWave;
constexpr int kRoQ = 16;                                // count vectors per lane per step
constexpr int kRoStep = kRoQ * 16 * kWave;              // counts per wave step (16384)
constexpr int kRoRuns = kRoStep * kRoWaves;             // counts per workgroup and iteration
constexpr size_t kRoMaxBlocks = FLRL_RL_RO_MAXB;        // workgroups: 256 (1 GiB runs32 call -2 %; 128: random bytes +13 %; 1024: the old cap)
static_assert(kRoMaxBlocks <= kMaxPrefixBlocks, "block_prefix_all bound");

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
    v += dpp_up0<0x111, 0xF>(v);
    v += dpp_up0<0x112, 0xF>(v);
    v += dpp_up0<0x114, 0xF>(v);
    v += dpp_up0<0x118, 0xF>(v);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 15) + (uint32_t)__builtin_amdgcn_readlane((int)v, 31) +
           (uint32_t)__builtin_amdgcn_readlane((int)v, 47) + (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

template <int TR>  // runs per decode tile
__global__ __launch_bounds__(kRoThreads, 4) void rl_offsets_kernel(  // 4 workgroups per CU
    const uint8_t *__restrict__ counts, uint64_t runs, uint64_t n, uint64_t *__restrict__ tile_base,
    uint32_t ntiles, uint32_t nblocks, uint32_t iters, Ctrl *ctrl, uint64_t *status)
{
    constexpr int TPS = kRoStep / TR;  // tiles per wave step
    constexpr int QPT = kRoQ / TPS;    // vectors per lane per tile
    static_assert(kRoStep % TR == 0 && TPS <= kWave, "whole tiles per wave step");
    __shared__ uint32_t s_ticket;
    __shared__ uint64_t s_wtot[kRoWaves];
    __shared__ uint64_t s_red[kRoWaves];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const uint32_t blk = take_ticket(ctrl, &s_ticket);
    if (blk >= nblocks) {  // the scratch's ticket was not reset for this launch
        if (threadIdx.x == 0)
            raise_error(ctrl, FLRL_E_ARG);
        return;
    }
    // this wave's span: iters steps of kRoStep counts
    const uint64_t w0 = ((uint64_t)blk * kRoWaves + wave) * iters * (uint64_t)kRoStep;
    uint64_t wrun = 0;  // output bytes of the wave's span so far
    uint64_t keep = 0;
    uint32_t zacc = 0;  // SWAR flags of zero counts
    for (uint32_t it = 0; it < iters; ++it) {
        const uint64_t wb = w0 + (uint64_t)it * kRoStep;
        if (wb >= runs)
            break;
        u32x4 cq[kRoQ];
        uint32_t sq[kRoQ];
        if (wb + kRoStep <= runs) {
#pragma unroll
            for (int q = 0; q < kRoQ; ++q)  // non-temporal: 1 GiB of counts 0.233 -> 0.191 ms
                cq[q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(counts + wb + 16 * (q * kWave + lane)));
#pragma unroll
            for (int q = 0; q < kRoQ; ++q) {
                sq[q] = 0;
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const uint32_t x = cq[q][d];
                    sq[q] = __builtin_amdgcn_udot4(x, 0x01010101u, sq[q], false);
                    zacc |= (x - 0x01010101u) & ~x & 0x80808080u;  // a zero count is malformed
                }
            }
        } else {  // the last counts: bytes past them are masked off
#pragma unroll
            for (int q = 0; q < kRoQ; ++q)
                cq[q] = load16_clamped(counts, wb + 16 * (q * kWave + lane), runs);
#pragma unroll
            for (int q = 0; q < kRoQ; ++q) {
                sq[q] = 0;
                const uint32_t valid = valid16(wb + 16 * (q * kWave + lane), runs);
#pragma unroll
                for (int d = 0; d < 4; ++d) {
                    const uint32_t x = mask_dword(cq[q][d], valid, d);
                    sq[q] = __builtin_amdgcn_udot4(x, 0x01010101u, sq[q], false);
                    zacc |= mask_dword((x - 0x01010101u) & ~x & 0x80808080u, valid, d);
                }
            }
        }
        // tile j of the step: vectors j QPT .. j QPT + QPT - 1 of every lane
        uint64_t run = wrun;
#pragma unroll
        for (int j = 0; j < TPS; ++j) {
            uint32_t pj = 0;
#pragma unroll
            for (int q = j * QPT; q < (j + 1) * QPT; ++q)
                pj += sq[q];
            const uint32_t tsum = wave_sum_u32(pj);
            const uint64_t tile = wb / TR + j;
            if (lane == j && tile < ntiles) {
                if (iters == 1)
                    keep = run;  // one step: the entry waits in a register for the base
                else
                    tile_base[tile] = run;  // wave-relative; the bases are added below
            }
            run += tsum;
        }
        wrun = run;
    }
    if (zacc != 0)
        raise_error(ctrl, FLRL_E_FORMAT);
    if (lane == 0)
        s_wtot[wave] = wrun;
    __syncthreads();
    uint64_t wbase = 0, local = 0;
#pragma unroll
    for (int v = 0; v < kRoWaves; ++v) {
        wbase += v < wave ? s_wtot[v] : 0ull;
        local += s_wtot[v];
    }
    // workgroup base from all predecessors (iters keeps the grid within kMaxPrefixBlocks)
    const uint64_t base = block_prefix_all<kRoThreads>(status, blk, local, ctrl, s_red) + wbase;
    // this wave's entries: tiles w0 / TR .. of its span, one per lane. They were
    // stored by other lanes of this wave: wait until those stores are done and
    // read past the L1 (agent-scope loads).
    const uint64_t t0 = w0 / TR, t1 = (w0 + (uint64_t)iters * kRoStep) / TR;
    if (iters == 1) {
        if (lane < TPS && t0 + lane < ntiles)
            tile_base[t0 + lane] = keep + base;
    } else {
        __builtin_amdgcn_s_waitcnt(0);
        for (uint64_t t = t0 + lane; t < t1 && t < ntiles; t += kWave)
            tile_base[t] = granule_load(&tile_base[t]) + base;
    }
    if (blk + 1 == nblocks && tid == 0) {
        tile_base[ntiles] = base - wbase + local;
        if (base - wbase + local != n)
            raise_error(ctrl, FLRL_E_FORMAT);
    }
}

// One 16-byte output chunk of a rank-decode window (block and wave decode):
// q = the chunk's index in the window; bm / pre = the window's start bitmap
// and the runs starting before each bitmap word; v32 = the tile's values (run
// indices tile-local); pfx = the byte-prefix popcount table; before = runs
// starting before the window. The run of the chunk's first byte is (runs
// before it) + (its start bit) - 1; byte i takes run r + k_i (k_i = start bits
// in bytes 1..i), gathered with byte permutes. (Gathering from the 16 values
// from run r on took three permutes per dword; two 8-value windows take one:
// VALU instructions -25 %, 1 GiB runs32 kernel -2..6 %.)
// Slot of byte-prefix table entry x. A ds_read_b64 serves 32 lanes per LDS
// cycle, entry slot s on banks 2s, 2s+1 (mod 64): plain slots put entries 0,
// 32, 64 and 128 on one bank pair, and with sparse start masks (runs32: a start
// every other chunk) those are most of the lookups -- ~5.5 LDS cycles per
// lookup instead of 2 in a model of runs32 masks; three padding slots per 32
// entries spread the single-bit entries over distinct banks (~2.2).
constexpr int kPfxSlots = 256 + 3 * 7 + 1;
__device__ __forceinline__ uint32_t pfx_slot(uint32_t x) { return x + 3u * (x >> 5); }

__device__ __forceinline__ u32x4 rd_chunk(const uint32_t *bm, const uint32_t *pre, const uint32_t *v32,
                                          const uint64_t *pfx, uint32_t q, uint32_t before)
{
    const uint32_t word = bm[q >> 1];
    const uint32_t m = (q & 1) ? word >> 16 : word & 0xFFFFu;
    const uint32_t pq = pre[q >> 1] + ((q & 1) ? __popc(word & 0xFFFFu) : 0u);
    int32_t r = (int32_t)(before + pq + (m & 1u)) - 1;  // run of byte 0
    uint32_t m1 = m & 0xFFFEu;                            // starts after byte 0
    if (r < 0) {  // bytes before the tile's first start are not stored
        m1 &= m1 - 1;
        r = 0;
    }
    // (no separate path for chunks without an inner start, m1 = 0: a wave
    // almost always holds both kinds, so it would run both; -2 %)
    // k_i <= i and k_(i+1) - k_i <= 1, so each 8-byte half needs only the 8
    // values from its own first run on: bytes 0-7 take values r + k_i (k_i <=
    // 7), bytes 8-15 values r8 + (k_i - k_8) with r8 = r + k_8 -- one byte
    // permute per output dword, selectors straight from the table
    const uint32_t a = (uint32_t)r >> 2, sh = (uint32_t)r & 3u;
    const uint32_t d0 = v32[a], d1 = v32[a + 1], d2 = v32[a + 2];
    const uint32_t r8 = (uint32_t)r + (uint32_t)__popc(m1 & 0x1FFu);
    const uint32_t a8 = r8 >> 2, sh8 = r8 & 3u;
    const uint32_t e0 = v32[a8], e1 = v32[a8 + 1], e2 = v32[a8 + 2];
    const uint64_t klo = pfx[pfx_slot(m1 & 0xFFu)], khi = pfx[pfx_slot((m1 >> 8) & 0xFEu)];
    const uint32_t w0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
    const uint32_t w1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    const uint32_t u0 = __builtin_amdgcn_alignbyte(e1, e0, sh8);
    const uint32_t u1 = __builtin_amdgcn_alignbyte(e2, e1, sh8);
    u32x4 o;
    o[0] = __builtin_amdgcn_perm(w1, w0, (uint32_t)klo);
    o[1] = __builtin_amdgcn_perm(w1, w0, (uint32_t)(klo >> 32));
    o[2] = __builtin_amdgcn_perm(u1, u0, (uint32_t)khi);
    o[3] = __builtin_amdgcn_perm(u1, u0, (uint32_t)(khi >> 32));
    return o;
}

// ---- decode by rank: output-driven windows ---------------------------------
// Every lane produces whole 16-byte output chunks, stored coalesced straight
// from registers. Per kRkWindow-byte window of a tile's output: (1) each run
// starting in the window sets its start bit in an LDS bitmap (ds_or), (2) a
// block scan of the bitmap words' popcounts gives, for every chunk, the number
// of runs that start before it, so (3) the run covering a chunk's first byte
// is (runs before the window) + (starts up to that byte) - 1; byte i of the
// chunk takes run r + k_i (k_i = start bits in bytes 1..i, an in-register byte
// prefix sum), gathered from the 16 values from run r on by byte permutes. No
// per-byte LDS stores, no LDS staging of the output. Lanes mark runs strided
// (lane t: runs t, t+256, ...) so one ds_or instruction targets consecutive
// runs' words, not words 16 runs apart (a 16-way bank conflict). Tiles with at
// most kRkDense bytes of output (mean run <= 8) keep the memset path. Output
// stores are plain (write-back) stores: with non-temporal stores the same
// kernel takes 0.335 instead of 0.281 ms on 1 GiB runs32 (scripts/ab_rl_decode.py).
// Measured against the LDS-window memset decode (scripts/ab_rl_decode.py, one
// process, decode call incl. offsets pre-pass): runs32 0.338 -> 0.290 ms,
// longruns 0.313 -> 0.272, random bytes 1.74 -> 1.24, lo4 1.79 -> 1.29.
// s_st index of run j: rows of 16 runs rotated by the row number, so the
// block scan's writes (thread t: runs 16t .. 16t + 15, one per instruction)
// spread over 16 banks instead of two; the marks' reads (consecutive j) stay
// conflict-free
__device__ __forceinline__ uint32_t rd_swz(uint32_t j) { return j ^ ((j >> 4) & 15u); }
constexpr int kRkWindow = 65536;            // output bytes per window
constexpr int kRkWords = kRkWindow / 32;    // bitmap words per window
constexpr int kRkDense = 32768;             // tiles with at most this much output: per-thread memsets

template <int T>
__global__ __launch_bounds__(T, 4) void rl_decode_kernel(  // 2nd: waves per SIMD (2 or 4 WG per CU)
    const uint8_t *__restrict__ counts, const uint8_t *__restrict__ values, uint64_t runs,
    uint8_t *__restrict__ out, uint64_t n, const uint64_t *__restrict__ tile_base, uint64_t ntiles,
    Ctrl *ctrl, uint32_t ticket0, bool tickets)
{
    constexpr int kRdRuns = 16 * T;  // runs per tile
    constexpr int RPT = kRdRuns / T;        // runs per thread
    constexpr int WPT = kRkWords / T;       // bitmap words per thread (scan)
    constexpr int CPT = kRkWindow / 16 / T; // chunks per thread per window
    static_assert(RPT == 16 && WPT % 4 == 0, "one 16-byte count/value vector, whole bitmap vectors per thread");
    // [bitmap: kRkWords][s_pre: kRkWords][s_st: kRdRuns + 1] u32; a dense tile
    // (output <= kRkDense bytes) uses the same LDS as its byte output window.
    // (Two bitmaps alternating by window, three barriers per window instead of
    // five: no change on any input kind)
    __shared__ u32x4 s_big4[(2 * kRkWords + kRdRuns + 1 + 3) / 4];
    __shared__ u32x4 s_val4[kRdRuns / 16 + 1];  // +16 B: the permute window reads up to 19 bytes past a run
    __shared__ uint32_t s_wave[T / kWave];
    __shared__ uint64_t s_pfx[kPfxSlots];  // byte i of s_pfx[pfx_slot(x)] = popcount(x & ((2 << i) - 1))
    static_assert(sizeof(s_big4) >= kRkDense, "dense window fits the aliased LDS");
    u32x4 *const s_bm4 = s_big4;
    uint32_t *const s_bm = reinterpret_cast<uint32_t *>(s_big4);
    uint32_t *const s_pre = s_bm + kRkWords;  // runs starting in the window before word w
    uint32_t *const s_st = s_pre + kRkWords;  // tile-local start of each run (+ the tile's total)
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;

    uint64_t tile = blockIdx.x;
    if (tile >= ntiles)
        return;
    // tickets: tiles from the third on by ticket, taken one tile ahead (the
    // pre-pass took tickets 0..ticket0-1), so the workgroups move through the
    // output together instead of drifting apart grid-stride (runs32: 1 GiB
    // -5 %, 4 GiB -10 %, runs of 1..64 -8 %); the first two tiles are
    // grid-stride, so no workgroup waits for a ticket at the start
    __shared__ uint32_t s_tk[2];
    uint32_t tslot = 0;
    bool first_round = true;  // the second tile is grid-stride too: no ticket wait at the start
    if (tid < 256) {
        static_assert(T >= 256, "one table entry per thread");
        uint64_t e = 0;
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            c += (tid >> i) & 1;
            e |= (uint64_t)c << (8 * i);
        }
        s_pfx[pfx_slot(tid)] = e;  // read after the first tile's barriers
    }
    u32x4 cv = load16_tail(counts, tile * kRdRuns + tid * RPT, runs);
    u32x4 vv = load16_tail(values, tile * kRdRuns + tid * RPT, runs);
    // The tile's output bounds come in by a VECTOR load (lane 0: start, lane 1:
    // end): a uniform scalar load of them counts in lgkmcnt, so every LDS wait
    // of the tile would also wait for that HBM round trip.
    uint64_t tbv = tile_base[tile + (lane & 1)];
    for (;;) {
        __syncthreads();  // the previous tile's LDS readers are done; s_tk written
        uint64_t next = tile + gridDim.x;
        if (tickets) {
            if (!first_round)
                next = s_tk[tslot ^ 1u];
            if (threadIdx.x == 0)  // the tile after next, read two barriers from now
                s_tk[tslot] = atomicAdd(&ctrl->ticket, 1u) - ticket0 + 2u * gridDim.x;
            tslot ^= 1u;
            first_round = false;
        }
        const uint64_t cbase = readlane64(tbv, 0), cend = readlane64(tbv, 1);
        const bool skip = cend > n || cbase >= cend;  // empty, or malformed (flagged by rl_offsets_kernel)
        s_val4[tid] = vv;
        const u32x4 vv_cur = vv;
        uint32_t c[RPT];
        uint32_t sum = 0;
#pragma unroll
        for (int i = 0; i < RPT; ++i) {
            c[i] = (cv[i >> 2] >> (8 * (i & 3))) & 0xFFu;
            sum += c[i];
        }
        if (next < ntiles) {  // next tile's loads in flight during this one
            cv = load16_tail(counts, next * kRdRuns + tid * RPT, runs);
            vv = load16_tail(values, next * kRdRuns + tid * RPT, runs);
            tbv = tile_base[next + (lane & 1)];
        }
        if (!skip) {
            const uint32_t inc = wave_incl_scan_u32(sum);
            if (lane == kWave - 1)
                s_wave[wave] = inc;
#pragma unroll
            for (int q = 0; q < WPT / 4; ++q)
                s_bm4[tid * (WPT / 4) + q] = u32x4{0u, 0u, 0u, 0u};
            __syncthreads();
            uint32_t before = 0;
#pragma unroll
            for (int v = 0; v < T / kWave; ++v)
                before += v < wave ? s_wave[v] : 0u;
            const uint64_t g0 = cbase & ~15ull;
            if (cend - g0 <= (uint64_t)kRkDense) {
                // dense tile (short runs): each thread memsets its own 16 runs from
                // registers into an LDS byte window, which leaves in 16-byte stores
                uint8_t *s_win = reinterpret_cast<uint8_t *>(s_big4);
                uint32_t p = (uint32_t)(cbase - g0) + before + inc - sum;
#pragma unroll
                for (int i = 0; i < RPT; ++i) {
                    const uint8_t v = (uint8_t)(vv_cur[i >> 2] >> (8 * (i & 3)));
                    const uint32_t q = p + c[i];
                    for (; p < q; ++p)
                        s_win[p] = v;
                }
                __syncthreads();
                const uint32_t wlen = (uint32_t)(cend - g0);
                // whole chunks from 16-byte stores; the (at most two) chunks shared with
                // the neighbouring tiles byte by byte, one byte per lane of waves 0 and 1
                // (one thread looping over them held the other waves at the next barrier)
                for (uint32_t ch = tid; ch * 16 < wlen; ch += T) {
                    const uint64_t gp = g0 + 16ull * ch;
                    if (gp >= cbase && gp + 16 <= cend)
                        *reinterpret_cast<u32x4 *>(out + gp) = s_big4[ch];  // plain: see the note above
                }
                if (wave < 2 && lane < 16) {
                    const uint32_t ch = wave == 0 ? 0u : (wlen - 1) / 16;
                    const uint64_t gp = g0 + 16ull * ch + (uint64_t)lane;
                    const bool edge = wave == 0 ? cbase > g0 || cend - g0 < 16 : (wlen & 15) != 0 && ch > 0;
                    if (edge && gp >= cbase && gp < cend)
                        out[gp] = reinterpret_cast<const uint8_t *>(s_big4)[16 * ch + lane];
                }
            } else {
            {
                uint32_t run = before + inc - sum;  // tile-local start of this thread's first run
#pragma unroll
                for (int i = 0; i < RPT; ++i) {
                    s_st[rd_swz(tid * RPT + i)] = run;
                    run += c[i];
                }
                if (tid == T - 1)
                    s_st[rd_swz(kRdRuns)] = run;
            }
            const uint32_t nr = (uint32_t)(runs - tile * kRdRuns < (uint64_t)kRdRuns ? runs - tile * kRdRuns
                                                                                      : kRdRuns);
            __syncthreads();
            uint32_t starts_before = 0;  // runs starting before the window
            for (uint64_t gw = g0; gw < cend; gw += kRkWindow) {
                // (1) start bits of the runs beginning in [gw, gw + W)
                // (strided: lane t takes runs t, t + T, ... so a wave's ds_or targets are
                // consecutive runs' start words -- distinct banks, not 16 words apart)
                // Only the runs that can start in this window: runs before it are
                // the first starts_before (counts >= 1), and starts are increasing.
                // Window-relative positions in 32 bits: a tile's output is at most
                // 16 T x 255 bytes, and the first window starts <= 15 bytes before it.
                const int32_t tb = (int32_t)(int64_t)(cbase - gw);  // tile start in the window
                const uint32_t ce = (uint32_t)(cend - gw);          // tile end in the window
                {
#pragma unroll 2  // (-1..1.5 % on runs32, runs of 1..32, long runs; 4: less)
                    for (int k = (int)(starts_before / T); k < RPT; ++k) {
                        const uint32_t j = (uint32_t)(k * T + tid);
                        if (j >= nr)
                            break;
                        const uint32_t x0 = s_st[rd_swz(j)], x1 = s_st[rd_swz(j + 1)];
                        const int32_t x = tb + (int32_t)x0;
                        if (x >= kRkWindow)
                            break;
                        if (x1 > x0 && x >= 0)
                            atomicOr(&s_bm[(uint32_t)x >> 5], 1u << (x & 31));
                    }
                }
                __syncthreads();
                // (2) popcount prefix over the window's words; thread t owns words [WPT t, WPT t + WPT)
                uint32_t pc[WPT];
                uint32_t tsum = 0;
#pragma unroll
                for (int q = 0; q < WPT / 4; ++q) {
                    const u32x4 w = s_bm4[tid * (WPT / 4) + q];
#pragma unroll
                    for (int d = 0; d < 4; ++d) {
                        pc[q * 4 + d] = __popc(w[d]);
                        tsum += pc[q * 4 + d];
                    }
                }
                const uint32_t tinc = wave_incl_scan_u32(tsum);
                if (lane == kWave - 1)
                    s_wave[wave] = tinc;
                __syncthreads();
                uint32_t wb = 0, wtot = 0;
#pragma unroll
                for (int v = 0; v < T / kWave; ++v) {
                    const uint32_t t = s_wave[v];
                    wb += v < wave ? t : 0u;
                    wtot += t;
                }
                {
                    uint32_t run = wb + tinc - tsum;
#pragma unroll
                    for (int q = 0; q < WPT; ++q) {
                        s_pre[tid * WPT + q] = run;
                        run += pc[q];
                    }
                }
                __syncthreads();
                // (3) chunks q = k*T + tid: 16 bytes each, coalesced stores
                const uint32_t wl = ce < (uint32_t)kRkWindow ? ce : (uint32_t)kRkWindow;
                const uint32_t b0 = tb > 0 ? (uint32_t)tb : 0u;
                uint8_t *const outw = out + gw;
#pragma unroll FLRL_RD_UNROLL
                for (int k = 0; k < CPT; ++k) {
                    const uint32_t q = (uint32_t)(k * T + tid);
                    const uint32_t off = 16u * q;
                    if (off >= wl)
                        break;
                    const u32x4 o = rd_chunk(s_bm, s_pre, reinterpret_cast<const uint32_t *>(s_val4), s_pfx, q,
                                             starts_before);
                    if (off >= b0 && off + 16 <= ce) {
                        *reinterpret_cast<u32x4 *>(outw + off) = o;  // plain: see the note above
                    } else {  // a chunk shared with a neighbouring tile: its bytes only
                        const uint32_t lo = off < b0 ? b0 - off : 0u;
                        const uint32_t hi = off + 16 > ce ? ce - off : 16u;
                        store_chunk_part(outw + off, o, lo, hi);
                    }
                }
                starts_before += wtot;
                if (gw + kRkWindow < cend) {
                    __syncthreads();  // chunk readers of the bitmap are done
#pragma unroll
                    for (int q = 0; q < WPT / 4; ++q)
                        s_bm4[tid * (WPT / 4) + q] = u32x4{0u, 0u, 0u, 0u};
                    __syncthreads();
                }
            }
            }
        }
        if (next >= ntiles)
            break;
        tile = next;
    }
}


// ---- decode, one wave per tile of 64 x RPL runs (dense inputs) -----------
// The block decode above spends its time on per-tile overhead when runs are
// short (a 4096-run tile of random bytes is only 4 KiB of output: three block
// barriers and a byte-memset loop that the compiler turns into ~30
// instructions per run). Here every wave decodes its own tiles (grid-stride
// over waves) with no block barrier: lane l holds runs RPL l .. RPL l + RPL - 1
// (RPL/16 count and value vectors), a wave scan places them, and the output is
// built by the same rank method per 8 KiB window -- each run's start bit is
// ds_or'ed into a wave-private bitmap (lane-contiguous runs: one instruction's
// targets are a lane's output length apart, <= 2 lanes per word for 1-byte
// runs), a wave scan of the words' popcounts ranks every 16-byte chunk, and
// each lane assembles whole chunks by byte permutes over the 16 values from the
// chunk's first run on and stores them coalesced. The two chunks a tile shares
// with its neighbours are stored as aligned 1/2/4/8-byte pieces. The offsets
// pre-pass runs at the wave tile's granularity for this kernel.
// Runs per lane: 32 (2048-run tiles), or 64 (4096-run tiles) for inputs with
// a mean run of at most kWd64Mean bytes (random bytes: -7 %; runs of 1..4 and
// longer: +2..4 %, so only the densest inputs take it).
constexpr int kWdRpl = 32;
constexpr int kWdRuns = kWave * kWdRpl;    // runs per wave tile (the finest tile_base granularity)
constexpr uint64_t kWd64Mean = FLRL_RL_WD64_MEAN;
constexpr int kWdWin = 8192;               // output bytes per window
constexpr int kWdWords = kWdWin / 32;      // bitmap words per window (4 per lane)
constexpr int kWdThreads = 256;
// resident workgroups per CU (VGPR-bound: 6 at 32 runs per lane, 5 at 64), also the launch bound
template <int RPL>
constexpr int wd_per_cu() { return RPL == 64 ? FLRL_RD_WD64_PER_CU : FLRL_RD_WD32_PER_CU; }
// inputs with a mean run of at most this many bytes take the wave decode
// (against the 512-thread block decode, 1 GiB: runs of 1..16 -15 %, 1..24
// equal, 1..32 +4 %)
constexpr uint64_t kWdDenseMean = FLRL_RL_DENSE_MEAN;
static_assert(kWdWords == 4 * kWave, "one bitmap vector per lane");



template <int RPL>
__global__ __launch_bounds__(kWdThreads, wd_per_cu<RPL>()) void rl_decode_wave_kernel(
    const uint8_t *__restrict__ counts, const uint8_t *__restrict__ values, uint64_t runs,
    uint8_t *__restrict__ out, uint64_t n, const uint64_t *__restrict__ tile_base, uint64_t ntiles)
{
    constexpr int NW = kWdThreads / kWave;
    static_assert(RPL % 16 == 0, "whole vectors per lane");
    constexpr int NV = RPL / 16;       // count / value vectors per lane
    constexpr int TR = kWave * RPL;    // runs per wave tile
    __shared__ u32x4 s_val4[NW][TR / 16 + 2];  // +32 B: the permute window reads up to 19 bytes past a run
    __shared__ u32x4 s_bm4[NW][kWdWords / 4 + 1];   // +1: a single-window tile's past-the-end marks
    __shared__ u32x4 s_pre4[NW][kWdWords / 4];      // starts in the window before word w
    __shared__ uint64_t s_pfx[kPfxSlots];           // byte i of s_pfx[pfx_slot(x)] = popcount(x & ((2 << i) - 1))
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    {
        static_assert(kWdThreads == 256, "one table entry per thread");
        uint64_t e = 0;
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            c += (tid >> i) & 1;
            e |= (uint64_t)c << (8 * i);
        }
        s_pfx[pfx_slot(tid)] = e;
    }
    __syncthreads();  // the only block barrier
    const uint64_t stride = (uint64_t)gridDim.x * NW;
    uint64_t tile = (uint64_t)blockIdx.x * NW + wave;
    if (tile >= ntiles)
        return;
    u32x4 *const sv4 = s_val4[wave];
    const uint32_t *const sv32 = reinterpret_cast<const uint32_t *>(sv4);
    u32x4 *const bm4 = s_bm4[wave];
    uint32_t *const bm = reinterpret_cast<uint32_t *>(bm4);
    u32x4 *const pre4 = s_pre4[wave];
    const uint32_t *const pre = reinterpret_cast<const uint32_t *>(pre4);
    if (lane < 2)
        sv4[TR / 16 + lane] = u32x4{0u, 0u, 0u, 0u};
    u32x4 cv[NV], vv[NV];
    // a tile's count and value vectors (zeros past the last run)
    auto load_tile = [&](uint64_t t) {
        const uint64_t r = t * TR + lane * RPL;
        if ((t + 1) * TR <= runs) {  // uniform: no per-load tail checks
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                cv[v] = *reinterpret_cast<const u32x4 *>(counts + r + 16 * v);  // (non-temporal: no change)
                vv[v] = *reinterpret_cast<const u32x4 *>(values + r + 16 * v);
            }
        } else {  // the last tile: counts are masked when used
#pragma unroll
            for (int v = 0; v < NV; ++v) {
                cv[v] = load16_clamped(counts, r + 16 * v, runs);
                vv[v] = load16_clamped(values, r + 16 * v, runs);
            }
        }
    };
    load_tile(tile);
    uint64_t tbv = tile_base[tile + (lane & 1)];  // vector load: lane 0 start, lane 1 end
    for (;;) {
        const uint64_t next = tile + stride;
        const uint64_t base = readlane64(tbv, 0), end = readlane64(tbv, 1);
        wave_lds_sync();  // the previous tile's readers of the values are done
        u32x4 cc[NV];     // counts stay packed
        uint32_t S = 0;
        const bool last = (tile + 1) * TR > runs;
#pragma unroll
        for (int v = 0; v < NV; ++v) {
            sv4[lane * NV + v] = vv[v];
            cc[v] = cv[v];
            if (last) {  // zero counts past the last run
                const uint32_t valid = valid16(tile * TR + lane * RPL + 16 * v, runs);
#pragma unroll
                for (int d = 0; d < 4; ++d)
                    cc[v][d] = mask_dword(cc[v][d], valid, d);
            }
#pragma unroll
            for (int d = 0; d < 4; ++d)
                S = __builtin_amdgcn_udot4(cc[v][d], 0x01010101u, S, false);
        }
        if (next < ntiles) {  // next tile's loads in flight during this one
            load_tile(next);
            tbv = tile_base[next + (lane & 1)];
        }
        if (end <= n && base < end) {  // else empty, or malformed (flagged by rl_offsets_kernel)
            const uint32_t inc = wave_incl_scan_u32(S);
            const uint64_t g0 = base & ~15ull;
            const uint32_t o = (uint32_t)(base - g0) + inc - S;  // window-relative start of the lane's first run
            const uint32_t len = (uint32_t)(end - g0);
            uint32_t starts_before = 0;  // runs starting before the window
            for (uint32_t w = 0; w < len; w += kWdWin) {
                bm4[lane] = u32x4{0u, 0u, 0u, 0u};
                wave_lds_sync();
                // (1) start bits of this lane's runs that begin in [w, w + W)
                // A zero count (past the last run; or malformed, flagged by the pre-pass)
                // marks the position of the next start or the tile's end again: harmless
                // (the bitmap has a word past the window for the latter).
                uint32_t p = o - w;
                if (len <= (uint32_t)kWdWin) {  // one window: every start is in it
#pragma unroll
                    for (int i = 0; i < RPL; ++i) {
                        atomicOr(bm + __builtin_amdgcn_ubfe(p, 5, 27), 1u << (p & 31));
                        p += (cc[i >> 4][(i >> 2) & 3] >> (8 * (i & 3))) & 0xFFu;
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < RPL; ++i) {
                        if (p <= (uint32_t)kWdWin)
                            atomicOr(bm + __builtin_amdgcn_ubfe(p, 5, 27), 1u << (p & 31));
                        p += (cc[i >> 4][(i >> 2) & 3] >> (8 * (i & 3))) & 0xFFu;
                    }
                }
                wave_lds_sync();
                // (2) popcount prefix over the window's words; lane owns words 4 lane .. 4 lane + 3
                const u32x4 wd = bm4[lane];
                const uint32_t p0 = __popc(wd[0]), p1 = __popc(wd[1]), p2 = __popc(wd[2]), p3 = __popc(wd[3]);
                const uint32_t tsum = p0 + p1 + p2 + p3;
                const uint32_t tinc = wave_incl_scan_u32(tsum);
                const uint32_t e0 = tinc - tsum;
                pre4[lane] = u32x4{e0, e0 + p0, e0 + p0 + p1, e0 + p0 + p1 + p2};
                const uint32_t wtot = (uint32_t)__builtin_amdgcn_readlane((int)tinc, kWave - 1);
                wave_lds_sync();
                // (3) chunks q = lane + 64 k of the window
                const uint32_t wl = len - w < (uint32_t)kWdWin ? len - w : (uint32_t)kWdWin;
                const uint32_t nch = (wl + 15) / 16;
                for (uint32_t q = lane; q < nch; q += kWave) {  // (unrolled by 2 or 4: +1..7 %)
                    const uint32_t gq = w + 16u * q;  // window-relative chunk start
                    const u32x4 ov = rd_chunk(bm, pre, sv32, s_pfx, q, starts_before);
                    const uint32_t b0 = (uint32_t)(base - g0);
                    const uint32_t lo = gq < b0 ? b0 - gq : 0u;
                    const uint32_t hi = gq + 16 > len ? len - gq : 16u;
                    if (lo == 0 && hi == 16)
                        *reinterpret_cast<u32x4 *>(out + g0 + gq) = ov;  // plain stores, as the block decode (nt: +4..17 %)
                    else  // a chunk shared with a neighbouring tile: its bytes only
                        store_chunk_part(out + g0 + gq, ov, lo, hi);
                }
                starts_before += wtot;
                wave_lds_sync();  // chunk readers of the bitmap are done before it is cleared
            }
        }
        if (next >= ntiles)
            break;
        tile = next;
    }
}

// [Ctrl][status: tiles, kRlStatusStride granules apart] (zeroed per call)
struct RlEncLayout {
    size_t tiles, zero, bytes;
    explicit RlEncLayout(size_t n)
    {
        tiles = div_up(n, (size_t)kRlTileBytes);
        zero = kRlStatusOff + round_up(tiles * 8 * kRlStatusStride, 16);  // ticket, error, status
        bytes = zero;
    }
};

struct RlDecLayout {
    size_t tiles, blocks, iters, zero, bytes;
    // tile_base is sized for the finer (wave) tiles; `tiles` counts the tiles
    // of the decode chosen for (runs, n)
    explicit RlDecLayout(size_t runs, size_t n = 0)
    {
        const bool dense = n != 0 && n <= kWdDenseMean * runs;
        const bool wide = n < kRdNarrowMean * runs;
        tiles = div_up(runs, (size_t)(dense ? kWdRuns : 16 * (wide ? kRdThreadsWide : kRdThreads)));
        // offsets rounds per workgroup: the grid stays within kMaxPrefixBlocks
        iters = div_up(div_up(runs, (size_t)kRoRuns), (size_t)kRoMaxBlocks);
        iters = iters ? iters : 1;
        blocks = div_up(runs, (size_t)kRoRuns * iters);
        zero = sizeof(Ctrl) + round_up(blocks * 8, 16);
        // the size a caller allocates must not shrink as runs grow (callers size
        // scratch for an upper bound of runs): bound blocks monotonically
        const size_t bmax = std::min(div_up(runs, (size_t)kRoRuns), (size_t)kMaxPrefixBlocks);
        bytes = sizeof(Ctrl) + round_up(bmax * 8, 16) + round_up((div_up(runs, (size_t)kWdRuns) + 1) * 8, 16);
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
    static_assert(kRlStatusOff % 16 == 0 && kRlStatusOff >= sizeof(Ctrl), "Ctrl area");
    FLRL_HIP(scratch_reset_strided(d_scratch, kRlStatusOff, L.tiles, 8 * kRlStatusStride, s));
    if (n == 0) {
        FLRL_HIP(zero_async(d_runs, sizeof(uint64_t), s));
        return FLRL_OK;
    }
    if (!d_in || !d_counts || !d_values)
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: null buffer");
    if (!aligned16(d_in))
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: input must be 16-byte aligned");
    if (L.tiles > 0xFFFFFFFFull)
        return set_error(FLRL_E_ARG, "flrl_rl_encode_device: input too large");
    Ctrl *ctrl = static_cast<Ctrl *>(d_scratch);
    uint64_t *status = reinterpret_cast<uint64_t *>(static_cast<uint8_t *>(d_scratch) + kRlStatusOff);
    kernel_timing_begin(s);
    hipLaunchKernelGGL((rl_encode_wave_kernel<kRlThreads, kRlLaneBytes, kRlSub>), dim3((uint32_t)L.tiles),
                       dim3(kRlThreads), 0, s, d_in, (uint64_t)n, (uint32_t)L.tiles, d_counts, d_values, d_runs,
                       ctrl, status, lookback_help_ticks(kRlHelpTicks));
    kernel_timing_end(s);
    FLRL_HIP(hipGetLastError());
    return FLRL_OK;
}

extern "C" int flrl_rl_decode_device(const uint8_t *d_counts, const uint8_t *d_values, size_t runs,
                                     uint8_t *d_out, size_t n, void *d_scratch,
                                     size_t scratch_bytes, void *stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    const RlDecLayout L(runs, n);
    const bool dense = n != 0 && n <= kWdDenseMean * runs;
    if (!d_scratch)
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: null scratch");
    if (scratch_bytes < L.bytes)
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: scratch %zu < required %zu",
                         scratch_bytes, L.bytes);
    if (!aligned16(d_scratch))
        return set_error(FLRL_E_ARG, "flrl_rl_decode_device: scratch not 16-byte aligned");
    FLRL_HIP(scratch_reset(d_scratch, L.zero, s));
    if (runs == 0) {
        if (n != 0)  // no runs cannot make n bytes: flagged like a malformed count
            FLRL_HIP(raise_error_async(d_scratch, FLRL_E_FORMAT, s));
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
    if (dense) {
        // mean run <= kWdDenseMean bytes: one wave per tile of 64 x RPL runs
        const bool densest = n <= kWd64Mean * runs;
        const size_t tiles = div_up(runs, (size_t)(densest ? 4096 : kWdRuns));
        if (densest)
            hipLaunchKernelGGL(rl_offsets_kernel<4096>, dim3((uint32_t)L.blocks), dim3(kRoThreads), 0, s,
                               d_counts, (uint64_t)runs, (uint64_t)n, tile_base, (uint32_t)tiles,
                               (uint32_t)L.blocks, (uint32_t)L.iters, ctrl, status);
        else
            hipLaunchKernelGGL(rl_offsets_kernel<kWdRuns>, dim3((uint32_t)L.blocks), dim3(kRoThreads), 0, s,
                               d_counts, (uint64_t)runs, (uint64_t)n, tile_base, (uint32_t)tiles,
                               (uint32_t)L.blocks, (uint32_t)L.iters, ctrl, status);
        FLRL_HIP(hipGetLastError());
        const size_t wgs = div_up(tiles, (size_t)(kWdThreads / kWave));
        const size_t wgrid = (size_t)(densest ? wd_per_cu<64>() : wd_per_cu<32>()) * (size_t)cu_count();
        const dim3 grid((uint32_t)(wgs < wgrid ? wgs : wgrid));
        kernel_timing_begin(s);
        if (densest)
            hipLaunchKernelGGL(rl_decode_wave_kernel<64>, grid, dim3(kWdThreads), 0, s, d_counts, d_values,
                               (uint64_t)runs, d_out, (uint64_t)n, tile_base, (uint64_t)tiles);
        else
            hipLaunchKernelGGL(rl_decode_wave_kernel<32>, grid, dim3(kWdThreads), 0, s, d_counts, d_values,
                               (uint64_t)runs, d_out, (uint64_t)n, tile_base, (uint64_t)tiles);
        kernel_timing_end(s);
        FLRL_HIP(hipGetLastError());
        return FLRL_OK;
    }
    const bool wide = n < kRdNarrowMean * runs;
    if (wide)
        hipLaunchKernelGGL(rl_offsets_kernel<16 * kRdThreadsWide>, dim3((uint32_t)L.blocks), dim3(kRoThreads), 0, s,
                           d_counts, (uint64_t)runs, (uint64_t)n, tile_base, (uint32_t)L.tiles,
                           (uint32_t)L.blocks, (uint32_t)L.iters, ctrl, status);
    else
        hipLaunchKernelGGL(rl_offsets_kernel<16 * kRdThreads>, dim3((uint32_t)L.blocks), dim3(kRoThreads), 0, s,
                           d_counts, (uint64_t)runs, (uint64_t)n, tile_base, (uint32_t)L.tiles,
                           (uint32_t)L.blocks, (uint32_t)L.iters, ctrl, status);
    FLRL_HIP(hipGetLastError());
    const size_t rgrid = (size_t)(wide ? rd_per_cu<kRdThreadsWide>() : rd_per_cu<kRdThreads>()) * (size_t)cu_count();
    const dim3 grid((uint32_t)(L.tiles < rgrid ? L.tiles : rgrid));
    kernel_timing_begin(s);
    // ticket order for the 512-thread decode from FLRL_RD_TICKET_MIN tiles per
    // workgroup on (long runs, 256-thread tiles: tickets +23 %)
    const bool tickets = wide && L.tiles >= (size_t)FLRL_RD_TICKET_MIN * grid.x;
    if (wide)
        hipLaunchKernelGGL(rl_decode_kernel<kRdThreadsWide>, grid, dim3(kRdThreadsWide), 0, s, d_counts, d_values,
                           (uint64_t)runs, d_out, (uint64_t)n, tile_base, (uint64_t)L.tiles, ctrl,
                           (uint32_t)L.blocks, tickets);
    else
        hipLaunchKernelGGL(rl_decode_kernel<kRdThreads>, grid, dim3(kRdThreads), 0, s, d_counts, d_values,
                           (uint64_t)runs, d_out, (uint64_t)n, tile_base, (uint64_t)L.tiles, ctrl,
                           (uint32_t)L.blocks, false);
    kernel_timing_end(s);
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
