// flrl_shard_layout.hpp — the arithmetic of the multi-GPU FL exchange, shared by
// the device code (size_scan_kernel, flrl_shard.hip) and the host C ABI
// (flrl_shard_* in include/flrl.h), so the CPU tests exercise the exact code
// the exchange runs.
//
//  * shard rule (file_io.cu:46-51, size_t instead of int): every shard but the
//    last is floor(N / (128 P)) * 128 bytes, the last takes the rest;
//  * gather layout: shard r runs on device r mod ndev as that device's local
//    shard r / ndev; each device holds S = ceil(P / ndev) slots of {F, V}
//    (2 u64) at ((r mod ndev) S + r / ndev) * 2, and the in-place all-gather
//    of every device's S slots leaves the same array on every device (in the
//    per-rank model ndev = P, S = 1: slot r at 2 r);
//  * the F word carries a "ragged" flag (bit 63) when the shard is not a whole
//    number of 128-byte frames; only the last shard may be ragged, otherwise
//    its successors' frames would start mid-frame and the concatenation would
//    no longer equal the whole-input encode;
//  * a shard whose rank failed locally (a bad argument, an allocation) still
//    joins the exchange, with a "failed" flag (bit 62) in its F word: every
//    rank's scan then reports FLRL_E_ARG, where returning before the
//    collective would leave every peer waiting in it;
//  * the record of shard `me` (FLRL_SZ_*): its F and V, the exclusive prefix
//    of F and V over shards 0..me-1 in shard order, and the totals.
#pragma once

#include <stdint.h>

#include "flrl.h"

#if defined(__HIPCC__)
#define FLRL_HD __host__ __device__
#else
#define FLRL_HD
#endif

namespace flrl {

constexpr uint64_t kRaggedBit = 1ull << 63;
constexpr uint64_t kFailedBit = 1ull << 62;
constexpr uint64_t kShardFlags = kRaggedBit | kFailedBit;

// shard_record's verdict bits
constexpr uint32_t kRecRagged = 1;  // a shard before the last is not whole frames
constexpr uint32_t kRecFailed = 2;  // some shard's rank failed locally

FLRL_HD inline void shard_range(uint64_t n, uint64_t P, uint64_t r, uint64_t *start, uint64_t *len)
{
    const uint64_t per = (n / (FLRL_FRAME_LENGTH * P)) * FLRL_FRAME_LENGTH;
    *start = r * per;
    *len = r + 1 == P ? n - (P - 1) * per : per;
}

FLRL_HD inline uint64_t shard_slot(uint64_t r, uint64_t ndev, uint64_t S)
{
    return ((r % ndev) * S + r / ndev) * 2;
}

// The F word a shard of n bytes puts into its slot.
FLRL_HD inline uint64_t shard_f_word(uint64_t n)
{
    return ((n + FLRL_FRAME_LENGTH - 1) / FLRL_FRAME_LENGTH) | (n % FLRL_FRAME_LENGTH ? kRaggedBit : 0);
}

// The F word (with V = 0) of a shard whose rank failed before its encode.
FLRL_HD inline uint64_t shard_failed_word() { return kFailedBit; }

// Record of shard `me` from the all-gathered slots (filled in every case; rec
// may be null). Returns 0, or kRecRagged / kRecFailed bits: a shard other than
// the last is ragged, or some shard's rank failed.
FLRL_HD inline uint32_t shard_record(const uint64_t *gather, uint32_t nshards, uint32_t ndev, uint32_t S,
                                     uint32_t me, uint64_t *rec)
{
    uint64_t F = 0, V = 0, Fo = 0, Vo = 0, Fr = 0, Vr = 0;
    uint32_t bad = 0;
    for (uint32_t r = 0; r < nshards; ++r) {
        const uint64_t *g = gather + shard_slot(r, ndev, S);
        const uint64_t fw = g[0], v = g[1];
        const uint64_t f = fw & ~kShardFlags;
        if ((fw & kRaggedBit) && r + 1 != nshards)
            bad |= kRecRagged;
        if (fw & kFailedBit)
            bad |= kRecFailed;
        if (r == me) {
            Fo = F;
            Vo = V;
            Fr = f;
            Vr = v;
        }
        F += f;
        V += v;
    }
    if (rec) {
        rec[FLRL_SZ_F] = Fr;
        rec[FLRL_SZ_V] = Vr;
        rec[FLRL_SZ_F_OFF] = Fo;
        rec[FLRL_SZ_V_OFF] = Vo;
        rec[FLRL_SZ_F_TOTAL] = F;
        rec[FLRL_SZ_V_TOTAL] = V;
    }
    return bad;
}

}  // namespace flrl
