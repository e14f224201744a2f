// flrl_tuning.hpp — the kernel shape constants, and the ONLY place where
// timing harnesses may override them or hook traces into the kernels.
//
// The shipped build (Makefile) defines none of the FLRL_* macros below: every
// constant then takes the value measured best (DESIGN.md §4 records the
// measurements). The A/B and trace harnesses under scripts/ (build_variant.sh,
// ubench_*.hip) define FLRL_TUNING_BUILD together with their overrides; an
// override without it is a compile error, so a stray -D cannot change a
// shipped library silently.
#pragma once

#if !defined(FLRL_TUNING_BUILD) &&                                                                  \
    (defined(FLRL_RL_TRACE) || defined(FLRL_RL_LB_STAT) || defined(FLRL_FL_TRACE) ||                \
     defined(FLRL_RL_THREADS) || defined(FLRL_RD_TICKET_MIN) || defined(FLRL_FL_LOOKG) || defined(FLRL_FL_LOOKL) ||\
     defined(FLRL_FL_STATUS_STRIDE) || defined(FLRL_FL_STATUS_OFF) || defined(FLRL_RL_LOOKL) || defined(FLRL_RL_LOOKG) || defined(FLRL_RL_PF) ||\
     defined(FLRL_RL_STATUS_STRIDE) || defined(FLRL_RL_STATUS_OFF) ||\
     defined(FLRL_RL_STAGE) || defined(FLRL_RL_WPS) || defined(FLRL_RD_NARROW_MEAN) || defined(FLRL_RL_RO_MAXB) ||          \
     defined(FLRL_RD_UNROLL) || defined(FLRL_HOST_WORKERS) || defined(FLRL_HOST_CHUNK) ||                \
     defined(FLRL_HOST_DIRECT) || defined(FLRL_HOST_PROFILE) || defined(FLRL_HOST_THP) || defined(FLRL_RL_WD64_MEAN) || defined(FLRL_RL_DENSE_MEAN) ||\
     defined(FLRL_FL_STORE_SPLIT) || defined(FLRL_FL_STORE_SKIP) || defined(FLRL_RL_SUB) || defined(FLRL_FL_STATIC_W) || defined(FLRL_RL_PMC_NOLB) || \
     defined(FLRL_RD_WD64_PER_CU) || defined(FLRL_RD_WD32_PER_CU))
#error "FLRL_* kernel overrides are for timing harnesses only (define FLRL_TUNING_BUILD)"
#endif

// ---- trace hooks (no-ops unless a harness supplies them) -------------------
// FL encode per-tile timestamps (scripts/ubench_fl.hip -DTRACE): 0 ticket,
// 1 widths done, 2 look-back resolved, 3 stores issued.
#ifndef FLRL_FL_TRACE
#define FLRL_FL_TRACE(tile, k) ((void)0)
#endif
// RL encode per-tile timestamps (scripts/ubench_rl.hip -DTRACE): 0 ticket,
// 1 all waves scanned, 2 map published, 3 look-back resolved, 4 wave 0 emitted.
#ifndef FLRL_RL_TRACE
#define FLRL_RL_TRACE(tile, k) ((void)0)
#endif
// RL encode look-back statistics: polls that found an unpublished
// predecessor, and windows composed.
#ifndef FLRL_RL_LB_STAT
#define FLRL_RL_LB_STAT(tile, spins, rounds) ((void)(spins), (void)(rounds))
#endif

// ---- RL encode shape ---------------------------------------------------------
#ifndef FLRL_RL_THREADS
#define FLRL_RL_THREADS 256  // 4 waves (LB 64: 94 VGPRs, < 32 KiB LDS, 5 per CU)
#endif
#ifndef FLRL_RL_SUB
#define FLRL_RL_SUB 8  // RL encode: 4 KiB sub-chunks per wave chunk (8: 32 KiB chunks, 128 KiB tiles)
#endif
#ifndef FLRL_FL_LOOKG
#define FLRL_FL_LOOKG 1  // FL encode look-back granules per lane (window 64 G tiles)
#endif
#ifndef FLRL_FL_LOOKL
#define FLRL_FL_LOOKL 32  // FL encode look-back lanes polled per window (G must be 1 below 64)
#endif
#ifndef FLRL_FL_STATUS_STRIDE
#define FLRL_FL_STATUS_STRIDE 16  // FL encode status: one 128-B line per tile (polls spread over lines)
#endif
#ifndef FLRL_FL_STORE_SPLIT
#define FLRL_FL_STORE_SPLIT 2  // FL encode: the staged tile leaves in this many parts of LDS reads + stores
#endif
#ifndef FLRL_FL_STORE_SKIP
#define FLRL_FL_STORE_SKIP 1  // FL encode: parts past the tile's packed bytes skipped (1 GiB lo4 -0.8 %, lo2 -2.3 %, zero -2.5 %, 16 GiB lo4 -1.0 %, u8 equal)
#endif
#ifndef FLRL_FL_STATIC_W
#define FLRL_FL_STATIC_W 0  // PMC/timing builds: FL encode tile offsets = tile x frames x W, no look-back (exact only when every frame has width W)
#endif
#ifndef FLRL_RD_WD64_PER_CU
#define FLRL_RD_WD64_PER_CU 5  // wave decode, 64 runs per lane: workgroups per CU, launch bound and grid (5: 96 VGPRs; 1 GiB random bytes -1.4 %, 4 GiB -5 %, 256 MiB +0.9 % against 4 at 104; 6 spills)
#endif
#ifndef FLRL_RD_WD32_PER_CU
#define FLRL_RD_WD32_PER_CU 6  // wave decode, 32 runs per lane: workgroups per CU, launch bound and grid (7: 72 VGPRs, runs of 1..3 to 1..12 -0.1..+1 %)
#endif
#ifndef FLRL_RL_PMC_NOLB
#define FLRL_RL_PMC_NOLB 0  // PMC builds: RL encode without its look-back (every tile at state (0, 0); output wrong)
#endif
#ifndef FLRL_FL_STATUS_OFF
#define FLRL_FL_STATUS_OFF 256  // FL encode status array offset (Ctrl with the ticket on its own lines)
#endif
#ifndef FLRL_RD_TICKET_MIN
#define FLRL_RD_TICKET_MIN 3  // RL block decode: tiles by ticket from this many tiles per workgroup on (2: 256 MiB +3 %)
#endif
#ifndef FLRL_RL_LOOKG
#define FLRL_RL_LOOKG 1  // RL encode look-back granules per lane (window 64 G tiles; G <= 4)
#endif
#ifndef FLRL_RL_LOOKL
#define FLRL_RL_LOOKL 64  // RL encode look-back lanes polled per window (G must be 1 below 64)
#endif
#ifndef FLRL_RL_STATUS_STRIDE
#define FLRL_RL_STATUS_STRIDE 4  // RL encode status: 32 B per tile, 4 tiles per 128-B line (16, one line each: equal time, +1 % fetch from the polls; 2: +0.6 %; 1: +4.5 %)
#endif
#ifndef FLRL_RL_STATUS_OFF
#define FLRL_RL_STATUS_OFF 256  // RL encode status array offset (Ctrl with the ticket on its own lines)
#endif
#ifndef FLRL_RL_STAGE
#define FLRL_RL_STAGE 15360  // LDS run staging per workgroup (bytes)
#endif

// RL encode: sub-chunks in flight per wave during the scan (register sets)
#ifndef FLRL_RL_PF
#define FLRL_RL_PF 2  // (1 GiB, ab_libs: runs32 -1.2 %, long runs -2.4 %, all-zero -3 %; random bytes +2 %, runs of 1..12 +2 %)
#endif

// RL encode: minimum waves per SIMD the kernels are compiled for (5: five
// 4-wave workgroups per CU, at most 96 VGPRs).
#ifndef FLRL_RL_WPS
#define FLRL_RL_WPS 5
#endif

// ---- RL decode shape ---------------------------------------------------------
// Block decode: 256 instead of 512 threads per workgroup from this mean run
// length (bytes) on.
#ifndef FLRL_RD_NARROW_MEAN
#define FLRL_RD_NARROW_MEAN 240
#endif
// Offsets pre-pass workgroups: 256 (1 GiB runs32 call -2 %; 128: random bytes
// +13 %; 1024: the old cap).
#ifndef FLRL_RL_RO_MAXB
#define FLRL_RL_RO_MAXB 256
#endif
// Block decode chunk loop unroll: 4. (8 was 3-4 % faster with the
// three-permute chunk assembly; with the two-window assembly it needs more
// than the 128 VGPRs of 4 waves per SIMD and spills: 256 MiB runs32 +11 %.)
#ifndef FLRL_RD_UNROLL
#define FLRL_RD_UNROLL 4
#endif
// Wave decode: 64 runs per lane up to this mean run length, and the wave
// decode at all up to FLRL_RL_DENSE_MEAN.
#ifndef FLRL_RL_WD64_MEAN
#define FLRL_RL_WD64_MEAN 2
#endif
#ifndef FLRL_RL_DENSE_MEAN
#define FLRL_RL_DENSE_MEAN 12
#endif

// ---- host-buffer API pipelines (flrl_fl_compress / flrl_fl_decompress) ------
// 8 pipelines x 16 MiB chunks through pinned staging, outputs on transparent
// huge pages (2 GiB u8: the first touch of fresh output pages bounds the call,
// not PCIe); DIRECT 1 copies from/to the caller's pageable buffers instead.
#ifndef FLRL_HOST_WORKERS
#define FLRL_HOST_WORKERS 8
#endif
#ifndef FLRL_HOST_CHUNK
#define FLRL_HOST_CHUNK (16ull << 20)
#endif
#ifndef FLRL_HOST_PROFILE
#define FLRL_HOST_PROFILE 0
#endif
#ifndef FLRL_HOST_DIRECT
#define FLRL_HOST_DIRECT 0
#endif
#ifndef FLRL_HOST_THP
#define FLRL_HOST_THP 1
#endif
