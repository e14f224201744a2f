/*
 * flrl oracle — CPU restatement of the reference codec. TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker for the MI355X HIP path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The
 * product path (libflrl.so, the `compress` CLI) never links or calls it.
 *
 * Pinning: the FL restatement is pinned by the plan's frame-length-3 example
 * (IMPLEMENTATION-PLAN.md:9-13) and checked against the golden vectors recorded
 * in SURVEY.md §8(c) (KATs + sha256 of fl-cpu output files from a survey-session
 * build with stand-in MPI/NCCL headers: they corroborate the restatement but do
 * not pin it; FL parity partially unpinned) — see tests/golden/. RL has no reference implementation
 * (SURVEY.md §0 item 2): RL parity is pinned only by the worked examples of
 * IMPLEMENTATION-PLAN.md:87-89,125,158-160 ("RL parity partially unpinned").
 */
#ifndef FLRL_ORACLE_H
#define FLRL_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* FRAME_LENGTH, src/fl/fl_common.cuh:9 */
#define ORC_FRAME_LENGTH 128

/* countLeadingZeroes, src/fl/fl_common.cuh:198-212 (bit loop kept: cost model) */
uint8_t orc_clz8(uint8_t v);

/* ceil(n/128) frames, src/fl/fl_cpu.cu:21 */
size_t orc_fl_frames(size_t n);

/* Upper bound on valuesSize (b <= 8 per value): n bytes. */
size_t orc_fl_values_bound(size_t n);

/* cpuCompress, src/fl/fl_cpu.cu:9-90. bits must hold orc_fl_frames(n) bytes,
 * values must hold >= the returned size (orc_fl_values_bound(n) is enough).
 * Returns valuesSize. n == 0 returns 0 and touches nothing (fl_cpu.cu:11-14). */
size_t orc_fl_compress(const uint8_t *data, size_t n, uint8_t *bits, uint8_t *values);

/* cpuDecompress, src/fl/fl_cpu.cu:92-147. Writes output_size bytes into out and
 * returns output_size, or returns 0 (writing nothing) on the reference's
 * early-out `valuesSize == 0 || bitsSize == 0` (fl_cpu.cu:94-97). Like the
 * reference it does not validate widths or sizes. */
size_t orc_fl_decompress(size_t output_size, const uint8_t *bits, size_t bits_size,
                         const uint8_t *values, size_t values_size, uint8_t *out);

/* The same two passes at any frame length (the reference fixes 128; the plan's
 * worked example, IMPLEMENTATION-PLAN.md:9-27, uses 3). Widths: bits[f] for
 * ceil(n/frame_len) frames, returns the total bit count. Starts: the plan's
 * frameStartIndices (bit offset of each frame, exclusive scan of b_f*frame_len). */
size_t orc_fl_widths_frame(const uint8_t *data, size_t n, size_t frame_len, uint8_t *bits);
void orc_fl_frame_starts(const uint8_t *bits, size_t frames, size_t frame_len, uint64_t *starts);
size_t orc_fl_compress_frame(const uint8_t *data, size_t n, size_t frame_len, uint8_t *bits,
                             uint8_t *values);
size_t orc_fl_decompress_frame(size_t output_size, size_t frame_len, const uint8_t *bits,
                               size_t bits_size, const uint8_t *values, size_t values_size,
                               uint8_t *out);

/* RL encode, IMPLEMENTATION-PLAN.md:85-152: maximal runs of equal bytes, runs
 * longer than 255 split into 255-chunks counted from the run start (:125).
 * counts/values must hold n bytes. Returns the number of runs R. */
size_t orc_rl_compress(const uint8_t *data, size_t n, uint8_t *counts, uint8_t *values);

/* RL decode, IMPLEMENTATION-PLAN.md:154-179. Returns bytes written (sum of
 * counts) or (size_t)-1 if that would exceed out_cap. */
size_t orc_rl_decompress(const uint8_t *counts, const uint8_t *values, size_t runs,
                         uint8_t *out, size_t out_cap);

/* Synthetic generator, SURVEY.md §8(d). kind: 0 u8, 1 lo4, 2 zero, 3 runs32,
 * 4 longruns (build-defined: len = 1 + r % 1023). word_offset shifts the
 * counter-based kinds (0-2) so a shard starting at byte 8*word_offset equals
 * the same bytes of the whole buffer; it must be 0 for the sequential kinds. */
int orc_gen(int kind, uint64_t seed, uint64_t word_offset, uint8_t *out, size_t n);

#ifdef __cplusplus
}
#endif

#endif
