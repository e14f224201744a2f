/*
 * flrl oracle — CPU restatement of the reference codec. TEST INFRASTRUCTURE ONLY
 * (see flrl_oracle.h). Never linked into the product path.
 *
 * FL: restates src/fl/fl_cpu.cu (cpuCompress :9-90, cpuDecompress :92-147) with
 * the same two-loop structure (per-frame width loop with the bit-loop clz, then a
 * serial bit-cursor pack loop) so its single-core cost model matches the
 * reference's fl-cpu. The reference's double-precision ceil() calls
 * (fl_cpu.cu:21,53) are exact integer ceilings for n < 2^53 and are written as
 * integer arithmetic here.
 *
 * RL: restates IMPLEMENTATION-PLAN.md:81-179 (no reference code exists).
 *
 * Generator: SURVEY.md §8(d) splitmix64 spec.
 */
#include "flrl_oracle.h"

#include <string.h>

uint8_t orc_clz8(uint8_t value)
{
    /* fl_common.cuh:198-212: clz8(0) = 8, else count leading zero bits */
    if (value == 0)
        return 8;
    uint8_t count = 0;
    uint8_t mask = 1u << 7;
    while (!(value & mask)) {
        count++;
        value = (uint8_t)(value << 1);
    }
    return count;
}

size_t orc_fl_frames(size_t n) { return (n + ORC_FRAME_LENGTH - 1) / ORC_FRAME_LENGTH; }

size_t orc_fl_values_bound(size_t n) { return n; }

/* The restatement is written for any frame length L (the reference fixes
 * L = FRAME_LENGTH = 128, fl_common.cuh:9; IMPLEMENTATION-PLAN.md:9-27 works its
 * example at L = 3), so the plan's worked example can pin it. */
size_t orc_fl_widths_frame(const uint8_t *data, size_t n, size_t frame_len, uint8_t *bits)
{
    /* width pass, fl_cpu.cu:35-50: b_f = max(1, max_i (8 - clz8(x_i))) */
    const size_t frames = (n + frame_len - 1) / frame_len;
    size_t total_bits = 0;
    for (size_t f = 0; f < frames; f++) {
        uint8_t min_bits = 1;
        for (size_t i = 0; i < frame_len && f * frame_len + i < n; i++) {
            uint8_t required = (uint8_t)(8 - orc_clz8(data[f * frame_len + i]));
            if (required > min_bits)
                min_bits = required;
        }
        bits[f] = min_bits;
        size_t cnt = n - frame_len * f;
        if (cnt > frame_len)
            cnt = frame_len;
        total_bits += (size_t)min_bits * cnt;
    }
    return total_bits;
}

void orc_fl_frame_starts(const uint8_t *bits, size_t frames, size_t frame_len, uint64_t *starts)
{
    /* frameStartIndices = Prescan(bits[f] * frame_len), IMPLEMENTATION-PLAN.md:20-29 */
    uint64_t acc = 0;
    for (size_t f = 0; f < frames; f++) {
        starts[f] = acc;
        acc += (uint64_t)bits[f] * frame_len;
    }
}

size_t orc_fl_compress_frame(const uint8_t *data, size_t n, size_t frame_len, uint8_t *bits,
                             uint8_t *values)
{
    if (n == 0 || frame_len == 0) /* fl_cpu.cu:11-14 */
        return 0;
    const size_t frames = (n + frame_len - 1) / frame_len;
    const size_t total_bits = orc_fl_widths_frame(data, n, frame_len, bits);

    /* valuesSize = ceil(totalBits/8), zero-filled, fl_cpu.cu:53-55 */
    const size_t values_size = (total_bits + 7) / 8;
    memset(values, 0, values_size);

    /* pack pass, fl_cpu.cu:62-84: LSB-first serial bit cursor */
    size_t used = 0;
    for (size_t f = 0; f < frames; f++) {
        const uint8_t b = bits[f];
        for (size_t i = 0; i < frame_len && f * frame_len + i < n; i++) {
            const uint8_t v = data[f * frame_len + i];
            const size_t id = used / 8;
            const uint8_t off = (uint8_t)(used % 8);
            values[id] |= (uint8_t)(v << off);
            if (off + b > 8)
                values[id + 1] |= (uint8_t)(v >> (8 - off));
            used += b;
        }
    }
    return values_size;
}

size_t orc_fl_compress(const uint8_t *data, size_t n, uint8_t *bits, uint8_t *values)
{
    return orc_fl_compress_frame(data, n, ORC_FRAME_LENGTH, bits, values);
}

size_t orc_fl_decompress_frame(size_t output_size, size_t frame_len, const uint8_t *bits,
                               size_t bits_size, const uint8_t *values, size_t values_size,
                               uint8_t *out)
{
    if (values_size == 0 || bits_size == 0 || frame_len == 0) /* fl_cpu.cu:94-97 */
        return 0;
    size_t consumed = 0;
    for (size_t f = 0; f < bits_size; f++) { /* fl_cpu.cu:117-141 */
        const uint8_t b = bits[f];
        for (size_t i = 0; i < frame_len && f * frame_len + i < output_size; i++) {
            const size_t id = consumed / 8;
            const uint8_t off = (uint8_t)(consumed % 8);
            const uint8_t mask = (uint8_t)((1u << b) - 1);
            uint8_t v = (uint8_t)((values[id] >> off) & mask);
            if (off + b > 8) {
                const uint8_t ob = (uint8_t)(off + b - 8);
                const uint8_t om = (uint8_t)((1u << ob) - 1);
                v |= (uint8_t)((values[id + 1] & om) << (b - ob));
            }
            out[f * frame_len + i] = v;
            consumed += b;
        }
    }
    return output_size;
}

size_t orc_fl_decompress(size_t output_size, const uint8_t *bits, size_t bits_size,
                         const uint8_t *values, size_t values_size, uint8_t *out)
{
    return orc_fl_decompress_frame(output_size, ORC_FRAME_LENGTH, bits, bits_size, values,
                                   values_size, out);
}

size_t orc_rl_compress(const uint8_t *data, size_t n, uint8_t *counts, uint8_t *values)
{
    /* IMPLEMENTATION-PLAN.md:85-152: startMask -> runs; a run longer than 255 is
     * split into 255-chunks from its start (:125-147); outputCount/outputValues. */
    size_t runs = 0;
    size_t i = 0;
    while (i < n) {
        const uint8_t v = data[i];
        size_t j = i + 1;
        while (j < n && data[j] == v)
            j++;
        size_t len = j - i;
        while (len > 0) {
            const size_t c = len > 255 ? 255 : len;
            counts[runs] = (uint8_t)c;
            values[runs] = v;
            runs++;
            len -= c;
        }
        i = j;
    }
    return runs;
}

size_t orc_rl_decompress(const uint8_t *counts, const uint8_t *values, size_t runs,
                         uint8_t *out, size_t out_cap)
{
    /* IMPLEMENTATION-PLAN.md:154-179: prescan of counts -> start indices; expand */
    size_t pos = 0;
    for (size_t r = 0; r < runs; r++) {
        const size_t c = counts[r];
        if (pos + c > out_cap)
            return (size_t)-1;
        memset(out + pos, values[r], c);
        pos += c;
    }
    return pos;
}

#define GOLDEN 0x9E3779B97F4A7C15ull

static uint64_t splitmix64(uint64_t *state)
{
    uint64_t z = (*state += GOLDEN);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int orc_gen(int kind, uint64_t seed, uint64_t word_offset, uint8_t *out, size_t n)
{
    if (kind >= 0 && kind <= 2) {
        const uint8_t mask = kind == 0 ? 0xFF : (kind == 1 ? 0x0F : 0x00);
        for (size_t w = 0; w * 8 < n; w++) {
            uint64_t st = seed + (word_offset + w) * GOLDEN;
            const uint64_t word = splitmix64(&st);
            for (size_t j = 0; j < 8 && w * 8 + j < n; j++)
                out[w * 8 + j] = (uint8_t)((word >> (8 * j)) & mask);
        }
        return 0;
    }
    if (kind == 3 || kind == 4) {
        if (word_offset != 0)
            return -1;
        const uint64_t modulus = kind == 3 ? 63 : 1023;
        uint64_t st = seed;
        size_t i = 0;
        uint8_t prev = 0;
        while (i < n) {
            const uint64_t r = splitmix64(&st);
            size_t len = (size_t)(1 + r % modulus);
            uint8_t val = (uint8_t)((r >> 32) & 0xFF);
            if (i > 0 && val == prev)
                val ^= 0x80;
            if (len > n - i)
                len = n - i;
            memset(out + i, val, len);
            i += len;
            prev = val;
        }
        return 0;
    }
    return -1;
}
