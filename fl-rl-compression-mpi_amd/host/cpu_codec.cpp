// cpu_codec.cpp — multi-threaded host codec for the CLI's fl-cpu / rl-cpu.
//
// Same format as the GPU path: frame f of width b_f (fl_cpu.cu:37-48) starts at
// byte 16*sum_{g<f} b_g and each group of 8 values packs into b bytes, so frames
// are encoded independently once a prefix of widths is known (instead of the
// reference's serial bit cursor, fl_cpu.cu:64-84).
#include "cpu_codec.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace flrl_cli {

namespace {

constexpr size_t kFrame = FLRL_FRAME_LENGTH;

uint64_t load_le64(const uint8_t *p, size_t avail)
{
    uint64_t x = 0;
    std::memcpy(&x, p, avail < 8 ? avail : 8);
    return x;
}

uint64_t pack8(uint64_t x, unsigned b)
{
    const uint64_t y = (x & 0x00FF00FF00FF00FFull) | ((x & 0xFF00FF00FF00FF00ull) >> (8 - b));
    const uint64_t z = (y & 0x0000FFFF0000FFFFull) | ((y & 0xFFFF0000FFFF0000ull) >> (16 - 2 * b));
    return (z & 0xFFFFFFFFull) | ((z >> 32) << (4 * b));
}

uint64_t unpack8(uint64_t w, unsigned b)
{
    const uint64_t m4 = b >= 8 ? 0xFFFFFFFFull : ((1ull << (4 * b)) - 1);
    const uint64_t z = (w & m4) | (((w >> (4 * b)) & m4) << 32);
    const uint64_t m2 = (1ull << (2 * b)) - 1;
    const uint64_t M2 = m2 | (m2 << 32);
    const uint64_t y = (z & M2) | (((z >> (2 * b)) & M2) << 16);
    const uint64_t M1 = ((1ull << b) - 1) * 0x0001000100010001ull;
    return (y & M1) | (((y >> b) & M1) << 8);
}

template <typename Fn>
void parallel_for(size_t count, unsigned threads, Fn fn)
{
    threads = std::max(1u, std::min<unsigned>(threads, (unsigned)std::max<size_t>(1, count / 4096)));
    if (threads == 1) {
        fn(0, count);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (count + threads - 1) / threads;
    for (unsigned t = 0; t < threads; ++t) {
        const size_t lo = std::min(count, t * per), hi = std::min(count, lo + per);
        th.emplace_back([=]() { fn(lo, hi); });
    }
    for (auto &x : th)
        x.join();
}

uint8_t *alloc_bytes(size_t n)
{
    uint8_t *p = static_cast<uint8_t *>(std::malloc(n ? n : 1));
    if (!p)
        throw std::runtime_error("Cannot allocate memory");
    return p;
}

}  // namespace

flrl_fl_buf cpuCompressFL(const uint8_t *data, size_t n, unsigned threads)
{
    flrl_fl_buf c{};
    if (n == 0)
        return c;
    const size_t F = (n + kFrame - 1) / kFrame;
    c.bits = alloc_bytes(F);
    c.bits_size = F;
    c.input_size = n;
    parallel_for(F, threads, [&](size_t lo, size_t hi) {
        for (size_t f = lo; f < hi; ++f) {
            const size_t cnt = std::min(kFrame, n - f * kFrame);
            uint8_t o = 0;
            for (size_t i = 0; i < cnt; ++i)
                o |= data[f * kFrame + i];
            unsigned b = 1;
            while (b < 8 && (o >> b))
                ++b;
            c.bits[f] = (uint8_t)b;
        }
    });
    std::vector<uint64_t> off;
    try {
        off.resize(F);
        uint64_t acc = 0;
        for (size_t f = 0; f < F; ++f) {
            off[f] = 16 * acc;
            acc += c.bits[f];
        }
        const size_t cnt_last = n - (F - 1) * kFrame;
        c.values_size = off[F - 1] + (cnt_last * c.bits[F - 1] + 7) / 8;
        c.values = alloc_bytes(c.values_size);
    } catch (...) {  // the caller gets nothing to free
        std::free(c.bits);
        throw;
    }
    parallel_for(F, threads, [&](size_t lo, size_t hi) {
        for (size_t f = lo; f < hi; ++f) {
            const unsigned b = c.bits[f];
            const size_t cnt = std::min(kFrame, n - f * kFrame);
            uint8_t *dst = c.values + off[f];
            for (size_t g = 0; g * 8 < cnt; ++g) {
                const size_t vals = std::min<size_t>(8, cnt - g * 8);
                const uint64_t w = pack8(load_le64(data + f * kFrame + g * 8, vals), b);
                std::memcpy(dst + g * b, &w, (vals * b + 7) / 8);
            }
        }
    });
    return c;
}

void cpuDecompressFL(const flrl_fl_buf &c, uint8_t **out, size_t *out_size, unsigned threads)
{
    *out = nullptr;
    *out_size = 0;
    if (c.values_size == 0 || c.bits_size == 0)
        return;
    const size_t n = c.input_size, F = c.bits_size;
    if (F != (n + kFrame - 1) / kFrame)
        throw std::runtime_error("bitsSize " + std::to_string(F) + " != ceil(inputSize/128)");
    std::vector<uint64_t> off(F);
    uint64_t acc = 0;
    for (size_t f = 0; f < F; ++f) {
        if (c.bits[f] < 1 || c.bits[f] > 8)
            throw std::runtime_error("frame " + std::to_string(f) + " has width " +
                                     std::to_string(c.bits[f]) + " (must be 1..8)");
        off[f] = 16 * acc;
        acc += c.bits[f];
    }
    const size_t cnt_last = n - (F - 1) * kFrame;
    if (off[F - 1] + (cnt_last * c.bits[F - 1] + 7) / 8 != c.values_size)
        throw std::runtime_error("valuesSize does not match the frame widths");
    uint8_t *o = alloc_bytes(n);
    parallel_for(F, threads, [&](size_t lo, size_t hi) {
        for (size_t f = lo; f < hi; ++f) {
            const unsigned b = c.bits[f];
            const size_t cnt = std::min(kFrame, n - f * kFrame);
            const uint8_t *src = c.values + off[f];
            const size_t avail = c.values_size - off[f];
            for (size_t g = 0; g * 8 < cnt; ++g) {
                const size_t vals = std::min<size_t>(8, cnt - g * 8);
                const uint64_t x = unpack8(load_le64(src + g * b, std::min<size_t>(b, avail - g * b)), b);
                std::memcpy(o + f * kFrame + g * 8, &x, vals);
            }
        }
    });
    *out = o;
    *out_size = n;
}

flrl_rl_buf cpuCompressRL(const uint8_t *data, size_t n)
{
    flrl_rl_buf c{};
    c.input_size = n;
    if (n == 0)
        return c;
    c.counts = alloc_bytes(n);
    c.values = static_cast<uint8_t *>(std::malloc(n));
    if (!c.values) {
        std::free(c.counts);
        throw std::runtime_error("Cannot allocate memory");
    }
    size_t r = 0, i = 0;
    while (i < n) {
        const uint8_t v = data[i];
        size_t j = i + 1;
        while (j < n && data[j] == v)
            ++j;
        for (size_t len = j - i; len > 0;) {  // 255-split from the run start
            const size_t k = len > 255 ? 255 : len;
            c.counts[r] = (uint8_t)k;
            c.values[r] = v;
            ++r;
            len -= k;
        }
        i = j;
    }
    c.runs = r;
    return c;
}

void cpuDecompressRL(const flrl_rl_buf &c, uint8_t **out, size_t *out_size)
{
    *out = nullptr;
    *out_size = 0;
    size_t total = 0;
    for (size_t r = 0; r < c.runs; ++r) {
        if (c.counts[r] == 0)
            throw std::runtime_error("run " + std::to_string(r) + " has count 0");
        total += c.counts[r];
    }
    if (total != c.input_size)
        throw std::runtime_error("RL counts sum to " + std::to_string(total) +
                                 ", header says " + std::to_string(c.input_size));
    if (total == 0)
        return;
    uint8_t *o = alloc_bytes(total);
    size_t pos = 0;
    for (size_t r = 0; r < c.runs; ++r) {
        std::memset(o + pos, c.values[r], c.counts[r]);
        pos += c.counts[r];
    }
    *out = o;
    *out_size = total;
}

}  // namespace flrl_cli
