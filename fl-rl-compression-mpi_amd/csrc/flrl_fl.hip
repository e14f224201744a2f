// flrl_fl.hip — fixed-length (FL) encode / decode for MI355X (gfx950).
//
// Format (reference src/fl/fl_cpu.cu:9-147): the input is cut into 128-byte
// frames; frame f gets width b_f = max(1, bitlen(max byte)) (fl_cpu.cu:37-48)
// and its values are packed LSB-first into a continuous bit stream
// (fl_cpu.cu:64-82). Because a full frame packs into exactly 16*b_f bytes, every
// frame starts byte-aligned at 16 * sum_{g<f} b_g, and every group of 8 values
// packs into exactly b bytes. One lane therefore owns
// 16 input bytes <-> 2b output bytes at a position known from a prefix sum of
// widths — no bit cursor, no atomics on the data path.
//
// Encode is a single pass over the input (read once, N+F+V bytes of HBM
// traffic): each 256-thread workgroup takes a 16*256*ITEMS-byte tile by ticket,
// keeps it in registers, computes frame widths (OR of the frame's bytes), scans
// them in LDS, publishes the tile's width sum and resolves its global offset by
// decoupled look-back while the other waves pack into an LDS staging tile; the
// packed tile then leaves in coalesced 16-byte stores (offsets are multiples of
// 16). Decode mirrors it: widths -> scan -> look-back -> the tile's contiguous
// packed bytes staged into LDS -> each lane unpacks 2b bytes into 16 bytes and
// stores them coalesced.
//
// Replaces the reference kernels compressCalculateOutputBits
// (fl_gpu.cu:648-685), compressInitializeFrameStartIndiciesBits + thrust scan
// (:687-698, :805-808), compressCalculateOutput (:700-726) and
// decompressCalculateOutput (:728-755). Indices are 64-bit throughout (the
// reference's 32-bit threadId wraps at 4 GiB, fl_gpu.cu:650,702,730).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "flrl.h"
#include "flrl_device.hpp"
#include "flrl_internal.hpp"

namespace flrl {

// Tile shape: 256 threads x ITEMS x 16 B. ITEMS = 16 -> 64 KiB tiles (512 frames).
constexpr int kFlItems = 16;
constexpr int kFlTileBytes = kThreads * 16 * kFlItems;

// Pack 8 bytes (each < 2^b) of x into the low 8b bits, value i at bit b*i.
__device__ __forceinline__ uint64_t pack8(uint64_t x, uint32_t b)
{
    const uint64_t y = (x & 0x00FF00FF00FF00FFull) | ((x & 0xFF00FF00FF00FF00ull) >> (8 - b));
    const uint64_t z = (y & 0x0000FFFF0000FFFFull) | ((y & 0xFFFF0000FFFF0000ull) >> (16 - 2 * b));
    return (z & 0xFFFFFFFFull) | ((z >> 32) << (4 * b));
}

// Inverse of pack8; bits of w at or above 8b are ignored.
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

template <int ITEMS>
__global__ __launch_bounds__(kThreads) void fl_encode_kernel(
    const uint8_t *__restrict__ in, uint64_t n, uint64_t nframes, uint64_t ntiles,
    uint8_t *__restrict__ bits, uint8_t *__restrict__ values, uint64_t *__restrict__ values_size,
    Ctrl *ctrl, uint64_t *status)
{
    constexpr int TB = kThreads * 16 * ITEMS;
    constexpr int TF = TB / kFrame;
    __shared__ u32x4 s_out[TB / 16];
    __shared__ u32x4 s_w4[TF / 16];
    __shared__ uint32_t s_pref[TF];
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_ticket;
    __shared__ uint64_t s_base;
    uint8_t *s_w = reinterpret_cast<uint8_t *>(s_w4);

    const int tid = threadIdx.x;
    const int wave = tid / kWave;
    const uint32_t tile = take_ticket(ctrl, &s_ticket);
    const uint64_t tile_off = (uint64_t)tile * TB;
    const uint64_t frame0 = (uint64_t)tile * TF;
    const bool full = tile_off + TB <= n;

    // ---- load the tile: 16 B per lane per item, coalesced -----------------
    u32x4 v[ITEMS];
    if (full) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(in + tile_off);
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            v[k] = __builtin_nontemporal_load(src + k * kThreads + tid);
    } else {
#pragma unroll
        for (int k = 0; k < ITEMS; ++k)
            v[k] = load16_tail(in, tile_off + (uint64_t)(k * kThreads + tid) * 16, n);
    }

    // ---- frame widths: OR over the frame's 8 lanes, b = max(1, bitlen) ---
    uint32_t bw[ITEMS];
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        uint32_t o = v[k].x | v[k].y | v[k].z | v[k].w;
        o |= o >> 16;
        o |= o >> 8;
        o &= 0xFFu;
        o |= __shfl_xor(o, 1, kWave);
        o |= __shfl_xor(o, 2, kWave);
        o |= __shfl_xor(o, 4, kWave);
        uint32_t b = o ? 32u - __clz(o) : 1u;
        const int ft = k * (kThreads / 8) + (tid >> 3);
        if (frame0 + ft >= nframes)
            b = 0;  // past the last frame: contributes nothing
        bw[k] = b;
        if ((tid & 7) == 0)
            s_w[ft] = (uint8_t)b;
    }
    __syncthreads();
    const uint32_t agg = block_excl_scan<TF>(s_w, s_pref, s_wave);
    __syncthreads();

    // ---- bits[] for this tile's frames -----------------------------------
    if (frame0 + TF <= nframes) {
        for (int i = tid; i < TF / 16; i += kThreads)
            reinterpret_cast<u32x4 *>(bits + frame0)[i] = s_w4[i];
    } else {
        for (int i = tid; i < TF; i += kThreads)
            if (frame0 + i < nframes)
                bits[frame0 + i] = s_w[i];
    }

    // ---- wave 0: global offset by look-back (overlaps the packing below) --
    if (wave == 0) {
        const uint64_t excl = lookback_sum(status, tile, agg, ctrl);
        if (tid == 0)
            s_base = excl;
    }

    // ---- pack each lane's 16 values into 2b bytes in the LDS staging tile -
    uint8_t *s_out_b = reinterpret_cast<uint8_t *>(s_out);
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const uint32_t b = bw[k];
        if (b == 0)
            continue;
        const int ft = k * (kThreads / 8) + (tid >> 3);
        const uint32_t off = 16u * s_pref[ft] + 2u * b * (uint32_t)(tid & 7);
        const uint64_t p0 = pack8(((uint64_t)v[k].y << 32) | v[k].x, b);
        const uint64_t p1 = pack8(((uint64_t)v[k].w << 32) | v[k].z, b);
        const uint64_t lo = b == 8 ? p0 : (p0 | (p1 << (8 * b)));
        const uint64_t hi = b == 8 ? p1 : (p1 >> (64 - 8 * b));
        uint16_t *d = reinterpret_cast<uint16_t *>(s_out_b + off);
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (i < (int)b)
                d[i] = (uint16_t)((i < 4 ? lo >> (16 * i) : hi >> (16 * (i - 4))) & 0xFFFFu);
    }
    __syncthreads();

    // ---- stream the packed tile out: 16-B aligned, coalesced --------------
    const uint64_t base = s_base;  // in 16-byte units
    u32x4 *dst = reinterpret_cast<u32x4 *>(values) + base;
    if (tile + 1 < ntiles) {
        for (uint32_t c = tid; c < agg; c += kThreads)
            __builtin_nontemporal_store(s_out[c], dst + c);
    } else {
        // last tile: valuesSize = 16*(frames before last) + ceil(cnt*b_last/8)
        const int fl = (int)(nframes - 1 - frame0);
        const uint64_t cnt = n - (nframes - 1) * kFrame;
        const uint64_t vsize = 16ull * (base + s_pref[fl]) + (cnt * s_w[fl] + 7) / 8;
        if (tid == 0)
            *values_size = vsize;
        for (uint32_t c = tid; c < agg; c += kThreads)
            store16_tail(values, 16ull * (base + c), vsize, s_out[c]);
    }
}

template <int ITEMS>
__global__ __launch_bounds__(kThreads) void fl_decode_kernel(
    const uint8_t *__restrict__ bits, uint64_t nframes, const uint8_t *__restrict__ values,
    uint64_t vsize, uint8_t *__restrict__ out, uint64_t n, uint64_t ntiles, Ctrl *ctrl,
    uint64_t *status)
{
    constexpr int TB = kThreads * 16 * ITEMS;
    constexpr int TF = TB / kFrame;
    __shared__ u32x4 s_in[TB / 16 + 2];  // +2: a lane may read 4 bytes past its 2b
    __shared__ u32x4 s_w4[TF / 16];
    __shared__ uint32_t s_pref[TF];
    __shared__ uint32_t s_wave[kWaves];
    __shared__ uint32_t s_ticket;
    __shared__ uint64_t s_base;
    uint8_t *s_w = reinterpret_cast<uint8_t *>(s_w4);

    const int tid = threadIdx.x;
    const int wave = tid / kWave;
    const uint32_t tile = take_ticket(ctrl, &s_ticket);
    const uint64_t tile_off = (uint64_t)tile * TB;
    const uint64_t frame0 = (uint64_t)tile * TF;

    // ---- widths of this tile's frames, validated to [1,8] -----------------
    if (frame0 + TF <= nframes) {
        for (int i = tid; i < TF / 16; i += kThreads)
            s_w4[i] = reinterpret_cast<const u32x4 *>(bits + frame0)[i];
    } else {
        for (int i = tid; i < TF; i += kThreads)
            s_w[i] = frame0 + i < nframes ? bits[frame0 + i] : 0;
    }
    __syncthreads();
    for (int i = tid; i < TF; i += kThreads) {
        const uint32_t b = s_w[i];
        if (frame0 + i < nframes && (b < 1 || b > 8)) {
            raise_error(ctrl, FLRL_E_FORMAT);
            s_w[i] = b < 1 ? 1 : 8;
        }
    }
    __syncthreads();
    const uint32_t agg = block_excl_scan<TF>(s_w, s_pref, s_wave);
    __syncthreads();

    if (wave == 0) {
        const uint64_t excl = lookback_sum(status, tile, agg, ctrl);
        if (tid == 0)
            s_base = excl;
    }
    __syncthreads();
    const uint64_t base = s_base;

    // ---- stage this tile's packed bytes (contiguous, 16-B aligned) --------
    const u32x4 *src = reinterpret_cast<const u32x4 *>(values) + base;
    if (16ull * (base + agg) <= vsize) {
        for (uint32_t c = tid; c < agg; c += kThreads)
            s_in[c] = __builtin_nontemporal_load(src + c);
    } else {
        for (uint32_t c = tid; c < agg; c += kThreads)
            s_in[c] = load16_tail(values, 16ull * (base + c), vsize);
    }
    if (tid < 2)
        s_in[agg + tid] = u32x4{0u, 0u, 0u, 0u};
    if (tile + 1 == ntiles && tid == 0) {
        const int fl = (int)(nframes - 1 - frame0);
        const uint64_t cnt = n - (nframes - 1) * kFrame;
        const uint64_t expect = 16ull * (base + s_pref[fl]) + (cnt * s_w[fl] + 7) / 8;
        if (expect != vsize)
            raise_error(ctrl, FLRL_E_FORMAT);
    }
    __syncthreads();

    // ---- unpack 2b bytes -> 16 values per lane, store coalesced -----------
    const uint32_t *s32 = reinterpret_cast<const uint32_t *>(s_in);
    const bool full = tile_off + TB <= n;
#pragma unroll
    for (int k = 0; k < ITEMS; ++k) {
        const int c = k * kThreads + tid;
        const int ft = c >> 3;
        const uint32_t b = s_w[ft];
        if (b == 0)
            continue;
        const uint32_t off = 16u * s_pref[ft] + 2u * b * (uint32_t)(tid & 7);
        const uint32_t a = off >> 2;
        const uint64_t w01 = ((uint64_t)s32[a + 1] << 32) | s32[a];
        const uint64_t w23 = ((uint64_t)s32[a + 3] << 32) | s32[a + 2];
        uint64_t lo = w01, hi = w23;
        if (off & 2) {  // 2-byte aligned start: funnel by 16 bits
            const uint64_t w4 = s32[a + 4];
            lo = (w01 >> 16) | (w23 << 48);
            hi = (w23 >> 16) | (w4 << 48);
        }
        const uint64_t p0 = lo;
        const uint64_t p1 = b == 8 ? hi : ((lo >> (8 * b)) | (hi << (64 - 8 * b)));
        const uint64_t x0 = unpack8(p0, b);
        const uint64_t x1 = unpack8(p1, b);
        const u32x4 r = u32x4{(uint32_t)x0, (uint32_t)(x0 >> 32), (uint32_t)x1,
                              (uint32_t)(x1 >> 32)};
        if (full)
            __builtin_nontemporal_store(r, reinterpret_cast<u32x4 *>(out + tile_off) + c);
        else
            store16_tail(out, tile_off + (uint64_t)c * 16, n, r);
    }
}

static size_t fl_tiles(size_t n) { return div_up(n, (size_t)kFlTileBytes); }

}  // namespace flrl

using namespace flrl;

extern "C" size_t flrl_fl_scratch_bytes(size_t n)
{
    return sizeof(Ctrl) + round_up(fl_tiles(n) * sizeof(uint64_t), 16);
}

extern "C" size_t flrl_fl_values_capacity(size_t n) { return round_up(n ? n : 1, 16); }

extern "C" int flrl_fl_encode_device(const uint8_t *d_in, size_t n, uint8_t *d_bits,
                                     uint8_t *d_values, uint64_t *d_values_size, void *d_scratch,
                                     size_t scratch_bytes, void *stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!d_values_size || !d_scratch)
        return set_error(FLRL_E_ARG, "flrl_fl_encode_device: null values_size/scratch");
    if (scratch_bytes < flrl_fl_scratch_bytes(n))
        return set_error(FLRL_E_ARG, "flrl_fl_encode_device: scratch %zu < required %zu",
                         scratch_bytes, flrl_fl_scratch_bytes(n));
    if (!aligned16(d_scratch))
        return set_error(FLRL_E_ARG, "flrl_fl_encode_device: scratch not 16-byte aligned");
    FLRL_HIP(hipMemsetAsync(d_scratch, 0, flrl_fl_scratch_bytes(n), s));
    if (n == 0) {
        FLRL_HIP(hipMemsetAsync(d_values_size, 0, sizeof(uint64_t), s));
        return FLRL_OK;
    }
    if (!d_in || !d_bits || !d_values)
        return set_error(FLRL_E_ARG, "flrl_fl_encode_device: null buffer");
    if (!aligned16(d_in) || !aligned16(d_bits) || !aligned16(d_values))
        return set_error(FLRL_E_ARG, "flrl_fl_encode_device: buffers must be 16-byte aligned");
    const size_t tiles = fl_tiles(n);
    if (tiles > 0xFFFFFFFFull)
        return set_error(FLRL_E_ARG, "flrl_fl_encode_device: input too large");
    Ctrl *ctrl = static_cast<Ctrl *>(d_scratch);
    uint64_t *status = reinterpret_cast<uint64_t *>(ctrl + 1);
    hipLaunchKernelGGL(fl_encode_kernel<kFlItems>, dim3((uint32_t)tiles), dim3(kThreads), 0, s,
                       d_in, (uint64_t)n, (uint64_t)div_up(n, kFrame), (uint64_t)tiles, d_bits,
                       d_values, d_values_size, ctrl, status);
    FLRL_HIP(hipGetLastError());
    return FLRL_OK;
}

extern "C" int flrl_fl_decode_device(const uint8_t *d_bits, size_t bits_size,
                                     const uint8_t *d_values, size_t values_size, uint8_t *d_out,
                                     size_t n, void *d_scratch, size_t scratch_bytes, void *stream)
{
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!d_scratch)
        return set_error(FLRL_E_ARG, "flrl_fl_decode_device: null scratch");
    if (scratch_bytes < flrl_fl_scratch_bytes(n))
        return set_error(FLRL_E_ARG, "flrl_fl_decode_device: scratch %zu < required %zu",
                         scratch_bytes, flrl_fl_scratch_bytes(n));
    if (!aligned16(d_scratch))
        return set_error(FLRL_E_ARG, "flrl_fl_decode_device: scratch not 16-byte aligned");
    FLRL_HIP(hipMemsetAsync(d_scratch, 0, flrl_fl_scratch_bytes(n), s));
    if (n == 0)
        return FLRL_OK;
    if (bits_size != div_up(n, kFrame))
        return set_error(FLRL_E_FORMAT, "bitsSize %zu != ceil(%zu/128)", bits_size, n);
    if (!d_bits || !d_values || !d_out)
        return set_error(FLRL_E_ARG, "flrl_fl_decode_device: null buffer");
    if (!aligned16(d_bits) || !aligned16(d_values) || !aligned16(d_out))
        return set_error(FLRL_E_ARG, "flrl_fl_decode_device: buffers must be 16-byte aligned");
    const size_t tiles = fl_tiles(n);
    if (tiles > 0xFFFFFFFFull)
        return set_error(FLRL_E_ARG, "flrl_fl_decode_device: output too large");
    Ctrl *ctrl = static_cast<Ctrl *>(d_scratch);
    uint64_t *status = reinterpret_cast<uint64_t *>(ctrl + 1);
    hipLaunchKernelGGL(fl_decode_kernel<kFlItems>, dim3((uint32_t)tiles), dim3(kThreads), 0, s,
                       d_bits, (uint64_t)bits_size, d_values, (uint64_t)values_size, d_out,
                       (uint64_t)n, (uint64_t)tiles, ctrl, status);
    FLRL_HIP(hipGetLastError());
    return FLRL_OK;
}

extern "C" int flrl_scratch_error(const void *d_scratch, void *stream)
{
    if (!d_scratch)
        return set_error(FLRL_E_ARG, "flrl_scratch_error: null scratch");
    Ctrl c;
    FLRL_HIP(hipMemcpyAsync(&c, d_scratch, sizeof(c), hipMemcpyDeviceToHost,
                            static_cast<hipStream_t>(stream)));
    FLRL_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
    return (int)c.error;
}

// ---------------------------------------------------------------------------
// Host-buffer entry points (synchronous), mirroring gpuCompress/gpuDecompress.
// ---------------------------------------------------------------------------

extern "C" int flrl_fl_compress(const uint8_t *data, size_t size, flrl_fl_buf *out)
{
    clear_error();
    if (!out || (!data && size))
        return set_error(FLRL_E_ARG, "flrl_fl_compress: null argument");
    memset(out, 0, sizeof(*out));
    if (size == 0)  // fl_gpu.cu:291-294 / fl_cpu.cu:11-14
        return FLRL_OK;
    if (flrl_device_count() <= 0)
        return set_error(FLRL_E_NODEV, "flrl_fl_compress: no HIP device visible");
    const size_t frames = div_up(size, kFrame);
    const size_t in_b = round_up(size, 16), bits_b = round_up(frames, 16);
    const size_t val_b = flrl_fl_values_capacity(size), scr_b = flrl_fl_scratch_bytes(size);
    DevBuf dev;
    if (dev.alloc(in_b + bits_b + val_b + 16 + scr_b) != hipSuccess)
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory (device, %zu bytes)",
                         in_b + bits_b + val_b + 16 + scr_b);
    uint8_t *d_in = dev.as<uint8_t>(0);
    uint8_t *d_bits = dev.as<uint8_t>(in_b);
    uint8_t *d_values = dev.as<uint8_t>(in_b + bits_b);
    uint64_t *d_vsize = dev.as<uint64_t>(in_b + bits_b + val_b);
    void *d_scr = dev.as<void>(in_b + bits_b + val_b + 16);
    FLRL_HIP(hipMemcpy(d_in, data, size, hipMemcpyHostToDevice));
    int rc = flrl_fl_encode_device(d_in, size, d_bits, d_values, d_vsize, d_scr, scr_b, nullptr);
    if (rc)
        return rc;
    uint64_t vsize = 0;
    FLRL_HIP(hipMemcpy(&vsize, d_vsize, sizeof(vsize), hipMemcpyDeviceToHost));
    const int kerr = flrl_scratch_error(d_scr, nullptr);
    if (kerr)
        return set_error(kerr, "flrl_fl_compress: device error %d", kerr);
    uint8_t *h_bits = static_cast<uint8_t *>(malloc(frames));
    uint8_t *h_vals = static_cast<uint8_t *>(malloc(vsize ? vsize : 1));
    if (!h_bits || !h_vals) {
        free(h_bits);
        free(h_vals);
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory");
    }
    hipError_t e1 = hipMemcpy(h_bits, d_bits, frames, hipMemcpyDeviceToHost);
    hipError_t e2 = hipMemcpy(h_vals, d_values, vsize, hipMemcpyDeviceToHost);
    if (e1 != hipSuccess || e2 != hipSuccess) {
        free(h_bits);
        free(h_vals);
        return set_error(FLRL_E_HIP, "flrl_fl_compress: copy-out failed: %s",
                         hipGetErrorString(e1 != hipSuccess ? e1 : e2));
    }
    out->bits = h_bits;
    out->bits_size = frames;
    out->values = h_vals;
    out->values_size = vsize;
    out->input_size = size;
    return FLRL_OK;
}

extern "C" int flrl_fl_decompress(size_t output_size, const uint8_t *bits, size_t bits_size,
                                  const uint8_t *values, size_t values_size, uint8_t **out,
                                  size_t *out_size)
{
    clear_error();
    if (!out || !out_size)
        return set_error(FLRL_E_ARG, "flrl_fl_decompress: null output pointer");
    *out = nullptr;
    *out_size = 0;
    if (values_size == 0 || bits_size == 0)  // fl_cpu.cu:94-97, fl_gpu.cu:539-542
        return FLRL_OK;
    if (!bits || !values)
        return set_error(FLRL_E_ARG, "flrl_fl_decompress: null input");
    if (flrl_device_count() <= 0)
        return set_error(FLRL_E_NODEV, "flrl_fl_decompress: no HIP device visible");
    // Format hardening: the reference reads out of
    // bounds on any of these; the output for valid files is unchanged.
    if (bits_size != div_up(output_size, kFrame))
        return set_error(FLRL_E_FORMAT, "bitsSize %zu != ceil(inputSize %zu / 128)", bits_size,
                         output_size);
    uint64_t sum_full = 0;
    for (size_t f = 0; f < bits_size; ++f) {
        if (bits[f] < 1 || bits[f] > 8)
            return set_error(FLRL_E_FORMAT, "frame %zu has width %u (must be 1..8)", f,
                             (unsigned)bits[f]);
        if (f + 1 < bits_size)
            sum_full += bits[f];
    }
    const uint64_t cnt_last = output_size - (bits_size - 1) * (uint64_t)kFrame;
    const uint64_t expect = 16 * sum_full + (cnt_last * bits[bits_size - 1] + 7) / 8;
    if (expect != values_size)
        return set_error(FLRL_E_FORMAT, "valuesSize %zu != %llu implied by the widths",
                         values_size, (unsigned long long)expect);

    const size_t bits_b = round_up(bits_size, 16), val_b = round_up(values_size, 16);
    const size_t out_b = round_up(output_size, 16), scr_b = flrl_fl_scratch_bytes(output_size);
    DevBuf dev;
    if (dev.alloc(bits_b + val_b + out_b + scr_b) != hipSuccess)
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory (device, %zu bytes)",
                         bits_b + val_b + out_b + scr_b);
    uint8_t *d_bits = dev.as<uint8_t>(0);
    uint8_t *d_vals = dev.as<uint8_t>(bits_b);
    uint8_t *d_out = dev.as<uint8_t>(bits_b + val_b);
    void *d_scr = dev.as<void>(bits_b + val_b + out_b);
    FLRL_HIP(hipMemcpy(d_bits, bits, bits_size, hipMemcpyHostToDevice));
    FLRL_HIP(hipMemcpy(d_vals, values, values_size, hipMemcpyHostToDevice));
    int rc = flrl_fl_decode_device(d_bits, bits_size, d_vals, values_size, d_out, output_size,
                                   d_scr, scr_b, nullptr);
    if (rc)
        return rc;
    const int kerr = flrl_scratch_error(d_scr, nullptr);
    if (kerr)
        return set_error(kerr, "flrl_fl_decompress: device error %d", kerr);
    uint8_t *h = static_cast<uint8_t *>(malloc(output_size));
    if (!h)
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory");
    hipError_t e = hipMemcpy(h, d_out, output_size, hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
        free(h);
        return set_error(FLRL_E_HIP, "flrl_fl_decompress: copy-out failed: %s",
                         hipGetErrorString(e));
    }
    *out = h;
    *out_size = output_size;
    return FLRL_OK;
}
