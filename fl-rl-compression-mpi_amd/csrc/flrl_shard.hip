// flrl_shard.hip — sharded FL encode across the GPUs of one node, one process.
//
// Replaces gpuNCCLCompress (src/fl/fl_gpu.cu:76-287) and gpuMPICompress
// (:41-74). The reference runs one MPI rank per GPU, exchanges the three sizes
// with MPI_Allgather, then ncclAllGather's every rank's padded outputs to every
// rank (O(P*N) traffic) and concatenates on rank 0. Here one process drives all
// GPUs: shards follow the reference rule (file_io.cu:46-51, in size_t: every
// shard but the last is floor(N/(128P))*128 bytes), each GPU encodes its shard
// in place, and a single RCCL ncclAllGather of {F_r, V_r} (16 B per GPU over
// xGMI) gives every GPU the exclusive scan that places its bits/values in the
// output. Concatenating 128-aligned shard outputs equals the whole-input output
// byte for byte, so the result is identical to
// flrl_fl_compress.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <thread>
#include <vector>

#include "flrl.h"
#include "flrl_internal.hpp"

using namespace flrl;

namespace {

struct Shard {
    int dev = 0;
    size_t off = 0, len = 0, frames = 0;
    hipStream_t stream = nullptr;
    void *base = nullptr;  // one device allocation per shard
    uint8_t *d_in = nullptr, *d_bits = nullptr, *d_vals = nullptr;
    uint64_t *d_sizes = nullptr, *d_all = nullptr;
    void *d_scr = nullptr;
    size_t scr_b = 0;
    uint64_t vsize = 0;
    int rc = 0;
    char err[256] = {0};
};

int shard_encode(Shard &s, const uint8_t *data, int ngpus)
{
    if (hipSetDevice(s.dev) != hipSuccess)
        return set_error(FLRL_E_HIP, "hipSetDevice(%d) failed", s.dev);
    const size_t in_b = round_up(s.len ? s.len : 1, 16), bits_b = round_up(s.frames + 1, 16);
    const size_t val_b = flrl_fl_values_capacity(s.len);
    const size_t sizes_b = round_up(16 + 16 * (size_t)ngpus, 16);
    s.scr_b = flrl_fl_scratch_bytes(s.len);
    if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess)
        return set_error(FLRL_E_HIP, "hipStreamCreate failed on device %d", s.dev);
    if (hipMalloc(&s.base, in_b + bits_b + val_b + sizes_b + s.scr_b) != hipSuccess)
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory (device %d)", s.dev);
    uint8_t *p = static_cast<uint8_t *>(s.base);
    s.d_in = p;
    s.d_bits = p + in_b;
    s.d_vals = p + in_b + bits_b;
    s.d_sizes = reinterpret_cast<uint64_t *>(p + in_b + bits_b + val_b);
    s.d_all = s.d_sizes + 2;
    s.d_scr = p + in_b + bits_b + val_b + sizes_b;
    if (s.len && hipMemcpyAsync(s.d_in, data + s.off, s.len, hipMemcpyHostToDevice, s.stream) !=
                     hipSuccess)
        return set_error(FLRL_E_HIP, "shard upload failed on device %d", s.dev);
    int rc = flrl_fl_encode_device(s.d_in, s.len, s.d_bits, s.d_vals, s.d_sizes + 1, s.d_scr,
                                   s.scr_b, s.stream);
    if (rc)
        return rc;
    const uint64_t f = s.frames;
    if (hipMemcpyAsync(s.d_sizes, &f, sizeof(f), hipMemcpyHostToDevice, s.stream) != hipSuccess)
        return set_error(FLRL_E_HIP, "frame-count upload failed on device %d", s.dev);
    if (hipStreamSynchronize(s.stream) != hipSuccess)  // also keeps &f alive for the copy
        return set_error(FLRL_E_HIP, "stream sync failed on device %d", s.dev);
    return FLRL_OK;
}

}  // namespace

extern "C" int flrl_fl_compress_sharded(const uint8_t *data, size_t size, int ngpus,
                                        flrl_fl_buf *out)
{
    clear_error();
    if (!out || (!data && size))
        return set_error(FLRL_E_ARG, "flrl_fl_compress_sharded: null argument");
    memset(out, 0, sizeof(*out));
    int ndev = flrl_device_count();
    if (ndev <= 0)
        return set_error(FLRL_E_NODEV, "flrl_fl_compress_sharded: no HIP device");
    if (ngpus <= 0)
        ngpus = ndev;
    if (ngpus > ndev)
        return set_error(FLRL_E_ARG, "flrl_fl_compress_sharded: %d GPUs requested, %d visible",
                         ngpus, ndev);
    if (size == 0)
        return FLRL_OK;

    const size_t P = (size_t)ngpus;
    const size_t per = (size / (FLRL_FRAME_LENGTH * P)) * FLRL_FRAME_LENGTH;
    std::vector<Shard> sh(P);
    for (size_t r = 0; r < P; ++r) {
        sh[r].dev = (int)r;
        sh[r].off = r * per;
        sh[r].len = r + 1 == P ? size - (P - 1) * per : per;
        sh[r].frames = div_up(sh[r].len, FLRL_FRAME_LENGTH);
    }
    auto cleanup = [&]() {
        for (auto &s : sh) {
            if (s.base) {
                (void)hipSetDevice(s.dev);
                (void)hipFree(s.base);
            }
            if (s.stream)
                (void)hipStreamDestroy(s.stream);
        }
    };

    {
        std::vector<std::thread> th;
        for (size_t r = 0; r < P; ++r)
            th.emplace_back([&, r]() {
                clear_error();
                sh[r].rc = shard_encode(sh[r], data, ngpus);
                if (sh[r].rc)  // the last-error string is per thread: keep the worker's
                    snprintf(sh[r].err, sizeof(sh[r].err), "%s", flrl_last_error());
            });
        for (auto &t : th)
            t.join();
    }
    for (size_t r = 0; r < P; ++r)
        if (sh[r].rc) {
            cleanup();
            return set_error(sh[r].rc, "flrl_fl_compress_sharded: shard %zu encode failed%s%s", r,
                             sh[r].err[0] ? ": " : "", sh[r].err);
        }

    // ---- the one exchange step: AllGather {F_r, V_r} over xGMI -------------
    std::vector<ncclComm_t> comms(P);
    std::vector<int> devs(P);
    for (size_t r = 0; r < P; ++r)
        devs[r] = (int)r;
    if (ncclCommInitAll(comms.data(), ngpus, devs.data()) != ncclSuccess) {
        cleanup();
        return set_error(FLRL_E_RCCL, "ncclCommInitAll failed");
    }
    ncclResult_t nr = ncclGroupStart();
    for (size_t r = 0; r < P && nr == ncclSuccess; ++r)
        nr = ncclAllGather(sh[r].d_sizes, sh[r].d_all, 2, ncclUint64, comms[r], sh[r].stream);
    ncclResult_t ne = ncclGroupEnd();
    std::vector<uint64_t> all(2 * P);
    int rc = FLRL_OK;
    if (nr != ncclSuccess || ne != ncclSuccess)
        rc = set_error(FLRL_E_RCCL, "ncclAllGather failed: %s",
                       ncclGetErrorString(nr != ncclSuccess ? nr : ne));
    for (size_t r = 0; r < P && rc == FLRL_OK; ++r) {
        (void)hipSetDevice(sh[r].dev);
        if (hipStreamSynchronize(sh[r].stream) != hipSuccess)
            rc = set_error(FLRL_E_HIP, "flrl_fl_compress_sharded: stream sync failed");
        const int kerr = flrl_scratch_error(sh[r].d_scr, sh[r].stream);
        if (kerr)
            rc = set_error(kerr, "flrl_fl_compress_sharded: device error %d on shard %zu", kerr, r);
    }
    if (rc == FLRL_OK) {
        (void)hipSetDevice(sh[0].dev);
        if (hipMemcpy(all.data(), sh[0].d_all, 16 * P, hipMemcpyDeviceToHost) != hipSuccess)
            rc = set_error(FLRL_E_HIP, "flrl_fl_compress_sharded: size read-back failed");
    }
    for (auto &c : comms)
        (void)ncclCommDestroy(c);
    if (rc) {
        cleanup();
        return rc;
    }

    // exclusive scan of {F_r, V_r} -> output placement
    std::vector<size_t> foff(P), voff(P);
    size_t F = 0, V = 0;
    for (size_t r = 0; r < P; ++r) {
        foff[r] = F;
        voff[r] = V;
        F += all[2 * r];
        V += all[2 * r + 1];
    }
    uint8_t *h_bits = static_cast<uint8_t *>(malloc(F ? F : 1));
    uint8_t *h_vals = static_cast<uint8_t *>(malloc(V ? V : 1));
    if (!h_bits || !h_vals) {
        free(h_bits);
        free(h_vals);
        cleanup();
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory");
    }
    {
        std::vector<std::thread> th;
        for (size_t r = 0; r < P; ++r)
            th.emplace_back([&, r]() {
                Shard &s = sh[r];
                (void)hipSetDevice(s.dev);
                const size_t fr = all[2 * r], vr = all[2 * r + 1];
                if ((fr && hipMemcpy(h_bits + foff[r], s.d_bits, fr, hipMemcpyDeviceToHost)) ||
                    (vr && hipMemcpy(h_vals + voff[r], s.d_vals, vr, hipMemcpyDeviceToHost)))
                    s.rc = FLRL_E_HIP;
            });
        for (auto &t : th)
            t.join();
    }
    for (size_t r = 0; r < P; ++r)
        if (sh[r].rc) {
            free(h_bits);
            free(h_vals);
            cleanup();
            return set_error(FLRL_E_HIP, "flrl_fl_compress_sharded: copy-out of shard %zu failed",
                             r);
        }
    cleanup();
    out->bits = h_bits;
    out->bits_size = F;
    out->values = h_vals;
    out->values_size = V;
    out->input_size = size;
    return FLRL_OK;
}
