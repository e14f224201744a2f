// flrl_shard.hip — multi-GPU FL encode: RCCL communicators, the one exchange
// step (an all-gather of {F_r, V_r} + exclusive scan) and the entry points
// built on it.
//
// Replaces gpuNCCLCompress (src/fl/fl_gpu.cu:76-287) and gpuMPICompress
// (:41-74). The reference runs one MPI rank per GPU, exchanges three sizes with
// MPI_Allgather (:101-106), then ncclAllGather's every rank's padded outputs to
// every rank (O(P*N) traffic, :144-194) and concatenates on rank 0. Here the
// only collective on the data path is one RCCL ncclAllGather of 16 bytes per
// shard over xGMI; every shard learns its output offsets {F_off, V_off} and the
// totals on the device, with no host round trip. Concatenating 128-aligned
// shard outputs equals the whole-input output byte for byte (SURVEY.md §0
// fact 7), so placing shard r at its offsets reproduces flrl_fl_compress.
//
// Two process models:
//  * one process per GPU (the reference's model, main.cu:46-70): a rank's comm
//    from flrl_comm_init_rank / flrl_comm_wrap; flrl_fl_encode_rank encodes the
//    rank's shard in place and runs the exchange on the caller's stream;
//    flrl_fl_compress_rank is the host-buffer twin of gpuNCCLCompress (rank 0
//    receives the merged result, ncclSend/ncclRecv of the payloads);
//  * one process driving the node's GPUs: flrl_comm_init (ncclCommInitAll over
//    distinct devices); flrl_fl_encode_sharded places shard r on device
//    r mod ndev, so any number of shards runs on any number of GPUs: shards of
//    one device exchange through a local slot array, devices through RCCL.
// A comm is created once and reused by every call (no per-call
// ncclCommInitAll); flrl_fl_compress_sharded keeps one per device set.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <mutex>
#include <vector>

#include "flrl.h"
#include "flrl_device.hpp"
#include "flrl_internal.hpp"
#include "flrl_shard_layout.hpp"

using namespace flrl;

namespace {

constexpr int kMaxLocal = 64;  // shards per device in one flrl_fl_encode_sharded call

// Sizes record of every shard (include/flrl.h FLRL_SZ_*), written on the device.
struct LocalOuts {
    uint32_t count;
    uint32_t index[kMaxLocal];   // global shard index
    uint64_t *sizes[kMaxLocal];  // its d_sizes (FLRL_SZ_COUNT u64)
    Ctrl *ctrl[kMaxLocal];       // its scratch (error word)
};

__global__ void put_u64_kernel(uint64_t *p, uint64_t v)
{
    if (threadIdx.x == 0 && blockIdx.x == 0)
        *p = v;
}

__global__ void put_pair_kernel(uint64_t *p, uint64_t a, uint64_t b)
{
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        p[0] = a;
        p[1] = b;
    }
}

// Each thread owns one local shard: its record from the all-gathered slots
// (shard_record, flrl_shard_layout.hpp: the layout the CPU tests check through
// flrl_shard_scan); a ragged shard before the last, or any shard whose rank
// failed, raises FLRL_E_ARG in that shard's scratch error word. A null sizes
// or ctrl pointer (a rank that failed on its own arguments) is skipped.
__global__ __launch_bounds__(kWave) void size_scan_kernel(const uint64_t *gather, uint32_t nshards,
                                                          uint32_t ndev, uint32_t S, LocalOuts outs)
{
    for (uint32_t i = threadIdx.x; i < outs.count; i += blockDim.x)
        if (shard_record(gather, nshards, ndev, S, outs.index[i], outs.sizes[i]) && outs.ctrl[i])
            raise_error(outs.ctrl[i], FLRL_E_ARG);
}

struct Dev {
    int id = 0;
    ncclComm_t nccl = nullptr;
    hipStream_t cstream = nullptr;  // exchange stream of the sharded path
    hipEvent_t cdone = nullptr;
    uint64_t *gather = nullptr;
    size_t gather_cap = 0;          // u64 entries
    // 8 u64: [0, 4) flrl_fl_compress_rank's {size, failed} all-reduce (send,
    // receive); [4, 8) constants written once at set-up: a failed exchange
    // pair {failed word, 0} and a failed all-reduce word {0, 1}, the sources a
    // rank that cannot stage its own words sends instead (no launch or copy
    // needed on the failure path, so it still completes every collective)
    uint64_t *red = nullptr;
    std::vector<hipEvent_t> ev;     // per local shard slot
};

int rccl_error(ncclResult_t r, const char *what)
{
    return set_error(FLRL_E_RCCL, "%s failed: %s", what, ncclGetErrorString(r));
}

}  // namespace

struct flrl_comm {
    int nranks = 0, rank = 0;  // RCCL ranks of this process's view
    bool owns = true;          // ncclCommDestroy on destroy (not for wrapped comms)
    std::vector<Dev> dev;      // one per local device
    std::mutex mu;             // calls on one comm are serialised
};

namespace {

int dev_setup(Dev &d, size_t gather_entries)
{
    if (hipSetDevice(d.id) != hipSuccess)
        return set_error(FLRL_E_HIP, "hipSetDevice(%d) failed", d.id);
    if (!d.cstream && hipStreamCreateWithFlags(&d.cstream, hipStreamNonBlocking) != hipSuccess)
        return set_error(FLRL_E_HIP, "hipStreamCreate failed on device %d", d.id);
    if (!d.cdone && hipEventCreateWithFlags(&d.cdone, hipEventDisableTiming) != hipSuccess)
        return set_error(FLRL_E_HIP, "hipEventCreate failed on device %d", d.id);
    if (!d.red) {
        if (hipMalloc(&d.red, 8 * sizeof(uint64_t)) != hipSuccess) {
            d.red = nullptr;
            return set_error(FLRL_E_NOMEM, "Cannot allocate memory (device %d)", d.id);
        }
        const uint64_t k[8] = {0, 0, 0, 0, shard_failed_word(), 0, 0, 1};
        if (hipMemcpy(d.red, k, sizeof(k), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipFree(d.red);
            d.red = nullptr;
            return set_error(FLRL_E_HIP, "hipMemcpy failed on device %d", d.id);
        }
    }
    if (gather_entries > d.gather_cap) {
        if (d.gather) {  // the previous call's exchange or scan may still read it
            (void)hipStreamSynchronize(d.cstream);
            (void)hipEventSynchronize(d.cdone);  // (a per-rank call's scan ran on the caller's stream)
            (void)hipFree(d.gather);
            d.gather = nullptr;
            d.gather_cap = 0;
        }
        if (hipMalloc(&d.gather, gather_entries * sizeof(uint64_t)) != hipSuccess)
            return set_error(FLRL_E_NOMEM, "Cannot allocate memory (device %d)", d.id);
        d.gather_cap = gather_entries;
        // complete before returning: the shards' streams are non-blocking, so a
        // null-stream hipMemset could land after their first size writes
        if (hipMemsetAsync(d.gather, 0, gather_entries * sizeof(uint64_t), d.cstream) != hipSuccess ||
            hipStreamSynchronize(d.cstream) != hipSuccess)
            return set_error(FLRL_E_HIP, "hipMemset failed on device %d", d.id);
    }
    return FLRL_OK;
}

void dev_release(Dev &d, bool destroy_nccl)
{
    (void)hipSetDevice(d.id);
    if (d.cstream)
        (void)hipStreamSynchronize(d.cstream);
    if (d.cdone)  // the last per-rank call's size scan (on the caller's stream) reads the gather array
        (void)hipEventSynchronize(d.cdone);
    if (d.gather)
        (void)hipFree(d.gather);
    if (d.red)
        (void)hipFree(d.red);
    for (hipEvent_t e : d.ev)
        (void)hipEventDestroy(e);
    if (d.cdone)
        (void)hipEventDestroy(d.cdone);
    if (d.cstream)
        (void)hipStreamDestroy(d.cstream);
    if (destroy_nccl && d.nccl)
        (void)ncclCommDestroy(d.nccl);
    d = Dev{};
}

int device_of(const void *p, int *dev)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // not sticky for the next launch check
        return -1;
    }
    if (a.type != hipMemoryTypeDevice && a.type != hipMemoryTypeManaged)
        return -1;  // host memory (registered or not) is not a shard buffer
    *dev = a.device;
    return 0;
}

int current_device()
{
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess)
        d = 0;
    return d;
}

}  // namespace

// ---- communicators ----------------------------------------------------------

extern "C" int flrl_comm_init(int ndev, const int *devs, flrl_comm **out)
{
    clear_error();
    if (!out)
        return set_error(FLRL_E_ARG, "flrl_comm_init: null output");
    *out = nullptr;
    const int visible = flrl_device_count();
    if (visible <= 0)
        return set_error(FLRL_E_NODEV, "flrl_comm_init: no HIP device");
    if (ndev <= 0)
        ndev = visible;
    std::vector<int> ids((size_t)ndev);
    for (int i = 0; i < ndev; ++i) {
        ids[(size_t)i] = devs ? devs[i] : i;
        if (ids[(size_t)i] < 0 || ids[(size_t)i] >= visible)
            return set_error(FLRL_E_ARG, "flrl_comm_init: device %d not visible (%d devices)",
                             ids[(size_t)i], visible);
        for (int j = 0; j < i; ++j)
            if (ids[(size_t)j] == ids[(size_t)i])
                return set_error(FLRL_E_ARG, "flrl_comm_init: device %d listed twice",
                                 ids[(size_t)i]);
    }
    const int prev = current_device();
    flrl_comm *c = new flrl_comm;
    c->nranks = ndev;
    c->rank = 0;
    c->dev.resize((size_t)ndev);
    std::vector<ncclComm_t> comms((size_t)ndev);
    ncclResult_t r = ncclCommInitAll(comms.data(), ndev, ids.data());
    if (r != ncclSuccess) {
        delete c;
        (void)hipSetDevice(prev);
        return rccl_error(r, "ncclCommInitAll");
    }
    int rc = FLRL_OK;
    for (int i = 0; i < ndev; ++i) {
        c->dev[(size_t)i].id = ids[(size_t)i];
        c->dev[(size_t)i].nccl = comms[(size_t)i];
        if (rc == FLRL_OK)
            rc = dev_setup(c->dev[(size_t)i], 2 * (size_t)ndev);
    }
    (void)hipSetDevice(prev);
    if (rc) {
        (void)flrl_comm_destroy(c);
        return rc;
    }
    *out = c;
    return FLRL_OK;
}

extern "C" int flrl_comm_unique_id(void *id)
{
    clear_error();
    if (!id)
        return set_error(FLRL_E_ARG, "flrl_comm_unique_id: null buffer");
    static_assert(sizeof(ncclUniqueId) == FLRL_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess)
        return rccl_error(r, "ncclGetUniqueId");
    memcpy(id, &u, sizeof(u));
    return FLRL_OK;
}

extern "C" int flrl_comm_init_rank(int nranks, const void *id, int rank, flrl_comm **out)
{
    clear_error();
    if (!out || !id)
        return set_error(FLRL_E_ARG, "flrl_comm_init_rank: null argument");
    *out = nullptr;
    if (nranks <= 0 || rank < 0 || rank >= nranks)
        return set_error(FLRL_E_ARG, "flrl_comm_init_rank: rank %d of %d", rank, nranks);
    if (flrl_device_count() <= 0)
        return set_error(FLRL_E_NODEV, "flrl_comm_init_rank: no HIP device");
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t nc = nullptr;
    const ncclResult_t r = ncclCommInitRank(&nc, nranks, u, rank);  // on the current device
    if (r != ncclSuccess)
        return rccl_error(r, "ncclCommInitRank");
    flrl_comm *c = new flrl_comm;
    c->nranks = nranks;
    c->rank = rank;
    c->dev.resize(1);
    c->dev[0].id = current_device();
    c->dev[0].nccl = nc;
    const int rc = dev_setup(c->dev[0], 2 * (size_t)nranks);
    if (rc) {
        (void)flrl_comm_destroy(c);
        return rc;
    }
    *out = c;
    return FLRL_OK;
}

extern "C" int flrl_comm_wrap(void *nccl_comm, flrl_comm **out)
{
    clear_error();
    if (!out || !nccl_comm)
        return set_error(FLRL_E_ARG, "flrl_comm_wrap: null argument");
    *out = nullptr;
    ncclComm_t nc = static_cast<ncclComm_t>(nccl_comm);
    int n = 0, r = 0, d = 0;
    ncclResult_t e;
    if ((e = ncclCommCount(nc, &n)) != ncclSuccess || (e = ncclCommUserRank(nc, &r)) != ncclSuccess ||
        (e = ncclCommCuDevice(nc, &d)) != ncclSuccess)
        return rccl_error(e, "flrl_comm_wrap: communicator query");
    const int prev = current_device();
    flrl_comm *c = new flrl_comm;
    c->nranks = n;
    c->rank = r;
    c->owns = false;
    c->dev.resize(1);
    c->dev[0].id = d;
    c->dev[0].nccl = nc;
    const int rc = dev_setup(c->dev[0], 2 * (size_t)n);
    (void)hipSetDevice(prev);
    if (rc) {
        (void)flrl_comm_destroy(c);
        return rc;
    }
    *out = c;
    return FLRL_OK;
}

extern "C" int flrl_comm_destroy(flrl_comm *c)
{
    if (!c)
        return FLRL_OK;
    const int prev = current_device();
    for (Dev &d : c->dev)
        dev_release(d, c->owns);
    (void)hipSetDevice(prev);
    delete c;
    return FLRL_OK;
}

extern "C" int flrl_comm_query(const flrl_comm *c, int *nranks, int *rank, int *ndev)
{
    if (!c)
        return set_error(FLRL_E_ARG, "flrl_comm_query: null comm");
    if (nranks)
        *nranks = c->nranks;
    if (rank)
        *rank = c->rank;
    if (ndev)
        *ndev = (int)c->dev.size();
    return FLRL_OK;
}

extern "C" int flrl_comm_rccl_info(const flrl_comm *c, int local, int *count, int *rank, int *device,
                                   char *pci_bus_id, int len)
{
    if (!c || local < 0 || (size_t)local >= c->dev.size())
        return set_error(FLRL_E_ARG, "flrl_comm_rccl_info: no local device %d", local);
    const Dev &d = c->dev[(size_t)local];
    int n = 0, r = 0, dv = -1;
    ncclResult_t e = ncclCommCount(d.nccl, &n);
    if (e == ncclSuccess)
        e = ncclCommUserRank(d.nccl, &r);
    if (e == ncclSuccess)
        e = ncclCommCuDevice(d.nccl, &dv);
    if (e != ncclSuccess)
        return rccl_error(e, "flrl_comm_rccl_info");
    if (count)
        *count = n;
    if (rank)
        *rank = r;
    if (device)
        *device = dv;
    if (pci_bus_id && len > 0) {
        pci_bus_id[0] = 0;
        if (hipDeviceGetPCIBusId(pci_bus_id, len, dv) != hipSuccess)
            return set_error(FLRL_E_HIP, "hipDeviceGetPCIBusId(%d) failed", dv);
    }
    return FLRL_OK;
}

// ---- the exchange layout on the host (flrl_shard_layout.hpp) ---------------

extern "C" int flrl_shard_range(size_t n, int nshards, int shard, size_t *start, size_t *length)
{
    if (nshards <= 0 || shard < 0 || shard >= nshards || !start || !length)
        return set_error(FLRL_E_ARG, "flrl_shard_range: shard %d of %d", shard, nshards);
    uint64_t s0 = 0, len = 0;
    shard_range(n, (uint64_t)nshards, (uint64_t)shard, &s0, &len);
    *start = s0;
    *length = len;
    return FLRL_OK;
}

extern "C" size_t flrl_shard_slot(int shard, int nshards, int ndev)
{
    if (nshards <= 0 || ndev <= 0 || shard < 0 || shard >= nshards)
        return (size_t)-1;
    return shard_slot((uint64_t)shard, (uint64_t)ndev, div_up((size_t)nshards, (size_t)ndev));
}

extern "C" uint64_t flrl_shard_size_word(size_t n) { return shard_f_word(n); }

extern "C" uint64_t flrl_shard_failed_word(void) { return shard_failed_word(); }

extern "C" int flrl_shard_scan(const uint64_t *gather, int nshards, int ndev, int shard, uint64_t *rec)
{
    clear_error();
    if (!gather || !rec || nshards <= 0 || ndev <= 0 || shard < 0 || shard >= nshards)
        return set_error(FLRL_E_ARG, "flrl_shard_scan: shard %d of %d on %d devices", shard, nshards, ndev);
    const uint32_t S = (uint32_t)div_up((size_t)nshards, (size_t)ndev);
    const uint32_t bad = shard_record(gather, (uint32_t)nshards, (uint32_t)ndev, S, (uint32_t)shard, rec);
    if (bad & kRecFailed)
        return set_error(FLRL_E_ARG, "flrl_shard_scan: a shard's rank failed before the exchange");
    if (bad & kRecRagged)
        return set_error(FLRL_E_ARG, "flrl_shard_scan: a shard before the last is not a multiple of %d bytes",
                         kFrame);
    return FLRL_OK;
}

// ---- device-resident encode + exchange ------------------------------------

namespace {

// flrl_fl_encode_rank's body. `local` != FLRL_OK: this rank has already failed
// (flrl_fl_compress_rank: an allocation or upload), so it joins the exchange
// with a failed slot instead of encoding. A local argument failure of the
// encode does the same. Either way the all-gather runs on every rank, every
// peer's scan raises FLRL_E_ARG, and this rank returns its own error; only a
// comm that cannot take part at all (null, multi-device) returns before it.
// A rank that cannot even reach its device or order its stream after the
// previous call (a failed hipSetDevice / hipStreamWaitEvent) still sends: its
// slot then comes from the comm's constant failed pair (Dev::red + 4), which
// needs no launch (RCCL switches to the comm's device itself).
int encode_rank_impl(flrl_comm *c, const uint8_t *d_in, size_t n, uint8_t *d_bits, uint8_t *d_values,
                     uint64_t *d_sizes, void *d_scratch, size_t scratch_bytes, void *stream, int local)
{
    if (!c)
        return set_error(FLRL_E_ARG, "flrl_fl_encode_rank: null comm");
    if (c->dev.size() != 1)
        return set_error(FLRL_E_ARG,
                         "flrl_fl_encode_rank: comm drives %zu devices (use flrl_fl_encode_sharded)",
                         c->dev.size());
    std::lock_guard<std::mutex> g(c->mu);
    Dev &d = c->dev[0];
    const int prev = current_device();
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (local == FLRL_OK && prev != d.id)
        local = set_error(FLRL_E_ARG, "flrl_fl_encode_rank: current device %d, comm on device %d", prev, d.id);
    if (local == FLRL_OK && !d_sizes)
        local = set_error(FLRL_E_ARG, "flrl_fl_encode_rank: null sizes");
    bool staged = true;  // this rank can write its own slot
    if (debug_fail_rank_step(FLRL_DEBUG_RANK_SET_DEVICE)) {
        if (local == FLRL_OK)
            local = set_error(FLRL_E_HIP, "flrl_fl_encode_rank: hipSetDevice(%d) failed (injected)", d.id);
        s = d.cstream;
        staged = false;
    } else if (local != FLRL_OK) {  // the caller's stream may be unusable: the comm's own
        s = d.cstream;
        staged = hipSetDevice(d.id) == hipSuccess;
    }
    // the previous call's scan may still read the gather array on another stream
    if (staged && (debug_fail_rank_step(FLRL_DEBUG_RANK_STREAM_WAIT) || hipStreamWaitEvent(s, d.cdone, 0) != hipSuccess)) {
        if (local == FLRL_OK)
            local = set_error(FLRL_E_HIP, "flrl_fl_encode_rank: event wait failed");
        s = d.cstream;
        // ordered on the host instead; failing that, the slot is not written
        // (the all-gather below still receives into the array: see there)
        staged = hipEventSynchronize(d.cdone) == hipSuccess;
    }
    uint64_t *slot = d.gather + shard_slot((uint64_t)c->rank, (uint64_t)c->nranks, 1);
    if (local == FLRL_OK) {
        hipLaunchKernelGGL(put_u64_kernel, dim3(1), dim3(kWave), 0, s, slot, shard_f_word(n));
        if (hipGetLastError() != hipSuccess)
            local = set_error(FLRL_E_HIP, "flrl_fl_encode_rank: launch failed");
        else
            local = flrl_fl_encode_device(d_in, n, d_bits, d_values, slot + 1, d_scratch, scratch_bytes, s);
        // on failure the failed pair follows the F word on the same stream (the
        // encode's argument checks precede every launch of it)
    }
    if (local != FLRL_OK && staged) {
        hipLaunchKernelGGL(put_pair_kernel, dim3(1), dim3(kWave), 0, s, slot, shard_failed_word(), (uint64_t)0);
        staged = hipGetLastError() == hipSuccess;
    }
    if (!staged) {
        // The constant failed pair is sent from d.cstream, and the all-gather
        // still RECEIVES into d.gather: order it after the previous call's scan
        // (which may still read the array on the caller's stream) -- on the
        // device, else on the host; if neither works the device is gone and
        // the send goes ahead regardless, so that the peers are not left
        // waiting in the collective.
        if (hipStreamWaitEvent(d.cstream, d.cdone, 0) != hipSuccess)
            (void)hipEventSynchronize(d.cdone);
        const ncclResult_t r = ncclAllGather(d.red + 4, d.gather, 2, ncclUint64, d.nccl, d.cstream);
        // the next call's slot write (ordered after d.cdone) must follow this
        // all-gather's write of the array
        if (r != ncclSuccess || hipEventRecord(d.cdone, d.cstream) != hipSuccess)
            (void)hipStreamSynchronize(d.cstream);
        (void)hipSetDevice(prev);
        return local ? local : rccl_error(r, "ncclAllGather");
    }
    const ncclResult_t r = ncclAllGather(slot, d.gather, 2, ncclUint64, d.nccl, s);  // in place
    if (r != ncclSuccess) {
        (void)hipSetDevice(prev);
        return local ? local : rccl_error(r, "ncclAllGather");
    }
    LocalOuts outs{};
    outs.count = 1;
    outs.index[0] = (uint32_t)c->rank;
    outs.sizes[0] = d_sizes;  // the failing rank's record too, when it gave one
    outs.ctrl[0] = local == FLRL_OK ? static_cast<Ctrl *>(d_scratch) : nullptr;
    hipLaunchKernelGGL(size_scan_kernel, dim3(1), dim3(kWave), 0, s, d.gather, (uint32_t)c->nranks,
                       (uint32_t)c->nranks, 1u, outs);
    const bool ok = hipGetLastError() == hipSuccess && hipEventRecord(d.cdone, s) == hipSuccess;
    (void)hipSetDevice(prev);
    if (local != FLRL_OK)
        return local;
    return ok ? FLRL_OK : set_error(FLRL_E_HIP, "flrl_fl_encode_rank: size scan failed");
}

}  // namespace

extern "C" int flrl_fl_encode_rank(flrl_comm *c, const uint8_t *d_in, size_t n, uint8_t *d_bits,
                                   uint8_t *d_values, uint64_t *d_sizes, void *d_scratch,
                                   size_t scratch_bytes, void *stream)
{
    clear_error();
    return encode_rank_impl(c, d_in, n, d_bits, d_values, d_sizes, d_scratch, scratch_bytes, stream, FLRL_OK);
}

extern "C" int flrl_fl_encode_sharded(flrl_comm *c, int nshards, const uint8_t *const *d_in,
                                      const size_t *n, uint8_t *const *d_bits,
                                      uint8_t *const *d_values, uint64_t *const *d_sizes,
                                      void *const *d_scratch, const size_t *scratch_bytes,
                                      void *const *streams)
{
    clear_error();
    if (!c || nshards <= 0 || !d_in || !n || !d_bits || !d_values || !d_sizes || !d_scratch ||
        !scratch_bytes || !streams)
        return set_error(FLRL_E_ARG, "flrl_fl_encode_sharded: null argument");
    if (c->rank != 0 || (size_t)c->nranks != c->dev.size())
        return set_error(FLRL_E_ARG, "flrl_fl_encode_sharded: needs a flrl_comm_init communicator");
    std::lock_guard<std::mutex> g(c->mu);
    const size_t ndev = c->dev.size();
    const size_t P = (size_t)nshards;
    const size_t S = div_up(P, ndev);  // slots per device
    if (S > (size_t)kMaxLocal)
        return set_error(FLRL_E_ARG, "flrl_fl_encode_sharded: %d shards on %zu devices (max %d per device)",
                         nshards, ndev, kMaxLocal);
    for (size_t r = 0; r + 1 < P; ++r)
        if (n[r] % kFrame)
            return set_error(FLRL_E_ARG,
                             "flrl_fl_encode_sharded: shard %zu has %zu bytes (every shard but the last "
                             "must be a multiple of %d)", r, n[r], kFrame);
    const int prev = current_device();
    // buffers of shard r must live on device r mod ndev
    for (size_t r = 0; r < P; ++r) {
        const int want = c->dev[r % ndev].id;
        int got = -1;
        if (!d_values[r] || !d_scratch[r] || !d_sizes[r] || device_of(d_values[r], &got) || got != want ||
            device_of(d_scratch[r], &got) || got != want || device_of(d_sizes[r], &got) || got != want) {
            (void)hipSetDevice(prev);
            return set_error(FLRL_E_ARG, "flrl_fl_encode_sharded: shard %zu buffers must be on device %d",
                             r, want);
        }
    }
    int rc = FLRL_OK;
    for (size_t k = 0; k < ndev && rc == FLRL_OK; ++k) {
        Dev &d = c->dev[k];
        rc = dev_setup(d, 2 * S * ndev);
        while (rc == FLRL_OK && d.ev.size() < S) {
            hipEvent_t e;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
                rc = set_error(FLRL_E_HIP, "hipEventCreate failed on device %d", d.id);
            else
                d.ev.push_back(e);
        }
    }
    // 1. every shard: F into its slot, encode (V lands in the slot), event
    for (size_t r = 0; r < P && rc == FLRL_OK; ++r) {
        Dev &d = c->dev[r % ndev];
        const size_t slot_i = shard_slot(r, ndev, S);
        hipStream_t s = static_cast<hipStream_t>(streams[r]);
        if (hipSetDevice(d.id) != hipSuccess) {
            rc = set_error(FLRL_E_HIP, "hipSetDevice(%d) failed", d.id);
            break;
        }
        // the previous call's scan may still read this device's gather array
        if (hipStreamWaitEvent(s, d.cdone, 0) != hipSuccess) {
            rc = set_error(FLRL_E_HIP, "flrl_fl_encode_sharded: event wait failed on device %d", d.id);
            break;
        }
        hipLaunchKernelGGL(put_u64_kernel, dim3(1), dim3(kWave), 0, s, d.gather + slot_i,
                           shard_f_word(n[r]));
        if (hipGetLastError() != hipSuccess) {
            rc = set_error(FLRL_E_HIP, "flrl_fl_encode_sharded: launch failed on device %d", d.id);
            break;
        }
        rc = flrl_fl_encode_device(d_in[r], n[r], d_bits[r], d_values[r], d.gather + slot_i + 1,
                                   d_scratch[r], scratch_bytes[r], streams[r]);
        if (rc)
            break;
        hipEvent_t e = d.ev[r / ndev];
        if (hipEventRecord(e, s) != hipSuccess || hipStreamWaitEvent(d.cstream, e, 0) != hipSuccess)
            rc = set_error(FLRL_E_HIP, "flrl_fl_encode_sharded: event failed on device %d", d.id);
    }
    // 2. the exchange: each device's S slots to every device
    if (rc == FLRL_OK) {
        ncclResult_t r1 = ncclGroupStart(), r2 = ncclSuccess;
        for (size_t k = 0; k < ndev && r1 == ncclSuccess; ++k) {
            Dev &d = c->dev[k];
            r1 = ncclAllGather(d.gather + k * S * 2, d.gather, 2 * S, ncclUint64, d.nccl, d.cstream);
        }
        r2 = ncclGroupEnd();
        if (r1 != ncclSuccess || r2 != ncclSuccess)
            rc = rccl_error(r1 != ncclSuccess ? r1 : r2, "ncclAllGather");
    }
    // 3. per device: offsets of its shards, then the shards' streams wait for them
    for (size_t k = 0; k < ndev && rc == FLRL_OK; ++k) {
        Dev &d = c->dev[k];
        LocalOuts outs{};
        for (size_t r = k; r < P; r += ndev) {
            outs.index[outs.count] = (uint32_t)r;
            outs.sizes[outs.count] = d_sizes[r];
            outs.ctrl[outs.count] = static_cast<Ctrl *>(d_scratch[r]);
            ++outs.count;
        }
        if (hipSetDevice(d.id) != hipSuccess) {
            rc = set_error(FLRL_E_HIP, "hipSetDevice(%d) failed", d.id);
            break;
        }
        hipLaunchKernelGGL(size_scan_kernel, dim3(1), dim3(kWave), 0, d.cstream, d.gather,
                           (uint32_t)P, (uint32_t)ndev, (uint32_t)S, outs);
        if (hipGetLastError() != hipSuccess || hipEventRecord(d.cdone, d.cstream) != hipSuccess) {
            rc = set_error(FLRL_E_HIP, "flrl_fl_encode_sharded: size scan failed on device %d", d.id);
            break;
        }
        for (size_t r = k; r < P; r += ndev)
            if (hipStreamWaitEvent(static_cast<hipStream_t>(streams[r]), d.cdone, 0) != hipSuccess)
                rc = set_error(FLRL_E_HIP, "flrl_fl_encode_sharded: event wait failed");
    }
    (void)hipSetDevice(prev);
    return rc;
}

// ---- host-buffer forms -------------------------------------------------------

namespace {

// Device buffers of one shard of a host-buffer call (freed after its stream).
struct ShardBufs {
    int dev = 0;
    size_t off = 0, len = 0;
    hipStream_t s = nullptr;
    void *base = nullptr;
    uint8_t *in = nullptr, *bits = nullptr, *vals = nullptr;
    uint64_t *sizes = nullptr;
    void *scr = nullptr;
    size_t scr_b = 0;
    int alloc(int device, size_t length)
    {
        dev = device;
        len = length;
        if (hipSetDevice(dev) != hipSuccess)
            return set_error(FLRL_E_HIP, "hipSetDevice(%d) failed", dev);
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
            return set_error(FLRL_E_HIP, "hipStreamCreate failed on device %d", dev);
        const size_t in_b = round_up(len ? len : 1, 16), bits_b = round_up(div_up(len, kFrame) + 1, 16);
        const size_t val_b = flrl_fl_values_capacity(len), sz_b = 64;
        scr_b = flrl_fl_scratch_bytes(len);
        if (hipMalloc(&base, in_b + bits_b + val_b + sz_b + scr_b) != hipSuccess)
            return set_error(FLRL_E_NOMEM, "Cannot allocate memory (device %d)", dev);
        uint8_t *p = static_cast<uint8_t *>(base);
        in = p;
        bits = p + in_b;
        vals = bits + bits_b;
        sizes = reinterpret_cast<uint64_t *>(vals + val_b);
        scr = vals + val_b + sz_b;
        return FLRL_OK;
    }
    ~ShardBufs()  // after its stream has drained, on its own device
    {
        if (!s && !base)
            return;
        (void)hipSetDevice(dev);
        if (s)
            (void)hipStreamSynchronize(s);
        if (base)
            (void)hipFree(base);
        if (s)
            (void)hipStreamDestroy(s);
    }
};

// One communicator per device count, created on first use and kept for the
// life of the process (RCCL init costs ~100 ms; a comm per call made the
// host-buffer sharded path unusable in a loop).
flrl_comm *cached_comm(int ndev, int *rc)
{
    static std::mutex m;
    static std::map<int, flrl_comm *> cache;
    std::lock_guard<std::mutex> g(m);
    auto it = cache.find(ndev);
    if (it != cache.end())
        return it->second;
    flrl_comm *c = nullptr;
    *rc = flrl_comm_init(ndev, nullptr, &c);
    if (*rc)
        return nullptr;
    cache[ndev] = c;
    return c;
}

int read_error(const ShardBufs &b, size_t r)
{
    (void)hipSetDevice(b.dev);
    const int kerr = flrl_scratch_error(b.scr, b.s);
    if (kerr)
        return set_error(kerr, "shard %zu: device error %d", r, kerr);
    return FLRL_OK;
}

}  // namespace

extern "C" int flrl_fl_compress_sharded(const uint8_t *data, size_t size, int nshards,
                                        flrl_fl_buf *out)
{
    clear_error();
    if (!out || (!data && size))
        return set_error(FLRL_E_ARG, "flrl_fl_compress_sharded: null argument");
    memset(out, 0, sizeof(*out));
    const int visible = flrl_device_count();
    if (visible <= 0)
        return set_error(FLRL_E_NODEV, "flrl_fl_compress_sharded: no HIP device");
    if (nshards <= 0)
        nshards = visible;
    if (nshards > kMaxLocal * visible)
        return set_error(FLRL_E_ARG, "flrl_fl_compress_sharded: %d shards (max %d)", nshards,
                         kMaxLocal * visible);
    if (size == 0)
        return FLRL_OK;
    const int ndev = nshards < visible ? nshards : visible;
    int rc = FLRL_OK;
    flrl_comm *c = cached_comm(ndev, &rc);
    if (!c)
        return rc;
    const int prev = current_device();

    // the reference shard rule (file_io.cu:46-51), size_t: every shard but the
    // last is floor(N/(128P))*128 bytes
    const size_t P = (size_t)nshards;
    std::vector<ShardBufs> sb(P);
    std::vector<const uint8_t *> in(P);
    std::vector<size_t> len(P), scr_b(P);
    std::vector<uint8_t *> bits(P), vals(P);
    std::vector<uint64_t *> sizes(P);
    std::vector<void *> scr(P), streams(P);
    for (size_t r = 0; r < P && rc == FLRL_OK; ++r) {
        uint64_t start = 0, L = 0;
        shard_range(size, P, r, &start, &L);
        rc = sb[r].alloc(c->dev[r % (size_t)ndev].id, L);
        if (rc)
            break;
        sb[r].off = start;
        if (L && hipMemcpyAsync(sb[r].in, data + sb[r].off, L, hipMemcpyHostToDevice, sb[r].s) != hipSuccess)
            rc = set_error(FLRL_E_HIP, "shard %zu upload failed", r);
        in[r] = sb[r].in;
        len[r] = L;
        bits[r] = sb[r].bits;
        vals[r] = sb[r].vals;
        sizes[r] = sb[r].sizes;
        scr[r] = sb[r].scr;
        scr_b[r] = sb[r].scr_b;
        streams[r] = sb[r].s;
    }
    if (rc == FLRL_OK)
        rc = flrl_fl_encode_sharded(c, nshards, in.data(), len.data(), bits.data(), vals.data(),
                                    sizes.data(), scr.data(), scr_b.data(), streams.data());
    std::vector<uint64_t> rec(P * FLRL_SZ_COUNT);
    for (size_t r = 0; r < P && rc == FLRL_OK; ++r) {
        (void)hipSetDevice(sb[r].dev);
        if (hipMemcpyAsync(&rec[r * FLRL_SZ_COUNT], sb[r].sizes, FLRL_SZ_COUNT * 8, hipMemcpyDeviceToHost,
                           sb[r].s) != hipSuccess ||
            hipStreamSynchronize(sb[r].s) != hipSuccess)
            rc = set_error(FLRL_E_HIP, "shard %zu: size read-back failed", r);
        else
            rc = read_error(sb[r], r);
    }
    uint8_t *h_bits = nullptr, *h_vals = nullptr;
    size_t F = 0, V = 0;
    if (rc == FLRL_OK) {
        F = rec[FLRL_SZ_F_TOTAL];
        V = rec[FLRL_SZ_V_TOTAL];
        h_bits = static_cast<uint8_t *>(malloc(F ? F : 1));
        h_vals = static_cast<uint8_t *>(malloc(V ? V : 1));
        if (!h_bits || !h_vals)
            rc = set_error(FLRL_E_NOMEM, "Cannot allocate memory");
    }
    for (size_t r = 0; r < P && rc == FLRL_OK; ++r) {
        const uint64_t *q = &rec[r * FLRL_SZ_COUNT];
        (void)hipSetDevice(sb[r].dev);
        if ((q[FLRL_SZ_F] && hipMemcpy(h_bits + q[FLRL_SZ_F_OFF], sb[r].bits, q[FLRL_SZ_F],
                                       hipMemcpyDeviceToHost) != hipSuccess) ||
            (q[FLRL_SZ_V] && hipMemcpy(h_vals + q[FLRL_SZ_V_OFF], sb[r].vals, q[FLRL_SZ_V],
                                       hipMemcpyDeviceToHost) != hipSuccess))
            rc = set_error(FLRL_E_HIP, "flrl_fl_compress_sharded: copy-out of shard %zu failed", r);
    }
    sb.clear();  // every shard's stream drained before its buffers are freed
    (void)hipSetDevice(prev);
    if (rc) {
        free(h_bits);
        free(h_vals);
        return rc;
    }
    out->bits = h_bits;
    out->bits_size = F;
    out->values = h_vals;
    out->values_size = V;
    out->input_size = size;
    return FLRL_OK;
}

extern "C" int flrl_fl_compress_rank(flrl_comm *c, const uint8_t *data, size_t size, flrl_fl_buf *out)
{
    clear_error();
    if (!c || !out || (!data && size))
        return set_error(FLRL_E_ARG, "flrl_fl_compress_rank: null argument");
    memset(out, 0, sizeof(*out));
    if (c->dev.size() != 1)
        return set_error(FLRL_E_ARG, "flrl_fl_compress_rank: needs a per-rank communicator");
    const int prev = current_device();
    Dev &dv = c->dev[0];
    // Collective on errors: a rank that fails anywhere
    // still completes (1) the exchange, with a failed slot, and (2) the
    // all-reduce of {size, failed}; (3) the payload send/recv runs only when no
    // rank failed, so no peer ever waits in a collective this rank skipped.
    ShardBufs b;
    int rc = b.alloc(dv.id, size);
    if (rc == FLRL_OK && size &&
        hipMemcpyAsync(b.in, data, size, hipMemcpyHostToDevice, b.s) != hipSuccess)
        rc = set_error(FLRL_E_HIP, "flrl_fl_compress_rank: upload failed");
    // (1) encode + exchange; a failed rank joins with a failed slot
    {
        const int e = encode_rank_impl(c, b.in, size, b.bits, b.vals, rc == FLRL_OK ? b.sizes : nullptr, b.scr,
                                       b.scr_b, b.s ? b.s : dv.cstream, rc);
        if (rc == FLRL_OK)
            rc = e;
    }
    const bool rcl_broken = rc == FLRL_E_RCCL;  // the comm itself failed: no further collectives
    const size_t R = (size_t)c->nranks;
    std::vector<uint64_t> all(2 * R);
    uint64_t rec[FLRL_SZ_COUNT] = {0};
    if (rc == FLRL_OK) {
        std::lock_guard<std::mutex> g(c->mu);
        if (hipMemcpyAsync(rec, b.sizes, sizeof(rec), hipMemcpyDeviceToHost, b.s) != hipSuccess ||
            hipMemcpyAsync(all.data(), dv.gather, 16 * R, hipMemcpyDeviceToHost, b.s) != hipSuccess ||
            hipStreamSynchronize(b.s) != hipSuccess)
            rc = set_error(FLRL_E_HIP, "flrl_fl_compress_rank: size read-back failed");
    }
    if (rc == FLRL_OK)
        rc = read_error(b, (size_t)c->rank);  // (a failed peer's slot raised FLRL_E_ARG here)
    // rank 0's merge buffer before the all-reduce, so its failure is reported in it
    uint8_t *d_all = nullptr;
    const uint64_t F = rec[FLRL_SZ_F_TOTAL], V = rec[FLRL_SZ_V_TOTAL];
    if (rc == FLRL_OK && c->rank == 0) {
        (void)hipSetDevice(dv.id);
        if (hipMalloc(&d_all, (F + V) ? F + V : 16) != hipSuccess) {
            d_all = nullptr;
            rc = set_error(FLRL_E_NOMEM, "Cannot allocate memory (device)");
        }
    }
    // (2) {whole input size (the reference all-gathers inputSize, fl_gpu.cu:105),
    // ranks that failed}, summed over the ranks on the comm's own buffer/stream.
    // The word is written by a kernel (its arguments travel with the launch, no
    // pageable copy); a rank that cannot stage it sends the comm's constant
    // {0, 1} instead (Dev::red + 6), so it is counted as failed either way.
    uint64_t total_n = 0, failed = 1;
    bool reduced = false;  // the all-reduce ran and its result was read back
    if (!rcl_broken) {
        std::lock_guard<std::mutex> g(c->mu);
        (void)hipSetDevice(dv.id);
        bool mine = !debug_fail_rank_step(FLRL_DEBUG_RANK_STAGE_WORD) &&
                    hipStreamWaitEvent(dv.cstream, dv.cdone, 0) == hipSuccess;
        if (mine) {
            hipLaunchKernelGGL(put_pair_kernel, dim3(1), dim3(kWave), 0, dv.cstream, dv.red, (uint64_t)size,
                               rc == FLRL_OK ? 0ull : 1ull);
            mine = hipGetLastError() == hipSuccess;
        }
        if (!mine && rc == FLRL_OK)
            rc = set_error(FLRL_E_HIP, "flrl_fl_compress_rank: staging {size, failed} failed");
        uint64_t sum[2] = {0, 1};
        const ncclResult_t r1 = ncclAllReduce(mine ? dv.red : dv.red + 6, dv.red + 2, 2, ncclUint64, ncclSum,
                                              dv.nccl, dv.cstream);
        if (r1 != ncclSuccess) {
            if (rc == FLRL_OK)
                rc = rccl_error(r1, "ncclAllReduce");
        } else if (debug_fail_rank_step(FLRL_DEBUG_RANK_READ_SUM) ||
                   hipMemcpyAsync(sum, dv.red + 2, sizeof(sum), hipMemcpyDeviceToHost, dv.cstream) != hipSuccess ||
                   hipStreamSynchronize(dv.cstream) != hipSuccess) {
            // the reduce completed on every rank, but this device cannot hand its
            // result to the host: a device failure in the middle of the call. The
            // peers decide (3) from the same sum; this rank cannot, so it leaves
            // here -- if no rank had failed, the peers' (3) then fails or waits
            // on this rank as any collective does on a dead device (RCCL).
            if (rc == FLRL_OK)
                rc = set_error(FLRL_E_HIP, "flrl_fl_compress_rank: size read-back failed");
        } else {
            reduced = true;
        }
        total_n = sum[0];
        failed = sum[1];
        if (reduced && rc == FLRL_OK && failed)
            rc = set_error(FLRL_E_ARG, "flrl_fl_compress_rank: %llu rank(s) failed", (unsigned long long)failed);
    }
    // (3) the payloads to rank 0 (the reference's rank-0 merge, fl_gpu.cu:144-238,
    // without padding or broadcasting them to every rank), gated on the
    // all-reduced count alone: every rank that reads failed == 0 contributed 0,
    // i.e. had succeeded so far, so all ranks take this branch or none
    if (reduced && failed == 0 && !rcl_broken) {
        std::lock_guard<std::mutex> g(c->mu);
        ncclComm_t nc = dv.nccl;
        ncclResult_t r1 = ncclGroupStart();
        if (c->rank == 0) {
            for (size_t q = 0; q < R && r1 == ncclSuccess; ++q) {
                // rank q's payload goes to its exchanged offsets (the same
                // record the device scan gave rank q)
                uint64_t qr[FLRL_SZ_COUNT];
                (void)shard_record(all.data(), (uint32_t)R, (uint32_t)R, 1, (uint32_t)q, qr);
                const uint64_t fq = qr[FLRL_SZ_F], vq = qr[FLRL_SZ_V];
                const uint64_t fo = qr[FLRL_SZ_F_OFF], vo = qr[FLRL_SZ_V_OFF];
                if (q == 0) {
                    if ((fq && hipMemcpyAsync(d_all, b.bits, fq, hipMemcpyDeviceToDevice, b.s) != hipSuccess) ||
                        (vq && hipMemcpyAsync(d_all + F, b.vals, vq, hipMemcpyDeviceToDevice, b.s) != hipSuccess))
                        r1 = ncclUnhandledCudaError;
                } else {
                    if (fq)
                        r1 = ncclRecv(d_all + fo, fq, ncclUint8, (int)q, nc, b.s);
                    if (r1 == ncclSuccess && vq)
                        r1 = ncclRecv(d_all + F + vo, vq, ncclUint8, (int)q, nc, b.s);
                }
            }
        } else {
            if (rec[FLRL_SZ_F])
                r1 = ncclSend(b.bits, rec[FLRL_SZ_F], ncclUint8, 0, nc, b.s);
            if (r1 == ncclSuccess && rec[FLRL_SZ_V])
                r1 = ncclSend(b.vals, rec[FLRL_SZ_V], ncclUint8, 0, nc, b.s);
        }
        const ncclResult_t r2 = ncclGroupEnd();
        if (r1 != ncclSuccess || r2 != ncclSuccess)
            rc = rccl_error(r1 != ncclSuccess ? r1 : r2, "flrl_fl_compress_rank: payload gather");
        else if (hipStreamSynchronize(b.s) != hipSuccess)
            rc = set_error(FLRL_E_HIP, "flrl_fl_compress_rank: stream failed");
    }
    if (rc == FLRL_OK && c->rank == 0) {
        uint8_t *h_bits = static_cast<uint8_t *>(malloc(F ? F : 1));
        uint8_t *h_vals = static_cast<uint8_t *>(malloc(V ? V : 1));
        if (!h_bits || !h_vals ||
            (F && hipMemcpy(h_bits, d_all, F, hipMemcpyDeviceToHost) != hipSuccess) ||
            (V && hipMemcpy(h_vals, d_all + F, V, hipMemcpyDeviceToHost) != hipSuccess)) {
            free(h_bits);
            free(h_vals);
            rc = set_error(FLRL_E_HIP, "flrl_fl_compress_rank: copy-out failed");
        } else {
            out->bits = h_bits;
            out->bits_size = F;
            out->values = h_vals;
            out->values_size = V;
            out->input_size = total_n;
        }
    }
    if (d_all) {
        (void)hipSetDevice(b.dev);
        (void)hipStreamSynchronize(b.s);
        (void)hipFree(d_all);
    }
    (void)hipSetDevice(prev);
    return rc;
}
