// flrl_stream.hip — FL file codec streamed through one or more GPUs.
//
// the reference CLI loads the whole file, encodes it
// with synchronous copies (fl_gpu.cu:330,393-394) and, for fl-mpi / fl-nccl,
// loads per-rank shards (file_io.cu:28-71) and gathers everything to rank 0; it
// has no multi-GPU decode (main.cu:139-147). Here a file is cut into
// frame-aligned chunks that `workers` pipelines (one host thread each, worker w
// on device w % devices) take round robin:
//   compress   pread chunk -> H2D -> flrl_fl_encode_device -> D2H bits/values,
//              two chunks in flight per worker on two streams (a chunk's D2H
//              overlaps the next chunk's read and H2D); a writer places bits at
//              24 + chunk_start/128 and values at 24 + F + (values of earlier
//              chunks) with pwrite, in chunk order, and writes the header last.
//   decompress the header, then one streamed pass over the widths gives every
//              chunk's value offset (a host prefix, 16 bytes per width unit);
//              each chunk (its widths and values read by its worker) is then
//              decoded independently and pwritten at its input offset.
// Chunks are frame-aligned, so the file is byte-identical to a whole-input
// encode (the concatenation identity). Memory is bounded
// by the chunk size (per worker: 2 x (2 chunks + chunk/128) pinned host bytes
// and as much device memory), so files larger than host RAM or HBM stream.
// Outputs are written to a temporary file next to the output and renamed into
// place on success (flrl_outfile.hpp): a failed call leaves an existing output
// untouched, and the input may be the output.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <list>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "flrl.h"
#include "flrl_internal.hpp"
#include "flrl_tuning.hpp"
#include "flrl_outfile.hpp"

namespace flrl {
namespace {

constexpr size_t kDefaultChunk = 64ull << 20;  // 64 MiB per chunk
constexpr size_t kHeader = 24;
constexpr size_t kFrame = FLRL_FRAME_LENGTH;

// First failure of any thread, re-raised on the calling thread. With a waiter
// (mutex + condition variable whose predicates test `failed`), set() wakes it:
// taking the waiters' mutex between the store and the notify means no waiter
// can have tested the predicate before the store and still be about to sleep.
// set() must not be called with the waiters' mutex held.
struct Failure {
    std::mutex m;
    std::atomic<bool> failed{false};
    int code = FLRL_OK;
    std::string msg;
    std::mutex *wait_m = nullptr;
    std::condition_variable *wait_cv = nullptr;
    void set(int c, const std::string &s)
    {
        {
            std::lock_guard<std::mutex> g(m);
            if (!failed.load()) {
                code = c;
                msg = s;
                failed.store(true);
            }
        }
        if (wait_cv) {
            { std::lock_guard<std::mutex> g(*wait_m); }
            wait_cv->notify_all();
        }
    }
};

struct Fd {
    int fd = -1;
    ~Fd()
    {
        if (fd >= 0)
            ::close(fd);
    }
};

bool pread_all(int fd, void *dst, size_t bytes, uint64_t off)
{
    uint8_t *p = static_cast<uint8_t *>(dst);
    while (bytes) {
        const ssize_t r = ::pread(fd, p, bytes, (off_t)off);
        if (r <= 0)
            return false;
        p += r;
        bytes -= (size_t)r;
        off += (uint64_t)r;
    }
    return true;
}

bool pwrite_all(int fd, const void *src, size_t bytes, uint64_t off)
{
    const uint8_t *p = static_cast<const uint8_t *>(src);
    while (bytes) {
        const ssize_t r = ::pwrite(fd, p, bytes, (off_t)off);
        if (r <= 0)
            return false;
        p += r;
        bytes -= (size_t)r;
        off += (uint64_t)r;
    }
    return true;
}

size_t requested_or(size_t requested) { return requested ? requested : kDefaultChunk; }

size_t chunk_size(size_t requested)
{
    size_t c = requested ? requested : kDefaultChunk;
    c -= c % kFrame;
    return c ? c : kFrame;
}

int worker_count(int workers, int *ndev)
{
    *ndev = 0;
    if (hipGetDeviceCount(ndev) != hipSuccess || *ndev <= 0)
        return 0;
    return workers > 0 ? workers : *ndev;
}

// Pipelines actually started: min(W, units), at least 1 (size_t: the unit
// count of a huge file with a small chunk can exceed INT_MAX).
int pipelines(int W, size_t units)
{
    const size_t u = units ? units : 1;
    return (size_t)W < u ? W : (int)u;
}

// Per-worker buffers: two slots, each with its stream, pinned host staging and
// device buffers.
struct Slot {
    hipStream_t s = nullptr;
    uint8_t *h_a = nullptr, *h_b = nullptr, *h_c = nullptr;  // pinned
    uint64_t *h_u64 = nullptr;                               // pinned
    uint8_t *d_a = nullptr, *d_b = nullptr, *d_c = nullptr;
    uint64_t *d_u64 = nullptr;
    void *d_scr = nullptr;
    size_t scr_bytes = 0;
};

struct Slots {
    Slot slot[2];
    int dev = -1;  // owning device (set before alloc when freed from another thread)
    ~Slots()
    {
        if (dev >= 0)
            (void)hipSetDevice(dev);
        for (Slot &x : slot) {
            if (x.s)
                (void)hipStreamSynchronize(x.s);
            (void)hipHostFree(x.h_a);
            (void)hipHostFree(x.h_b);
            (void)hipHostFree(x.h_c);
            (void)hipHostFree(x.h_u64);
            (void)hipFree(x.d_a);
            (void)hipFree(x.d_b);
            (void)hipFree(x.d_c);
            (void)hipFree(x.d_u64);
            (void)hipFree(x.d_scr);
            if (x.s)
                (void)hipStreamDestroy(x.s);
        }
    }
    // a, b, c: byte capacities of the three buffer pairs
    hipError_t alloc(size_t a, size_t b, size_t c, size_t scr)
    {
        for (Slot &x : slot) {
            hipError_t e;
            if ((e = hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking)) != hipSuccess ||
                (e = hipHostMalloc((void **)&x.h_a, a ? a : 16, 0)) != hipSuccess ||
                (e = hipHostMalloc((void **)&x.h_b, b ? b : 16, 0)) != hipSuccess ||
                (e = hipHostMalloc((void **)&x.h_c, c ? c : 16, 0)) != hipSuccess ||
                (e = hipHostMalloc((void **)&x.h_u64, 16, 0)) != hipSuccess ||
                (e = hipMalloc(&x.d_a, a ? a : 16)) != hipSuccess ||
                (e = hipMalloc(&x.d_b, b ? b : 16)) != hipSuccess ||
                (e = hipMalloc(&x.d_c, c ? c : 16)) != hipSuccess ||
                (e = hipMalloc(&x.d_u64, 16)) != hipSuccess || (e = hipMalloc(&x.d_scr, scr)) != hipSuccess)
                return e;
            x.scr_bytes = scr;
        }
        return hipSuccess;
    }
};

// Hand-off of finished compress chunks to the in-order writer.
struct Ready {
    bool done = false;
    const uint8_t *bits = nullptr, *values = nullptr;
    size_t nbits = 0, nvalues = 0;
    std::atomic<bool> *released = nullptr;  // set by the writer once written
};

// The in-order writer has stopped (done, or after a failure): every chunk
// handed over but not written is released, and chunks finished later are not
// handed over, so no worker waits for a writer that is gone.
void release_unwritten(std::mutex &m, std::condition_variable &cv, std::vector<Ready> &ready,
                       bool &writer_stopped)
{
    {
        std::lock_guard<std::mutex> g(m);
        writer_stopped = true;
        for (Ready &r : ready)
            if (r.done && r.released)
                r.released->store(true);
    }
    cv.notify_all();
}

}  // namespace
}  // namespace flrl

using namespace flrl;

namespace flrl {
namespace {

// ---- FL pipelines over any source / sink -----------------------------------
// Byte sources and sinks of the FL pipelines. Compress reads the raw input and
// writes the container's two arrays; decompress reads the container's arrays
// and writes the raw output. File forms use pread/pwrite (container at its
// on-disk offsets), memory forms memcpy (the flrl_fl_compress/_decompress host
// API). Every call is made by a worker thread on a disjoint range.
// `direct` (memory forms only): the pipelines copy between the caller's
// pageable memory and HBM with hipMemcpyAsync instead of memcpy through the
// pinned staging; ptr()/wptr() give the addresses.
struct FdRaw {  // raw bytes of a file
    int fd;
    bool direct = false;
    const uint8_t *ptr(uint64_t) const { return nullptr; }
    uint8_t *wptr(uint64_t) const { return nullptr; }
    bool read(void *d, size_t len, uint64_t off) { return pread_all(fd, d, len, off); }
    bool write(const void *p, size_t len, uint64_t off) { return pwrite_all(fd, p, len, off); }
};
struct MemRawIn {
    const uint8_t *p;
    bool direct = false;
    const uint8_t *ptr(uint64_t off) const { return p + off; }
    bool read(void *d, size_t len, uint64_t off)
    {
        memcpy(d, p + off, len);
        return true;
    }
};
struct MemRawOut {
    uint8_t *p;
    bool direct = false;
    uint8_t *wptr(uint64_t off) const { return p + off; }
    bool write(const void *q, size_t len, uint64_t off)
    {
        memcpy(p + off, q, len);
        return true;
    }
};
struct FdFl {  // FL container file: u64 header[3] | bits[F] | values[V]
    int fd;
    uint64_t F;
    bool direct = false;
    const uint8_t *bits_ptr(uint64_t) const { return nullptr; }
    const uint8_t *values_ptr(uint64_t) const { return nullptr; }
    uint8_t *bits_wptr(uint64_t) const { return nullptr; }
    uint8_t *values_wptr(uint64_t) const { return nullptr; }
    bool read_bits(void *d, size_t len, uint64_t f) { return pread_all(fd, d, len, kHeader + f); }
    bool read_values(void *d, size_t len, uint64_t v) { return pread_all(fd, d, len, kHeader + F + v); }
    bool write_bits(const void *q, size_t len, uint64_t f) { return pwrite_all(fd, q, len, kHeader + f); }
    bool write_values(const void *q, size_t len, uint64_t v) { return pwrite_all(fd, q, len, kHeader + F + v); }
};
struct MemFl {  // FL arrays in host memory
    const uint8_t *rbits = nullptr, *rvalues = nullptr;
    uint8_t *wbits = nullptr, *wvalues = nullptr;
    bool direct = false;
    const uint8_t *bits_ptr(uint64_t f) const { return rbits + f; }
    const uint8_t *values_ptr(uint64_t v) const { return rvalues + v; }
    uint8_t *bits_wptr(uint64_t f) const { return wbits + f; }
    uint8_t *values_wptr(uint64_t v) const { return wvalues + v; }
    bool read_bits(void *d, size_t len, uint64_t f)
    {
        memcpy(d, rbits + f, len);
        return true;
    }
    bool read_values(void *d, size_t len, uint64_t v)
    {
        memcpy(d, rvalues + v, len);
        return true;
    }
    bool write_bits(const void *q, size_t len, uint64_t f)
    {
        memcpy(wbits + f, q, len);
        return true;
    }
    bool write_values(const void *q, size_t len, uint64_t v)
    {
        memcpy(wvalues + v, q, len);
        return true;
    }
};

// Pinned staging + device buffers of one pipeline, kept across calls: a
// pipeline's hipHostMalloc/hipMalloc of 2 x ~2 chunks costs more than a
// 16 MiB chunk's transfer. Idle sets wait in one pool, most recently used
// last; past kPoolBytes of idle pinned memory the least recently used sets are
// freed (a set holds as much HBM as pinned memory), and flrl_release_staging
// frees every idle set. The host-buffer API's 8 pipelines of 16 MiB chunks
// hold 8 x 2 x (16 MiB + 128 KiB + 16 MiB + 16) ~ 514 MiB of pinned memory per
// direction (compress, decompress); the cap keeps both directions' sets (plus
// slack), so alternating compress and decompress never reallocates. The file
// APIs take workers and chunk sizes at run time, so the cap also grows to
// twice the most pinned memory ever leased at once (both directions of the
// largest call shape seen): more or larger pipelines than the host API's do
// not re-allocate on every call either. That growth is bounded
// (ADVICE r05): it follows the most leased at once in the current and the last
// kPoolEpochs busy periods (a busy period ends when no set is leased), so one
// large call's pinned memory leaves the idle pool after a few smaller calls,
// and it never exceeds an eighth of the host's physical memory.
constexpr size_t kHostSetBound = 2 * (2 * (size_t)FLRL_HOST_CHUNK + (size_t)FLRL_HOST_CHUNK / 128 + 16);
constexpr size_t kPoolBytes = 2 * (size_t)FLRL_HOST_WORKERS * kHostSetBound + (64ull << 20);
constexpr int kPoolEpochs = 4;
size_t g_leased_bytes = 0;                 // pinned bytes of the sets leased right now
size_t g_epoch_peak = 0;                   // the most leased at once in the current busy period
size_t g_epoch_peaks[kPoolEpochs] = {0};   // ... in the last kPoolEpochs busy periods
int g_epoch_i = 0;
size_t pool_ceiling()
{
    static const size_t c = [] {
        const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGESIZE);
        return pages > 0 && psz > 0 ? (size_t)pages * (size_t)psz / 8 : kPoolBytes;
    }();
    return std::max(kPoolBytes, c);
}
size_t pool_cap()
{
    size_t peak = g_epoch_peak;
    for (size_t p : g_epoch_peaks)
        peak = std::max(peak, p);
    return std::min(pool_ceiling(), std::max(kPoolBytes, 2 * peak + ((size_t)64 << 20)));
}
struct PoolKey {
    int dev;
    size_t a, b, c, scr;
    bool operator==(const PoolKey &o) const
    {
        return dev == o.dev && a == o.a && b == o.b && c == o.c && scr == o.scr;
    }
    size_t pinned() const { return 2 * (a + b + c + 16); }
};
struct PoolEntry {
    PoolKey key;
    Slots *x;
};
std::mutex g_pool_m;
std::list<PoolEntry> g_pool;  // idle sets, least recently used first
size_t g_pool_bytes = 0;      // their pinned bytes

// Frees `v`'s sets and restores the calling thread's device.
void free_sets(std::vector<Slots *> &v)
{
    if (v.empty())
        return;
    int prev = 0;
    const bool had = hipGetDevice(&prev) == hipSuccess;
    for (Slots *x : v)
        delete x;
    if (had)
        (void)hipSetDevice(prev);
    v.clear();
}

Slots *slots_acquire(int dev, size_t a, size_t b, size_t c, size_t scr)
{
    const PoolKey k{dev, a, b, c, scr};
    {
        std::lock_guard<std::mutex> g(g_pool_m);
        g_leased_bytes += k.pinned();  // (given back by slots_release, also for a failed lease)
        g_epoch_peak = std::max(g_epoch_peak, g_leased_bytes);
        for (auto it = g_pool.rbegin(); it != g_pool.rend(); ++it)
            if (it->key == k) {
                Slots *x = it->x;
                g_pool_bytes -= k.pinned();
                g_pool.erase(std::next(it).base());
                return x;
            }
    }
    Slots *x = new Slots;
    x->dev = dev;
    if (x->alloc(a, b, c, scr) != hipSuccess) {
        delete x;
        // an allocation can fail because idle sets hold the memory: free them, retry once
        if (flrl_release_staging() == 0)
            return nullptr;
        x = new Slots;
        x->dev = dev;
        if (x->alloc(a, b, c, scr) != hipSuccess) {
            delete x;
            return nullptr;
        }
    }
    return x;
}

void slots_release(Slots *x, size_t a, size_t b, size_t c, size_t scr)
{
    {
        std::lock_guard<std::mutex> g(g_pool_m);
        g_leased_bytes -= PoolKey{0, a, b, c, scr}.pinned();
        if (g_leased_bytes == 0) {  // a busy period ends
            g_epoch_peaks[g_epoch_i] = g_epoch_peak;
            g_epoch_i = (g_epoch_i + 1) % kPoolEpochs;
            g_epoch_peak = 0;
        }
    }
    if (!x)
        return;
    for (Slot &y : x->slot)  // idle: nothing of a previous call still in flight
        (void)hipStreamSynchronize(y.s);
    std::vector<Slots *> evict;
    {
        std::lock_guard<std::mutex> g(g_pool_m);
        const PoolKey k{x->dev, a, b, c, scr};
        g_pool.push_back(PoolEntry{k, x});
        g_pool_bytes += k.pinned();
        while (g_pool_bytes > pool_cap() && !g_pool.empty()) {
            g_pool_bytes -= g_pool.front().key.pinned();
            evict.push_back(g_pool.front().x);
            g_pool.pop_front();
        }
    }
    free_sets(evict);
}

}  // namespace
}  // namespace flrl

extern "C" size_t flrl_release_staging(void)
{
    using namespace flrl;
    std::vector<Slots *> v;
    size_t freed = 0;
    {
        std::lock_guard<std::mutex> g(g_pool_m);
        for (PoolEntry &e : g_pool) {
            freed += e.key.pinned();
            v.push_back(e.x);
        }
        g_pool.clear();
        g_pool_bytes = 0;
    }
    free_sets(v);
    return freed;
}

namespace flrl {
namespace {

struct SlotsLease {
    Slots *x = nullptr;
    size_t a = 0, b = 0, c = 0, scr = 0;
    SlotsLease(int dev, size_t a_, size_t b_, size_t c_, size_t s_) : a(a_), b(b_), c(c_), scr(s_)
    {
        x = slots_acquire(dev, a, b, c, scr);
    }
    ~SlotsLease() { slots_release(x, a, b, c, scr); }
};

// FL compress of n bytes from `src` into `dst`, frame-aligned chunks through
// W pipelines (pipeline w on devs[w % devs.size()], two chunks in flight).
// Bits land at frame c*chunk/128; a chunk's values at the sum of the earlier
// chunks' sizes, which each pipeline learns from the chunk before its own (a
// chain of u64s, no writer thread): every pipeline writes its own bytes, so
// host copies (memcpy or pwrite) run W-wide and a pipeline's buffers are never
// read by another thread. *V_total = valuesSize.
// FLRL_HOST_PROFILE (tuning builds): per-phase wall time of the compress
// pipelines summed over workers, printed to stderr per call.
#if FLRL_HOST_PROFILE
static inline uint64_t prof_now()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}
struct HostProf {
    std::atomic<uint64_t> ns[8];
    const char *name[8] = {"read", "submit", "wait", "offsets", "write", "lease", "worker_wall", "thread_start"};
    uint64_t t0 = prof_now();
    HostProf() { for (auto &x : ns) x = 0; }
    ~HostProf()
    {
        fprintf(stderr, "[host-prof] core_wall %.1f ms", (prof_now() - t0) * 1e-6);
        for (int i = 0; i < 8; ++i)
            fprintf(stderr, " %s %.1f ms", name[i], ns[i].load() * 1e-6);
        fprintf(stderr, "\n");
    }
};
#define PROF_T(v) const uint64_t v = prof_now()
#define PROF_ADD(k, t0) prof.ns[k] += prof_now() - (t0)
#else
#define PROF_T(v) ((void)0)
#define PROF_ADD(k, t0) ((void)0)
#endif

template <class Src, class Dst>
int fl_compress_core(Src &src, Dst &dst, uint64_t n, const std::vector<int> &devs, int W, size_t chunk,
                     uint64_t *V_total, const char *who)
{
#if FLRL_HOST_PROFILE
    HostProf prof;
#endif
    const size_t cf = chunk / kFrame;
    const size_t nchunks = n ? (size_t)((n + chunk - 1) / chunk) : 0;
    *V_total = 0;
    if (!nchunks)
        return FLRL_OK;
    Failure fail;
    std::mutex m;
    std::condition_variable cv;
    fail.wait_m = &m;
    fail.wait_cv = &cv;
    std::vector<uint64_t> voff(nchunks + 1, 0);
    std::vector<char> known(nchunks + 1, 0);  // under m
    known[0] = 1;
    const int nw = pipelines(W, nchunks);
    const size_t scr_b = flrl_fl_scratch_bytes(chunk), vcap = flrl_fl_values_capacity(chunk);

    auto worker = [&](int w) {
#if FLRL_HOST_PROFILE
        const uint64_t tw0 = prof_now();
        prof.ns[7] += tw0 - prof.t0;
        struct WallEnd {
            HostProf &p;
            uint64_t t;
            ~WallEnd() { p.ns[6] += prof_now() - t; }
        } wall_end{prof, tw0};
#endif
        const int dev = devs[(size_t)w % devs.size()];
        if (hipSetDevice(dev) != hipSuccess) {
            fail.set(FLRL_E_HIP, "hipSetDevice failed");
            return;
        }
        PROF_T(tl);
        SlotsLease lease(dev, chunk, cf, vcap, scr_b);
        PROF_ADD(5, tl);
        if (!lease.x) {
            fail.set(FLRL_E_NOMEM, "Cannot allocate memory (pinned staging)");
            return;
        }
        Slots &S = *lease.x;
        auto finish = [&](size_t c, int k) -> bool {  // chunk c in slot k: check, place
            Slot &x = S.slot[k];
            PROF_T(tw);
            if (hipStreamSynchronize(x.s) != hipSuccess) {
                fail.set(FLRL_E_HIP, "fl encode: stream failed");
                return false;
            }
            const int kerr = flrl_scratch_error(x.d_scr, x.s);
            if (kerr) {
                fail.set(kerr, "fl encode: device error");
                return false;
            }
            const uint64_t len = (c + 1 == nchunks) ? n - (uint64_t)c * chunk : chunk;
            const size_t fb = (size_t)((len + kFrame - 1) / kFrame);
            const size_t vb = (size_t)x.h_u64[0];
            if (vb > vcap) {
                fail.set(FLRL_E_HIP, "fl encode: values size out of range");
                return false;
            }
            if (!dst.direct && hipMemcpyAsync(x.h_c, x.d_c, vb, hipMemcpyDeviceToHost, x.s) != hipSuccess) {
                fail.set(FLRL_E_HIP, "fl encode: copy-out failed");
                return false;
            }
            PROF_ADD(2, tw);
            PROF_T(to);
            uint64_t vo;
            {  // this chunk's values offset, then the next chunk's
                std::unique_lock<std::mutex> g(m);
                cv.wait(g, [&] { return known[c] || fail.failed.load(); });
                if (!known[c])
                    return false;
                vo = voff[c];
                voff[c + 1] = vo + vb;
                known[c + 1] = 1;
            }
            cv.notify_all();
            if (dst.direct) {
                if ((vb && hipMemcpyAsync(dst.values_wptr(vo), x.d_c, vb, hipMemcpyDeviceToHost, x.s) != hipSuccess) ||
                    hipStreamSynchronize(x.s) != hipSuccess) {
                    fail.set(FLRL_E_HIP, "fl encode: copy-out failed");
                    return false;
                }
                return true;
            }
            if (hipStreamSynchronize(x.s) != hipSuccess) {
                fail.set(FLRL_E_HIP, "fl encode: copy-out failed");
                return false;
            }
            PROF_ADD(3, to);
            PROF_T(tr);
            if (!dst.write_bits(x.h_b, fb, (uint64_t)c * cf) || !dst.write_values(x.h_c, vb, vo)) {
                fail.set(FLRL_E_ARG, "[FileIO] Cannot write to file");
                return false;
            }
            PROF_ADD(4, tr);
            return true;
        };
        size_t pend = SIZE_MAX;  // chunk in flight in slot pend_k
        int pend_k = 0;
        int i = 0;
        for (size_t c = (size_t)w; c < nchunks && !fail.failed.load(); c += (size_t)nw, ++i) {
            const int k = i & 1;  // slot k last held chunk c - 2*nw, finished an iteration ago
            Slot &x = S.slot[k];
            const uint64_t off = (uint64_t)c * chunk;
            const size_t len = (size_t)((c + 1 == nchunks) ? n - off : chunk);
            const size_t fb = (len + kFrame - 1) / kFrame;
            if (debug_fail_chunk(c)) {
                fail.set(FLRL_E_HIP, "injected failure (flrl_debug_fail_chunk)");
                break;
            }
            PROF_T(trd);
            if (!src.direct && !src.read(x.h_a, len, off)) {
                fail.set(FLRL_E_ARG, "[FileIO] Cannot read file content");
                break;
            }
            PROF_ADD(0, trd);
            PROF_T(ts);
            uint8_t *bits_to = dst.direct ? dst.bits_wptr((uint64_t)c * cf) : x.h_b;
            if (hipMemcpyAsync(x.d_a, src.direct ? src.ptr(off) : x.h_a, len, hipMemcpyHostToDevice, x.s) != hipSuccess ||
                flrl_fl_encode_device(x.d_a, len, x.d_b, x.d_c, x.d_u64, x.d_scr, x.scr_bytes, x.s) != FLRL_OK ||
                hipMemcpyAsync(x.h_u64, x.d_u64, 8, hipMemcpyDeviceToHost, x.s) != hipSuccess ||
                hipMemcpyAsync(bits_to, x.d_b, fb, hipMemcpyDeviceToHost, x.s) != hipSuccess) {
                fail.set(FLRL_E_HIP, std::string("fl encode: ") + flrl_last_error());
                break;
            }
            PROF_ADD(1, ts);
            if (pend != SIZE_MAX && !finish(pend, pend_k))
                break;
            pend = c;
            pend_k = k;
        }
        if (!fail.failed.load() && pend != SIZE_MAX)
            (void)finish(pend, pend_k);
    };
    std::vector<std::thread> threads;
    for (int w = 0; w < nw; ++w)
        threads.emplace_back(worker, w);
    for (auto &t : threads)
        t.join();
    if (fail.failed.load())
        return set_error(fail.code ? fail.code : FLRL_E_HIP, "%s: %s", who, fail.msg.c_str());
    *V_total = voff[nchunks];
    return FLRL_OK;
}

// Value offset of every chunk (16 x the widths of all earlier frames) in one
// pass over the widths, 4 MiB at a time, validating them (1..8) and the
// values size they imply. voff has nchunks + 1 entries.
template <class Src>
int fl_chunk_offsets(Src &src, uint64_t n, uint64_t F, uint64_t V, size_t chunk, std::vector<uint64_t> &voff)
{
    const size_t cf = chunk / kFrame;
    const size_t nchunks = (size_t)((n + chunk - 1) / chunk);
    voff.assign(nchunks + 1, 0);
    std::vector<uint8_t> win(4u << 20);
    uint64_t acc = 0;  // width units before the current window's chunk
    uint8_t last_w = 0;
    for (size_t c = 0; c < nchunks; ++c) {
        voff[c] = 16 * acc;
        const uint64_t f0 = (uint64_t)c * cf, f1 = f0 + cf < F ? f0 + cf : F;
        for (uint64_t f = f0; f < f1;) {
            const size_t k = (size_t)(f1 - f < win.size() ? f1 - f : win.size());
            if (!src.read_bits(win.data(), k, f))
                return set_error(FLRL_E_ARG, "[FileIO] Cannot read file content");
            uint32_t bad = 0;
            uint64_t s = 0;
            for (size_t i = 0; i < k; ++i) {  // vectorised: sum and range check
                const uint8_t b = win[i];
                bad |= (uint8_t)(b - 1) > 7u;
                s += b;
            }
            if (bad) {
                for (size_t i = 0; i < k; ++i)
                    if ((uint8_t)(win[i] - 1) > 7u)
                        return set_error(FLRL_E_FORMAT, "frame %llu has width %u (must be 1..8)",
                                         (unsigned long long)(f + i), (unsigned)win[i]);
            }
            acc += s;
            last_w = win[k - 1];
            f += k;
        }
    }
    // the last frame holds cnt_last bytes: (cnt_last * b + 7) / 8 of its 16 b
    const uint64_t cnt_last = n - (F - 1) * kFrame;
    const uint64_t expect = 16 * (acc - last_w) + (cnt_last * last_w + 7) / 8;
    if (expect != V)
        return set_error(FLRL_E_FORMAT, "valuesSize %llu != %llu implied by the widths",
                         (unsigned long long)V, (unsigned long long)expect);
    voff[nchunks] = V;
    return FLRL_OK;
}

// FL decompress of n bytes: each chunk's widths and values read by its
// pipeline, decoded, written at its output offset.
template <class Src, class Dst>
int fl_decompress_core(Src &src, Dst &dst, uint64_t n, uint64_t F, uint64_t V, const std::vector<int> &devs,
                       int W, size_t chunk, const char *who)
{
    const size_t cf = chunk / kFrame;
    const size_t nchunks = (size_t)((n + chunk - 1) / chunk);
    std::vector<uint64_t> voff;
    int rc = fl_chunk_offsets(src, n, F, V, chunk, voff);
    if (rc)
        return rc;
    Failure fail;
    const int nw = pipelines(W, nchunks);
    const size_t vcap = flrl_fl_values_capacity(chunk), scr_b = flrl_fl_scratch_bytes(chunk);
    auto worker = [&](int w) {
        const int dev = devs[(size_t)w % devs.size()];
        if (hipSetDevice(dev) != hipSuccess) {
            fail.set(FLRL_E_HIP, "hipSetDevice failed");
            return;
        }
        SlotsLease lease(dev, cf, vcap, chunk, scr_b);
        if (!lease.x) {
            fail.set(FLRL_E_NOMEM, "Cannot allocate memory (pinned staging)");
            return;
        }
        Slots &S = *lease.x;
        auto finish = [&](size_t c, int k) -> bool {  // wait, check, write chunk c
            Slot &x = S.slot[k];
            if (hipStreamSynchronize(x.s) != hipSuccess) {
                fail.set(FLRL_E_HIP, "fl decode: stream failed");
                return false;
            }
            const int kerr = flrl_scratch_error(x.d_scr, x.s);
            if (kerr) {
                fail.set(kerr, "fl decode: malformed data (widths or valuesSize)");
                return false;
            }
            const uint64_t off = (uint64_t)c * chunk;
            const size_t len = (size_t)((c + 1 == nchunks) ? n - off : chunk);
            if (!dst.direct && !dst.write(x.h_c, len, off)) {
                fail.set(FLRL_E_ARG, "[FileIO] Cannot write to file");
                return false;
            }
            return true;
        };
        size_t pend = SIZE_MAX;
        int pend_k = 0;
        int i = 0;
        for (size_t c = (size_t)w; c < nchunks && !fail.failed.load(); c += (size_t)nw, ++i) {
            const int k = i & 1;
            Slot &x = S.slot[k];
            // slot k last held chunk c - 2*nw, finished (written) in the previous iteration
            const uint64_t off = (uint64_t)c * chunk;
            const size_t len = (size_t)((c + 1 == nchunks) ? n - off : chunk);
            const size_t fb = (len + kFrame - 1) / kFrame;
            const uint64_t vo = voff[c], vb = voff[c + 1] - voff[c];
            if (vb > vcap || voff[c + 1] < voff[c]) {
                fail.set(FLRL_E_FORMAT, "valuesSize larger than the widths imply");
                break;
            }
            if (debug_fail_chunk(c)) {
                fail.set(FLRL_E_HIP, "injected failure (flrl_debug_fail_chunk)");
                break;
            }
            if (!src.direct &&
                (!src.read_bits(x.h_a, fb, (uint64_t)c * cf) || !src.read_values(x.h_b, (size_t)vb, vo))) {
                fail.set(FLRL_E_ARG, "[FileIO] Cannot read file content");
                break;
            }
            if (hipMemcpyAsync(x.d_a, src.direct ? src.bits_ptr((uint64_t)c * cf) : x.h_a, fb, hipMemcpyHostToDevice,
                               x.s) != hipSuccess ||
                (vb && hipMemcpyAsync(x.d_b, src.direct ? src.values_ptr(vo) : x.h_b, (size_t)vb,
                                      hipMemcpyHostToDevice, x.s) != hipSuccess) ||
                flrl_fl_decode_device(x.d_a, fb, x.d_b, (size_t)vb, x.d_c, len, x.d_scr, x.scr_bytes, x.s) !=
                    FLRL_OK ||
                hipMemcpyAsync(dst.direct ? dst.wptr(off) : x.h_c, x.d_c, len, hipMemcpyDeviceToHost, x.s) !=
                    hipSuccess) {
                fail.set(FLRL_E_HIP, std::string("fl decode: ") + flrl_last_error());
                break;
            }
            if (pend != SIZE_MAX && !finish(pend, pend_k))
                break;
            pend = c;
            pend_k = k;
        }
        if (!fail.failed.load() && pend != SIZE_MAX)
            (void)finish(pend, pend_k);
    };
    std::vector<std::thread> threads;
    for (int w = 0; w < nw; ++w)
        threads.emplace_back(worker, w);
    for (auto &t : threads)
        t.join();
    if (fail.failed.load())
        return set_error(fail.code ? fail.code : FLRL_E_HIP, "%s: %s", who, fail.msg.c_str());
    return FLRL_OK;
}

std::vector<int> all_devices(int ndev)
{
    std::vector<int> d((size_t)ndev);
    for (int i = 0; i < ndev; ++i)
        d[(size_t)i] = i;
    return d;
}

}  // namespace

// Host-buffer FL (flrl_fl_compress / flrl_fl_decompress, flrl_fl.hip): the
// same pipelines memory to memory on the current device, kHostWorkers wide.
// Measured on 2 GiB u8 (scripts/bench_stream.py --mem-only over variant
// builds of the FLRL_HOST_* knobs, flrl_tuning.hpp): the first touch of the freshly malloc'd output pages bounds the call
// (~10 GB/s single-threaded), not PCIe (57 GB/s each way); huge pages for the
// outputs roughly double the rate; 8 pipelines x 16 MiB chunks through pinned
// staging beat direct hipMemcpyAsync from/to the pageable buffers.
constexpr int kHostWorkers = FLRL_HOST_WORKERS;
constexpr size_t kHostChunk = FLRL_HOST_CHUNK;
struct HostCfg {
    int workers = kHostWorkers;
    size_t chunk = chunk_size(kHostChunk);
    bool direct = FLRL_HOST_DIRECT != 0;
};

// malloc for a large host output, backed by transparent huge pages where the
// kernel allows (madvise before the first touch): the first touch of freshly
// mapped 4 KiB pages, not PCIe, bounds the host-buffer API otherwise.
uint8_t *host_alloc(size_t bytes)
{
    uint8_t *p = static_cast<uint8_t *>(malloc(bytes ? bytes : 1));
    if (p && bytes >= (8u << 20) && FLRL_HOST_THP) {
        const uintptr_t a = ((uintptr_t)p + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
        const uintptr_t e = ((uintptr_t)p + bytes) & ~(uintptr_t)((2u << 20) - 1);
        if (e > a)
            (void)madvise(reinterpret_cast<void *>(a), e - a, MADV_HUGEPAGE);
    }
    return p;
}

int fl_compress_host(const uint8_t *data, size_t size, flrl_fl_buf *out)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return set_error(FLRL_E_NODEV, "flrl_fl_compress: no HIP device visible");
    const size_t F = (size + kFrame - 1) / kFrame;
    uint8_t *bits = host_alloc(F);
    uint8_t *vals = host_alloc(size);  // V <= n; shrunk below
    if (!bits || !vals) {
        free(bits);
        free(vals);
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory");
    }
    const HostCfg cfg;
    MemRawIn src{data};
    src.direct = cfg.direct;
    MemFl dst;
    dst.wbits = bits;
    dst.wvalues = vals;
    dst.direct = cfg.direct;
    uint64_t V = 0;
    const int rc = fl_compress_core(src, dst, size, std::vector<int>{dev}, cfg.workers, cfg.chunk, &V,
                                    "flrl_fl_compress");
    (void)hipSetDevice(dev);
    if (rc) {
        free(bits);
        free(vals);
        return rc;
    }
    if (V < size) {
        uint8_t *v2 = static_cast<uint8_t *>(realloc(vals, V ? V : 1));
        if (v2)
            vals = v2;
    }
    out->bits = bits;
    out->bits_size = F;
    out->values = vals;
    out->values_size = V;
    out->input_size = size;
    return FLRL_OK;
}

int fl_decompress_host(size_t n, const uint8_t *bits, size_t F, const uint8_t *values, size_t V, uint8_t **out)
{
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return set_error(FLRL_E_NODEV, "flrl_fl_decompress: no HIP device visible");
    uint8_t *h = host_alloc(n);
    if (!h)
        return set_error(FLRL_E_NOMEM, "Cannot allocate memory");
    const HostCfg cfg;
    MemFl src;
    src.rbits = bits;
    src.rvalues = values;
    src.direct = cfg.direct;
    MemRawOut dst{h};
    dst.direct = cfg.direct;
    const int rc = fl_decompress_core(src, dst, n, F, V, std::vector<int>{dev}, cfg.workers, cfg.chunk,
                                      "flrl_fl_decompress");
    (void)hipSetDevice(dev);
    if (rc) {
        free(h);
        return rc;
    }
    *out = h;
    return FLRL_OK;
}

}  // namespace flrl

using namespace flrl;

extern "C" int flrl_fl_compress_file(const char *in_path, const char *out_path, int workers,
                                     size_t chunk_bytes)
{
    clear_error();
    if (!in_path || !out_path)
        return set_error(FLRL_E_ARG, "flrl_fl_compress_file: null path");
    int ndev = 0;
    const int W = worker_count(workers, &ndev);
    if (W <= 0)
        return set_error(FLRL_E_NODEV, "flrl_fl_compress_file: no HIP device");
    Fd in;
    OutFile out;
    if ((in.fd = ::open(in_path, O_RDONLY)) < 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot open file: %s", in_path);
    struct stat st;
    if (::fstat(in.fd, &st) != 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot stat file: %s", in_path);
    const uint64_t n = (uint64_t)st.st_size;
    if (!out.open(out_path, false, in.fd))
        return set_error(FLRL_E_ARG, "[FileIO] Cannot open file: %s", out_path);
    const uint64_t F = (n + kFrame - 1) / kFrame;
    FdRaw src{in.fd};
    FdFl dst{out.fd, F};
    uint64_t V = 0;
    const int prev = [] { int d = 0; (void)hipGetDevice(&d); return d; }();
    const int rc = fl_compress_core(src, dst, n, all_devices(ndev), W, chunk_size(chunk_bytes), &V,
                                    "flrl_fl_compress_file");
    (void)hipSetDevice(prev);
    if (rc)
        return rc;
    const uint64_t hdr[3] = {n, F, V};
    if (!pwrite_all(out.fd, hdr, sizeof(hdr), 0) || !out.truncate(kHeader + F + V) || !out.commit())
        return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
    return FLRL_OK;
}

extern "C" int flrl_fl_decompress_file(const char *in_path, const char *out_path, int workers,
                                       size_t chunk_bytes)
{
    clear_error();
    if (!in_path || !out_path)
        return set_error(FLRL_E_ARG, "flrl_fl_decompress_file: null path");
    int ndev = 0;
    const int W = worker_count(workers, &ndev);
    if (W <= 0)
        return set_error(FLRL_E_NODEV, "flrl_fl_decompress_file: no HIP device");
    Fd in;
    OutFile out;
    if ((in.fd = ::open(in_path, O_RDONLY)) < 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot open file: %s", in_path);
    struct stat st;
    if (::fstat(in.fd, &st) != 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot stat file: %s", in_path);
    const uint64_t fsize = (uint64_t)st.st_size;
    uint64_t hdr[3];
    if (fsize < kHeader || !pread_all(in.fd, hdr, sizeof(hdr), 0))
        return set_error(FLRL_E_FORMAT, "[FileIO] truncated FL header");
    const uint64_t n = hdr[0], F = hdr[1], V = hdr[2];
    // format hardening: header invariants before any allocation
    if (F != (n + kFrame - 1) / kFrame || F > fsize || V > fsize || kHeader + F + V != fsize)
        return set_error(FLRL_E_FORMAT,
                         "[FileIO] inconsistent FL header (inputSize %llu, bitsSize %llu, valuesSize %llu, "
                         "file %llu bytes)",
                         (unsigned long long)n, (unsigned long long)F, (unsigned long long)V,
                         (unsigned long long)fsize);
    if (!out.open(out_path, false, in.fd))
        return set_error(FLRL_E_ARG, "[FileIO] Cannot open file: %s", out_path);
    if (n == 0 || V == 0) {  // the reference's early-out: empty result (fl_cpu.cu:94-97)
        if (!out.commit())
            return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
        return FLRL_OK;
    }
    if (!out.truncate(n))
        return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
    FdFl src{in.fd, F};
    FdRaw dst{out.fd};
    const int prev = [] { int d = 0; (void)hipGetDevice(&d); return d; }();
    const int rc = fl_decompress_core(src, dst, n, F, V, all_devices(ndev), W, chunk_size(chunk_bytes),
                                      "flrl_fl_decompress_file");
    (void)hipSetDevice(prev);
    if (rc)
        return rc;
    if (!out.commit())
        return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
    return FLRL_OK;
}

// ---------------------------------------------------------------------------
// RL, file to file. Chunks are encoded independently on the GPUs; the writer
// stitches them in order: a run crossing a chunk boundary is re-split into
// 255-byte pieces from its true start (IMPLEMENTATION-PLAN.md:125-147), so the
// file equals a whole-input encode. A chunk's records split into its first run
// (which may continue the pending run of earlier chunks), the runs wholly
// inside it (written verbatim) and its last run (kept pending). Runs are
// maximal, so consecutive records with one value are pieces of one run.
// counts[] are written in place; values[] go to a side file appended at the
// end, since R (and so the values offset) is known only then.
// ---------------------------------------------------------------------------
namespace flrl {
namespace {

struct RlWriter {
    int out = -1, side = -1;
    uint64_t runs = 0;                     // records written so far
    uint8_t pend_v = 0;
    uint64_t pend_len = 0;                 // pending run (0: none)
    uint8_t fill_c[4096], fill_v[4096];
    bool put(const uint8_t *c, const uint8_t *v, size_t k)
    {
        if (!k)
            return true;
        if (!pwrite_all(out, c, k, 16 + runs) || !pwrite_all(side, v, k, runs))
            return false;
        runs += k;
        return true;
    }
    bool emit(uint8_t v, uint64_t len)  // one run of len bytes, split from its start
    {
        memset(fill_c, 255, sizeof(fill_c));
        memset(fill_v, v, sizeof(fill_v));
        uint64_t full = len / 255;
        while (full) {
            const size_t k = full < sizeof(fill_c) ? (size_t)full : sizeof(fill_c);
            if (!put(fill_c, fill_v, k))
                return false;
            full -= k;
        }
        if (len % 255) {
            const uint8_t c = (uint8_t)(len % 255);
            return put(&c, &v, 1);
        }
        return true;
    }
    bool chunk(const uint8_t *cnt, const uint8_t *val, size_t R)
    {
        if (!R)
            return true;
        size_t j1 = 1;  // records of the chunk's first run
        uint64_t l0 = cnt[0];
        while (j1 < R && val[j1] == val[0])
            l0 += cnt[j1++];
        if (j1 == R) {  // the whole chunk is one run
            if (pend_len && pend_v == val[0]) {
                pend_len += l0;
            } else {
                if (pend_len && !emit(pend_v, pend_len))
                    return false;
                pend_v = val[0];
                pend_len = l0;
            }
            return true;
        }
        size_t start = 0;
        if (pend_len && pend_v == val[0]) {
            if (!emit(pend_v, pend_len + l0))
                return false;
            start = j1;
        } else if (pend_len && !emit(pend_v, pend_len)) {
            return false;
        }
        size_t jl = R - 1;  // first record of the chunk's last run
        uint64_t ll = cnt[R - 1];
        while (jl > j1 && val[jl - 1] == val[R - 1])
            ll += cnt[--jl];
        if (!put(cnt + start, val + start, jl - start))
            return false;
        pend_v = val[R - 1];
        pend_len = ll;
        return true;
    }
};

}  // namespace
}  // namespace flrl

extern "C" int flrl_rl_compress_file(const char *in_path, const char *out_path, int workers,
                                     size_t chunk_bytes)
{
    clear_error();
    if (!in_path || !out_path)
        return set_error(FLRL_E_ARG, "flrl_rl_compress_file: null path");
    int ndev = 0;
    const int W = worker_count(workers, &ndev);
    if (W <= 0)
        return set_error(FLRL_E_NODEV, "flrl_rl_compress_file: no HIP device");
    Fd in, side;
    OutFile out;
    if ((in.fd = ::open(in_path, O_RDONLY)) < 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot open file: %s", in_path);
    struct stat st;
    if (::fstat(in.fd, &st) != 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot stat file: %s", in_path);
    const uint64_t n = (uint64_t)st.st_size;
    // values[] until R is known: an anonymous file next to the output (else in
    // $TMPDIR or /tmp). Created BEFORE the output is opened: an output in a
    // read-only directory is truncated in place at open (OutFile), so nothing
    // that can fail may come between that open and the first write
    if ((side.fd = anon_file_near(out_path)) < 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot create a temporary file for %s", out_path);
    if (!out.open(out_path, false, in.fd))
        return set_error(FLRL_E_ARG, "[FileIO] Cannot open file: %s", out_path);
    const size_t chunk = requested_or(chunk_bytes);
    const size_t nchunks = n ? (size_t)((n + chunk - 1) / chunk) : 0;

    Failure fail;
    std::mutex m;
    std::condition_variable cv;
    fail.wait_m = &m;
    fail.wait_cv = &cv;
    std::vector<Ready> ready(nchunks);
    const int nw = pipelines(W, nchunks);
    std::vector<std::atomic<bool>> slot_free((size_t)nw * 2);
    for (auto &f : slot_free)
        f.store(true);
    bool writer_stopped = false;  // under m: chunks handed over later are never read

    auto worker = [&](int w) {
        if (hipSetDevice(w % ndev) != hipSuccess) {
            fail.set(FLRL_E_HIP, "hipSetDevice failed");
            cv.notify_all();
            return;
        }
        Slots S;
        if (S.alloc(chunk, chunk, chunk, flrl_rl_scratch_bytes(chunk)) != hipSuccess) {
            fail.set(FLRL_E_NOMEM, "Cannot allocate memory");
            cv.notify_all();
            return;
        }
        auto finish = [&](size_t c, int k) -> bool {
            Slot &x = S.slot[k];
            if (hipStreamSynchronize(x.s) != hipSuccess)
                return false;
            const int kerr = flrl_scratch_error(x.d_scr, x.s);
            if (kerr) {
                fail.set(kerr, "rl encode: device error");
                return false;
            }
            const size_t R = (size_t)x.h_u64[0];
            if (hipMemcpyAsync(x.h_b, x.d_b, R, hipMemcpyDeviceToHost, x.s) != hipSuccess ||
                hipMemcpyAsync(x.h_c, x.d_c, R, hipMemcpyDeviceToHost, x.s) != hipSuccess ||
                hipStreamSynchronize(x.s) != hipSuccess)
                return false;
            std::atomic<bool> *rel = &slot_free[(size_t)w * 2 + k];
            {
                std::lock_guard<std::mutex> g(m);
                if (!writer_stopped)
                    rel->store(false);
                Ready &r = ready[c];
                r.bits = x.h_b;  // counts
                r.values = x.h_c;
                r.nbits = r.nvalues = R;
                r.released = rel;
                r.done = true;
            }
            cv.notify_all();
            return true;
        };
        size_t pend = SIZE_MAX;
        int pend_k = 0;
        int i = 0;
        for (size_t c = (size_t)w; c < nchunks && !fail.failed.load(); c += (size_t)nw, ++i) {
            const int k = i & 1;
            Slot &x = S.slot[k];
            {
                std::unique_lock<std::mutex> g(m);
                cv.wait(g, [&] { return slot_free[(size_t)w * 2 + k].load() || fail.failed.load(); });
            }
            if (fail.failed.load())
                break;
            const uint64_t off = (uint64_t)c * chunk;
            const size_t len = (size_t)((c + 1 == nchunks) ? n - off : chunk);
            if (debug_fail_chunk(c)) {
                fail.set(FLRL_E_HIP, "injected failure (flrl_debug_fail_chunk)");
                break;
            }
            if (!pread_all(in.fd, x.h_a, len, off)) {
                fail.set(FLRL_E_ARG, "[FileIO] Cannot read file content");
                break;
            }
            if (hipMemcpyAsync(x.d_a, x.h_a, len, hipMemcpyHostToDevice, x.s) != hipSuccess ||
                flrl_rl_encode_device(x.d_a, len, x.d_b, x.d_c, x.d_u64, x.d_scr, x.scr_bytes, x.s) != FLRL_OK ||
                hipMemcpyAsync(x.h_u64, x.d_u64, 8, hipMemcpyDeviceToHost, x.s) != hipSuccess) {
                fail.set(FLRL_E_HIP, std::string("rl encode: ") + flrl_last_error());
                break;
            }
            if (pend != SIZE_MAX && !finish(pend, pend_k)) {
                fail.set(FLRL_E_HIP, "rl encode: stream failed");
                break;
            }
            pend = c;
            pend_k = k;
        }
        if (!fail.failed.load() && pend != SIZE_MAX && !finish(pend, pend_k))
            fail.set(FLRL_E_HIP, "rl encode: stream failed");
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return slot_free[(size_t)w * 2].load() && slot_free[(size_t)w * 2 + 1].load(); });
    };
    std::vector<std::thread> threads;
    for (int w = 0; w < nw && nchunks; ++w)
        threads.emplace_back(worker, w);

    RlWriter wr;
    wr.out = out.fd;
    wr.side = side.fd;
    for (size_t c = 0; c < nchunks; ++c) {
        Ready r;
        {
            std::unique_lock<std::mutex> g(m);
            cv.wait(g, [&] { return ready[c].done || fail.failed.load(); });
            if (fail.failed.load())
                break;
            r.bits = ready[c].bits;
            r.values = ready[c].values;
            r.nbits = ready[c].nbits;
            r.released = ready[c].released;
        }
        const bool ok = wr.chunk(r.bits, r.values, r.nbits);
        {
            std::lock_guard<std::mutex> g(m);
            r.released->store(true);
        }
        cv.notify_all();
        if (!ok) {
            fail.set(FLRL_E_ARG, "[FileIO] Cannot write to file");
            cv.notify_all();
            break;
        }
    }
    release_unwritten(m, cv, ready, writer_stopped);
    for (auto &t : threads)
        t.join();
    if (fail.failed.load())
        return set_error(fail.code ? fail.code : FLRL_E_HIP, "%s", fail.msg.c_str());
    if (wr.pend_len && !wr.emit(wr.pend_v, wr.pend_len))
        return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
    // header, then values[] after counts[]
    const uint64_t R = wr.runs;
    const uint64_t hdr[2] = {n, R};
    if (!pwrite_all(out.fd, hdr, sizeof(hdr), 0))
        return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
    {
        std::vector<uint8_t> buf(R < (4u << 20) ? (size_t)R + 1 : (4u << 20));
        for (uint64_t o = 0; o < R;) {
            const size_t k = (size_t)(R - o < buf.size() ? R - o : buf.size());
            if (!pread_all(side.fd, buf.data(), k, o) || !pwrite_all(out.fd, buf.data(), k, 16 + R + o))
                return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
            o += k;
        }
    }
    if (!out.truncate(16 + 2 * R) || !out.commit())
        return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
    return FLRL_OK;
}

extern "C" int flrl_rl_decompress_file(const char *in_path, const char *out_path, int workers,
                                       size_t chunk_bytes)
{
    clear_error();
    if (!in_path || !out_path)
        return set_error(FLRL_E_ARG, "flrl_rl_decompress_file: null path");
    int ndev = 0;
    const int W = worker_count(workers, &ndev);
    if (W <= 0)
        return set_error(FLRL_E_NODEV, "flrl_rl_decompress_file: no HIP device");
    Fd in;
    OutFile out;
    if ((in.fd = ::open(in_path, O_RDONLY)) < 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot open file: %s", in_path);
    struct stat st;
    if (::fstat(in.fd, &st) != 0)
        return set_error(FLRL_E_ARG, "[FileIO] Cannot stat file: %s", in_path);
    const uint64_t fsize = (uint64_t)st.st_size;
    uint64_t hdr[2];
    if (fsize < 16 || !pread_all(in.fd, hdr, sizeof(hdr), 0))
        return set_error(FLRL_E_FORMAT, "[FileIO] truncated RL header");
    const uint64_t n = hdr[0], R = hdr[1];
    if (R > fsize || 16 + 2 * R != fsize)
        return set_error(FLRL_E_FORMAT, "[FileIO] RL runs %llu do not match the file (%llu bytes)",
                         (unsigned long long)R, (unsigned long long)fsize);
    const size_t chunk = requested_or(chunk_bytes) < 256 ? 256 : requested_or(chunk_bytes);
    // blocks of runs with at most `chunk` output bytes (a run is <= 255 bytes)
    struct Block {
        uint64_t r0, r1, o0;
    };
    std::vector<Block> blocks;
    {
        std::vector<uint8_t> buf(1u << 22);
        uint64_t out_pos = 0, r0 = 0, acc = 0;
        for (uint64_t o = 0; o < R;) {
            const size_t k = (size_t)(R - o < buf.size() ? R - o : buf.size());
            if (!pread_all(in.fd, buf.data(), k, 16 + o))
                return set_error(FLRL_E_ARG, "[FileIO] Cannot read file content");
            for (size_t i = 0; i < k; ++i) {
                const uint32_t c = buf[i];
                if (c == 0)
                    return set_error(FLRL_E_FORMAT, "RL count 0 at run %llu", (unsigned long long)(o + i));
                if (acc && acc + c > chunk) {
                    blocks.push_back({r0, o + i, out_pos});
                    out_pos += acc;
                    r0 = o + i;
                    acc = 0;
                }
                acc += c;
            }
            o += k;
        }
        if (R) {
            blocks.push_back({r0, R, out_pos});
            out_pos += acc;
        }
        if (out_pos != n)
            return set_error(FLRL_E_FORMAT, "RL counts sum to %llu, header says %llu",
                             (unsigned long long)out_pos, (unsigned long long)n);
    }
    if (!out.open(out_path, false, in.fd))
        return set_error(FLRL_E_ARG, "[FileIO] Cannot open file: %s", out_path);
    if (!out.truncate(n))
        return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
    const size_t nb = blocks.size();
    Failure fail;
    const int nw = nb ? pipelines(W, nb) : 0;
    auto worker = [&](int w) {
        if (hipSetDevice(w % ndev) != hipSuccess) {
            fail.set(FLRL_E_HIP, "hipSetDevice failed");
            return;
        }
        Slots S;
        if (S.alloc(chunk, chunk, chunk, flrl_rl_decode_scratch_bytes(chunk)) != hipSuccess) {
            fail.set(FLRL_E_NOMEM, "Cannot allocate memory");
            return;
        }
        auto len_of = [&](size_t b) {
            return (size_t)((b + 1 < nb ? blocks[b + 1].o0 : n) - blocks[b].o0);
        };
        auto finish = [&](size_t b, int k) -> bool {
            Slot &x = S.slot[k];
            if (hipStreamSynchronize(x.s) != hipSuccess) {
                fail.set(FLRL_E_HIP, "rl decode: stream failed");
                return false;
            }
            const int kerr = flrl_scratch_error(x.d_scr, x.s);
            if (kerr) {
                fail.set(kerr, "rl decode: malformed counts");
                return false;
            }
            if (!pwrite_all(out.fd, x.h_c, len_of(b), blocks[b].o0)) {
                fail.set(FLRL_E_ARG, "[FileIO] Cannot write to file");
                return false;
            }
            return true;
        };
        size_t pend = SIZE_MAX;
        int pend_k = 0;
        int i = 0;
        for (size_t b = (size_t)w; b < nb && !fail.failed.load(); b += (size_t)nw, ++i) {
            const int k = i & 1;  // slot k last held block b - 2*nw, written in the previous iteration
            Slot &x = S.slot[k];
            const size_t nr = (size_t)(blocks[b].r1 - blocks[b].r0);
            const size_t len = len_of(b);
            if (debug_fail_chunk(b)) {
                fail.set(FLRL_E_HIP, "injected failure (flrl_debug_fail_chunk)");
                break;
            }
            if (!pread_all(in.fd, x.h_a, nr, 16 + blocks[b].r0) ||
                !pread_all(in.fd, x.h_b, nr, 16 + R + blocks[b].r0)) {
                fail.set(FLRL_E_ARG, "[FileIO] Cannot read file content");
                break;
            }
            if (hipMemcpyAsync(x.d_a, x.h_a, nr, hipMemcpyHostToDevice, x.s) != hipSuccess ||
                hipMemcpyAsync(x.d_b, x.h_b, nr, hipMemcpyHostToDevice, x.s) != hipSuccess ||
                flrl_rl_decode_device(x.d_a, x.d_b, nr, x.d_c, len, x.d_scr, x.scr_bytes, x.s) != FLRL_OK ||
                hipMemcpyAsync(x.h_c, x.d_c, len, hipMemcpyDeviceToHost, x.s) != hipSuccess) {
                fail.set(FLRL_E_HIP, std::string("rl decode: ") + flrl_last_error());
                break;
            }
            if (pend != SIZE_MAX && !finish(pend, pend_k))
                break;
            pend = b;
            pend_k = k;
        }
        if (!fail.failed.load() && pend != SIZE_MAX)
            (void)finish(pend, pend_k);
    };
    std::vector<std::thread> threads;
    for (int w = 0; w < nw; ++w)
        threads.emplace_back(worker, w);
    for (auto &t : threads)
        t.join();
    if (fail.failed.load())
        return set_error(fail.code ? fail.code : FLRL_E_HIP, "%s", fail.msg.c_str());
    if (!out.commit())
        return set_error(FLRL_E_ARG, "[FileIO] Cannot write to file");
    return FLRL_OK;
}
