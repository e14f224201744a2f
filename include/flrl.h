/*
 * flrl.h — C ABI of the MI355X-native fixed-length (FL) / run-length (RL) codec.
 *
 * Drop-in boundary for the reference's codec functions (namespace FixedLength in
 * Polyphemus980/fl-rl-compression-MPI). Every entry point is plain C: pointers,
 * sizes, int status codes; no HIP or torch types. Streams are passed as `void*`
 * (a hipStream_t; NULL = the default stream).
 *
 * Status codes: 0 = ok, nonzero = error (see FLRL_E_*); flrl_last_error()
 * returns the message of the calling thread's last failure. Host-buffer
 * functions are synchronous and return malloc'd buffers the caller releases
 * with free() (the reference's ownership rule: fl_cpu.cu:23,54,104 malloc,
 * main.cu:126-128,155-156,168 free). Device functions are asynchronous on the
 * given stream; their data-dependent errors (bad widths, size mismatch) land in
 * the scratch area and are read with flrl_scratch_error().
 *
 * File formats:
 *  FL (byte-identical to the reference, file_io.cu:222-280 / :117-192):
 *     u64 inputSize | u64 bitsSize | u64 valuesSize | u8 bits[bitsSize] | u8 values[valuesSize]
 *  RL (build-defined; the reference has no RL code):
 *     u64 inputSize | u64 runs | u8 counts[runs] | u8 values[runs]
 */
#ifndef FLRL_H
#define FLRL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FLRL_FRAME_LENGTH 128 /* FRAME_LENGTH, src/fl/fl_common.cuh:9 */

enum {
    FLRL_OK = 0,
    FLRL_E_ARG = 1,        /* bad argument (null pointer, capacity too small) */
    FLRL_E_HIP = 2,        /* HIP runtime error (message in flrl_last_error) */
    FLRL_E_NOMEM = 3,      /* host/device allocation failed ("Cannot allocate memory") */
    FLRL_E_FORMAT = 4,     /* malformed compressed data (width not in [1,8], size mismatch) */
    FLRL_E_TIMEOUT = 5,    /* in-kernel look-back did not complete (should never happen) */
    FLRL_E_NODEV = 6,      /* no HIP device */
    FLRL_E_RCCL = 7        /* RCCL error in the sharded path */
};

/* Mirrors FixedLength::FLCompressed, src/fl/fl_common.cuh:11-34. */
typedef struct flrl_fl_buf {
    uint8_t *bits;        /* per-frame bit width b in [1,8], bits_size = ceil(n/128) */
    size_t bits_size;
    uint8_t *values;      /* LSB-first packed values, values_size bytes */
    size_t values_size;
    size_t input_size;
} flrl_fl_buf;

/* RL analogue (build-defined). */
typedef struct flrl_rl_buf {
    uint8_t *counts;      /* run lengths, each in [1,255] */
    uint8_t *values;      /* run byte values */
    size_t runs;
    size_t input_size;
} flrl_rl_buf;

/* ---- library / errors ---------------------------------------------------- */
const char *flrl_last_error(void);       /* thread-local; "" when none */
const char *flrl_version(void);
int flrl_device_count(void);             /* number of visible HIP devices (0 if none) */

/* ---- FL, host buffers (synchronous) ---------------------------------------
 * flrl_fl_compress replaces FixedLength::gpuCompress (src/fl/fl_gpu.cuh:14,
 * fl_gpu.cu:289-423) and its CPU twin cpuCompress (src/fl/fl_cpu.cuh:9). On
 * size == 0 it returns an all-zero flrl_fl_buf (fl_gpu.cu:291-294). Runs on
 * the current device through pinned staging in 16 MiB chunks, 8 pipelines with
 * two chunks in flight each (the staging is allocated once and kept for
 * later calls), so host copies, PCIe transfers and the kernels overlap. */
int flrl_fl_compress(const uint8_t *data, size_t size, flrl_fl_buf *out);

/* The host-buffer and file paths keep their pinned staging and device buffers
 * for later calls (per device and chunk shape; after a flrl_fl_compress plus a
 * flrl_fl_decompress: ~1 GiB of pinned host memory and ~1 GiB of HBM). Idle
 * sets are capped at both directions' sets plus 64 MiB (~1.07 GiB of pinned
 * memory; least recently used freed first) and
 * freed when an allocation fails; this frees every idle set now and returns
 * the pinned bytes released (sets in use by running calls are not touched). */
size_t flrl_release_staging(void);

/* Replaces FixedLength::gpuDecompress (src/fl/fl_gpu.cuh:15, fl_gpu.cu:537-645)
 * and cpuDecompress (src/fl/fl_cpu.cuh:10). Keeps the reference's early-out: if
 * values_size == 0 || bits_size == 0 the result is empty (*out = NULL,
 * *out_size = 0; fl_cpu.cu:94-97). Unlike the reference it validates the
 * frame widths (each in [1,8]), bits_size == ceil(output_size/128) and
 * values_size == the size the widths imply, returning FLRL_E_FORMAT otherwise. */
int flrl_fl_decompress(size_t output_size, const uint8_t *bits, size_t bits_size,
                       const uint8_t *values, size_t values_size,
                       uint8_t **out, size_t *out_size);

/* Sharded encode of a host buffer in `nshards` 128-aligned shards (<= 0: one
 * per visible GPU), one process; shard r runs on device r mod ndev, ndev =
 * min(nshards, visible devices), so any shard count runs on any node.
 * Replaces FixedLength::gpuNCCLCompress (src/fl/fl_gpu.cuh:16,
 * fl_gpu.cu:76-287) and gpuMPICompress (fl_gpu.cuh:13, fl_gpu.cu:41-74) for a
 * caller holding the whole input: shards by the reference rule
 * (file_io.cu:46-51, size_t here), flrl_fl_encode_sharded on a communicator
 * cached per device count (created once per process, not per call). The result
 * is byte-identical to flrl_fl_compress. */
int flrl_fl_compress_sharded(const uint8_t *data, size_t size, int nshards, flrl_fl_buf *out);

/* ---- FL, multi-GPU: communicators and the size exchange -------------------
 * The only collective on the data path is one RCCL all-gather of {F_r, V_r}
 * (16 B per shard over xGMI) followed by an exclusive scan on the device; every
 * shard learns where its bits/values go in the whole-input output. A comm is
 * created once and reused (ncclCommInitAll/InitRank cost ~100 ms). */
typedef struct flrl_comm flrl_comm;
#define FLRL_UNIQUE_ID_BYTES 128 /* sizeof(ncclUniqueId) */

/* Per-shard sizes record (device u64[FLRL_SZ_COUNT]) the exchange writes. */
enum {
    FLRL_SZ_F = 0,       /* this shard's bitsSize  (= ceil(n_r/128)) */
    FLRL_SZ_V = 1,       /* this shard's valuesSize */
    FLRL_SZ_F_OFF = 2,   /* byte offset of its bits in the whole output */
    FLRL_SZ_V_OFF = 3,   /* byte offset of its values in the whole output */
    FLRL_SZ_F_TOTAL = 4, /* whole-input bitsSize */
    FLRL_SZ_V_TOTAL = 5, /* whole-input valuesSize */
    FLRL_SZ_COUNT = 6
};

/* One process driving `ndev` GPUs of this node (devs NULL: 0..ndev-1; ndev <= 0:
 * all visible); ncclCommInitAll. */
int flrl_comm_init(int ndev, const int *devs, flrl_comm **out);
/* One process per GPU (the reference's MPI model, main.cu:46-70): rank 0 calls
 * flrl_comm_unique_id and distributes the FLRL_UNIQUE_ID_BYTES bytes (MPI_Bcast,
 * torch.distributed, a file ...); every rank calls flrl_comm_init_rank with the
 * current HIP device set to its GPU (ncclCommInitRank). */
int flrl_comm_unique_id(void *id);
int flrl_comm_init_rank(int nranks, const void *id, int rank, flrl_comm **out);
/* Wrap an existing ncclComm_t (e.g. MpiNcclData::ncclComm, mpi_common.cuh);
 * not destroyed by flrl_comm_destroy. */
int flrl_comm_wrap(void *nccl_comm, flrl_comm **out);
int flrl_comm_destroy(flrl_comm *c);
int flrl_comm_query(const flrl_comm *c, int *nranks, int *rank, int *ndev);
/* What RCCL itself reports for the comm's local device `local` (0 for a
 * per-rank comm): ncclCommCount, ncclCommUserRank, ncclCommCuDevice and that
 * device's PCI bus id (hipDeviceGetPCIBusId, `len` bytes incl. the NUL) -- so a
 * multi-GPU run can show that RCCL saw N ranks on N distinct GPUs. Any output
 * pointer may be NULL. */
int flrl_comm_rccl_info(const flrl_comm *c, int local, int *count, int *rank, int *device,
                        char *pci_bus_id, int len);

/* Per-rank device-resident encode + exchange (per-rank comm): encodes this
 * rank's shard like flrl_fl_encode_device, then fills d_sizes
 * (u64[FLRL_SZ_COUNT], device) with its sizes, offsets and the totals, all on
 * `stream` with no host synchronisation. Every rank of the comm must call it
 * (collective). Shards of ranks 0..nranks-2 must be multiples of 128 bytes:
 * otherwise every rank's scratch error word reads FLRL_E_ARG after the
 * exchange. A rank whose arguments fail locally (null or undersized scratch,
 * misaligned buffers, the current device not the comm's) still joins the
 * exchange with a failed slot (flrl_shard_failed_word) and returns its own
 * error code; every other rank's scratch error word then reads FLRL_E_ARG
 * (instead of waiting forever in the all-gather, as gpuNCCLCompress's peers
 * would). The device half of gpuNCCLCompress (fl_gpu.cu:76-143). */
int flrl_fl_encode_rank(flrl_comm *c, const uint8_t *d_in, size_t n, uint8_t *d_bits,
                        uint8_t *d_values, uint64_t *d_sizes, void *d_scratch,
                        size_t scratch_bytes, void *stream);

/* Host-buffer per-rank twin of gpuNCCLCompress(data, size, MpiNcclData)
 * (fl_gpu.cuh:16): each rank passes its own shard (loadFileMpi, file_io.cu:28-71);
 * rank 0 receives the merged whole-input result (input_size = sum of the
 * ranks' sizes), the other ranks an empty flrl_fl_buf — the reference's rank-0
 * merge (fl_gpu.cu:196-238). Payloads travel ncclSend/ncclRecv to rank 0 only.
 * Collective on errors too: a rank that fails (allocation, upload, device
 * error, rank 0's merge buffer) still completes the exchange and an all-reduce
 * of {size, failed}, so every rank returns an error and none waits in the
 * payload send/recv.
 * ONE EXCEPTION (not collective): a device that fails between that all-reduce
 * and copying its result to the host (csrc/flrl_shard.hip, the read-back after
 * ncclAllReduce). That rank cannot learn whether the payload step runs, so it
 * returns FLRL_E_HIP without joining it; if no rank had failed before, its
 * peers then block in the payload ncclSend/ncclRecv as in any collective with
 * a dead member (RCCL's own behaviour; the job's launcher has to end the
 * ranks). A second confirmation round would only move this window, not close
 * it. */
int flrl_fl_compress_rank(flrl_comm *c, const uint8_t *data, size_t size, flrl_fl_buf *out);

/* The exchange's layout, host-callable (the device scan runs the same code,
 * csrc/flrl_shard_layout.hpp); for callers that place shards themselves and
 * for tests.
 *  flrl_shard_range: shard `shard` of `nshards` of an n-byte input by the
 *    reference rule (loadFileMpi, file_io.cu:46-51, in size_t): every shard but
 *    the last is floor(n / (128 nshards)) * 128 bytes.
 *  flrl_shard_slot: u64 index of shard's {F word, V} pair in the all-gathered
 *    array when nshards shards run on ndev devices (shard r on device r mod ndev;
 *    one process per GPU: ndev = nshards); (size_t)-1 for bad arguments.
 *  flrl_shard_size_word: the F word a shard of n bytes contributes (ceil(n/128),
 *    bit 63 set when n is not a multiple of 128).
 *  flrl_shard_failed_word: the F word (bit 62; V = 0) of a shard whose rank
 *    failed locally but still joins the exchange.
 *  flrl_shard_scan: shard's record (u64[FLRL_SZ_COUNT]) from the gathered
 *    array; FLRL_E_ARG if a shard before the last is ragged or any shard
 *    carries the failed word (the record is still written). */
int flrl_shard_range(size_t n, int nshards, int shard, size_t *start, size_t *length);
size_t flrl_shard_slot(int shard, int nshards, int ndev);
uint64_t flrl_shard_size_word(size_t n);
uint64_t flrl_shard_failed_word(void);
int flrl_shard_scan(const uint64_t *gather, int nshards, int ndev, int shard, uint64_t *rec);

/* Single-process device-resident sharded encode (flrl_comm_init comm): shard r
 * (d_in[r], n[r]; all but the last a multiple of 128 bytes, else FLRL_E_ARG)
 * with its buffers on
 * device devs[r mod ndev], encoded on streams[r]; after the call every
 * streams[r] is ordered after the exchange, and d_sizes[r] holds shard r's
 * record. At most 64 shards per device. */
int flrl_fl_encode_sharded(flrl_comm *c, int nshards, const uint8_t *const *d_in, const size_t *n,
                           uint8_t *const *d_bits, uint8_t *const *d_values,
                           uint64_t *const *d_sizes, void *const *d_scratch,
                           const size_t *scratch_bytes, void *const *streams);

/* ---- FL, file to file, streamed through GPUs ---
 * The CLI's `c|d fl` (workers = 1) and `fl-mpi` / `fl-nccl` / `fl-shmem`
 * (workers <= 0: one per visible GPU) paths; replaces main.cu:81-117 (load,
 * encode, save) and :139-161 without holding the file in memory: frame-aligned
 * chunks of `chunk_bytes` (0: 64 MiB; rounded down to a multiple of 128) go
 * through `workers` pipelines (worker w on device w % devices; more workers
 * than devices is allowed), pread -> H2D -> device codec -> D2H -> pwrite, two
 * chunks in flight per worker. Output files are byte-identical to
 * flrl_fl_compress + the FL container (file_io.cu:222-280). Decompression
 * validates the header (bitsSize == ceil(inputSize/128), file length ==
 * 24 + bitsSize + valuesSize) and every width before decoding (FLRL_E_FORMAT).
 * Outputs go to a temporary file next to out_path, renamed into place on
 * success: on error an existing output is left as it was, and in_path may
 * equal out_path. */
int flrl_fl_compress_file(const char *in_path, const char *out_path, int workers, size_t chunk_bytes);
int flrl_fl_decompress_file(const char *in_path, const char *out_path, int workers, size_t chunk_bytes);

/* RL, file to file, same pipelines (the CLI's `c|d rl`). Compression encodes
 * chunks independently and re-splits a run that crosses a chunk boundary from
 * its true start, so the file equals flrl_rl_compress + the RL container;
 * values[] go through an unlinked side file until R is known. Decompression
 * validates the header (file length == 16 + 2*runs), every count (>= 1) and
 * their sum (== inputSize), then decodes blocks of runs of <= chunk_bytes
 * output (0: 64 MiB; at least 256) on all pipelines. */
int flrl_rl_compress_file(const char *in_path, const char *out_path, int workers, size_t chunk_bytes);
int flrl_rl_decompress_file(const char *in_path, const char *out_path, int workers, size_t chunk_bytes);

/* ---- FL, device-resident (asynchronous on `stream`) -----------------------
 * Replaces FixedLength::gpuCompressDevice (src/fl/fl_gpu.cuh:17,
 * fl_gpu.cu:425-535) — outputs stay in HBM.
 * All device pointers must be 16-byte aligned (hipMalloc / torch allocations
 * are); FLRL_E_ARG otherwise.
 *   d_in        n input bytes
 *   d_bits      ceil(n/128) bytes
 *   d_values    capacity >= flrl_fl_values_capacity(n) bytes
 *   d_values_size  device u64 receiving valuesSize
 *   d_scratch   >= flrl_fl_scratch_bytes(n) bytes of device memory, 16-B aligned
 * n == 0 writes 0 to *d_values_size. */
size_t flrl_fl_scratch_bytes(size_t n);
size_t flrl_fl_values_capacity(size_t n);
int flrl_fl_encode_device(const uint8_t *d_in, size_t n, uint8_t *d_bits, uint8_t *d_values,
                          uint64_t *d_values_size, void *d_scratch, size_t scratch_bytes,
                          void *stream);

/* Device decode: n output bytes from bits/values. The kernel flags
 * FLRL_E_FORMAT in the scratch area when a width is outside [1,8] or
 * values_size differs from the size the widths imply; the output is then
 * undefined. values_size == n (every frame stored at width 8, e.g.
 * incompressible data) skips the offsets pre-pass: the decode kernel derives
 * the offsets and checks each width itself. */
int flrl_fl_decode_device(const uint8_t *d_bits, size_t bits_size, const uint8_t *d_values,
                          size_t values_size, uint8_t *d_out, size_t n, void *d_scratch,
                          size_t scratch_bytes, void *stream);

/* Reads (synchronising `stream`) the error word a device call left in scratch:
 * 0 = ok, else an FLRL_E_* code. */
int flrl_scratch_error(const void *d_scratch, void *stream);

/* Measurement hook (no reference counterpart): the next flrl_*_device call of
 * this thread that launches its kernels records `start_event` on its stream
 * immediately before its main kernel (fl_encode, fl_decode, rl_encode,
 * rl_decode) and `stop_event` immediately after it, so the caller's
 * hipEventElapsedTime covers that kernel alone (not the scratch memset or the
 * decode offsets pre-pass). Events are hipEvent_t created by the caller; both
 * NULL cancels a pending pair. */
int flrl_time_next_kernel(void *start_event, void *stop_event);

/* Test hook (no reference counterpart): the next `calls` device calls of this
 * thread skip their per-call scratch reset, so their kernels see the previous
 * launch's ticket. Every ticketed kernel then raises FLRL_E_ARG in the scratch
 * error word instead of running (or silently doing nothing) on stale state.
 * 0 cancels. Never needed by callers. */
int flrl_debug_skip_scratch_resets(int calls);

/* Test hook (no reference counterpart): the RL encode look-backs of this
 * thread's later launches compute an unpublished predecessor tile's map
 * (its aggregate) from the input once it has been
 * unpublished for `microseconds` (0: at the first unpublished poll) instead of
 * after the default 200 us -- the decoupled fallback that keeps them
 * independent of workgroup dispatch order. -1 restores the default. Output is
 * identical either way; never needed by callers. */
int flrl_debug_lookback_help_us(int microseconds);

/* Test hook: the streamed file paths (flrl_*_file) fail when a worker reaches
 * chunk (or RL decode block) `chunk`, as a failed read or device call would.
 * Process-wide; a negative value cancels. */
int flrl_debug_fail_chunk(long long chunk);

/* Test hook: the next flrl_fl_encode_rank / flrl_fl_compress_rank call of this
 * thread fails once at `step`, as the runtime call there would, to exercise the
 * collective-on-error paths (every rank still completes every collective,
 * except after FLRL_DEBUG_RANK_READ_SUM):
 *   FLRL_DEBUG_RANK_SET_DEVICE   the rank cannot reach its device: its exchange
 *                                slot is sent from the comm's constant failed pair
 *   FLRL_DEBUG_RANK_STREAM_WAIT  the stream cannot be ordered after the previous
 *                                call: ordered on the host, failed slot
 *   FLRL_DEBUG_RANK_STAGE_WORD   (compress_rank) the {size, failed} word cannot be
 *                                staged: the constant {0, 1} is reduced instead
 *   FLRL_DEBUG_RANK_READ_SUM     (compress_rank) the reduced word cannot be read
 *                                back (a device failure after the all-reduce; the
 *                                one case that is NOT collective: with two or more
 *                                ranks and no earlier failure the peers then wait
 *                                in the payload send/recv, see flrl_fl_compress_rank)
 * 0 cancels. Never needed by callers. */
#define FLRL_DEBUG_RANK_SET_DEVICE 1
#define FLRL_DEBUG_RANK_STREAM_WAIT 2
#define FLRL_DEBUG_RANK_STAGE_WORD 3
#define FLRL_DEBUG_RANK_READ_SUM 4
int flrl_debug_fail_rank_step(int step);

/* ---- RL, host buffers (synchronous) --------------------------------------- */
int flrl_rl_compress(const uint8_t *data, size_t size, flrl_rl_buf *out);
int flrl_rl_decompress(size_t output_size, const uint8_t *counts, const uint8_t *values,
                       size_t runs, uint8_t **out, size_t *out_size);

/* ---- RL, device-resident (asynchronous) ----------------------------------
 * d_counts / d_values capacity n bytes each; d_runs receives R (device u64).
 * One kernel: 128 KiB tiles chained by a decoupled look-back (DESIGN.md §4
 * "RL encode"). (A three-pass scan / state / emit form without the look-back
 * wait was removed in round 4: it lost alone and in the encode/decode loop.) */
size_t flrl_rl_scratch_bytes(size_t n);
int flrl_rl_encode_device(const uint8_t *d_in, size_t n, uint8_t *d_counts, uint8_t *d_values,
                          uint64_t *d_runs, void *d_scratch, size_t scratch_bytes, void *stream);
/* Decode R runs into n = sum(counts) bytes; flags FLRL_E_FORMAT in scratch if a
 * count is 0 or the counts do not sum to n. */
size_t flrl_rl_decode_scratch_bytes(size_t runs);
int flrl_rl_decode_device(const uint8_t *d_counts, const uint8_t *d_values, size_t runs,
                          uint8_t *d_out, size_t n, void *d_scratch, size_t scratch_bytes,
                          void *stream);

/* ---- synthetic inputs on device (SURVEY.md §8(d) generator) ---------------
 * kind 0 u8, 1 lo4, 2 zero (counter-based; word_offset = global 8-byte word index
 * of d_out[0], so a shard at byte offset 8*k reproduces the whole buffer's bytes). */
int flrl_gen_device(int kind, uint64_t seed, uint64_t word_offset, uint8_t *d_out, size_t n,
                    void *stream);

/* Same generator on the host, all kinds: 0 u8, 1 lo4, 2 zero (word_offset as
 * above), 3 runs32 (runs of 1..63 equal bytes), 4 longruns (runs of 1..1023);
 * the run kinds are sequential and need word_offset == 0. */
int flrl_gen_host(int kind, uint64_t seed, uint64_t word_offset, uint8_t *out, size_t n);

#ifdef __cplusplus
}
#endif

#endif /* FLRL_H */
