// ubench_fl.hip — timing of the library's FL encode/decode on device-resident
// data, with an optional per-tile timestamp trace of the encode (-DTRACE:
// s_memrealtime at tile start / aggregate published / look-back resolved /
// stores issued, written to gpurun_out/fl_trace.bin for offline analysis).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DTRACE] -I include \
//         -I fl-rl-compression-mpi_amd/csrc scripts/ubench_fl.hip -o scripts/ubench_fl.bin -lrccl
//   scripts/ubench_fl.bin [kind=0 (u8)] [n=1 GiB] [reps=20]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define FLRL_TUNING_BUILD 1  // trace hooks below (csrc/flrl_tuning.hpp)

#ifdef TRACE
__device__ uint64_t *g_trace;
__device__ __forceinline__ uint64_t fl_rtime()
{
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#define FLRL_FL_TRACE(tile, k)                                         \
    do {                                                               \
        if ((threadIdx.x & 63) == 0)                                   \
            g_trace[(uint64_t)(tile) * 4 + (k)] = fl_rtime();          \
    } while (0)
#endif

#include "flrl_common.hip"
#include "flrl_fl.hip"

// the host-buffer pipelines live in flrl_stream.hip, which this harness does
// not build: flrl_fl_compress / flrl_fl_decompress are never called here
namespace flrl {
int fl_compress_host(const uint8_t *, size_t, flrl_fl_buf *) { return FLRL_E_ARG; }
int fl_decompress_host(size_t, const uint8_t *, size_t, const uint8_t *, size_t, uint8_t **) { return FLRL_E_ARG; }
}  // namespace flrl

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

int main(int argc, char **argv)
{
    const int kind = argc > 1 ? atoi(argv[1]) : 0;
    const size_t n = argc > 2 ? strtoull(argv[2], nullptr, 0) : (1ull << 30);
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    const size_t F = (n + 127) / 128;
    uint8_t *d_in, *d_bits, *d_vals, *d_out;
    uint64_t *d_vs;
    void *d_scr;
    const size_t scr = flrl_fl_scratch_bytes(n);
    CK(hipMalloc(&d_in, n + 64));
    CK(hipMalloc(&d_bits, F + 64));
    CK(hipMalloc(&d_vals, n + 64));
    CK(hipMalloc(&d_out, n + 64));
    CK(hipMalloc(&d_vs, 8));
    CK(hipMalloc(&d_scr, scr));
#ifdef TRACE
    // the trace buffer must exist before ANY encode call (the hook writes it)
    const size_t ntiles = (n + 131071) / 131072;
    uint64_t *d_tr;
    CK(hipMalloc(&d_tr, ntiles * 32));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &d_tr, sizeof(d_tr)));
#endif
    if (flrl_gen_device(kind, 42, 0, d_in, n, nullptr) != FLRL_OK) {
        fprintf(stderr, "gen: %s\n", flrl_last_error());
        return 1;
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float se = 0, sd = 0, be = 1e30f, bd = 1e30f;
    uint64_t vs = 0;
    for (int r = 0; r < reps + 3; ++r) {
        float ms;
        CK(hipEventRecord(e0, nullptr));
        if (flrl_fl_encode_device(d_in, n, d_bits, d_vals, d_vs, d_scr, scr, nullptr) != FLRL_OK) {
            fprintf(stderr, "encode: %s\n", flrl_last_error());
            return 1;
        }
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) {
            se += ms;
            be = ms < be ? ms : be;
        }
        CK(hipMemcpy(&vs, d_vs, 8, hipMemcpyDeviceToHost));
        CK(hipEventRecord(e0, nullptr));
        if (flrl_fl_decode_device(d_bits, F, d_vals, vs, d_out, n, d_scr, scr, nullptr) != FLRL_OK) {
            fprintf(stderr, "decode: %s\n", flrl_last_error());
            return 1;
        }
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) {
            sd += ms;
            bd = ms < bd ? ms : bd;
        }
    }
    bool rt_ok;
    {  // round trip of the last encode/decode
        uint8_t *h_a = (uint8_t *)malloc(n), *h_b = (uint8_t *)malloc(n);
        CK(hipMemcpy(h_a, d_in, n, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h_b, d_out, n, hipMemcpyDeviceToHost));
        rt_ok = memcmp(h_a, h_b, n) == 0;
        free(h_a);
        free(h_b);
    }
    const double alg = (double)n + F + vs;
    printf("fl kind %d n %zu V %llu: encode avg %.4f best %.4f ms (%.1f GB/s alg)  decode avg %.4f best %.4f ms "
           "(%.1f GB/s alg)  err %d  roundtrip %s\n",
           kind, n, (unsigned long long)vs, se / reps, be, alg / (se / reps) / 1e6, sd / reps, bd,
           alg / (sd / reps) / 1e6, flrl_scratch_error(d_scr, nullptr), rt_ok ? "ok" : "MISMATCH");
#ifdef TRACE
    CK(hipMemset(d_tr, 0, ntiles * 32));
    flrl_fl_encode_device(d_in, n, d_bits, d_vals, d_vs, d_scr, scr, nullptr);
    CK(hipDeviceSynchronize());
    uint64_t *tr = (uint64_t *)malloc(ntiles * 32);
    CK(hipMemcpy(tr, d_tr, ntiles * 32, hipMemcpyDeviceToHost));
    FILE *f = fopen("gpurun_out/fl_trace.bin", "wb");
    if (f) {
        fwrite(tr, 32, ntiles, f);
        fclose(f);
    }
    printf("trace written: %zu tiles\n", ntiles);
#endif
    return 0;
}
