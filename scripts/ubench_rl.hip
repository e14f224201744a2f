// ubench_rl.hip — timing + per-phase cycle breakdown of the library's RL encode
// (the product kernel itself, compiled in with its phase hooks enabled).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 [-DSTAMP] -I include \
//         -I fl-rl-compression-mpi_amd/csrc scripts/ubench_rl.hip -o scripts/ubench_rl.bin
//   scripts/ubench_rl.bin [kind=3 (runs32); 100+M: runs of 1..M] [n=1 GiB] [reps=20]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define FLRL_TUNING_BUILD 1  // trace hooks below (csrc/flrl_tuning.hpp)

__device__ unsigned long long g_ph[64];
__device__ __forceinline__ uint64_t rl_stamp()
{
    uint64_t t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
#ifdef STAMP
#define FLRL_RL_PHASE_BEGIN() uint64_t _t0 = rl_stamp(), _t1 = 0, _ph[6] = {0, 0, 0, 0, 0, 0}
#define FLRL_RL_PHASE(k)                                                                   \
    do {                                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                 \
        _t1 = rl_stamp();                                                                  \
        _ph[k] += _t1 - _t0;                                                               \
        _t0 = _t1;                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                 \
    } while (0)
#define FLRL_RL_PHASE_END()                                                                \
    do {                                                                                   \
        if ((threadIdx.x & 63) == 0)                                                       \
            for (int _i = 0; _i < 6; ++_i)                                                 \
                atomicAdd(&g_ph[(threadIdx.x / 64) * 8 + _i], (unsigned long long)_ph[_i]); \
    } while (0)
#else
#define FLRL_RL_PHASE_BEGIN() ((void)0)
#define FLRL_RL_PHASE(k) ((void)0)
#define FLRL_RL_PHASE_END() ((void)0)
#endif

#ifdef TRACE
__device__ uint64_t *g_trace;
__device__ __forceinline__ uint64_t rl_rtime()
{
    uint64_t t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    return t;
}
// slot 7 (at k == 0): where the tile ran -- XCC id << 32 | HW_ID (wave, SIMD,
// CU, SH, SE fields)
__device__ __forceinline__ uint64_t rl_where()
{
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    return ((uint64_t)xcc << 32) | hw;
}
#define FLRL_RL_TRACE(tile, k)                                                   \
    do {                                                                         \
        if ((threadIdx.x & 63) == 0) {                                           \
            g_trace[(uint64_t)(tile) * 8 + (k)] = rl_rtime();                    \
            if ((k) == 0)                                                        \
                g_trace[(uint64_t)(tile) * 8 + 7] = rl_where();                  \
        }                                                                        \
    } while (0)
#define FLRL_RL_LB_STAT(tile, spins, rounds)                                      \
    do {                                                                          \
        if ((threadIdx.x & 63) == 0) {                                            \
            g_trace[(uint64_t)(tile) * 8 + 5] = (spins);                           \
            g_trace[(uint64_t)(tile) * 8 + 6] = (rounds);                          \
        }                                                                         \
    } while (0)
#endif
#include "flrl_common.hip"
#include "flrl_rl.hip"

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

int main(int argc, char **argv)
{
    const int kind = argc > 1 ? atoi(argv[1]) : 3;  // 3 = runs32
    const size_t n = argc > 2 ? strtoull(argv[2], nullptr, 0) : (1ull << 30);
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    uint8_t *d_in, *d_c, *d_v;
    uint64_t *d_runs;
    void *d_scr;
    const size_t scr = flrl_rl_scratch_bytes(n);
    CK(hipMalloc(&d_in, n + 64));
    CK(hipMalloc(&d_c, n + 64));
    CK(hipMalloc(&d_v, n + 64));
    CK(hipMalloc(&d_runs, 8));
    CK(hipMalloc(&d_scr, scr));
    {
        uint8_t *h = (uint8_t *)malloc(n);
        if (kind >= 100) {  // runs of 1..(kind-100) bytes, fresh value per run
            const uint32_t maxrun = (uint32_t)(kind - 100);
            uint64_t x = 88172645463325252ull;
            uint8_t v = 0;
            for (size_t i = 0; i < n;) {
                x ^= x << 13, x ^= x >> 7, x ^= x << 17;
                size_t L = 1 + (size_t)(x % maxrun);
                v = (uint8_t)(v + 1 + (x >> 32) % 254);
                for (size_t k = 0; k < L && i < n; ++k)
                    h[i++] = v;
            }
        } else if (flrl_gen_host(kind, 42, 0, h, n) != FLRL_OK) {
            fprintf(stderr, "gen: %s\n", flrl_last_error());
            return 1;
        }
        CK(hipMemcpy(d_in, h, n, hipMemcpyHostToDevice));
        if (getenv("INPUT_OUT")) {  // the input, for per-tile statistics on the host
            FILE *f = fopen(getenv("INPUT_OUT"), "wb");
            if (f) {
                fwrite(h, 1, n, f);
                fclose(f);
            }
        }
        free(h);
    }
#ifdef TRACE
    const size_t ntiles = (n + flrl::kRlTileBytes - 1) / flrl::kRlTileBytes;
    uint64_t *d_tr;
    CK(hipMalloc(&d_tr, ntiles * 64));
    CK(hipMemset(d_tr, 0, ntiles * 64));
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &d_tr, sizeof(d_tr)));
#endif
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e30f, sum = 0;
    for (int r = 0; r < reps + 3; ++r) {
        if (r == 3) {
            unsigned long long z[64] = {};
            CK(hipMemcpyToSymbol(HIP_SYMBOL(g_ph), z, sizeof(z)));
        }
        CK(hipEventRecord(e0, nullptr));
        if (flrl_rl_encode_device(d_in, n, d_c, d_v, d_runs, d_scr, scr, nullptr) != FLRL_OK) {
            fprintf(stderr, "encode: %s\n", flrl_last_error());
            return 1;
        }
        CK(hipEventRecord(e1, nullptr));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) {
            sum += ms;
            best = ms < best ? ms : best;
        }
    }
    uint64_t runs = 0;
    CK(hipMemcpy(&runs, d_runs, 8, hipMemcpyDeviceToHost));
    printf("rl_encode kind %d n %zu runs %llu: avg %.4f ms best %.4f ms (%.1f GB/s alg avg)  err %d\n", kind, n,
           (unsigned long long)runs, sum / reps, best, (n + 2.0 * runs) / (sum / reps) / 1e6,
           flrl_scratch_error(d_scr, nullptr));
    if (getenv("NO_DECODE"))  // ablation builds: the encode output is wrong by design
        return 0;
    {  // decode of what was just encoded, checked against the input
        uint8_t *d_out;
        CK(hipMalloc(&d_out, n + 64));
        const size_t dscr = flrl_rl_decode_scratch_bytes(runs);
        void *d_dscr;
        CK(hipMalloc(&d_dscr, dscr));
        float dsum = 0, dbest = 1e30f;
        for (int r = 0; r < reps + 3; ++r) {
            CK(hipEventRecord(e0, nullptr));
            if (flrl_rl_decode_device(d_c, d_v, runs, d_out, n, d_dscr, dscr, nullptr) != FLRL_OK) {
                fprintf(stderr, "decode: %s\n", flrl_last_error());
                return 1;
            }
            CK(hipEventRecord(e1, nullptr));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 3) {
                dsum += ms;
                dbest = ms < dbest ? ms : dbest;
            }
        }
        uint8_t *h_a = (uint8_t *)malloc(n), *h_b = (uint8_t *)malloc(n);
        CK(hipMemcpy(h_a, d_in, n, hipMemcpyDeviceToHost));
        CK(hipMemcpy(h_b, d_out, n, hipMemcpyDeviceToHost));
        printf("rl_decode: avg %.4f ms best %.4f ms (%.1f GB/s alg avg)  err %d  roundtrip %s\n", dsum / reps, dbest,
               (n + 2.0 * runs) / (dsum / reps) / 1e6, flrl_scratch_error(d_dscr, nullptr),
               memcmp(h_a, h_b, n) == 0 ? "ok" : "MISMATCH");
        free(h_a);
        free(h_b);
    }
#ifdef TRACE
    {
        CK(hipMemset(d_tr, 0, ntiles * 64));
        flrl_rl_encode_device(d_in, n, d_c, d_v, d_runs, d_scr, scr, nullptr);
        CK(hipDeviceSynchronize());
        uint64_t *h = (uint64_t *)malloc(ntiles * 64);
        CK(hipMemcpy(h, d_tr, ntiles * 64, hipMemcpyDeviceToHost));
        FILE *f = fopen(getenv("TRACE_OUT") ? getenv("TRACE_OUT") : "gpurun_out/rl_trace.bin", "wb");
        if (f) {
            fwrite(h, 64, ntiles, f);
            fclose(f);
        }
        free(h);
    }
#endif
#ifdef STAMP
    unsigned long long ph[64];
    CK(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_ph), sizeof(ph)));
    const char *names[6] = {"load", "scan", "lookback+barrier", "emit",
                            "-", "-"};
    for (int w = 0; w < 4; ++w) {
        unsigned long long tot = 0;
        for (int i = 0; i < 6; ++i)
            tot += ph[w * 8 + i];
        printf("wave %d:", w);
        for (int i = 0; i < 6; ++i)
            printf("  %s %.1f%%", names[i], 100.0 * ph[w * 8 + i] / (tot ? tot : 1));
        printf("\n");
    }
#endif
    return 0;
}
