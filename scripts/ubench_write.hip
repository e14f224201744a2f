// ubench_write.hip — does the RL block decode's write pattern reach the write
// ceiling, and do its writes overlap a compute phase? 1 GiB written by:
//   fill:  grid-stride 16-byte stores from every CU (the ceiling)
//   tiles: the decode's pattern — 512-thread workgroups (2 per CU) take
//          256 KiB tiles by ticket, each in four 64 KiB windows, store k of
//          thread t at chunk k*512 + t of the window
//   tiles+work: the same with a VALU-only phase of `spin` iterations before
//          each window's stores (the decode's marks and scan), barrier-separated
//   work:  the phases alone, no stores (spin < 0: -spin LDS write+read round trips per phase instead of VALU; spin <= -1000: -(spin+1000) LDS reads only)
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_write.hip -o scripts/ubench_write.bin
//   scripts/ubench_write.bin [spin=2000] [reps=20] [gather=0: 1 = store data read from LDS, 2 = all gathers then all stores, 3 = from ds_bpermute] [gridstride=0]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));           \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int T = 512;
constexpr uint64_t kTile = 256 << 10, kWin = 64 << 10;

__global__ __launch_bounds__(256) void fill_kernel(u32x4 *out, uint64_t n16)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride)
        out[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

__device__ __forceinline__ uint32_t spin_work(uint32_t x, int spin)
{
    if (spin >= 0) {
        for (int i = 0; i < spin; ++i)  // a dependent VALU chain
            x = x * 1664525u + 1013904223u;
        return x;
    }
    __shared__ uint32_t s_buf[T * 4];
    if (spin <= -1000) {  // -(spin + 1000) dependent LDS reads, no LDS writes
        for (int i = 0; i < -(spin + 1000); ++i)
            x += s_buf[(threadIdx.x * 4 + i + (x & 63)) & (T * 4 - 1)] * 3u;
        return x;
    }
    // spin < 0: -spin dependent LDS round trips (write, read back a neighbour's word)
    for (int i = 0; i < -spin; ++i) {
        s_buf[(threadIdx.x * 4 + i) & (T * 4 - 1)] = x;
        x += s_buf[(threadIdx.x * 4 + i + 64) & (T * 4 - 1)] * 3u;
    }
    return x;
}

__shared__ uint32_t s_gat[T * 8];

template <bool STORE>
__global__ __launch_bounds__(T, 4) void tiles_kernel(uint8_t *out, uint32_t ntiles, uint32_t *ticket, int spin,
                                                      int gather, int gridstride)
{
    __shared__ uint32_t s_tile;
    uint32_t gs_tile = blockIdx.x;
    for (int i = threadIdx.x; i < T * 8; i += T)
        s_gat[i] = i * 2654435761u;
    uint32_t x = threadIdx.x;
    for (;;) {
        uint32_t tile;
        if (gridstride) {  // no ticket: tiles blockIdx, blockIdx + grid, ...
            tile = gs_tile;
            gs_tile += gridDim.x;
        } else {
            if (threadIdx.x == 0)
                s_tile = atomicAdd(ticket, 1u);
            __syncthreads();
            tile = s_tile;
            __syncthreads();
        }
        if (tile >= ntiles)
            break;
        for (uint64_t w = 0; w < kTile / kWin; ++w) {
            x = spin_work(x, spin);
            __syncthreads();
            u32x4 *o = reinterpret_cast<u32x4 *>(out + (uint64_t)tile * kTile + w * kWin);
            if (gather == 2) {  // all gathers of the window first, then all stores
                constexpr int K = (int)(kWin / 16 / T);
                u32x4 g[K];
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    const uint32_t a = (x + k * 977u + threadIdx.x * 5u) & (T * 8 - 8);
                    g[k] = u32x4{s_gat[a], s_gat[a + 1], s_gat[a + 2] ^ x, s_gat[a + 5]};
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    if (STORE)
                        o[k * T + threadIdx.x] = g[k];
                    else
                        asm volatile("" ::"v"(g[k][0]), "v"(g[k][1]));
                }
                __syncthreads();
                continue;
            }
#pragma unroll
            for (int k = 0; k < (int)(kWin / 16 / T); ++k) {
                u32x4 v = u32x4{x, (uint32_t)k, tile, 0u};
                if (gather == 3) {  // store data from other lanes by ds_bpermute (no LDS memory access)
                    const int src = (int)(((x + k * 977u) & 63u) << 2);
                    v = u32x4{(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)x),
                              (uint32_t)__builtin_amdgcn_ds_bpermute(src + 4, (int)(x ^ k)),
                              (uint32_t)__builtin_amdgcn_ds_bpermute(src + 8, (int)tile), x};
                } else if (gather) {  // store data gathered from LDS at data-dependent words, as the decode's chunks
                    const uint32_t a = (x + k * 977u + threadIdx.x * 5u) & (T * 8 - 8);
                    v = u32x4{s_gat[a], s_gat[a + 1], s_gat[a + 2] ^ x, s_gat[a + 5]};
                }
                if (STORE)
                    o[k * T + threadIdx.x] = v;
                else
                    asm volatile("" ::"v"(v[0]), "v"(v[1]));
            }
            __syncthreads();
        }
    }
    if (x == 0xFFFFFFFFu)  // keep the work
        out[0] = 1;
}

int main(int argc, char **argv)
{
    const int spin = argc > 1 ? atoi(argv[1]) : 2000;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const int gather = argc > 3 ? atoi(argv[3]) : 0;  // 1: store data gathered from LDS
    const int gridstride = argc > 4 ? atoi(argv[4]) : 0;  // 1: tiles grid-stride instead of by ticket
    const uint64_t n = 1ull << 30;
    uint8_t *out;
    uint32_t *ticket;
    CK(hipMalloc(&out, n));
    CK(hipMalloc(&ticket, 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const uint32_t ntiles = (uint32_t)(n / kTile);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        float tot = 0;
        for (int r = 0; r < reps + 2; ++r) {
            CK(hipMemset(ticket, 0, 4));
            CK(hipEventRecord(e0, nullptr));
            launch();
            CK(hipEventRecord(e1, nullptr));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r >= 2)
                tot += ms;
        }
        printf("%-28s %.4f ms  %.1f GB/s written\n", name, tot / reps, n / (tot / reps) / 1e6);
    };
    timeit("fill", [&] { hipLaunchKernelGGL(fill_kernel, dim3(cus * 8), dim3(256), 0, nullptr, (u32x4 *)out, n / 16); });
    timeit("tiles (no work)", [&] {
        hipLaunchKernelGGL(tiles_kernel<true>, dim3(cus * 2), dim3(T), 0, nullptr, out, ntiles, ticket, 0, gather, gridstride);
    });
    char name[64];
    snprintf(name, sizeof name, "tiles + work(%d)", spin);
    timeit(name, [&] {
        hipLaunchKernelGGL(tiles_kernel<true>, dim3(cus * 2), dim3(T), 0, nullptr, out, ntiles, ticket, spin, gather, gridstride);
    });
    snprintf(name, sizeof name, "work(%d) alone", spin);
    timeit(name, [&] {
        hipLaunchKernelGGL(tiles_kernel<false>, dim3(cus * 2), dim3(T), 0, nullptr, out, ntiles, ticket, spin, gather, gridstride);
    });
    CK(hipDeviceSynchronize());
    return 0;
}
