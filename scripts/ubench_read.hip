// ubench_read.hip — read-only streaming rate for the RL encode's access shape:
// one workgroup per 128 KiB tile (non-persistent), 16-byte loads per lane,
// SUB sub-tiles loaded one after another, occupancy set by a dummy LDS array.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/ubench_read.hip -o scripts/ubench_read.bin
#include <hip/hip_runtime.h>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int T, int LDSB, int PF>
__global__ __launch_bounds__(T) void rd(const uint8_t *in, uint64_t n, uint32_t *out)
{
    __shared__ uint32_t s[LDSB / 4];
    constexpr int TILE = 131072, PER = TILE / T / 16;  // 16-byte loads per lane per tile
    const uint64_t off = (uint64_t)blockIdx.x * TILE;
    u32x4 acc = {0, 0, 0, 0};
    if (PF) {
#pragma unroll
        for (int k = 0; k < PER; ++k)
            acc ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(in + off + ((uint64_t)k * T + threadIdx.x) * 16));
    } else {
        constexpr int SUBL = PER / 4;
        for (int sub = 0; sub < 4; ++sub) {
            u32x4 a = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < SUBL; ++k)
                a ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(in + off + ((uint64_t)(sub * SUBL + k) * T + threadIdx.x) * 16));
            s[threadIdx.x] = a.x ^ a.y ^ a.z ^ a.w;
            __syncthreads();
            acc.x ^= s[(threadIdx.x + 1) % T];
            __syncthreads();
        }
    }
    const uint32_t r = acc.x ^ acc.y ^ acc.z ^ acc.w;
    if (r == 0x12345678u)
        out[blockIdx.x] = r;
}

template <int T, int LDSB, int PF>
void run(const char *name, const uint8_t *d, uint64_t n, uint32_t *o)
{
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const uint32_t g = (uint32_t)(n / 131072);
    float best = 1e9, sum = 0;
    for (int r = 0; r < 23; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL((rd<T, LDSB, PF>), dim3(g), dim3(T), 0, 0, d, n, o);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (r >= 3) {
            sum += ms;
            best = ms < best ? ms : best;
        }
    }
    printf("%-28s avg %.4f ms best %.4f ms  %.1f GB/s\n", name, sum / 20, best, n / (sum / 20) / 1e6);
}

int main()
{
    const uint64_t n = 1ull << 30;
    uint8_t *d;
    uint32_t *o;
    hipMalloc(&d, n);
    hipMalloc(&o, 1 << 20);
    hipMemset(d, 1, n);
    run<256, 49152, 0>("T256 3/CU 4 sub serial", d, n, o);
    run<256, 49152, 1>("T256 3/CU all in flight", d, n, o);
    run<256, 32768, 0>("T256 5/CU 4 sub serial", d, n, o);
    run<256, 16384, 0>("T256 8/CU 4 sub serial", d, n, o);
    run<256, 16384, 1>("T256 8/CU all in flight", d, n, o);
    run<512, 81920, 0>("T512 2/CU 4 sub serial", d, n, o);
    run<512, 32768, 1>("T512 4/CU all in flight", d, n, o);
    run<1024, 16384, 1>("T1024 2/CU all in flight", d, n, o);
    return 0;
}
