// pcie_probe.hip — host<->device transfer shapes on one MI355X (for the
// host-buffer API design, DESIGN.md §4 "File paths"): DMA copies one way and
// both ways at once, and device->host by a kernel storing straight into pinned
// host memory (concurrent with a DMA host->device copy).
//   hipcc --offload-arch=gfx950 -O3 scripts/pcie_probe.hip -o scripts/pcie_probe.bin
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__global__ void copy_kernel(const u32x4 *__restrict__ src, u32x4 *__restrict__ dst, size_t n16)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        __builtin_nontemporal_store(src[i], dst + i);
}

int main(int argc, char **argv)
{
    const size_t n = (argc > 1 ? strtoull(argv[1], nullptr, 0) : (1ull << 30));
    const int reps = 5;
    uint8_t *h1, *h2, *d1, *d2;
    CK(hipHostMalloc((void **)&h1, n, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&h2, n, hipHostMallocDefault));
    CK(hipMalloc((void **)&d1, n));
    CK(hipMalloc((void **)&d2, n));
    for (size_t i = 0; i < n; i += 4096) { h1[i] = 1; h2[i] = 2; }
    CK(hipMemset(d1, 3, n));
    CK(hipMemset(d2, 4, n));
    hipStream_t sa, sb;
    CK(hipStreamCreate(&sa));
    CK(hipStreamCreate(&sb));
    int blocks = 0;
    CK(hipDeviceGetAttribute(&blocks, hipDeviceAttributeMultiprocessorCount, 0));
    auto timeit = [&](const char *name, double moved, auto &&fn) {
        double best = 1e30;
        for (int r = 0; r < reps; ++r) {
            CK(hipDeviceSynchronize());
            auto t0 = __builtin_readcyclecounter();
            (void)t0;
            timespec a, b;
            clock_gettime(CLOCK_MONOTONIC, &a);
            fn();
            CK(hipDeviceSynchronize());
            clock_gettime(CLOCK_MONOTONIC, &b);
            const double s = (b.tv_sec - a.tv_sec) + (b.tv_nsec - a.tv_nsec) * 1e-9;
            best = s < best ? s : best;
        }
        printf("%-44s %7.2f ms  %6.1f GB/s moved\n", name, best * 1e3, moved / best / 1e9);
    };
    timeit("DMA H2D", n, [&] { CK(hipMemcpyAsync(d1, h1, n, hipMemcpyHostToDevice, sa)); });
    timeit("DMA D2H", n, [&] { CK(hipMemcpyAsync(h2, d2, n, hipMemcpyDeviceToHost, sb)); });
    timeit("DMA H2D + DMA D2H (two streams)", 2.0 * n, [&] {
        CK(hipMemcpyAsync(d1, h1, n, hipMemcpyHostToDevice, sa));
        CK(hipMemcpyAsync(h2, d2, n, hipMemcpyDeviceToHost, sb));
    });
    for (int mult : {1, 4}) {
        char nm[64];
        snprintf(nm, sizeof nm, "kernel D2H (%d WG/CU)", mult);
        timeit(nm, n, [&] {
            hipLaunchKernelGGL(copy_kernel, dim3(blocks * mult), dim3(256), 0, sb, (const u32x4 *)d2, (u32x4 *)h2, n / 16);
        });
        snprintf(nm, sizeof nm, "DMA H2D + kernel D2H (%d WG/CU)", mult);
        timeit(nm, 2.0 * n, [&] {
            CK(hipMemcpyAsync(d1, h1, n, hipMemcpyHostToDevice, sa));
            hipLaunchKernelGGL(copy_kernel, dim3(blocks * mult), dim3(256), 0, sb, (const u32x4 *)d2, (u32x4 *)h2, n / 16);
        });
    }
    timeit("kernel H2D (1 WG/CU)", n, [&] {
        hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(256), 0, sa, (const u32x4 *)h1, (u32x4 *)d1, n / 16);
    });
    return 0;
}
