// Host-memory micro-benchmark for the staging decisions (run on the GPU box):
// pinned allocation cost, H2D rates (pageable / pinned), CPU read rate of
// mapped pinned memory written by a kernel.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>
static double ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
__global__ void fill(uint32_t* p, size_t n) { for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = uint32_t(i * 2654435761u); }
int main() {
    hipFree(0);
    void* dev; hipMalloc(&dev, 256 << 20);
    for (size_t mb : {1, 4, 16, 64}) {
        for (unsigned flags : {unsigned(hipHostMallocMapped), unsigned(hipHostMallocDefault), unsigned(hipHostMallocMapped | hipHostMallocNonCoherent), unsigned(hipHostMallocMapped | hipHostMallocCoherent)}) {
            void* h; double t0 = ms();
            if (hipHostMalloc(&h, mb << 20, flags) != hipSuccess) { printf("alloc fail\n"); continue; }
            double t1 = ms();
            std::memset(h, 1, mb << 20);
            double t2 = ms();
            hipMemcpy(dev, h, mb << 20, hipMemcpyHostToDevice);
            double t3 = ms();
            hipMemcpy(dev, h, mb << 20, hipMemcpyHostToDevice);
            double t4 = ms();
            // kernel writes into mapped memory, CPU reads it
            void* dp = nullptr;
            double rd = -1;
            if (flags & hipHostMallocMapped) {
                hipHostGetDevicePointer(&dp, h, 0);
                hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, (uint32_t*)dp, (mb << 20) / 4);
                hipDeviceSynchronize();
                double t5 = ms();
                uint64_t s = 0; const uint32_t* q = (const uint32_t*)h;
                for (size_t i = 0; i < (mb << 20) / 4; ++i) s += q[i];
                double t6 = ms();
                rd = (mb / 1024.0) / ((t6 - t5) / 1000.0);
                if (s == 42) printf("x");
            }
            printf("%3zu MB flags %2u: alloc %.2f ms, first touch %.2f ms, H2D %.1f GB/s (2nd %.1f GB/s), CPU read of GPU-written %.2f GB/s\n",
                   mb, flags, t1 - t0, t2 - t1, (mb / 1024.0) / ((t3 - t2) / 1000.0), (mb / 1024.0) / ((t4 - t3) / 1000.0), rd);
            hipHostFree(h);
        }
        std::vector<char> pg(mb << 20, 1);
        double t0 = ms(); hipMemcpy(dev, pg.data(), mb << 20, hipMemcpyHostToDevice); double t1 = ms();
        hipMemcpy(dev, pg.data(), mb << 20, hipMemcpyHostToDevice); double t2 = ms();
        printf("%3zu MB pageable H2D %.1f GB/s (2nd %.1f GB/s)\n", mb, (mb / 1024.0) / ((t1 - t0) / 1000.0), (mb / 1024.0) / ((t2 - t1) / 1000.0));
    }
    return 0;
}
