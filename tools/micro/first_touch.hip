// First use of freshly allocated device memory: H2D into it, or a memset first.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
static double ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    hipFree(0);
    const size_t B = 64u << 20;
    void* h; hipHostMalloc(&h, B, hipHostMallocMapped); std::memset(h, 1, B);
    hipStream_t s; hipStreamCreate(&s);
    for (int mode = 0; mode < 3; ++mode) {
        void* d; double t0 = ms(); hipMalloc(&d, B); double t1 = ms();
        double tm = 0;
        if (mode == 1) { double a = ms(); hipMemsetAsync(d, 0, B, s); hipStreamSynchronize(s); tm = ms() - a; }
        if (mode == 2) { double a = ms(); hipMemsetAsync(d, 0, 4096, s); hipStreamSynchronize(s); tm = ms() - a; }
        double t2 = ms(); hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, s); hipStreamSynchronize(s); double t3 = ms();
        hipMemcpyAsync(d, h, B, hipMemcpyHostToDevice, s); hipStreamSynchronize(s); double t4 = ms();
        printf("mode %d (%s): malloc %.2f ms, memset %.2f ms, first H2D %.2f ms, second H2D %.2f ms\n", mode,
               mode == 0 ? "H2D first" : (mode == 1 ? "memset whole first" : "memset 4 KiB first"), t1 - t0, tm, t3 - t2, t4 - t3);
    }
    return 0;
}
