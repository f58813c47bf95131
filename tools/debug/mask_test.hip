// Standalone unit test of the W-word mask helpers on the device.
#include <cstdio>
#include "../../spark-fsm_amd/csrc/device_util.h"
using namespace fsm;
template <int W> __global__ void k(const uint64_t* in, uint32_t* lohi, uint64_t* out, int n, int lo_clear) {
    int i = threadIdx.x;
    if (i >= n) return;
    uint64_t m[W];
    load_mask<W>(in + i * W, m);
    lohi[2 * i] = mask_lo<W>(m);
    lohi[2 * i + 1] = mask_hi<W>(m);
    mask_clear_upto<W>(m, uint32_t(lo_clear));
    store_mask<W>(out + i * W, m);
}
int main() {
    const int W = 4, n = 4;
    uint64_t h[n * W] = {0};
    int bits[n][2] = {{10, 200}, {10, 140}, {195, 200}, {64, 255}};
    for (int i = 0; i < n; ++i)
        for (int b : bits[i]) h[i * W + b / 64] |= 1ull << (b % 64);
    uint64_t *din, *dout; uint32_t* dl;
    hipMalloc(&din, sizeof h); hipMalloc(&dout, sizeof h); hipMalloc(&dl, 8 * n);
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    for (int clr : {10, 150, 196}) {
        hipLaunchKernelGGL(k<W>, 1, 64, 0, 0, din, dl, dout, n, clr);
        uint32_t l[2 * n]; uint64_t o[n * W];
        hipMemcpy(l, dl, sizeof l, hipMemcpyDeviceToHost);
        hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
        for (int i = 0; i < n; ++i)
            printf("bits {%d,%d} lo=%u hi=%u clear<=%d -> %016llx %016llx %016llx %016llx\n", bits[i][0], bits[i][1],
                   l[2 * i], l[2 * i + 1], clr, (unsigned long long)o[i * W], (unsigned long long)o[i * W + 1],
                   (unsigned long long)o[i * W + 2], (unsigned long long)o[i * W + 3]);
    }
    return 0;
}
