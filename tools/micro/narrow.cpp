// Host narrowing rate (int64 -> int32) by thread count, into pageable and pinned memory.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdint>
#include <thread>
#include <vector>
static double ms() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
    const size_t T = 17u << 20;
    std::vector<int64_t> src(T);
    for (size_t i = 0; i < T; ++i) src[i] = int64_t(i % 10007) - 2;
    std::vector<int32_t> dst(T, 0);
    void* pin; hipHostMalloc(&pin, T * 4, hipHostMallocMapped);
    printf("hardware_concurrency %u\n", std::thread::hardware_concurrency());
    for (int rep = 0; rep < 2; ++rep)
    for (int nt : {1, 2, 4, 8, 16, 32}) {
        for (int dp = 0; dp < 2; ++dp) {
            int32_t* d = dp ? (int32_t*)pin : dst.data();
            double t0 = ms();
            std::vector<std::thread> th;
            for (int t = 0; t < nt; ++t)
                th.emplace_back([&, t] { size_t a = T * t / nt, z = T * (t + 1) / nt; for (size_t i = a; i < z; ++i) d[i] = int32_t(src[i]); });
            for (auto& x : th) x.join();
            double t1 = ms();
            printf("threads %2d %s: %.2f ms (%.1f GB/s read)\n", nt, dp ? "pinned  " : "pageable", t1 - t0, T * 8 / 1e6 / (t1 - t0));
        }
    }
    return 0;
}
