// host_prof.cpp — a small SIGPROF sampler for the host side of a mine
// (FSM_HOST_PROF=<file>: diagnostics only, off by default).  Every 50 us of
// wall time (a CLOCK_MONOTONIC POSIX timer aimed at the mining thread) the
// interrupted instruction pointer of that thread is recorded; at the end each sample is written as "<object> <offset>" so the
// offsets can be symbolized offline (llvm-symbolizer --obj=libfsm.so).
#include <dlfcn.h>
#include <signal.h>
#include <sys/syscall.h>
#include <sys/time.h>
#include <time.h>
#include <unistd.h>
#include <ucontext.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <string>
#include <vector>

#include "fsm_internal.h"

namespace fsm {
namespace {

constexpr size_t kMaxSamples = 1u << 20;
uintptr_t g_ip[kMaxSamples];
std::atomic<size_t> g_n{0};
std::atomic<bool> g_on{false};
timer_t g_timer;

void on_prof(int, siginfo_t*, void* uc) {
    if (!g_on.load(std::memory_order_relaxed)) return;
    const size_t k = g_n.fetch_add(1, std::memory_order_relaxed);
    if (k < kMaxSamples) g_ip[k] = uintptr_t(static_cast<ucontext_t*>(uc)->uc_mcontext.gregs[REG_RIP]);
}

}  // namespace

bool host_prof_start() {
    if (!std::getenv("FSM_HOST_PROF")) return false;
    g_n = 0;
    struct sigaction sa {};
    sa.sa_sigaction = on_prof;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGPROF, &sa, nullptr);
    sigevent sev{};
    sev.sigev_notify = SIGEV_THREAD_ID;
    sev.sigev_signo = SIGPROF;
    sev._sigev_un._tid = pid_t(syscall(SYS_gettid));
    if (timer_create(CLOCK_MONOTONIC, &sev, &g_timer) != 0) return false;
    g_on = true;
    itimerspec ts{{0, 50000}, {0, 50000}};
    timer_settime(g_timer, 0, &ts, nullptr);
    return true;
}

void host_prof_stop() {
    g_on = false;
    timer_delete(g_timer);
    const char* path = std::getenv("FSM_HOST_PROF");
    if (!path) return;
    std::FILE* f = std::fopen(path, "a");
    if (!f) return;
    const size_t n = std::min(g_n.load(), kMaxSamples);
    std::map<std::pair<std::string, uintptr_t>, size_t> hist;
    for (size_t k = 0; k < n; ++k) {
        Dl_info di{};
        if (dladdr(reinterpret_cast<void*>(g_ip[k]), &di) && di.dli_fname)
            hist[{di.dli_fname, g_ip[k] - uintptr_t(di.dli_fbase)}] += 1;
        else
            hist[{"?", 0}] += 1;
    }
    std::fprintf(f, "# samples %zu\n", n);
    for (const auto& [k, v] : hist) std::fprintf(f, "%zu %s 0x%llx\n", v, k.first.c_str(), (unsigned long long)k.second);
    std::fclose(f);
}

}  // namespace fsm
