// One-time, per-device kernel attributes (host side). hipFuncSetAttribute acts on the calling
// thread's current device, and the C-ABI allows distinct contexts (possibly on distinct devices)
// to be driven from concurrent threads, so a process-wide `static bool` set once is
// both a data race and wrong for the second device. Each call site keeps one LdsAttrOnce (a
// function-local static: its construction is thread-safe) holding a bit per device, set under the
// object's mutex once the attribute call succeeded; the fast path is one acquire load.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>

namespace orbhip {

struct LdsAttrOnce {
    std::atomic<unsigned long long> done{0};   // bit d: set on device d
    std::mutex m;
    // the dynamic-LDS limit of kernels fs[0..n) on the current device (all or nothing)
    hipError_t ensure(const void* const* fs, int n, int bytes) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
        const unsigned long long bit = 1ull << dev;
        if (done.load(std::memory_order_acquire) & bit) return hipSuccess;
        std::lock_guard<std::mutex> g(m);
        if (done.load(std::memory_order_relaxed) & bit) return hipSuccess;
        for (int i = 0; i < n; i++) {
            const hipError_t e = hipFuncSetAttribute(fs[i], hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
            if (e != hipSuccess) return e;
        }
        done.fetch_or(bit, std::memory_order_release);
        return hipSuccess;
    }
    hipError_t ensure(const void* f, int bytes) { return ensure(&f, 1, bytes); }
};

}  // namespace orbhip
