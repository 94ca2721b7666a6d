// Launch-sequence replay for the per-frame entry points (orbhip_extract_batch_device,
// orbhip_match_*_device).
//
// One C2 frame is six dependent kernels. Submitting them one by one costs the host ~2.9 us per
// hipLaunchKernel on this runtime (tools/ubench/launch_cost.hip), more than the GPU needs for a
// pipelined frame. With ORBHIP_GRAPH=1, a call whose launch sequence is fully fixed by its
// arguments (pointers, sizes, stream, the context's scratch buffers) is captured into a hipGraph
// the SECOND time the same key is seen and replayed by one hipGraphLaunch from then on; one-off
// calls (tests, changing buffers) stay direct and pay no capture. The kernels and their
// arguments are the same either way, so results are identical. Direct launches are kept for the
// legacy NULL stream, a stream that is already capturing (the caller's own graph) and an active
// stage timer (its events are per-launch).
// Off by default: on ROCm 7.2 / MI355X a replay costs the host about a third of the direct
// launches but adds ~10 us of device time per C2 frame (sequential 70 -> 81 us per frame in the
// same run), so it only pays for a host-bound pipelined stream ("Launch graphs").
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <unordered_map>

namespace orbhip {

struct GraphKey {
    static constexpr int kWords = 48;
    uint64_t w[kWords] = {};
    int n = 0;
    bool overflow = false;   // more words than kWords: the key is not exact, never replay it
    GraphKey& add(uint64_t v) {
        if (n < kWords) w[n++] = v;
        else overflow = true;
        return *this;
    }
    GraphKey& ptr(const void* p) { return add((uint64_t)(uintptr_t)p); }
    GraphKey& f32(float f) {
        uint32_t u;
        std::memcpy(&u, &f, 4);
        return add(u);
    }
    bool operator==(const GraphKey& o) const {
        return !overflow && !o.overflow && n == o.n && std::memcmp(w, o.w, sizeof(uint64_t) * n) == 0;
    }
};

struct GraphKeyHash {
    size_t operator()(const GraphKey& k) const {
        uint64_t h = 1469598103934665603ull;   // FNV-1a over the words
        for (int i = 0; i < k.n; i++) {
            h ^= k.w[i];
            h *= 1099511628211ull;
        }
        return (size_t)(h ^ (h >> 29));
    }
};

class GraphCache {
public:
    static constexpr size_t kMaxEntries = 256;
    ~GraphCache() { clear(); }
    void clear() {
        for (auto& kv : map_)
            if (kv.second.exec) (void)hipGraphExecDestroy(kv.second.exec);
        map_.clear();
    }
    int graphs() const {
        int c = 0;
        for (const auto& kv : map_) c += kv.second.exec != nullptr;
        return c;
    }
    // fn(stream) issues the launch sequence and returns an ORBHIP status; `direct` forces the
    // plain path. Returns fn's status, or the replay's.
    template <class F>
    int run(const GraphKey& key, hipStream_t st, bool direct, F&& fn) {
        const char* on = std::getenv("ORBHIP_GRAPH");
        if (!on || !on[0] || on[0] == '0' || direct || st == nullptr || key.overflow) return fn(st);
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return fn(st);
        auto it = map_.find(key);
        if (it == map_.end()) {
            if (map_.size() >= kMaxEntries) clear();
            map_.emplace(key, Entry{});
            return fn(st);   // first sighting: direct
        }
        Entry& e = it->second;
        if (!e.exec) {
            if (e.failed) return fn(st);
            if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
                e.failed = true;
                return fn(st);
            }
            const int rc = fn(st);
            hipGraph_t g = nullptr;
            const hipError_t ce = hipStreamEndCapture(st, &g);
            (void)hipGetLastError();
            if (rc != 0 || ce != hipSuccess || !g ||
                hipGraphInstantiate(&e.exec, g, nullptr, nullptr, 0) != hipSuccess) {
                if (g) (void)hipGraphDestroy(g);
                e.exec = nullptr;
                e.failed = true;
                (void)hipGetLastError();
                return rc != 0 ? rc : fn(st);   // nothing ran during the capture: run it now
            }
            (void)hipGraphDestroy(g);
        }
        return hipGraphLaunch(e.exec, st) == hipSuccess ? 0 : -3;   // ORBHIP_ERR_DEVICE
    }

private:
    struct Entry {
        hipGraphExec_t exec = nullptr;
        bool failed = false;
    };
    std::unordered_map<GraphKey, Entry, GraphKeyHash> map_;
};

}  // namespace orbhip
