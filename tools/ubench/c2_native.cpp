// C2 stream driven from C++ through the C-ABI (no Python in the loop): S contexts / streams,
// frames in flight with the bench's event hand-offs. Frames: raw 640x480 u8 file of NF frames
// (written by tools/ubench/c2_frames.py). Prints frames/s and host submit us/frame.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/orbhip.h"

#define CK(x) do { if ((x) != 0) { std::printf("fail %s line %d\n", #x, __LINE__); return 1; } } while (0)

int main(int argc, char** argv) {
    const char* path = argc > 1 ? argv[1] : "gpurun_out/c2_frames.u8";
    const int S = argc > 2 ? std::atoi(argv[2]) : 4;
    const int K = argc > 3 ? std::atoi(argv[3]) : 2000;
    const int D = argc > 4 ? std::atoi(argv[4]) : 0;   // host throttle: at most D frames queued (0 = none)
    const int W = 640, H = 480, NF = 32;
    std::vector<uint8_t> host((size_t)W * H * NF);
    FILE* f = std::fopen(path, "rb");
    if (!f || std::fread(host.data(), 1, host.size(), f) != host.size()) { std::printf("no frames\n"); return 1; }
    std::fclose(f);
    uint8_t* dframes;
    CK(hipMalloc(&dframes, host.size()));
    CK(hipMemcpy(dframes, host.data(), host.size(), hipMemcpyHostToDevice));
    orbhip_orb_params prm = {1000, 1.2f, 8, 20, 7};
    std::vector<orbhip_ctx*> ctx(S);
    std::vector<hipStream_t> st(S);
    // streams first: HIP assigns hardware queues round-robin at stream creation (each context
    // creates one stream of its own), so interleaving would put two of ours on one queue
    const int mode = std::getenv("C2N_MODE") ? std::atoi(std::getenv("C2N_MODE")) : 0;
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    if (mode == 1)   // contexts first, as the Python bench does
        for (int j = 0; j < S; j++) CK(orbhip_create(&ctx[j], 0, &prm));
    for (int j = 0; j < S; j++) {
        if (mode == 2) CK(hipStreamCreateWithPriority(&st[j], hipStreamNonBlocking, hi));
        else if (mode == 3) CK(hipStreamCreateWithPriority(&st[j], hipStreamNonBlocking, lo));
        else CK(hipStreamCreateWithFlags(&st[j], hipStreamNonBlocking));
    }
    if (mode != 1)
        for (int j = 0; j < S; j++) CK(orbhip_create(&ctx[j], 0, &prm));
    std::printf("mode %d (priority range %d..%d)\n", mode, lo, hi);
    const int cap = orbhip_max_keypoints(ctx[0], W, H);
    const int ns = S > 1 ? S : 2;
    orbhip_kp* kps; uint8_t* desc; int32_t *n, *mono, *mm, *nm;
    CK(hipMalloc(&kps, sizeof(orbhip_kp) * cap * ns));
    CK(hipMalloc(&desc, 32 * (size_t)cap * ns));
    CK(hipMalloc(&n, 4 * ns)); CK(hipMalloc(&mono, 4 * ns)); CK(hipMalloc(&nm, 4 * ns));
    CK(hipMalloc(&mm, 4 * 3 * (size_t)cap * ns));
    std::vector<hipEvent_t> ev_x(ns), ev_m(ns), ev_done(64);
    for (int i = 0; i < ns; i++) {
        CK(hipEventCreateWithFlags(&ev_x[i], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&ev_m[i], hipEventDisableTiming));
    }
    for (auto& e : ev_done) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    auto step = [&](int k) -> int {
        const int j = k % S, cur = k % ns, prev = (k - 1 + ns) % ns;
        if (S > 1 && k >= ns) CK(hipStreamWaitEvent(st[j], ev_m[cur], 0));
        CK(orbhip_extract_batch_device(ctx[j], dframes + (size_t)(k % NF) * W * H, 1, W, H, W, (int64_t)W * H, 0, 1000,
                                       kps + (size_t)cur * cap, desc + (size_t)cur * cap * 32, cap, n + cur, mono + cur,
                                       st[j]));
        if (S > 1) {
            CK(hipEventRecord(ev_x[cur], st[j]));
            if (k >= 1) CK(hipStreamWaitEvent(st[j], ev_x[prev], 0));
        }
        int32_t* m = mm + (size_t)cur * 3 * cap;
        CK(orbhip_match_frames_device(ctx[j], kps + (size_t)prev * cap, desc + (size_t)prev * cap * 32, n + prev,
                                      kps + (size_t)cur * cap, desc + (size_t)cur * cap * 32, n + cur, cap, 50, 0.9f, 1,
                                      m, m + cap, m + 2 * cap, nm + cur, st[j]));
        if (S > 1) CK(hipEventRecord(ev_m[prev], st[j]));
        if (D > 0) {
            CK(hipEventRecord(ev_done[k % 64], st[j]));
            if (k >= D) CK(hipEventSynchronize(ev_done[(k - D) % 64]));
        }
        return 0;
    };
    int k = 0;
    for (; k < 100; k++) if (step(k)) return 1;
    CK(hipDeviceSynchronize());
    for (int rep = 0; rep < 3; rep++) {
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < K; i++, k++) if (step(k)) return 1;
        auto t1 = std::chrono::steady_clock::now();
        CK(hipDeviceSynchronize());
        auto t2 = std::chrono::steady_clock::now();
        const double sub = std::chrono::duration<double, std::micro>(t1 - t0).count() / K;
        const double tot = std::chrono::duration<double>(t2 - t0).count();
        std::printf("D=%d S=%d: %.1f frames/s, host submit %.2f us/frame\n", D, S, K / tot, sub);
    }
    return 0;
}
