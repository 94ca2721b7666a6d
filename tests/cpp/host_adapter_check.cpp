// C++ host-side check of include/orbhip.hpp (the ORBextractor / ORBmatcher / Optimizer mirror)
// against a golden fixture unpacked by tests/test_host_cpp.py into raw files:
//   <dir>/image.u8 (h*w), <dir>/meta.i32 {w, h, nfeatures, lap0, lap1, mono, n},
//   <dir>/kps.f32 (n x 6), <dir>/desc.u8 (n x 32),
//   <dir>/ba_*.bin (BA problem arrays) + ba_meta.f32 {fx, fy, cx, cy, huber, iters, P, M, E, L}
//   <dir>/ba_out_*.f32 (expected poses / points), ba_out_meta.f64 {chi2_0, chi2_1}
// Exit 0 = identical keypoints/descriptors/monoIndex and BA within 1e-4 relative.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "orbhip.hpp"

template <typename T>
static std::vector<T> load(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("missing " + path);
    std::vector<char> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<T> v(b.size() / sizeof(T));
    std::memcpy(v.data(), b.data(), v.size() * sizeof(T));
    return v;
}

static int check_extract(const std::string& d) {
    const auto meta = load<int32_t>(d + "/meta.i32");
    const int w = meta[0], h = meta[1], nf = meta[2], mono_ref = meta[5], n_ref = meta[6];
    const auto img = load<uint8_t>(d + "/image.u8");
    const auto kref = load<float>(d + "/kps.f32");
    const auto dref = load<uint8_t>(d + "/desc.u8");
    orbhip::ORBextractor ext(nf, 1.2f, 8, 20, 7);
    std::vector<orbhip::KeyPoint> kps;
    std::vector<uint8_t> desc;
    std::vector<int> lap = {meta[3], meta[4]};
    const int mono = ext(img.data(), w, h, w, kps, desc, lap);
    if (mono != mono_ref || (int)kps.size() != n_ref) {
        std::printf("FAIL extract: mono %d/%d n %zu/%d\n", mono, mono_ref, kps.size(), n_ref);
        return 1;
    }
    for (int i = 0; i < n_ref; i++) {
        const float* r = &kref[6 * i];
        const orbhip::KeyPoint& k = kps[i];
        if (k.x != r[0] || k.y != r[1] || k.size != r[2] || k.angle != r[3] || k.response != r[4] ||
            k.octave != (int)r[5] || k.class_id != -1) {
            std::printf("FAIL kp %d\n", i);
            return 1;
        }
    }
    if (desc != dref) { std::printf("FAIL descriptors\n"); return 1; }
    // ORBmatcher::DescriptorDistance and the ctor tables
    if (orbhip::ORBmatcher::DescriptorDistance(&desc[0], &desc[0]) != 0) return 1;
    const auto sc = ext.GetScaleFactors();
    if (ext.GetLevels() != 8 || sc[0] != 1.0f || std::fabs(sc[1] - 1.2f) > 1e-6f) { std::printf("FAIL tables\n"); return 1; }
    // an empty image returns -1 like the reference
    std::vector<orbhip::KeyPoint> k2;
    std::vector<uint8_t> d2;
    if (ext(nullptr, 0, 0, 0, k2, d2, lap) != -1) { std::printf("FAIL empty\n"); return 1; }
    std::printf("extract OK: %d keypoints, monoIndex %d\n", n_ref, mono);
    return 0;
}

static int check_ba(const std::string& d, orbhip_ctx* ctx) {
    const auto meta = load<float>(d + "/ba_meta.f32");
    orbhip::BAProblem p;
    p.fx = meta[0]; p.fy = meta[1]; p.cx = meta[2]; p.cy = meta[3]; p.huber_delta = meta[4];
    p.iterations = (int)meta[5];
    p.pose_q = load<float>(d + "/ba_pose_q.f32");
    p.pose_t = load<float>(d + "/ba_pose_t.f32");
    p.pose_fixed = load<uint8_t>(d + "/ba_pose_fixed.u8");
    p.points = load<float>(d + "/ba_points.f32");
    p.edge_pose = load<int32_t>(d + "/ba_edge_pose.i32");
    p.edge_point = load<int32_t>(d + "/ba_edge_point.i32");
    p.edge_uv = load<float>(d + "/ba_edge_uv.f32");
    p.edge_octave = load<int32_t>(d + "/ba_edge_octave.i32");
    p.inv_sigma2 = load<float>(d + "/ba_inv_sigma2.f32");
    const auto r = orbhip::Optimizer::LocalBundleAdjustment(ctx, p);
    const auto chi = load<double>(d + "/ba_out_meta.f64");
    const auto t_ref = load<float>(d + "/ba_out_pose_t.f32");
    const auto x_ref = load<float>(d + "/ba_out_points.f32");
    double dt = 0, dx = 0, st = 1, sx = 1;
    for (size_t i = 0; i < t_ref.size(); i++) { dt = std::fmax(dt, std::fabs(r.pose_t[i] - t_ref[i])); st = std::fmax(st, std::fabs(t_ref[i])); }
    for (size_t i = 0; i < x_ref.size(); i++) { dx = std::fmax(dx, std::fabs(r.points[i] - x_ref[i])); sx = std::fmax(sx, std::fabs(x_ref[i])); }
    const double dchi = std::fabs(r.final_chi2 - chi[1]) / chi[1];
    std::printf("BA: chi2 %.6f -> %.6f (ref %.6f), rel dt %.2e dx %.2e dchi %.2e\n", r.initial_chi2, r.final_chi2,
                chi[1], dt / st, dx / sx, dchi);
    return (dt / st < 1e-4 && dx / sx < 1e-4 && dchi < 1e-4) ? 0 : 1;
}

int main(int argc, char** argv) {
    if (argc < 2) { std::fprintf(stderr, "usage: %s <fixture dir>\n", argv[0]); return 2; }
    try {
        const std::string d = argv[1];
        if (check_extract(d)) return 1;
        orbhip::ORBextractor ctx_owner(1000, 1.2f, 8, 20, 7);
        if (check_ba(d, ctx_owner.context())) return 1;
        std::printf("host adapter OK\n");
        return 0;
    } catch (const std::exception& e) {
        std::printf("FAIL exception: %s\n", e.what());
        return 1;
    }
}
