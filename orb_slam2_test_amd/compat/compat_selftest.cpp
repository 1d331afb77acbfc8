// compat_selftest.cpp -- drives the C++ compat layer the way Tracking.cc drives the
// reference (extract two frames, SearchForInitialization, brute-force knn2) and dumps the
// results as raw files for tests/test_gpu_compat.py to compare against the oracle.
//
//   compat_selftest nogpu
//       expects the Extractor constructor to throw (no HIP device: no CPU fallback)
//   compat_selftest run <w> <h> <frame0.raw> <frame1.raw> <outdir> <nfeatures>
//       writes kps0/kps1 (28-B cv::KeyPoint records), desc0/desc1 (N x 32),
//       m12 (int32 per F1 keypoint), knn (int32 triples per F2 keypoint), nm.txt,
//       stereo_ur / stereo_depth (StereoFrame of frame0 as left, frame1 as right)
//   compat_selftest bench <w> <h> <frames.raw> <nimages> <nframes> <nfeatures>
//       the monocular per-frame loop of Tracking.cc as C++ drives it (Frame ctor ->
//       ExtractORB, then MonocularInitialization's SearchForInitialization against the
//       previous frame), host images in, host vectors out; one JSON line of per-frame
//       latency percentiles (the Python mirror's interpreter overhead excluded)
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "orbg_compat.hpp"

static std::vector<uint8_t> read_file(const std::string &p, size_t n)
{
    std::vector<uint8_t> b(n);
    std::ifstream f(p, std::ios::binary);
    f.read((char *)b.data(), (std::streamsize)n);
    if ((size_t)f.gcount() != n) throw std::runtime_error("short read: " + p);
    return b;
}

template <class T>
static void write_file(const std::string &p, const std::vector<T> &v)
{
    std::ofstream f(p, std::ios::binary);
    f.write((const char *)v.data(), (std::streamsize)(v.size() * sizeof(T)));
}

static int bench(char **argv)
{
    using clk = std::chrono::steady_clock;
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]);
    const int nimg = std::atoi(argv[5]), nframes = std::atoi(argv[6]), nfeat = std::atoi(argv[7]);
    const size_t px = (size_t)w * h;
    std::vector<uint8_t> imgs = read_file(argv[4], px * (size_t)nimg);
    orbg_compat::Extractor ext(nfeat, 1.2f, 8, 20, 7);
    orbg_compat::Matcher matcher(0.9f, true, ext.context());
    std::vector<orbg_keypoint> kp[2];
    std::vector<uint8_t> ds[2];
    std::vector<float> prev;
    std::vector<int> m12;
    std::vector<double> lat, lext;
    int n[2] = {0, 0};
    long matches = 0;
    for (int t = -3; t < nframes; t++) {  // three warm-up frames
        const int cur = (t + 3) & 1, old = cur ^ 1;
        const auto t0 = clk::now();
        n[cur] = ext(imgs.data() + px * (size_t)(((t % nimg) + nimg) % nimg), w, h, (size_t)w,
                     kp[cur], ds[cur]);
        const auto t1 = clk::now();
        if (t > -3) {
            prev.resize(2 * (size_t)n[old]);
            for (int i = 0; i < n[old]; i++) {
                prev[2 * i] = kp[old][i].x;
                prev[2 * i + 1] = kp[old][i].y;
            }
            orbg_compat::FrameView F1{kp[old].data(), ds[old].data(), n[old],
                                      {0.f, (float)w, 0.f, (float)h}};
            orbg_compat::FrameView F2{kp[cur].data(), ds[cur].data(), n[cur],
                                      {0.f, (float)w, 0.f, (float)h}};
            matches += matcher.SearchForInitialization(F1, F2, prev, m12, 100);
        }
        const auto t2 = clk::now();
        if (t >= 0) {
            lat.push_back(std::chrono::duration<double, std::milli>(t2 - t0).count());
            lext.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
        }
    }
    auto pct = [](std::vector<double> v, double q) {
        std::sort(v.begin(), v.end());
        return v[std::min(v.size() - 1, (size_t)(q * (double)v.size()))];
    };
    double mean = 0;
    for (double v : lat) mean += v;
    mean /= (double)std::max<size_t>(lat.size(), 1);
    std::printf("{\"frames\": %d, \"ms_per_frame\": {\"mean\": %.4f, \"p50\": %.4f, "
                "\"p90\": %.4f}, \"extract_ms_per_frame\": {\"p50\": %.4f}, "
                "\"match_ms_per_frame\": {\"p50\": %.4f}, \"frames_per_s\": %.1f, "
                "\"matches_per_frame\": %.1f}\n",
                nframes, mean, pct(lat, 0.5), pct(lat, 0.9), pct(lext, 0.5),
                pct(lat, 0.5) - pct(lext, 0.5), 1e3 / mean, (double)matches / (nframes + 2));
    return 0;
}

int main(int argc, char **argv)
{
    if (argc >= 2 && std::string(argv[1]) == "nogpu") {
        try {
            orbg_compat::Extractor e(2000, 1.2f, 8, 20, 7);
            std::cerr << "constructor succeeded without a GPU\n";
            return 1;
        } catch (const orbg_compat::Error &err) {
            std::cout << "no-gpu ok (" << err.code << "): " << err.what() << "\n";
            return err.code == ORBG_EIO ? 0 : 2;
        }
    }
    if (argc >= 8 && std::string(argv[1]) == "bench") return bench(argv);
    if (argc < 8 || std::string(argv[1]) != "run") {
        std::cerr << "usage: compat_selftest nogpu | run w h f0 f1 outdir nfeatures\n";
        return 2;
    }
    const int w = std::atoi(argv[2]), h = std::atoi(argv[3]);
    const std::string out = argv[6];
    const int nfeat = std::atoi(argv[7]);
    std::vector<uint8_t> im0 = read_file(argv[4], (size_t)w * h);
    std::vector<uint8_t> im1 = read_file(argv[5], (size_t)w * h);

    // Tracking.cc:127 / Frame.cc:310-316: one extractor per role, reused every frame
    orbg_compat::Extractor ext(nfeat, 1.2f, 8, 20, 7);
    std::vector<orbg_keypoint> k0, k1;
    std::vector<uint8_t> d0, d1;
    // empty image: outputs untouched (ORBextractor.cc:1333-1334)
    k0.resize(3);
    if (ext(nullptr, 0, 0, 0, k0, d0) != 0 || k0.size() != 3) return 3;
    const int n0 = ext(im0.data(), w, h, (size_t)w, k0, d0);
    const int n1 = ext(im1.data(), w, h, (size_t)w, k1, d1);
    int lw = 0, lh = 0;
    std::vector<uint8_t> top = ext.ImagePyramidLevel(ext.GetLevels() - 1, &lw, &lh);
    if ((int)top.size() != lw * lh || lw <= 0) return 4;

    // Tracking::MonocularInitialization (Tracking.cc:781-782): ORBmatcher(0.9, true),
    // vbPrevMatched = F1 keypoint positions, window 100
    orbg_compat::Matcher matcher(0.9f, true, ext.context());
    orbg_compat::FrameView F1{k0.data(), d0.data(), n0, {0.f, (float)w, 0.f, (float)h}};
    orbg_compat::FrameView F2{k1.data(), d1.data(), n1, {0.f, (float)w, 0.f, (float)h}};
    std::vector<float> prev(2 * (size_t)n0);
    for (int i = 0; i < n0; i++) {
        prev[2 * i] = k0[i].x;
        prev[2 * i + 1] = k0[i].y;
    }
    std::vector<int> m12;
    const int nm = matcher.SearchForInitialization(F1, F2, prev, m12, 100);
    std::vector<int32_t> bi, bd, sd;
    matcher.HammingKnn2(d1.data(), n1, d0.data(), n0, bi, bd, sd);
    std::vector<int32_t> knn(3 * (size_t)n1);
    for (int i = 0; i < n1; i++) {
        knn[3 * i] = bi[i];
        knn[3 * i + 1] = bd[i];
        knn[3 * i + 2] = sd[i];
    }
    if (n0 > 1 && orbg_compat::Matcher::DescriptorDistance(d0.data(), d0.data()) != 0) return 5;

    // stereo Frame constructor on (frame0, frame1) as (left, right), KITTI00 bf / fx
    const float bf = 386.1448f, fx = 718.856f;
    orbg_compat::StereoFrame SF(ext, im0.data(), im1.data(), w, h, (size_t)w, bf, bf / fx);
    if (SF.N != n0 || (int)SF.mvDepth.size() != n0) return 6;
    write_file(out + "/stereo_ur", SF.mvuRight);
    write_file(out + "/stereo_depth", SF.mvDepth);

    write_file(out + "/kps0", k0);
    write_file(out + "/kps1", k1);
    write_file(out + "/desc0", d0);
    write_file(out + "/desc1", d1);
    write_file(out + "/m12", std::vector<int32_t>(m12.begin(), m12.end()));
    write_file(out + "/knn", knn);
    std::ofstream(out + "/nm.txt") << nm << "\n";
    std::cout << "compat ok: " << n0 << " + " << n1 << " keypoints, " << nm << " matches\n";
    return 0;
}
