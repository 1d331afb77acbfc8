// Developer tool: cycle split of SearchForInitialization's single-pair resolver
// (k_init_resolve_single) over the C++ drop-in loop of compat_selftest's bench, from the
// counters of a developer build (make OUT=../lib/dev DEV=1).
//   g++ -std=c++17 -O2 -I include -I orb_slam2_test_amd/compat tools/resolve_prof.cpp \
//       -L orb_slam2_test_amd/lib/dev -lorbg -Wl,-rpath,<repo>/orb_slam2_test_amd/lib/dev -o ...
//   resolve_prof <w> <h> <frames.raw> <nimages> <nframes> <nfeatures>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#include "orbg_compat.hpp"

extern "C" int orbg_dev_resolve_prof(unsigned long long out[8], int reset);

int main(int argc, char **argv)
{
    if (argc < 7) return 2;
    const int w = std::atoi(argv[1]), h = std::atoi(argv[2]);
    const int nimg = std::atoi(argv[4]), nframes = std::atoi(argv[5]), nfeat = std::atoi(argv[6]);
    const size_t px = (size_t)w * h;
    std::vector<uint8_t> imgs(px * nimg);
    std::ifstream f(argv[3], std::ios::binary);
    f.read((char *)imgs.data(), (std::streamsize)imgs.size());
    orbg_compat::Extractor ext(nfeat, 1.2f, 8, 20, 7);
    orbg_compat::Matcher matcher(0.9f, true, ext.context());
    std::vector<orbg_keypoint> kp[2];
    std::vector<uint8_t> ds[2];
    std::vector<float> prev;
    std::vector<int> m12;
    int n[2] = {0, 0};
    unsigned long long c[8];
    for (int t = -3; t < nframes; t++) {
        if (t == 0) orbg_dev_resolve_prof(c, 1);
        const int cur = (t + 3) & 1, old = cur ^ 1;
        n[cur] = ext(imgs.data() + px * (size_t)(((t % nimg) + nimg) % nimg), w, h, (size_t)w,
                     kp[cur], ds[cur]);
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
            matcher.SearchForInitialization(F1, F2, prev, m12, 100);
        }
    }
    orbg_dev_resolve_prof(c, 0);
    const double calls = (double)(c[7] ? c[7] : 1);
    std::printf("{\"calls\": %llu, \"cycles_per_call\": {\"init\": %.0f, \"chunk_walk\": %.0f, "
                "\"rescan\": %.0f, \"chunk_barrier\": %.0f, \"tail\": %.0f}, "
                "\"rounds_per_call\": %.2f, \"rescans_per_call\": %.2f}\n",
                c[7], c[0] / calls, c[1] / calls, c[2] / calls, c[3] / calls, c[4] / calls,
                c[5] / calls, c[6] / calls);
    return 0;
}
