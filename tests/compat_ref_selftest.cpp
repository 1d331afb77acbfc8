// tests/compat_ref_selftest.cpp -- TEST PROGRAM: the reference-facing drop-in layer
// (orb_slam2_test_amd/compat/orbg_compat.hpp's ORB_SLAM2::ORBextractor and
// orbg_reference.hpp) driven the way Tracking.cc / Optimizer.cc call it, on stand-ins of the
// reference's Frame / KeyFrame / MapPoint (same member names and types) and the test-only
// cv:: subset in tests/compat_stub/.  Built by tests/test_compat_ref.py (CPU: it compiles);
// run there on the GPU.  usage: compat_ref_selftest img1.raw img2.raw w h
#include <cmath>
#include <cstdio>
#include <fstream>
#include <list>
#include <map>
#include <vector>

#include <opencv2/core/core.hpp>

#include "orbg_compat.hpp"
#include "orbg_reference.hpp"

#define REQUIRE(c)                                                                           \
    do {                                                                                     \
        if (!(c)) {                                                                          \
            std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #c);              \
            return 1;                                                                        \
        }                                                                                    \
    } while (0)

struct KeyFrame;

struct MapPoint {  // include/MapPoint.h members the hot path reads
    long unsigned int mnId = 0;
    cv::Mat pos, desc;
    bool bad = false;
    bool mbTrackInView = false;
    float mTrackProjX = 0, mTrackProjY = 0, mTrackProjXR = -1;
    int mnTrackScaleLevel = 0;
    float mTrackViewCos = 1;
    std::map<KeyFrame *, size_t> obs;
    cv::Mat GetWorldPos() const { return pos.clone(); }
    cv::Mat GetDescriptor() const { return desc.clone(); }
    int Observations() const { return (int)obs.size(); }
    bool isBad() const { return bad; }
    std::map<KeyFrame *, size_t> GetObservations() const { return obs; }
};

struct Frame {  // include/Frame.h
    static float fx, fy, cx, cy, mnMinX, mnMaxX, mnMinY, mnMaxY;
    int N = 0;
    std::vector<cv::KeyPoint> mvKeys, mvKeysUn;
    std::vector<float> mvuRight, mvInvLevelSigma2;
    cv::Mat mDescriptors, mTcw;
    std::vector<MapPoint *> mvpMapPoints;
    std::vector<bool> mvbOutlier;
    float mbf = 0, mb = 0;
    void SetPose(cv::Mat T) { mTcw = T.clone(); }
};
float Frame::fx, Frame::fy, Frame::cx, Frame::cy, Frame::mnMinX, Frame::mnMaxX, Frame::mnMinY,
    Frame::mnMaxY;

struct KeyFrame {  // include/KeyFrame.h
    long unsigned int mnId = 0;
    float fx, fy, cx, cy, mbf;
    std::vector<cv::KeyPoint> mvKeysUn;
    std::vector<float> mvuRight, mvInvLevelSigma2;
    cv::Mat Tcw;
    cv::Mat GetPose() const { return Tcw.clone(); }
    bool isBad() const { return false; }
};

static std::vector<uint8_t> read_raw(const char *path, size_t n)
{
    std::vector<uint8_t> b(n);
    std::ifstream f(path, std::ios::binary);
    f.read((char *)b.data(), (std::streamsize)n);
    return b;
}

int main(int argc, char **argv)
{
    if (argc < 5) return 2;
    const int w = atoi(argv[3]), h = atoi(argv[4]);
    std::vector<uint8_t> im1 = read_raw(argv[1], (size_t)w * h), im2 = read_raw(argv[2], (size_t)w * h);
    cv::Mat I1(h, w, CV_8U, im1.data()), I2(h, w, CV_8U, im2.data());

    // ---- ORBextractor as Frame::ExtractORB calls it (Frame.cc:310-316) ----
    ORB_SLAM2::ORBextractor ext(2000, 1.2f, 8, 20, 7);
    Frame F1, F2;
    ext(I1, cv::Mat(), F1.mvKeys, F1.mDescriptors);
    ext(I2, cv::Mat(), F2.mvKeys, F2.mDescriptors);
    REQUIRE(F1.mvKeys.size() > 500 && F2.mvKeys.size() > 500);
    REQUIRE(F1.mDescriptors.rows == (int)F1.mvKeys.size() && F1.mDescriptors.cols == 32);
    // the pyramid is downloaded on first access, and is the last image's (level 0 = input)
    REQUIRE(ext.mvImagePyramid.size() == 8);
    const cv::Mat &L0 = ext.mvImagePyramid[0];
    REQUIRE(L0.rows == h && L0.cols == w);
    REQUIRE(std::memcmp(L0.ptr<uint8_t>(h / 2), im2.data() + (size_t)(h / 2) * w, w) == 0);
    REQUIRE(ext.mvImagePyramid[1].cols == (int)std::lround(w / 1.2));
    const std::vector<float> inv2 = ext.GetInverseScaleSigmaSquares();
    Frame::fx = Frame::fy = 718.856f;
    Frame::cx = 607.1928f;
    Frame::cy = 185.2157f;
    Frame::mnMinX = 0;
    Frame::mnMaxX = (float)w;
    Frame::mnMinY = 0;
    Frame::mnMaxY = (float)h;
    for (Frame *F : {&F1, &F2}) {
        F->N = (int)F->mvKeys.size();
        F->mvKeysUn = F->mvKeys;
        F->mvuRight.assign(F->N, -1.f);
        F->mvpMapPoints.assign(F->N, nullptr);
        F->mvbOutlier.assign(F->N, false);
        F->mvInvLevelSigma2 = inv2;
        F->mTcw = cv::Mat::eye(4, 4, CV_32F);
        F->mbf = 386.1448f;
        F->mb = F->mbf / Frame::fx;
    }
    orbg_ctx *ctx = orbg_compat::ref::default_ctx();

    // ---- ORBmatcher(0.9, true).SearchForInitialization (Tracking::MonocularInitialization) ----
    std::vector<cv::Point2f> prev(F1.N);
    for (int i = 0; i < F1.N; i++) prev[i] = F1.mvKeysUn[i].pt;
    std::vector<int> m12;
    const int nsfi = orbg_compat::ref::SearchForInitialization(ctx, 0.9f, true, F1, F2, prev, m12, 100);
    {   // the same call through the plain-buffer layer
        std::vector<orbg_keypoint> k1 = orbg_compat::ref::keys_of(F1.mvKeysUn),
                                   k2 = orbg_compat::ref::keys_of(F2.mvKeysUn);
        orbg_compat::FrameView v1{k1.data(), F1.mDescriptors.data, F1.N, {0, (float)w, 0, (float)h}};
        orbg_compat::FrameView v2{k2.data(), F2.mDescriptors.data, F2.N, {0, (float)w, 0, (float)h}};
        std::vector<float> p2(2 * F1.N);
        for (int i = 0; i < F1.N; i++) {
            p2[2 * i] = F1.mvKeysUn[i].pt.x;
            p2[2 * i + 1] = F1.mvKeysUn[i].pt.y;
        }
        std::vector<int> r12;
        orbg_compat::Matcher m(0.9f, true, ctx);
        REQUIRE(m.SearchForInitialization(v1, v2, p2, r12, 100) == nsfi);
        REQUIRE(r12 == m12);
        for (int i = 0; i < F1.N; i++) REQUIRE(prev[i].x == p2[2 * i] && prev[i].y == p2[2 * i + 1]);
    }
    REQUIRE(nsfi > 100);
    int nm12 = 0;
    for (int v : m12) nm12 += v >= 0;
    REQUIRE(nm12 == nsfi);

    // ---- SearchByProjection(CurrentFrame, LastFrame, 15, mono) (TrackWithMotionModel) ----
    // map points of F1's keypoints back-projected at 10 m with the identity pose, each
    // observed by one key frame (a matched slot then counts as taken, ORBmatcher.cc:1602)
    KeyFrame K[3];
    std::vector<MapPoint> mps(F1.N);
    for (int i = 0; i < F1.N; i++) {
        MapPoint &mp = mps[i];
        mp.mnId = 100 + i;
        mp.pos = cv::Mat(3, 1, CV_32F);
        mp.pos.at<float>(0) = (F1.mvKeysUn[i].pt.x - Frame::cx) * 10.f / Frame::fx;
        mp.pos.at<float>(1) = (F1.mvKeysUn[i].pt.y - Frame::cy) * 10.f / Frame::fy;
        mp.pos.at<float>(2) = 10.f;
        mp.desc = cv::Mat(1, 32, CV_8U);
        std::memcpy(mp.desc.data, F1.mDescriptors.ptr<uint8_t>(i), 32);
        mp.obs[&K[2]] = (size_t)i;
        F1.mvpMapPoints[i] = &mp;
    }
    const int nproj = orbg_compat::ref::SearchByProjection(ctx, true, F2, F1, 15.f, true);
    int nset = 0;
    for (int i = 0; i < F2.N; i++) {
        if (!F2.mvpMapPoints[i]) continue;
        nset++;
        const MapPoint *pMP = F2.mvpMapPoints[i];
        const int j = (int)(pMP - mps.data());
        REQUIRE(j >= 0 && j < F1.N);
        REQUIRE(orbg_descriptor_distance(F2.mDescriptors.ptr<uint8_t>(i), pMP->desc.data) <= 100);
    }
    REQUIRE(nproj > 50 && nset == nproj);

    // ---- Optimizer::PoseOptimization(&CurrentFrame) ----
    const int ninl = orbg_compat::ref::PoseOptimization(ctx, &F2);
    REQUIRE(ninl > 20 && ninl <= nproj);
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 4; c++) REQUIRE(std::isfinite(F2.mTcw.at<float>(r, c)));
    REQUIRE(std::fabs(F2.mTcw.at<float>(0, 0) - 1.f) < 0.05f);

    // ---- LocalBundleAdjustment window + BlockSolver<6,3> layout ----
    for (int k = 0; k < 3; k++) {
        K[k].mnId = (long unsigned)(2 - k) * 5;  // ids not in list order: hessian order by id
        K[k].fx = K[k].fy = Frame::fx;
        K[k].cx = Frame::cx;
        K[k].cy = Frame::cy;
        K[k].mbf = F1.mbf;
        K[k].mvKeysUn = F1.mvKeysUn;
        K[k].mvuRight.assign(F1.N, -1.f);
        for (int i = 0; i < F1.N; i += 3) K[k].mvuRight[i] = F1.mvKeysUn[i].pt.x - 20.f;  // stereo
        K[k].mvInvLevelSigma2 = inv2;
        K[k].Tcw = cv::Mat::eye(4, 4, CV_32F);
        K[k].Tcw.at<float>(0, 3) = 0.01f * (float)k;  // small baseline: nonzero residuals
    }
    std::list<KeyFrame *> local{&K[0], &K[1]}, fixed{&K[2]};
    std::list<MapPoint *> points;
    for (int i = 0; i < 300 && i < F1.N; i++) {
        for (int k = 0; k < 3; k++) mps[i].obs[&K[k]] = (size_t)i;
        points.push_back(&mps[i]);
    }
    auto win = orbg_compat::ref::build_lba_window(local, fixed, points);
    REQUIRE(win.poses.size() == 3 && win.poses[2].fixed == 1 && win.poses[1].fixed == 0);
    REQUIRE(win.poses[0].fixed == 0 || K[0].mnId == 0);
    REQUIRE(win.edges.size() == 3 * points.size());
    const auto sys = orbg_compat::ref::linearize_lba_window(ctx, win);
    const orbg_compat::BASystem raw = orbg_compat::linearize_local_ba(ctx, win.poses, win.points, win.edges);
    int nfree = 0;
    for (int i = 0; i < 3; i++) nfree += sys.pose_hidx[i] >= 0;
    REQUIRE(sys.b.size() == (size_t)6 * nfree + 3 * points.size());
    REQUIRE(sys.pose_hidx[1] == 0);  // K[1] (id 5) before K[0] (id 10)
    for (int i = 0; i < 3; i++) {
        const int hx = sys.pose_hidx[i];
        if (hx < 0) continue;
        for (int r = 0; r < 6; r++)
            for (int c = 0; c < 6; c++)
            {  // pose blocks are summed over edge slices in either order: 1e-9 relative
                const double a = sys.Hpp[(size_t)hx * 36 + c * 6 + r];
                const double b = raw.hpose[(size_t)i * 36 + r * 6 + c];
                REQUIRE(std::fabs(a - b) <= 1e-9 * (std::fabs(b) + 1e-12));
            }
    }
    REQUIRE(sys.Hpl.size() == (size_t)nfree * points.size());
    REQUIRE(sys.active_robust_chi2 > 0);
    double bn = 0;
    for (double v : sys.b) bn += v * v;
    REQUIRE(bn > 0 && std::isfinite(bn));
    std::printf("compat_ref ok: %d + %d keypoints, SearchForInitialization %d, SearchByProjection %d, "
                "PoseOptimization inliers %d, LBA edges %zu, chi2 %.6g\n",
                F1.N, F2.N, nsfi, nproj, ninl, win.edges.size(), sys.active_robust_chi2);
    return 0;
}
