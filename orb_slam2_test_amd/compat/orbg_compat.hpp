// orbg_compat.hpp -- header-only C++ host layer over the liborbg C ABI (include/orbg.h).
//
// Two layers:
//   orbg_compat::Extractor / Matcher / linearize_local_ba
//       RAII C++ classes over plain buffers (std::vector), always compiled.  They keep the
//       reference's names, argument meaning and error behaviour:
//         ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
//                                           include/ORBextractor.h:64-65
//         operator()(image, keypoints, descriptors) ... include/ORBextractor.h:74-76,
//             src/ORBextractor.cc:1330-1397 (empty image: outputs untouched; 0 keypoints:
//             empty descriptors)
//         GetLevels/GetScaleFactor/GetScaleFactors/GetInverseScaleFactors/
//         GetScaleSigmaSquares/GetInverseScaleSigmaSquares ... include/ORBextractor.h:78-98
//         mvImagePyramid (downloaded on demand) ............ include/ORBextractor.h:101
//         ORBmatcher(nnratio, checkOri), DescriptorDistance, SearchForInitialization
//                                           include/ORBmatcher.h:47,51,128
//         StereoFrame: the stereo Frame constructor (two extractions + ComputeStereoMatches)
//                                           src/Frame.cc:86-161, 619-834
//   ORB_SLAM2::ORBextractor (only when OpenCV headers are present)
//       the reference's exact cv::InputArray / std::vector<cv::KeyPoint> / cv::OutputArray
//       signatures, so Tracking.cc and Frame.cc compile unchanged.  This
//       image has no OpenCV: tests/test_compat_ref.py compiles and runs that block against
//       tests/compat_stub/, a test-only stand-in of the cv:: subset it uses.
//   orbg_reference.hpp: ORBmatcher / Optimizer call sites over the reference's own Frame,
//       KeyFrame and MapPoint classes.
//
// Errors: the C ABI returns negative errno codes; this layer throws orbg_compat::Error
// (std::runtime_error) with orbg_last_error()'s message.  There is no CPU fallback: without
// a HIP device the constructor throws.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "orbg.h"

namespace orbg_compat {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &what)
        : std::runtime_error(what + ": " + orbg_last_error()), code(c) {}
};

inline void check(int rc, const char *what)
{
    if (rc != ORBG_OK) throw Error(rc, what);
}

class Extractor {
public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    Extractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
              int device = 0)
    {
        orbg_params p;
        orbg_params_default(&p);
        p.nfeatures = nfeatures;
        p.scale_factor = scaleFactor;
        p.nlevels = nlevels;
        p.ini_th_fast = iniThFAST;
        p.min_th_fast = minThFAST;
        check(orbg_create(device, &p, &ctx_), "orbg_create");
        int32_t nl = 0;
        float sf = 0.f;
        scale_.resize(ORBG_MAX_LEVELS);
        inv_scale_.resize(ORBG_MAX_LEVELS);
        sigma2_.resize(ORBG_MAX_LEVELS);
        inv_sigma2_.resize(ORBG_MAX_LEVELS);
        fpl_.resize(ORBG_MAX_LEVELS);
        umax_.resize(16);
        check(orbg_get_scale_tables(ctx_, &nl, &sf, scale_.data(), inv_scale_.data(),
                                    sigma2_.data(), inv_sigma2_.data(), fpl_.data(),
                                    umax_.data()),
              "orbg_get_scale_tables");
        nlevels_ = nl;
        scale_factor_ = sf;
        for (auto *v : {&scale_, &inv_scale_, &sigma2_, &inv_sigma2_}) v->resize(nl);
        fpl_.resize(nl);
    }
    ~Extractor() { orbg_destroy(ctx_); }
    Extractor(const Extractor &) = delete;
    Extractor &operator=(const Extractor &) = delete;

    // operator()(image, mask, keypoints, descriptors): `image` is 8-bit grey, `step` bytes
    // per row.  Returns the number of keypoints.  An empty image (w or h == 0) returns 0 and
    // leaves both outputs untouched, like the reference (ORBextractor.cc:1333-1334).
    int operator()(const uint8_t *image, int w, int h, size_t step,
                   std::vector<orbg_keypoint> &keypoints, std::vector<uint8_t> &descriptors)
    {
        if (!image || w <= 0 || h <= 0) return 0;
        int n = 0;
        if (cap_ == 0) cap_ = 4096;
        for (;;) {
            keypoints.resize(cap_);
            descriptors.resize((size_t)cap_ * 32);
            const int rc = orbg_extract(ctx_, image, w, h, step, keypoints.data(),
                                        descriptors.data(), cap_, &n);
            if (rc == ORBG_ERANGE) {
                cap_ = n;
                continue;
            }
            check(rc, "orbg_extract");
            break;
        }
        // the context's per-frame output capacity (known after the first extraction): every
        // later frame fits it, and the resize above then value-initialises only the few
        // entries between the last frame's count and that capacity, not up to 4096
        int32_t fc = 0;
        if (orbg_batch_outputs(ctx_, nullptr, nullptr, nullptr, &fc) == ORBG_OK && fc > 0)
            cap_ = fc;
        keypoints.resize(n);
        descriptors.resize((size_t)n * 32);
        levels_valid_ = true;
        return n;
    }

    int GetLevels() const { return nlevels_; }
    float GetScaleFactor() const { return scale_factor_; }
    std::vector<float> GetScaleFactors() const { return scale_; }
    std::vector<float> GetInverseScaleFactors() const { return inv_scale_; }
    std::vector<float> GetScaleSigmaSquares() const { return sigma2_; }
    std::vector<float> GetInverseScaleSigmaSquares() const { return inv_sigma2_; }
    const std::vector<int32_t> &FeaturesPerLevel() const { return fpl_; }

    // mvImagePyramid[level] of the last operator() call (downloaded from HBM)
    std::vector<uint8_t> ImagePyramidLevel(int level, int *w, int *h) const
    {
        if (!levels_valid_) throw Error(ORBG_EINVAL, "no image extracted yet");
        int lw = 0, lh = 0;
        check(orbg_get_level(ctx_, 0, level, nullptr, 0, &lw, &lh), "orbg_get_level(size)");
        std::vector<uint8_t> buf((size_t)lw * lh);
        check(orbg_get_level(ctx_, 0, level, buf.data(), (size_t)lw, &lw, &lh), "orbg_get_level");
        if (w) *w = lw;
        if (h) *h = lh;
        return buf;
    }

    orbg_ctx *context() const { return ctx_; }

private:
    orbg_ctx *ctx_ = nullptr;
    int nlevels_ = 0;
    float scale_factor_ = 0.f;
    int cap_ = 0;
    bool levels_valid_ = false;
    std::vector<float> scale_, inv_scale_, sigma2_, inv_sigma2_;
    std::vector<int32_t> fpl_, umax_;
};

// Minimal frame view SearchForInitialization needs: mvKeysUn (x, y, angle, octave),
// mDescriptors (N x 32) and the image bounds Frame::mnMinX/mnMaxX/mnMinY/mnMaxY.
struct FrameView {
    const orbg_keypoint *keys = nullptr;
    const uint8_t *desc = nullptr;
    int n = 0;
    orbg_bounds bounds{0.f, 0.f, 0.f, 0.f};
};

class Matcher {
public:
    static const int TH_LOW = 50;
    static const int TH_HIGH = 100;
    static const int HISTO_LENGTH = 30;

    explicit Matcher(float nnratio = 0.6f, bool checkOri = true, orbg_ctx *ctx = nullptr)
        : nnratio_(nnratio), check_ori_(checkOri), ctx_(ctx) {}

    static int DescriptorDistance(const uint8_t *a, const uint8_t *b)
    {
        return orbg_descriptor_distance(a, b);
    }

    // SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
    // vbPrevMatched: 2*F1.n floats (x, y), updated in place; vnMatches12 resized to F1.n.
    int SearchForInitialization(const FrameView &F1, const FrameView &F2,
                                std::vector<float> &vbPrevMatched,
                                std::vector<int> &vnMatches12, int windowSize = 10) const
    {
        if (!ctx_) throw Error(ORBG_EINVAL, "Matcher needs an orbg context");
        if ((int)vbPrevMatched.size() < 2 * F1.n)
            throw Error(ORBG_EINVAL, "vbPrevMatched smaller than 2 * F1.n");
        static_assert(sizeof(int) == sizeof(int32_t), "vnMatches12 is written in place");
        vnMatches12.resize(F1.n);  // every entry is written by the call
        int nm = 0;
        check(orbg_search_for_initialization(ctx_, F1.keys, F1.desc, F1.n, F2.keys, F2.desc,
                                             F2.n, &F2.bounds, vbPrevMatched.data(),
                                             (int32_t *)vnMatches12.data(), windowSize, nnratio_,
                                             check_ori_ ? 1 : 0, &nm),
              "orbg_search_for_initialization");
        return nm;
    }

    // all-pairs best/second (query -> train), strict <, lowest index on ties
    void HammingKnn2(const uint8_t *qdesc, int nq, const uint8_t *tdesc, int nt,
                     std::vector<int32_t> &best_idx, std::vector<int32_t> &best,
                     std::vector<int32_t> &second) const
    {
        if (!ctx_) throw Error(ORBG_EINVAL, "Matcher needs an orbg context");
        best_idx.resize(nq);
        best.resize(nq);
        second.resize(nq);
        check(orbg_hamming_knn2(ctx_, qdesc, nq, tdesc, nt, best_idx.data(), best.data(),
                                second.data()),
              "orbg_hamming_knn2");
    }

private:
    float nnratio_;
    bool check_ori_;
    orbg_ctx *ctx_;
};

// The stereo Frame constructor (Frame.cc:86-161): both extractions + ComputeStereoMatches.
// mb is Frame::mb, read uninitialised by the reference (Frame.cc:661 vs :148); pass bf / fx.
struct StereoFrame {
    std::vector<orbg_keypoint> mvKeys, mvKeysRight;
    std::vector<uint8_t> mDescriptors, mDescriptorsRight;  // N x 32, Nr x 32
    std::vector<float> mvuRight, mvDepth;                  // -1 where unmatched
    int N = 0;
    float mbf = 0.f, mb = 0.f;

    StereoFrame(Extractor &ext, const uint8_t *imLeft, const uint8_t *imRight, int w, int h,
                size_t step, float bf, float mb_)
        : mbf(bf), mb(mb_)
    {
        int cap = 4096, nl = 0, nr = 0;
        for (;;) {
            mvKeys.resize(cap);
            mvKeysRight.resize(cap);
            mDescriptors.resize((size_t)cap * 32);
            mDescriptorsRight.resize((size_t)cap * 32);
            mvuRight.resize(cap);
            mvDepth.resize(cap);
            const int rc = orbg_stereo_frame(ext.context(), imLeft, imRight, w, h, step, bf, mb_,
                                             mvKeys.data(), mDescriptors.data(), cap, &nl,
                                             mvKeysRight.data(), mDescriptorsRight.data(), cap,
                                             &nr, mvuRight.data(), mvDepth.data());
            if (rc == ORBG_ERANGE) {
                cap = nl > nr ? nl : nr;
                continue;
            }
            check(rc, "orbg_stereo_frame");
            break;
        }
        N = nl;
        mvKeys.resize(nl);
        mDescriptors.resize((size_t)nl * 32);
        mvKeysRight.resize(nr);
        mDescriptorsRight.resize((size_t)nr * 32);
        mvuRight.resize(nl);
        mvDepth.resize(nl);
    }
};

// Optimizer::LocalBundleAdjustment's per-edge arithmetic (computeActiveErrors +
// buildSystem for EdgeSE3ProjectXYZ / EdgeStereoSE3ProjectXYZ, Optimizer.cc:762-851).
struct BASystem {
    std::vector<orbg_edge_out> edges;
    std::vector<double> hpose, bpose, hpoint, bpoint;
};

inline BASystem linearize_local_ba(orbg_ctx *ctx, const std::vector<orbg_pose> &poses,
                                   const std::vector<double> &points,
                                   const std::vector<orbg_edge> &edges)
{
    BASystem s;
    const int np = (int)poses.size(), nx = (int)(points.size() / 3), ne = (int)edges.size();
    s.edges.resize(ne);
    s.hpose.resize((size_t)np * 36);
    s.bpose.resize((size_t)np * 6);
    s.hpoint.resize((size_t)nx * 9);
    s.bpoint.resize((size_t)nx * 3);
    check(orbg_ba_linearize(ctx, poses.data(), np, points.data(), nx, edges.data(), ne,
                            s.edges.data(), s.hpose.data(), s.bpose.data(), s.hpoint.data(),
                            s.bpoint.data()),
          "orbg_ba_linearize");
    return s;
}

}  // namespace orbg_compat

#if defined(ORBG_WITH_OPENCV) || __has_include(<opencv2/core/core.hpp>)
#include <opencv2/core/core.hpp>
#include <opencv2/features2d/features2d.hpp>

namespace ORB_SLAM2 {

// Drop-in for include/ORBextractor.h: same public surface, backed by liborbg.
class ORBextractor {
    class LazyPyramid;

public:
    enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST)
        : mvImagePyramid(this), ext_(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST),
          levels_(nlevels), fresh_(nlevels, false)
    {
    }
    ~ORBextractor() {}
    ORBextractor(const ORBextractor &) = delete;
    ORBextractor &operator=(const ORBextractor &) = delete;

    void operator()(cv::InputArray image, cv::InputArray mask,
                    std::vector<cv::KeyPoint> &keypoints, cv::OutputArray descriptors)
    {
        (void)mask;
        if (image.empty()) return;
        cv::Mat im = image.getMat();
        CV_Assert(im.type() == CV_8UC1);
        // the staging vectors persist across frames (no allocation per frame)
        std::vector<orbg_keypoint> &kps = kps_;
        std::vector<uint8_t> &desc = desc_;
        const int n = ext_(im.data, im.cols, im.rows, im.step[0], kps, desc);
        keypoints.clear();
        keypoints.reserve(n);
        for (const orbg_keypoint &k : kps)
            keypoints.emplace_back(k.x, k.y, k.size, k.angle, k.response, k.octave, k.class_id);
        if (n == 0) {
            descriptors.release();
        } else {
            descriptors.create(n, 32, CV_8U);
            std::memcpy(descriptors.getMat().data, desc.data(), desc.size());
        }
        // the pyramid stays in HBM: only stereo callers read it (Frame.cc:626, 738)
        fresh_.assign(fresh_.size(), false);
    }

    int inline GetLevels() { return ext_.GetLevels(); }
    float inline GetScaleFactor() { return ext_.GetScaleFactor(); }
    std::vector<float> inline GetScaleFactors() { return ext_.GetScaleFactors(); }
    std::vector<float> inline GetInverseScaleFactors() { return ext_.GetInverseScaleFactors(); }
    std::vector<float> inline GetScaleSigmaSquares() { return ext_.GetScaleSigmaSquares(); }
    std::vector<float> inline GetInverseScaleSigmaSquares()
    {
        return ext_.GetInverseScaleSigmaSquares();
    }

private:
    std::vector<orbg_keypoint> kps_;
    std::vector<uint8_t> desc_;
    // mvImagePyramid[l]: level l of the last operator() call, downloaded from HBM on its first
    // access after that call (std::vector<cv::Mat>'s indexing and size in the reference)
    class LazyPyramid {
    public:
        explicit LazyPyramid(ORBextractor *o) : o_(o) {}
        cv::Mat &operator[](size_t l) { return o_->level(l); }
        const cv::Mat &operator[](size_t l) const { return o_->level(l); }
        size_t size() const { return o_->levels_.size(); }

    private:
        ORBextractor *o_;
    };

public:
    LazyPyramid mvImagePyramid;

private:
    cv::Mat &level(size_t l) const
    {
        if (!fresh_[l]) {
            int w = 0, h = 0;
            std::vector<uint8_t> lv = ext_.ImagePyramidLevel((int)l, &w, &h);
            levels_[l] = cv::Mat(h, w, CV_8U, lv.data()).clone();
            fresh_[l] = true;
        }
        return levels_[l];
    }

    orbg_compat::Extractor ext_;
    mutable std::vector<cv::Mat> levels_;
    mutable std::vector<bool> fresh_;
};

}  // namespace ORB_SLAM2
#endif
