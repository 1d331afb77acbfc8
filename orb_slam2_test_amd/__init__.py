"""orb_slam2_test_amd: MI355X-native (gfx950) ORB-SLAM2 per-frame hot path.

ORBextractor (pyramid, FAST-9 + quadtree distribution, IC_Angle, rBRIEF), ORBmatcher's
Hamming matching (DescriptorDistance, brute-force 2-NN, SearchForInitialization),
Frame::ComputeStereoMatches, the tracking matchers (SearchByProjection), PoseOptimization,
DBoW2's vocabulary transform (Frame::ComputeBoW), the LBA Schur solve and
the per-edge arithmetic of Optimizer::LocalBundleAdjustment, as hand-written HIP
kernels behind the C ABI in include/orbg.h (lib/liborbg.so).  The Python classes mirror
the reference's C++ interfaces; see DESIGN.md.
"""
from ._lib import KP_DTYPE, EDGE_DTYPE, EDGE_OUT_DTYPE, POSE_DTYPE, LIB_PATH  # noqa: F401
from .orbextractor import ORBextractor  # noqa: F401
from .orbmatcher import Frame, MapPointProjections, ORBmatcher  # noqa: F401
from .frame import StereoFrame  # noqa: F401
from .optimizer import PoseOptimization, linearize_local_ba  # noqa: F401
from .vocabulary import ORBVocabulary, BowVector, FeatureVector  # noqa: F401

__all__ = ["ORBextractor", "ORBmatcher", "Frame", "MapPointProjections", "StereoFrame", "PoseOptimization", "linearize_local_ba",
           "ORBVocabulary", "BowVector", "FeatureVector", "KP_DTYPE",
           "EDGE_DTYPE", "EDGE_OUT_DTYPE", "POSE_DTYPE"]
