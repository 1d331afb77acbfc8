#!/usr/bin/env python3
"""The per-frame path Tracking.cc calls (mono_kitti.cc:78-90 -> TrackMonocular -> Frame ->
ORBextractor::operator(), Frame.cc:310-316; MonocularInitialization ->
ORBmatcher::SearchForInitialization, Tracking.cc:664): one frame at a time, host image in,
host keypoints / descriptors / vnMatches12 out, through the C ABI (orbg_extract,
orbg_search_for_initialization).  Timed per frame, next to the oracle (the C restatement)
on one host thread doing the same per-frame work.

usage: single_frame_bench.py [nframes] [w h nfeatures]  -> one JSON line
       single_frame_bench.py --write-frames <path> [nimages] [w h]
           (no GPU call) writes the same synthetic frames as raw bytes for the C++ loop,
           orb_slam2_test_amd/lib/compat_selftest bench <w> <h> <path> <nimages> <nframes>
           <nfeatures> (the drop-in as C++ drives it, no interpreter in the loop)
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def write_frames():
    path = sys.argv[2]
    nimg = int(sys.argv[3]) if len(sys.argv) > 3 else 16
    w, h = (int(v) for v in sys.argv[4:6]) if len(sys.argv) > 5 else (1241, 376)
    from orb_slam2_test_amd import synthetic as S
    frames = S.sequence(nimg, h, w, seed=S.DEFAULT_SEED + 77)
    np.ascontiguousarray(np.stack(frames), np.uint8).tofile(path)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--write-frames":
        return write_frames()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    w, h, nf = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1241, 376, 2000)
    from orb_slam2_test_amd import ORBextractor, ORBmatcher, Frame, synthetic as S
    from oracle import pyoracle as O
    frames = S.sequence(min(n, 64), h, w, seed=S.DEFAULT_SEED + 77)
    ext = ORBextractor(nf, 1.2, 8, 20, 7)
    m = ORBmatcher(0.9, True)

    # warm-up (plans the buffers, loads the code objects)
    for t in range(3):
        ext(frames[t])
    lat, lext = [], []
    t_all = time.perf_counter()
    kprev, dprev = ext(frames[0])
    for t in range(1, n + 1):
        t0 = time.perf_counter()
        k, d = ext(frames[t % len(frames)])
        lext.append(time.perf_counter() - t0)
        F1 = Frame.from_extraction(kprev, dprev, w, h)
        F2 = Frame.from_extraction(k, d, w, h)
        pm = np.ascontiguousarray(np.stack([kprev["x"], kprev["y"]], 1).astype(np.float32))
        m.SearchForInitialization(F1, F2, pm, 100)
        lat.append(time.perf_counter() - t0)
        kprev, dprev = k, d
    gpu_total = time.perf_counter() - t_all
    lat = np.array(lat) * 1e3
    lext = np.array(lext) * 1e3
    # oracle, one thread, same per-frame work
    p = O.params(nfeatures=nf)
    no = max(8, min(40, n // 5))
    olat = []
    rp = O.extract(p, frames[0])
    for t in range(1, no + 1):
        t0 = time.perf_counter()
        r = O.extract(p, frames[t % len(frames)])
        prevxy = np.ascontiguousarray(np.stack([rp["kps"]["x"], rp["kps"]["y"]], 1))
        O.search_for_initialization(rp["kps"], rp["desc"], r["kps"], r["desc"], prevxy,
                                    (0, w, 0, h), 100, 0.9, True)
        olat.append(time.perf_counter() - t0)
        rp = r
    olat = np.array(olat) * 1e3
    out = {
        "metric": "single-frame drop-in path: orbg_extract + orbg_search_for_initialization, "
                  "host image in, host outputs out (B=1)",
        "image": [w, h], "nfeatures": nf, "frames": n,
        "gpu_ms_per_frame": {"mean": round(float(lat.mean()), 3), "p50": round(float(np.median(lat)), 3),
                             "p90": round(float(np.percentile(lat, 90)), 3)},
        "gpu_extract_ms_per_frame": {"mean": round(float(lext.mean()), 3),
                                     "p50": round(float(np.median(lext)), 3)},
        "gpu_frames_per_s": round(n / gpu_total, 1),
        "cpu_oracle_1thread_ms_per_frame": {"mean": round(float(olat.mean()), 3),
                                            "p50": round(float(np.median(olat)), 3)},
        "cpu_oracle_1thread_frames_per_s": round(1e3 / float(olat.mean()), 2),
        "cpu_frames": no,
        "note": "includes the PCIe upload of the image and the download of keypoints, "
                "descriptors and matches; Python ctypes mirror over the C ABI",
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
