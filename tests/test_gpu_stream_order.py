"""GPU: liborbg's writes into caller buffers are ordered after the caller's context stream.

orbg_batch_summary, orbg_batch_matches, orbg_match_pose_batch_device and orbg_stereo_summary
write caller-owned device buffers on liborbg's non-blocking match stream.  Each records an
event on the context stream at entry and makes the match stream wait for it (include/orbg.h),
so a zero fill the caller queued on the context stream before the call -- here held back
behind a ~50 ms GPU spin, with no host synchronisation anywhere -- can never land after
liborbg's write.  Round 3 saw exactly that race on MI355X (an all-zero vnMatches12 row); the
outputs are checked against the oracle (SearchForInitialization ORBmatcher.cc:487-631, the pose
stub Optimizer.cc:356-631, ComputeStereoMatches Frame.cc:619-834).
"""
import numpy as np
import pytest
import torch

from orb_slam2_test_amd import ORBextractor, sequence, synthetic as S

pytestmark = pytest.mark.gpu

W, H = 1241, 376
SPIN = 120_000_000  # torch.cuda._sleep cycles on the context stream (~50 ms)


def _ctx_stream(ext):
    st = torch.cuda.Stream()
    ext.ctx.set_stream(st.cuda_stream)
    return st


@pytest.mark.parametrize("pipelined", [True, False])
def test_writes_ordered_after_context_stream_fills(oracle, pipelined):
    n = 5
    frames = S.sequence_block(n, 0, n, H, W, seed=S.DEFAULT_SEED + 29)
    p = oracle.params(nfeatures=2000)
    ex = [oracle.extract(p, im) for im in frames]
    ref_m, ref_pose = [], []
    for t in range(1, n):
        a, b = ex[t - 1], ex[t]
        prev = np.ascontiguousarray(np.stack([a["kps"]["x"], a["kps"]["y"]], 1))
        k, m, _ = oracle.search_for_initialization(a["kps"], a["desc"], b["kps"], b["desc"],
                                                   prev, (0, W, 0, H), 100, 0.9, True)
        ref_m.append((k, m))
        ref_pose.append(oracle.match_pose(p, a["kps"], b["kps"], m, sequence.POSE_CAM,
                                          sequence.POSE_DEPTH))
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=n)
    ext.ctx.set_pipeline(pipelined)
    st = _ctx_stream(ext)
    with torch.cuda.stream(st):
        d = torch.from_numpy(frames).cuda()
        ext.extract_batch_device(d.data_ptr(), n, W, H)
        ext.match_batch_device(np.arange(n - 1), np.arange(1, n), 100, 0.9, True)
        cap = ext.ctx.batch_matches(None)
        summary = torch.empty(2 * n, dtype=torch.int32, device="cuda")
        m12 = torch.empty((n - 1, cap), dtype=torch.int32, device="cuda")
        dq = torch.empty((n - 1, 4), dtype=torch.float64, device="cuda")
        dt = torch.empty((n - 1, 3), dtype=torch.float64, device="cuda")
        dn = torch.empty(n - 1, dtype=torch.int32, device="cuda")
        # the fills run late on the context stream; no synchronize before the calls
        torch.cuda._sleep(SPIN)
        for t in (summary, m12, dn):
            t.fill_(-7)
        dq.fill_(0.0)
        dt.fill_(0.0)
        ext.ctx.batch_summary(summary.data_ptr())
        ext.ctx.batch_matches(m12.data_ptr())
        ext.match_pose_batch_device(sequence.POSE_CAM, sequence.POSE_DEPTH, dq.data_ptr(),
                                    dt.data_ptr(), dn.data_ptr())
    ext.ctx.sync()
    torch.cuda.synchronize()
    s, rows = summary.cpu().numpy(), m12.cpu().numpy()
    q, tt, ni = dq.cpu().numpy(), dt.cpu().numpy(), dn.cpu().numpy()
    for f in range(n):
        assert s[f] == len(ex[f]["kps"]), ("keypoints", f)
    for i, (k, m) in enumerate(ref_m):
        assert s[n + i] == k, ("nmatches", i)
        assert np.array_equal(rows[i, :len(m)], m), ("vnMatches12", i)
        assert (rows[i, len(m):] == -1).all(), ("vnMatches12 tail", i)
        rn, rq, rt = ref_pose[i]
        assert ni[i] == rn and np.array_equal(q[i], rq) and np.array_equal(tt[i], rt), ("pose", i)
    assert min(k for k, _ in ref_m) > 100
    ext.close()


def test_stereo_summary_ordered_after_context_stream_fill(oracle):
    B = 3
    lefts, rights, _ = S.stereo_sequence(B, H, W, seed=97)
    frames = np.empty((2 * B, H, W), np.uint8)
    frames[0::2], frames[1::2] = lefts, rights
    p = oracle.params(nfeatures=2000)
    ref = []
    for i in range(B):
        rl = oracle.extract(p, lefts[i], with_pyramid=True)
        rr = oracle.extract(p, rights[i], with_pyramid=True)
        _, dp = oracle.stereo_matches(p, rl, rr, W, H, S.KITTI_BF, S.KITTI_BF / S.KITTI_FX)
        ref.append((len(rl["kps"]), int((dp > 0).sum())))
    ext = ORBextractor(2000, 1.2, 8, 20, 7, max_batch=2 * B)
    ext.ctx.set_pipeline(True)
    st = _ctx_stream(ext)
    with torch.cuda.stream(st):
        d = torch.from_numpy(frames).cuda()
        ext.extract_batch_device(d.data_ptr(), 2 * B, W, H)
        ext.stereo_batch_device(np.arange(B) * 2, np.arange(B) * 2 + 1, S.KITTI_BF,
                                S.KITTI_BF / S.KITTI_FX)
        out = torch.empty(2 * B, dtype=torch.int32, device="cuda")
        torch.cuda._sleep(SPIN)
        out.fill_(-7)
        ext.ctx.stereo_summary(out.data_ptr())
    ext.ctx.sync()
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for i, (nk, nd) in enumerate(ref):
        assert o[i] == nk and o[B + i] == nd, i
    assert sum(nd for _, nd in ref) > 0
    ext.close()
