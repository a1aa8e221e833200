"""Two keyframes of the synthetic KITTI-shaped sequence for SearchForTriangulation tests:
features (oracle extraction + stereo), GT poses, FeatureVectors from a synthetic vocabulary,
map-point flags and LocalMapping::ComputeF12 (src/LocalMapping.cc:676-693)."""
import numpy as np

from scenario import frame_data


def compute_f12(T1, T2, cam):
    """F12 = K1^-T [t12]x R12 K2^-1 (float32 inputs, float64 arithmetic: an input to both sides)."""
    T1, T2 = np.asarray(T1, np.float64), np.asarray(T2, np.float64)
    R1, t1, R2, t2 = T1[:3, :3], T1[:3, 3], T2[:3, :3], T2[:3, 3]
    R12 = R1 @ R2.T
    t12 = -R1 @ R2.T @ t2 + t1
    tx = np.array([[0, -t12[2], t12[1]], [t12[2], 0, -t12[0]], [-t12[1], t12[0], 0]])
    K = np.array([[cam.fx, 0, cam.cx], [0, cam.fy, cam.cy], [0, 0, 1.0]])
    return (np.linalg.inv(K.T) @ tx @ R12 @ np.linalg.inv(K)).astype(np.float32)


def keyframe_pair(f1=3, f2=4, seed=0, vocab_L=5, levelsup=4, mp_frac=0.3, drop_stereo=0.0):
    from oracle import oracle_ctypes as O
    from orb_slam2_with_comment_amd import synth, synth_map as SM
    from orb_slam2_with_comment_amd.types import FeatureVector, Frame
    from orb_slam2_with_comment_amd.vocabulary import Vocabulary
    cam = synth.KITTI
    v = Vocabulary.synthetic(k=10, L=vocab_L, seed=21)
    rng = np.random.default_rng(seed)
    out = []
    for f in (f1, f2):
        kl, dl, u, _, T = frame_data(f)
        u = u.copy()
        u[rng.random(len(u)) < drop_stereo] = -1.0  # monocular keypoints (epipole test)
        fr = Frame(kl, dl, u, SM.tcw_from_twc(T), cam)
        _, _, node, off, feat = O.transform(v, dl, levelsup)
        has_mp = (rng.random(len(kl)) < mp_frac).astype(np.uint8)
        out.append((fr, has_mp, FeatureVector.from_csr(node, off, feat)))
    F12 = compute_f12(out[0][0].tcw, out[1][0].tcw, cam)
    return out[0], out[1], F12
