"""Test infrastructure: a numpy Gauss-Newton reduced camera system (no robust kernel, lambda 0)
of an EdgeSE3ProjectXYZ problem, used to check that landmark shards'
partial systems add up to the full one. Not a solver, and not used by the product."""
import numpy as np


def quat_to_mat(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def reduced_system(prob):
    """S (n x n) and bs (n) over the optimised poses, Hpp/bp from the problem's edges and the
    Schur complement of its landmarks."""
    p = prob.normalized()
    opt = np.cumsum(1 - p.pose_fixed.astype(np.int64)) - 1
    opt[p.pose_fixed == 1] = -1
    npo = int((p.pose_fixed == 0).sum())
    n = 6 * npo
    S = np.zeros((n, n))
    bs = np.zeros(n)
    R = [quat_to_mat(q.astype(np.float64)) for q in p.pose_q]
    Hll = np.zeros((p.points.shape[0], 3, 3))
    bl = np.zeros((p.points.shape[0], 3))
    Hpl = {}
    for e in range(p.edge_pose.shape[0]):
        i, m = int(p.edge_pose[e]), int(p.edge_point[e])
        X = p.points[m].astype(np.float64)
        Xc = R[i] @ X + p.pose_t[i]
        x, y, z = Xc
        pj = np.array([[p.fx / z, 0, -p.fx * x / (z * z)], [0, p.fy / z, -p.fy * y / (z * z)]])
        err = p.edge_uv[e] - np.array([p.fx * x / z + p.cx, p.fy * y / z + p.cy])
        info = float(p.inv_sigma2[p.edge_octave[e]])
        JX = -pj @ R[i]
        JT = -pj @ np.array([[0, z, -y, 1, 0, 0], [-z, 0, x, 0, 1, 0], [y, -x, 0, 0, 0, 1]])
        Hll[m] += info * JX.T @ JX
        bl[m] -= info * JX.T @ err
        oi = opt[i]
        if oi >= 0:
            S[6 * oi:6 * oi + 6, 6 * oi:6 * oi + 6] += info * JT.T @ JT
            bs[6 * oi:6 * oi + 6] -= info * JT.T @ err
            Hpl.setdefault(m, []).append((oi, info * JT.T @ JX))
    for m, lst in Hpl.items():
        Di = np.linalg.inv(Hll[m])
        for a, Ha in lst:
            bs[6 * a:6 * a + 6] -= Ha @ Di @ bl[m]
            for b, Hb in lst:
                S[6 * a:6 * a + 6, 6 * b:6 * b + 6] -= Ha @ Di @ Hb.T
    return S, bs
