"""CPU oracle (test infrastructure only) for the detection metrics: a
scalar-loop restatement of air/evaluation_detection.py, used to check the
vectorised host implementation mog_air/evaluation.py.

IoU_evaluation: evaluation_detection.py:5-25; evaluation: :28-98 (boxes
:43-57, empty cases :66-74, thresholds 0.5 + 0.05 i :76-84, best IoUs
:85-86, Hungarian global IoU :88-90).  Pinned by the known-answer cases in
tests/test_pipeline.py and, since round 6, by outputs of the reference
module itself (tests/golden/eval_detection.npz, scripts/make_eval_golden.py,
checked in tests/test_eval_golden.py).
"""
import numpy as np
from scipy.optimize import linear_sum_assignment


def iou(a, b):
    w = max(0, min(a[2], b[2]) - max(a[0], b[0]) + 1)
    h = max(0, min(a[3], b[3]) - max(a[1], b[1]) + 1)
    inter = w * h
    area_a = (a[2] - a[0] + 1) * (a[3] - a[1] + 1)
    area_b = (b[2] - b[0] + 1) * (b[3] - b[1] + 1)
    return inter / float(area_a + area_b - inter)


def evaluation(gt_pos, gt_size, shifts, scales, nums, csize=50):
    n = len(gt_pos)
    P, R = np.zeros([n, 11]), np.zeros([n, 11])
    gbest, dbest, glob = np.zeros(n), np.zeros(n), np.zeros(n)
    for i in range(n):
        ng, nd = len(gt_pos[i]) // 2, int(nums[i])
        M = np.zeros([ng, nd])
        for a in range(ng):
            x1, y1 = gt_pos[i][2 * a], gt_pos[i][2 * a + 1]
            g = [x1, y1, x1 + gt_size[i][2 * a], y1 + gt_size[i][2 * a + 1]]
            for b in range(nd):
                h = csize / 2
                cx, cy, s = shifts[i, b, 0], shifts[i, b, 1], scales[i, b, 0]
                d = [(cx + 1) * h - s * h, (cy + 1) * h - s * h, (cx + 1) * h + s * h,
                     (cy + 1) * h + s * h]
                M[a, b] = iou(g, d)
        if ng == 0 and nd == 0:
            P[i], R[i], gbest[i], dbest[i], glob[i] = 1, 1, 1, 1, 1
        elif ng == 0:
            R[i] = 1
        elif nd == 0:
            pass
        else:
            for t in range(11):
                tp = np.sum(np.max((M > t * 0.05 + 0.5).astype(np.int32), 0))
                P[i, t], R[i, t] = tp / nd, tp / ng
            gbest[i] = np.mean(np.max(M, 1))
            dbest[i] = np.mean(np.max(M, 0))
            r, c = linear_sum_assignment(-M)
            glob[i] = np.sum(M[r, c]) / max(nd, ng)
    return P.mean(0), R.mean(0), gbest.mean(), dbest.mean(), glob.mean()
