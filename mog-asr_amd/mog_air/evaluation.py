"""Detection metrics of the inferred objects, restating
air/evaluation_detection.py:5-98 on the host: per image, the IoU matrix of
ground-truth boxes against the boxes implied by the inferred (scale, shift),
precision / recall at IoU thresholds 0.50, 0.55, ..., 1.00, the mean best IoU
per ground-truth box and per detection, and the Hungarian-matched global IoU
(scipy.optimize.linear_sum_assignment, as the reference).

Box conventions (evaluation_detection.py:5-25, :43-57): ground truth
[x1, y1, x1 + w, y1 + h] from (positions, boxes); a detection is the square
of half-side scale * C/2 centred at ((tx + 1) C/2, (ty + 1) C/2); IoU uses
the inclusive-pixel "+1" areas.
"""
from __future__ import annotations

import numpy as np
from scipy.optimize import linear_sum_assignment

THRESHOLDS = 0.5 + 0.05 * np.arange(11)


def iou_matrix(gt: np.ndarray, det: np.ndarray) -> np.ndarray:
    """IoU of every gt box [G, 4] against every detection [D, 4]
    (evaluation_detection.py:5-25, vectorised)."""
    xa = np.maximum(gt[:, None, 0], det[None, :, 0])
    ya = np.maximum(gt[:, None, 1], det[None, :, 1])
    xb = np.minimum(gt[:, None, 2], det[None, :, 2])
    yb = np.minimum(gt[:, None, 3], det[None, :, 3])
    inter = np.maximum(0, xb - xa + 1) * np.maximum(0, yb - ya + 1)
    area_g = (gt[:, 2] - gt[:, 0] + 1) * (gt[:, 3] - gt[:, 1] + 1)
    area_d = (det[:, 2] - det[:, 0] + 1) * (det[:, 3] - det[:, 1] + 1)
    return inter / (area_g[:, None] + area_d[None, :] - inter).astype(np.float64)


def detection_boxes(shifts: np.ndarray, scales: np.ndarray, n: int, csize: int) -> np.ndarray:
    half = csize / 2
    cx = (shifts[:n, 0] + 1) * half
    cy = (shifts[:n, 1] + 1) * half
    r = scales[:n, 0] * half
    return np.stack([cx - r, cy - r, cx + r, cy + r], axis=1)


def evaluation(gt_position_xy, gt_scale_xy, inf_shifts, inf_scales, inf_num, csize=50):
    """(mean precision[11], mean recall[11], mean gt best-IoU, mean detection
    best-IoU, mean global IoU) over the images (evaluation_detection.py:28-98).
    inf_shifts [N, T, 2], inf_scales [N, T, 1], inf_num [N]."""
    inf_shifts = np.asarray(inf_shifts, np.float64)
    inf_scales = np.asarray(inf_scales, np.float64)
    n_img = len(gt_position_xy)
    precision = np.zeros((n_img, THRESHOLDS.size))
    recall = np.zeros((n_img, THRESHOLDS.size))
    gt_best = np.zeros(n_img)
    det_best = np.zeros(n_img)
    global_iou = np.zeros(n_img)
    for i in range(n_img):
        pos = np.asarray(gt_position_xy[i], np.float64)
        size = np.asarray(gt_scale_xy[i], np.float64)
        n_gt, n_det = len(pos) // 2, int(inf_num[i])
        if n_gt == 0 and n_det == 0:
            precision[i] = recall[i] = 1.0
            gt_best[i] = det_best[i] = global_iou[i] = 1.0
            continue
        if n_gt == 0:
            recall[i] = 1.0
            continue
        if n_det == 0:
            continue
        xy = pos.reshape(-1, 2)
        gt = np.concatenate([xy, xy + size.reshape(-1, 2)], axis=1)
        iou = iou_matrix(gt, detection_boxes(inf_shifts[i], inf_scales[i], n_det, csize))
        hit = (iou[None, :, :] > THRESHOLDS[:, None, None]).any(axis=1).sum(axis=1)
        precision[i] = hit / n_det
        recall[i] = hit / n_gt
        gt_best[i] = iou.max(axis=1).mean()
        det_best[i] = iou.max(axis=0).mean()
        r, c = linear_sum_assignment(-iou)
        global_iou[i] = iou[r, c].sum() / max(n_det, n_gt)
    return (precision.mean(0), recall.mean(0), gt_best.mean(), det_best.mean(),
            global_iou.mean())
