"""Row F4 pinned by the reference itself: mog_air/evaluation.py against
outputs of /root/reference/air/evaluation_detection.py:28-98 run in the
build container (tests/golden/eval_detection.npz, made by
scripts/make_eval_golden.py; nothing of the reference travels with it).

Bar: bit-exact (assert_array_equal) on float64 detections -- the
reference's arithmetic under the NumPy 1.x it ran on -- for the batch means
and every image evaluated alone; the float32-detection run of the reference
under NumPy 2 (float32 scalar arithmetic) within 1e-6."""
import os

import numpy as np
import pytest

from mog_air.evaluation import evaluation

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "eval_detection.npz")


def _case(g, name):
    def unflat(a, off):
        return [a[off[i]:off[i + 1]] for i in range(len(off) - 1)]
    return (unflat(g[f"{name}_pos"], g[f"{name}_pos_off"]),
            unflat(g[f"{name}_box"], g[f"{name}_box_off"]),
            g[f"{name}_shifts"], g[f"{name}_scales"], g[f"{name}_num"])


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD) as f:
        return dict(f)


@pytest.mark.parametrize("name", ["random", "edges", "hungary"])
def test_batch_means_bit_exact(gold, name):
    p, r, gi, di, gl = evaluation(*_case(gold, name), csize=50)
    np.testing.assert_array_equal(p, gold[f"{name}_precision"])
    np.testing.assert_array_equal(r, gold[f"{name}_recall"])
    np.testing.assert_array_equal(np.array([gi, di, gl]), gold[f"{name}_means"])


@pytest.mark.parametrize("name", ["random", "edges", "hungary"])
def test_every_image_bit_exact(gold, name):
    pos, box, sh, sc, num = _case(gold, name)
    ref = gold[f"{name}_per_image"]
    for i in range(len(pos)):
        p, r, gi, di, gl = evaluation([pos[i]], [box[i]], sh[i:i + 1], sc[i:i + 1],
                                      num[i:i + 1], csize=50)
        got = np.concatenate([p, r, [gi, di, gl]])
        np.testing.assert_array_equal(got, ref[i], err_msg=f"{name} image {i}")


def test_edge_cases_hit_the_exact_thresholds(gold):
    """The fixture holds what it claims: IoU exactly 1.0 (no hit at the
    `> 1.0` threshold) and exactly 0.5 (no hit at `> 0.5`), empty sides."""
    per = gold["edges_per_image"]
    np.testing.assert_array_equal(per[0], np.ones(25))           # nothing either side
    assert per[1].sum() == 0.0                                   # boxes, no detections
    np.testing.assert_array_equal(per[2][11:22], np.ones(11))    # no boxes: recall 1
    assert per[3][10] == 0.0 and per[3][9] == 1.0 and per[3][22] == 1.0
    assert per[4][0] == 0.0 and per[4][22] == 0.5


def test_hungarian_beats_greedy(gold):
    """The Hungarian case: the global IoU is the optimal assignment's, above
    what a row-greedy pairing reaches on at least one image."""
    from mog_air.evaluation import detection_boxes, iou_matrix
    pos, box, sh, sc, num = _case(gold, "hungary")
    better = 0
    for i in range(len(pos)):
        xy = pos[i].reshape(-1, 2).astype(np.float64)
        gt = np.concatenate([xy, xy + box[i].reshape(-1, 2)], 1)
        iou = iou_matrix(gt, detection_boxes(sh[i], sc[i], int(num[i]), 50))
        used, greedy = set(), 0.0
        for row in iou:
            j = max((j for j in range(iou.shape[1]) if j not in used), key=lambda j: row[j])
            used.add(j)
            greedy += row[j]
        better += gold["hungary_per_image"][i][24] * 3 > greedy + 1e-12
    assert better == len(pos)


def test_float32_detections_close(gold):
    pos, box, sh, sc, num = _case(gold, "random")
    p, r, gi, di, gl = evaluation(pos, box, sh.astype(np.float32), sc.astype(np.float32), num,
                                  csize=50)
    np.testing.assert_allclose(p, gold["random_f32_precision"], atol=1e-6)
    np.testing.assert_allclose(r, gold["random_f32_recall"], atol=1e-6)
    np.testing.assert_allclose([gi, di, gl], gold["random_f32_means"], atol=1e-6)
