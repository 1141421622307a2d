"""The quantised 4-wide node (rt_qnode, include/rt_wide.h; rt_quantize_wide): every used child's decoded
box contains its fp32 box, decoding is exact in fp32, unused slots are empty boxes, and boxes beyond an
fp32 grid are refused. CPU only (the GPU walk over these nodes: test_gpu_parity.py
test_resumable_walks_closest_hits[...-16])."""
import numpy as np
import pytest

import rtamd


def _decode(q, which):
    planes = np.zeros((len(q), 3, 4), dtype=np.float64)
    for a in range(3):
        for k in range(4):
            byte = (q[which][:, a] >> np.uint32(8 * k)) & np.uint32(255)
            # fp32 fma(q, s, o): q * s is exact (q < 2^8, s a power of two), the sum exact by construction
            exact = byte.astype(np.float64) * q["scale"][:, a].astype(np.float64) + q["origin"][:, a].astype(np.float64)
            f32 = (byte.astype(np.float32) * q["scale"][:, a] + q["origin"][:, a]).astype(np.float64)
            assert np.array_equal(exact, f32), "decoding is not exact in fp32"
            planes[:, a, k] = exact
    return planes


@pytest.mark.parametrize("name,param", [("stress_spheres", 3000), ("random_book_one", 0), ("three_spheres", 0)])
def test_quantised_boxes_contain_the_fp32_boxes(name, param):
    sc, _ = rtamd.make_scene(name, rtamd.randGen(1024), param=param)
    rb = rtamd.rebuilt_scene(sc)
    w, _ = rtamd.wide_bvh(rb)
    q = rtamd.quantize_wide(w)
    assert q.dtype.itemsize == 64 and len(q) == len(w)
    assert np.array_equal(q["child"], w["child"])
    lo, hi = _decode(q, "qlo"), _decode(q, "qhi")
    used = np.all(w["lo"] <= w["hi"], axis=1)  # (node, child)
    for a in range(3):
        assert np.all(lo[:, a][used] <= w["lo"][:, a][used])
        assert np.all(hi[:, a][used] >= w["hi"][:, a][used])
        # unused slots: qlo 255, qhi 0 (an empty box on every axis)
        assert np.all(lo[:, a][~used] > hi[:, a][~used])
    # the grid is not much coarser than the node: a child's quantised extent within 2 steps of its own
    step = q["scale"][:, :, None].astype(np.float64)
    slack = ((hi - lo) - (w["hi"] - w["lo"]).astype(np.float64)) / step
    assert np.all(slack[np.broadcast_to(used[:, None, :], slack.shape)] <= 2.0 + 1e-9)


def test_quantise_refuses_boxes_beyond_fp32():
    w = np.zeros(1, dtype=rtamd.WNODE_DTYPE)
    w["child"][:] = -1
    w["lo"][:] = -np.inf
    w["hi"][:] = np.inf
    with pytest.raises(rtamd.RTError):
        rtamd.quantize_wide(w)
    w["lo"][:] = 3.3e38  # every decodable plane must stay finite: no grid of 2^k steps fits
    w["hi"][:] = 3.4e38
    with pytest.raises(rtamd.RTError):
        rtamd.quantize_wide(w)
    w["lo"][:] = 1e-30  # tiny boxes far below 1 on a fine grid
    w["hi"][:] = 2e-30
    q = rtamd.quantize_wide(w)
    assert np.all(_decode(q, "qlo")[0] <= 1e-30) and np.all(_decode(q, "qhi")[0] >= 2e-30)
