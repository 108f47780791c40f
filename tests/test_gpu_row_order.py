"""bdpt_set_row_order / bdpt_get_row_costs: the claim order of a shard's rows.

The order changes which samples run last, never a sample (each keeps its
(pixel, sample) seed, renderer.cpp:155 per SURVEY §8c), so a reordered shard is
the reference's frame to float-addition order; the per-row query counts of a
counting pass sum to the pass's queries.
"""
import numpy as np
import pytest

import bdpt_amd
from conftest import load_golden
from test_gpu_parity import TOL, integrator, report

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,stride", [("G2_caustic_64x64_spp16", 1), ("G6_caustic_512x512_spp4_rows16", 16)])
def test_gpu_row_order_keeps_the_reference_frame(name, stride, golden_manifest):
    m = golden_manifest["framebuffers"][name]
    assert m["row_stride"] == stride
    it = integrator(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"])
    nrows = len(range(0, m["height"], stride))
    # costs of the shard from a counting pass, then costly rows first
    it.render_frame(row_offset=0, row_stride=stride, flags=bdpt_amd.FLAG_COUNT)
    costs = it.row_costs(nrows)
    st = it.stats()
    # every sample issues its primary query at least; the closest-hit queries are all the owners'
    assert costs.sum() >= st["samples"] and costs.sum() >= st["counters"]["closest_rays"]
    assert (costs > 0).all()
    order = bdpt_amd.cost_row_order(costs)
    assert sorted(order.tolist()) == list(range(nrows))
    assert all(costs[order[i]] >= costs[order[i + 1]] for i in range(nrows - 1))
    it.set_row_order(order)
    it.rgb[:] = 0  # (render_frame adds to the host framebuffer)
    fb = it.render_frame(row_offset=0, row_stride=stride).reshape(-1).copy()
    worst, exact, _ = report(fb, load_golden(name))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f})"
    # reversed and random orders too
    rng = np.random.default_rng(7)
    for o in (order[::-1].copy(), rng.permutation(nrows).astype(np.int32)):
        it.set_row_order(o)
        it.rgb[:] = 0
        worst, _, _ = report(it.render_frame(row_offset=0, row_stride=stride).reshape(-1), load_golden(name))
        assert worst <= TOL
    it.set_row_order(None)


def test_gpu_row_order_rejects_bad_orders():
    it = integrator("caustic", 16, 8, 2, 8)
    with pytest.raises(bdpt_amd.BdptError):
        it.set_row_order([0, 0, 1, 2, 3, 4, 5, 6])  # not a permutation
    it.set_row_order(list(range(4)))  # 4 rows: a shard of 8 rows cannot use it
    with pytest.raises(bdpt_amd.BdptError):
        it.render_frame()
    it.rgb[:] = 0
    it.render_frame(row_offset=0, row_stride=2)  # the 4-row shard can
    it.set_row_order(None)
    it.render_frame()
