"""Express mode of the Russian-roulette megakernel (bdpt_kernels.hip).

A wave holding a subpath deeper than the express depth (512 bounces by default,
DevFrame::express_depth) stops refilling and shades at one ready lane; while it
holds 2-4 busy lanes whose closest-hit walks have begun, the wave walks them at
once in groups of 32 / 16 lanes (coop_closest_groups: group partition, stack
ranges [gi*cap, gi*cap + cap), the owner / result shuffle); with
BDPT_COOP_GROUPS=0, or with one such lane, it walks them one after another with
all 64 lanes (coop_closest). On the golden frames no walk reaches 512 bounces,
so these tests lower the express depth per render (BDPT_EXPRESS_DEPTH) until
those waves are common, and check that both schedules ran (bdpt_stats:
rr_long_walks_max, rr_express_iters = waves-iterations with 1 / 2-4 / more long
walks) and that the frames are still the reference's (NO_RR = 0 goldens
R1-R6, per-pixel relative L2 <= 1e-4).
"""
import pytest

from conftest import load_golden
from test_gpu_parity import TOL, report, rr_integrator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("chain", ["1", "0"])
@pytest.mark.parametrize("groups", ["1", "0"])
@pytest.mark.parametrize("depth", ["3", "12"])
@pytest.mark.parametrize("name", ["R1_caustic_rr_64x64_spp16", "R2_hardlight_rr_64x64_spp16",
                                  "R6_caustic_rr_512x512_spp2_rows32"])
def test_gpu_express_walks_match_reference_golden(name, depth, groups, chain, golden_manifest, monkeypatch):
    """chain: the build that runs a lone walk's delta bounces inline (bdpt_kernels_rrc.hip, chosen for
    scenes with glass) or the plain RR build, forced either way (BDPT_RR_CHAIN)."""
    monkeypatch.setenv("BDPT_EXPRESS_DEPTH", depth)
    monkeypatch.setenv("BDPT_COOP_GROUPS", groups)
    monkeypatch.setenv("BDPT_RR_CHAIN", chain)
    m = golden_manifest["rr_framebuffers"][name]
    it = rr_integrator(m["scene"], m["width"], m["height"], m["spp"], m["rr_depth"])
    fb = it.render_frame(row_offset=0, row_stride=m["row_stride"]).reshape(-1)
    st = it.stats()
    assert st["kernel"] == ("bdpt_frame_kernel_rrc" if chain == "1" else "bdpt_frame_kernel_rr"), st["kernel"]
    assert st["capped_samples"] == 0 and st["schedule_errors"] == 0
    # express waves ran, with one and with 2-4 long walks at once
    assert st["rr_long_walks_max"] >= 2, st
    assert st["rr_express_iters"][0] > 0 and st["rr_express_iters"][1] > 0, st["rr_express_iters"]
    worst, exact, _ = report(fb, load_golden(name))
    assert worst <= TOL, f"max per-pixel rel L2 {worst:.3g} (bit-exact floats {exact:.4f})"
