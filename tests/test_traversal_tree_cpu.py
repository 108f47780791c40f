"""The traversal tree's exactness preconditions (wide_bvh.hpp), checked
on the host layout the library uploads (bdpt_scene_export_traversal; no GPU):

* every triangle sits in exactly one traversal leaf, and its record carries the
  reference geometry bit-for-bit (v0, e1 = v1 - v0, e2 = v2 - v0 in float32), its
  reference leaf-order index and the id of the reference leaf that holds it;
* lbox[k] is the reference's k-th leaf box (preorder), bit-for-bit — the box the
  device tests exactly before a candidate hit may win (ref_leaf_passes);
* every child box of a wide node contains every triangle below it, grown by the
  culling tolerance (kTriBoxPad x scene diagonal) for the triangle tree;
* links are well formed: leaves of 1..kTriLeafMax triangles, empty slots
  0xffffffff, depth within the reported wide_depth.

Both trees are covered: the default SAH tree over single triangles and the
reference-leaf tree (BDPT_TRAV_TREE=refleaf at scene load)."""
import numpy as np
import pytest

import bdpt_amd
import variants

LEAF_BIT, EMPTY = 0x80000000, 0xFFFFFFFF
TRI_LEAF_MAX, TRI_BOX_PAD = 4, 1e-4  # wide_bvh.hpp kTriLeafMax / kTriBoxPad


def ref_leaves(nu):
    """(start, count) of the reference's leaves in preorder (right_offset == 0)."""
    return [(int(s), int(c)) for s, c, r in nu if r == 0]


def check_tree(scene, tri_tree):
    info = scene.info()
    assert info["triangle_tree"] == int(tri_tree)
    tf, _, nf, nu = scene.export()
    wn, wt, lb, root = scene.export_traversal()
    n = info["triangles"]
    V = tf[:, :9].reshape(n, 3, 3)  # reference vertices, leaf order

    # triangle records: a permutation of the reference order, exact geometry
    ref_idx = wt[:, 0, 3].view(np.uint32).astype(np.int64)
    assert np.array_equal(np.sort(ref_idx), np.arange(n))
    if not tri_tree:
        assert np.array_equal(ref_idx, np.arange(n))
    v = V[ref_idx]
    assert np.array_equal(wt[:, 0, :3].view(np.uint32), v[:, 0].view(np.uint32))
    assert np.array_equal(wt[:, 1, :3].view(np.uint32), (v[:, 1] - v[:, 0]).view(np.uint32))
    assert np.array_equal(wt[:, 2, :3].view(np.uint32), (v[:, 2] - v[:, 0]).view(np.uint32))

    # reference leaf ids and their exact boxes
    leaves = ref_leaves(nu)
    assert info["bvh_leaves"] == len(leaves) == lb.shape[0]
    leaf_id = wt[:, 1, 3].view(np.uint32).astype(np.int64)
    starts = np.array([s for s, _ in leaves])
    counts = np.array([c for _, c in leaves])
    assert np.all((ref_idx >= starts[leaf_id]) & (ref_idx < starts[leaf_id] + counts[leaf_id]))
    leaf_nodes = np.flatnonzero(nu[:, 2] == 0)
    if nu[0, 2] == 0:  # one leaf: the reference tests no box
        assert np.all(np.isinf(lb[0, 0, :3])) and np.all(lb[0, 0, :3] < 0) and np.all(lb[0, 1, :3] > 0)
    else:
        assert np.array_equal(lb[:, 0, :3].view(np.uint32), nf[leaf_nodes, :3].view(np.uint32))
        assert np.array_equal(lb[:, 1, :3].view(np.uint32), nf[leaf_nodes, 3:].view(np.uint32))

    # the hierarchy: every triangle once, boxes contain (padded) subtrees
    lo_all, hi_all = V.reshape(-1, 3).min(0), V.reshape(-1, 3).max(0)
    pad = np.float32(TRI_BOX_PAD * np.sqrt(((hi_all.astype(np.float64) - lo_all) ** 2).sum())) if tri_tree else 0
    grow = np.float32(pad * 0.999)
    seen = np.zeros(n, np.int64)
    max_leaf = TRI_LEAF_MAX if tri_tree else 4

    def walk(link, depth):
        if link & LEAF_BIT:
            start, count = (link & 0x7FFFFFFF) >> 3, link & 7
            assert 1 <= count <= max_leaf and start + count <= n
            seen[start:start + count] += 1
            t = V[ref_idx[start:start + count]].reshape(-1, 3)
            return t.min(0), t.max(0), depth
        assert 0 <= link < wn.shape[0]
        node = wn[link]
        links = node[6].view(np.uint32)
        used = links != EMPTY
        assert used.sum() >= 2 or (link == root and used.sum() >= 1)
        assert np.all(used[:used.sum()])  # empty slots trail
        los, his, deepest = [], [], depth
        for j in np.flatnonzero(used):
            lo, hi, d = walk(int(links[j]), depth + 1)
            blo = np.array([node[0, j], node[2, j], node[4, j]], np.float32)
            bhi = np.array([node[1, j], node[3, j], node[5, j]], np.float32)
            assert np.all(blo <= lo - grow) and np.all(bhi >= hi + grow), (link, j)
            los.append(lo), his.append(hi)
            deepest = max(deepest, d)
        return np.min(los, 0), np.max(his, 0), deepest

    _, _, depth = walk(root, 0)
    assert np.all(seen == 1)
    if not root & LEAF_BIT:
        assert depth <= info["wide_depth"] + 1


SCENES = ["cbox_low", "caustic", "hardlight_mirror"]


@pytest.mark.parametrize("scene_name", SCENES)
def test_triangle_tree_preconditions(scene_name):
    check_tree(bdpt_amd.Scene(variants.obj_path(scene_name)), tri_tree=True)


@pytest.mark.parametrize("scene_name", SCENES)
def test_reference_leaf_tree_preconditions(scene_name, monkeypatch):
    monkeypatch.setenv("BDPT_TRAV_TREE", "refleaf")
    check_tree(bdpt_amd.Scene(variants.obj_path(scene_name)), tri_tree=False)


@pytest.mark.parametrize("gen", ["many_shapes_obj", "closed_box_obj"])
def test_tree_preconditions_on_generated_scenes(gen, tmp_path):
    check_tree(bdpt_amd.Scene(getattr(variants, gen)(str(tmp_path))), tri_tree=True)


def test_single_triangle_scene_is_one_leaf(tmp_path):
    """The whole scene one reference leaf: no node, the leaf box infinite."""
    (tmp_path / "one.mtl").write_text("newmtl a\nKd 0.5 0.5 0.5\nKe 1 1 1\nillum 7\n")
    p = tmp_path / "one.obj"
    p.write_text("mtllib one.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nvn 0 0 1\nusemtl a\nf 1//1 2//1 3//1\n")
    s = bdpt_amd.Scene(str(p))
    _, _, _, root = s.export_traversal()
    assert root == (LEAF_BIT | (0 << 3) | 1)
    check_tree(s, tri_tree=True)


@pytest.mark.parametrize("scene_name", SCENES)
def test_greedy_collapse_tree_preconditions_and_dp_is_smaller(scene_name, monkeypatch):
    """The 4-wide grouping by SAH dynamic programming (the default, wide_bvh.cpp
    DpCollapse) and the earlier largest-child-first rule (BDPT_WIDE_COLLAPSE=greedy)
    group the same binary tree: same traversal leaves, both meet the preconditions,
    and the DP tree needs no more nodes (it fills the 4 slots where the SAH says so)."""
    dp = bdpt_amd.Scene(variants.obj_path(scene_name))
    monkeypatch.setenv("BDPT_WIDE_COLLAPSE", "greedy")
    greedy = bdpt_amd.Scene(variants.obj_path(scene_name))
    check_tree(greedy, tri_tree=True)
    a, b = dp.info(), greedy.info()
    assert a["wide_leaves"] == b["wide_leaves"]
    assert a["wide_nodes"] <= b["wide_nodes"]


@pytest.mark.parametrize("name,diags", [("caustic", 250.0), ("caustic", 350.0), ("hardlight", 100.0)])
def test_tree_preconditions_on_translated_scenes(name, diags, tmp_path):
    """The scenes test_gpu_parity.py's translated-scene cases render: every vertex
    moved ~diags scene diagonals from 0 (variants.translated_obj), so float
    coordinates are coarse relative to the scene, and the padded boxes must still
    hold their triangles (the slack-free interior test's precondition there)."""
    with open(variants.obj_path(name)) as f:
        v = np.array([line.split()[1:4] for line in f if line.startswith("v ")], np.float64)
    off = np.full(3, diags * np.linalg.norm(v.max(0) - v.min(0)))
    path = variants.translated_obj(name, str(tmp_path), off)
    with open(path) as f:
        w = np.array([line.split()[1:4] for line in f if line.startswith("v ")], np.float64)
    assert w.shape == v.shape and np.abs(w - v - off).max() < 1e-5
    check_tree(bdpt_amd.Scene(path), tri_tree=True)
