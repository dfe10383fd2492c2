"""Host-side checks of the BVH builder behind the trace kernel (no GPU): the spatial-split
tree, its coded copy and the 16-bit quantized / octant copies (tools/bvh_check.cpp).

The GPU parity tests compare whole renders with the oracle; these check the builder's
invariants directly on CPU: every triangle referenced, quantized boxes contain the f32 boxes,
and closest hits through both trees equal brute force for random rays."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import REPO

CSRC = os.path.join(REPO, "audiorenderingv2_amd", "csrc")


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path_factory.mktemp("bvh") / "bvh_check")
    subprocess.run([gxx, "-O2", "-std=c++17", "-pthread", "-I", CSRC, os.path.join(REPO, "tools", "bvh_check.cpp"),
                    os.path.join(CSRC, "arx_bvh.cpp"), "-o", exe], check=True)
    return exe


def run(checker, tri_v, tmp_path, n_rays=1500, env=None):
    path = tmp_path / "scene.f32"
    np.ascontiguousarray(tri_v, np.float32).tofile(path)
    res = subprocess.run([checker, str(path), str(len(tri_v)), str(n_rays)], capture_output=True, text=True,
                         env={**os.environ, **(env or {})})
    assert res.returncode == 0, res.stdout + res.stderr
    assert res.stdout.startswith("ok"), res.stdout
    return res.stdout


def cylinders_scene(n_cyl=60, n_box=20, seed=3):
    """A small conference-like soup: a room, boxes and tessellated cylinders (long slivers and
    fan caps, the triangles spatial splits clip)."""
    from audiorenderingv2_amd.scene import _box_tris, _cyl_tris

    rng = np.random.default_rng(seed)
    room = _box_tris(np.array([[-6, 0, -4]], np.float32), np.array([[6, 3, 4]], np.float32))
    lo = np.stack([rng.uniform(-5, 4, n_box), np.zeros(n_box), rng.uniform(-3, 2, n_box)], -1).astype(np.float32)
    boxes = _box_tris(lo, lo + rng.uniform(0.2, 1.0, (n_box, 3)).astype(np.float32))
    cc = rng.uniform([-5, -3], [5, 3], (n_cyl, 2)).astype(np.float32)
    y0 = rng.uniform(0, 0.2, n_cyl).astype(np.float32)
    cyl = _cyl_tris(cc, rng.uniform(0.1, 0.3, n_cyl).astype(np.float32), y0,
                    y0 + rng.uniform(0.5, 2.5, n_cyl).astype(np.float32))
    return np.concatenate([room, boxes, cyl]).astype(np.float32)


def test_sbvh_conservative_and_exact(checker, tmp_path):
    tv = cylinders_scene()
    out = run(checker, tv, tmp_path)
    n_refs = int(out.split(",")[1].split()[0])
    assert n_refs > len(tv), "the spatial splits should duplicate some references on this scene"


def test_object_split_builder(checker, tmp_path):
    run(checker, cylinders_scene(seed=5), tmp_path, env={"ARX_SBVH": "0"})


def test_degenerate_and_random_soup(checker, tmp_path):
    rng = np.random.default_rng(9)
    tv = rng.uniform(-3, 3, (6000, 9)).astype(np.float32)
    tv[:50, 3:6] = tv[:50, 0:3]  # degenerate (zero-area) triangles
    tv[50:100, 1::3] = 1.0       # triangles in one plane y = 1
    run(checker, tv, tmp_path, n_rays=800)


@pytest.mark.parametrize("k", ["0", "1", "7", "100000"])
def test_breadth_first_renumbering(checker, tmp_path, k):
    """bfs_prefix_order (the scene-tree numbering arx_set_scene uses): the first k inner nodes
    in breadth-first order, the tree still valid and closest hits still exact (k = 100000:
    the whole tree renumbered)."""
    run(checker, cylinders_scene(seed=11), tmp_path, n_rays=600, env={"BFS_K": k})


def test_threaded_build_is_deterministic(tmp_path):
    """The spatial builder builds the top subtrees on threads (arx_bvh.cpp SpatialBuilder::inner):
    the node and triangle arrays must not depend on thread timing, within a process or across
    processes, at a size where the thread path is taken (> 4096 references per subtree)."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "tree_hash")
    subprocess.run([gxx, "-O2", "-std=c++17", "-pthread", "-I", CSRC, os.path.join(REPO, "tests", "cpp", "tree_hash.cpp"),
                    os.path.join(CSRC, "arx_bvh.cpp"), "-o", exe], check=True)
    tri_v = cylinders_scene(n_cyl=400, n_box=200, seed=11)
    path = tmp_path / "scene.f32"
    np.ascontiguousarray(tri_v, np.float32).tofile(path)
    outs = [subprocess.run([exe, str(path), str(len(tri_v))], capture_output=True, text=True, check=True).stdout.split()
            for _ in range(2)]
    assert int(outs[0][2]) > 8 * 4096 // 4, outs  # big enough for the threaded top levels
    assert outs[0][0] == outs[0][1] == outs[1][0] == outs[1][1], outs


def wide_stats(tri_v, tri_abs, emitter, n_rays=400, bounces=8, seed=5):
    """arx_debug_wide_stats: the BVH2 (16-bit quantized) and its 4-wide compressed copy (CW4)
    traversed on the CPU over the same bouncing rays."""
    import ctypes as C

    from audiorenderingv2_amd import _lib

    tv = np.ascontiguousarray(tri_v, np.float32)
    ta = np.ascontiguousarray(tri_abs, np.float32)
    em = np.asarray(emitter, np.float32)
    out = np.zeros(16)
    _lib.check(_lib.lib().arx_debug_wide_stats(_lib.fptr(tv), _lib.fptr(ta), ta.size, _lib.fptr(em), n_rays, bounces,
                                               seed, out.ctypes.data_as(C.POINTER(C.c_double)), 16))
    return dict(zip(["queries", "q2_steps", "q2_tris", "q4_steps", "q4_tris", "q4_max_stack", "mismatches",
                     "q4_nodes", "q4_depth", "q2_nodes", "q2_depth", "quantize_failures", "misses"], out))


@pytest.mark.parametrize("which", ["c1", "cylinders", "soup"])
def test_cw4_collapse_finds_the_same_closest_hits(which, c1_scene):
    """The CW4 copy (BVH2 collapsed to 4 children, 6-bit planes on per-node frames, arx_wide.cpp)
    finds the BVH2's closest hit for every query, quantizes every node onto the grid, and takes
    fewer node steps than the BVH2."""
    rng = np.random.default_rng(11)
    if which == "c1":
        tv, ta, em = c1_scene.tri_v, c1_scene.tri_abs, (0.5, 3.0, 1.0)
    elif which == "cylinders":
        tv = cylinders_scene().reshape(-1, 9)
        ta, em = np.full(len(tv), 0.3, np.float32), tuple(tv.reshape(-1, 3).mean(0))
    else:  # a closed box of random triangles, some degenerate
        tv = rng.uniform(-5, 5, (3000, 9)).astype(np.float32)
        tv[::17, 3:6] = tv[::17, 0:3]  # zero-area triangles
        ta, em = np.full(len(tv), 0.2, np.float32), (0.1, 0.2, 0.3)
    st = wide_stats(tv, ta, em)
    assert st["queries"] > 400
    assert st["mismatches"] == 0 and st["quantize_failures"] == 0
    assert st["q4_steps"] < st["q2_steps"]
    assert st["q4_depth"] < st["q2_depth"] + 2
