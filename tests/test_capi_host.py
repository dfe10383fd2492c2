"""Host-side checks of libarx.so (no GPU needed): the C ABI loads, exports every symbol
include/arx.h declares, and its host-only pieces match the reference's own outputs."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from audiorenderingv2_amd import _lib
from audiorenderingv2_amd.renderer import frac_bits, place_receiver_vertices
from audiorenderingv2_amd.scene import load_meshes_npz, material_absorption, reference_config_materials
from conftest import GOLDEN, REPO

import pyoracle as po


def header_functions():
    src = open(os.path.join(REPO, "include", "arx.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(arx_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    declared = header_functions()
    assert len(declared) >= 30
    missing = [f for f in declared if not hasattr(L, f)]
    assert not missing, missing
    # and the ctypes binding covers all of them
    assert set(declared) <= set(_lib.SIGNATURES), set(declared) - set(_lib.SIGNATURES)
    assert L.arx_abi_version() == 2


def test_trace_kernel_id_is_the_build_source_hash():
    """The library reports the identity build.py hashed from the trace kernel's sources (the guard
    of every stored PMC profile); an experiment macro gives another identity, a measurement-only
    macro does not."""
    from audiorenderingv2_amd import build
    kid = int(_lib.lib().arx_trace_kernel_id())
    assert kid != 0
    assert kid == int(build.trace_source_id()[:-3], 16)
    assert build.trace_source_id(("ARX_TRACE_COUNT=1",)) == build.trace_source_id()
    assert build.trace_source_id(("ARX_TRACE_LEAFFLAT=1",)) != build.trace_source_id()


def test_status_strings_and_errors():
    L = _lib.lib()
    assert L.arx_status_string(0) == b"ok"
    assert L.arx_status_string(1) == b"invalid argument"
    # invalid config is rejected before touching the GPU
    cfg = _lib.ArxConfig()
    L.arx_default_config(C.byref(cfg))
    cfg.rays_x = 0
    h = C.c_void_p()
    st = L.arx_create(C.byref(cfg), C.byref(h))
    assert st == 1 and not h.value
    assert b"rays" in L.arx_last_error()
    with pytest.raises(_lib.ArxError):
        _lib.check(st)


def test_default_config_matches_reference_defaults():
    cfg = _lib.ArxConfig()
    _lib.lib().arx_default_config(C.byref(cfg))
    # Context.cpp:19-117 (+ round(0.9) for hrtf, :145)
    assert (cfg.rays_x, cfg.rays_y, cfg.rays_z) == (100, 100, 100)
    assert cfg.ir_length_in_seconds == 2 and cfg.max_bounces == 10
    assert cfg.base_power == 100.0 and cfg.energy_thres == 0.0 and cfg.hrtf_absorption_rate == 1.0


@pytest.mark.parametrize("fixture,pos,yaw", [("receiver_c1.npz", (2.5, 9.9, 0.0), 0.0),
                                             ("receiver_rot.npz", (-1.25, 2.0, 3.5), 37.5)])
def test_receiver_placement_matches_reference_glm(fixture, pos, yaw):
    """place_receiver_half (OptixModel.cpp:159-257) via the reference's glm, bit for bit."""
    local = {m.name: m for m in load_meshes_npz(os.path.join(GOLDEN, "receiver_local.npz"))}
    placed = {m.name: m for m in load_meshes_npz(os.path.join(GOLDEN, fixture))}
    for name in ("receiver_left", "receiver_right"):
        got = place_receiver_vertices(local[name].vertices, pos, yaw)
        assert np.array_equal(local[name].faces, placed[name].faces)
        assert np.array_equal(got.view(np.uint32), placed[name].vertices.view(np.uint32)), name


def test_material_absorption_rules():
    names = [b"low", b"med", b"receiver_left"]
    arr = (C.c_char_p * 3)(*names)
    ab = np.array([0.1, 0.3, 0.9], np.float32)
    f = _lib.lib().arx_material_absorption
    assert f(b"receiver_left", arr, _lib.fptr(ab), 3) == -1.0
    assert f(b"receiver_right", arr, _lib.fptr(ab), 3) == -2.0
    assert f(b"med", arr, _lib.fptr(ab), 3) == np.float32(0.3)
    assert f(b"Amarillo", arr, _lib.fptr(ab), 3) == 0.5
    mats = reference_config_materials()
    for n in ("low", "blue", "Rojo", "receiver_right"):
        assert material_absorption(n, mats) == f(n.encode(), (C.c_char_p * len(mats))(*[m[0].encode() for m in mats]),
                                                 _lib.fptr(np.array([m[1] for m in mats], np.float32)), len(mats))


def test_frac_bits_agree_with_oracle():
    for n in (1, 2, 1000, 1024, 1 << 20, 10**6, 10**7, 10**9):
        assert frac_bits(n) == po.frac_bits(n)


def test_no_silent_fallback_without_library(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    with pytest.raises(_lib.ArxError):
        _lib.lib()


def test_scene_image_roundtrip_and_hash(c1_scene):
    """The byte image rank 0 broadcasts to the other ranks (arx_group_set_scene) reads back as the
    same tree; the content hash (arx_stats.tree_hash, the stored-profile guard) is stable across
    builds and changes with the geometry."""
    L = _lib.lib()
    tv = np.ascontiguousarray(c1_scene.tri_v, np.float32)
    ta = np.ascontiguousarray(c1_scene.tri_abs, np.float32)

    def roundtrip(v, a):
        h, n = C.c_uint64(), C.c_uint64()
        _lib.check(L.arx_debug_scene_roundtrip(_lib.fptr(v), _lib.fptr(a), a.size, C.byref(h), C.byref(n)))
        return h.value, n.value

    before = L.arx_scene_build_count()
    h1, n1 = roundtrip(tv, ta)
    h2, n2 = roundtrip(tv, ta)
    assert L.arx_scene_build_count() == before + 2
    assert h1 == h2 and n1 == n2 and n1 > 64 * len(ta) // 4
    tv2 = tv.copy()
    tv2[0, 0] += 0.25
    assert roundtrip(tv2, ta)[0] != h1
    bad = ta.copy()
    bad[0] = 1.5  # absorption outside [0, 1]
    h, n = C.c_uint64(), C.c_uint64()
    assert L.arx_debug_scene_roundtrip(_lib.fptr(tv), _lib.fptr(bad), bad.size, C.byref(h), C.byref(n)) == 1


@pytest.mark.parametrize("case", ["ok", "root_fails", "stage_fails", "consume_fails", "rank0_skips"])
def test_rank_path_scene_share_protocol(case, tmp_path):
    """arx_group_set_scene's rank path (arx_scene_share.hpp) with three ranks as threads: a failed
    input check or build on rank 0, a rank that cannot stage the image and a rank that cannot read it
    make every rank return the same error instead of leaving the others in a collective.  The
    round-3 shape -- rank 0 returning before the first collective -- hangs (the watchdog's exit 2)."""
    import shutil
    import subprocess

    gxx = shutil.which("g++")
    if not gxx:
        pytest.skip("g++ not available")
    exe = str(tmp_path / "scene_share_test")
    subprocess.run([gxx, "-O1", "-std=c++17", "-pthread", "-Wall", "-Werror", "-I",
                    os.path.join(REPO, "audiorenderingv2_amd", "csrc"),
                    os.path.join(REPO, "tests", "cpp", "scene_share_test.cpp"), "-o", exe], check=True)
    res = subprocess.run([exe, case], capture_output=True, text=True, timeout=60)
    if case == "rank0_skips":
        assert res.returncode == 2 and "HANG" in res.stdout, res.stdout
    else:
        want = {"ok": "ok", "root_fails": "root_failed", "stage_fails": "staging_failed",
                "consume_fails": "consume_failed"}[case]
        assert res.returncode == 0, res.stdout
        assert res.stdout.count(f": {want} ") == 3, res.stdout


def test_main_style_caller_compiles_against_reference_glm(tmp_path):
    """main.cpp:40-67's full_render over the C++ shim builds with the reference's own glm::vec3 (the
    glm the reference vendors, read in place; this container only) and links against libarx.so.
    The GPU run of the same program is tests/test_gpu_shim.py::test_main_style_full_render_matches_oracle."""
    import shutil
    import subprocess

    glm = "/root/reference/prebuild/common"
    gxx = shutil.which("g++")
    if not gxx or not os.path.exists(os.path.join(glm, "glm", "glm.hpp")):
        pytest.skip("g++ or the reference's glm not available")
    pkg = os.path.join(REPO, "audiorenderingv2_amd")
    subprocess.run([gxx, "-std=c++17", "-O1", "-Wall", "-Werror", "-DARX_DEMO_GLM", "-I", glm, "-I",
                    os.path.join(REPO, "include"), os.path.join(REPO, "tests", "cpp", "main_style_demo.cpp"),
                    "-L", pkg, "-larx", f"-Wl,-rpath,{pkg}", "-o", str(tmp_path / "main_style_demo")], check=True)


def test_tree_limits_guard_the_kernels_offsets_and_leaf_codes():
    """check_buffer_offsets (arx_debug_check_tree_limits) admits a tree up to the trace kernel's 31-bit
    buffer offsets and rejects one node / one triangle record beyond; at that limit the largest leaf
    code ~(index * 16 + count) and the largest inner-node code (its index) still fit int32, and stay
    clear of the empty-child code -- so the code width never binds before the offsets do."""
    from audiorenderingv2_amd._lib import ARX_OK, lib

    max_off = 0x7FFFFFFF
    tris_max, nodes_max = max_off // 48, max_off // 64
    L = lib()
    assert L.arx_debug_check_tree_limits(1, tris_max) == ARX_OK
    assert L.arx_debug_check_tree_limits(nodes_max, 1) == ARX_OK
    assert L.arx_debug_check_tree_limits(1, tris_max + 1) == 1  # ARX_ERR_INVALID_ARGUMENT
    assert L.arx_debug_check_tree_limits(nodes_max + 1, 1) == 1
    assert "31-bit buffer offsets" in L.arx_last_error().decode()
    last_leaf = (tris_max - 1) * 16 + 15  # the leaf code's positive form (count <= 15)
    assert last_leaf <= 0x7FFFFFFF and (nodes_max - 1) <= 0x7FFFFFFF
    assert ~last_leaf != ~16 and last_leaf != 16  # kEmptyChildCode = ~16 (a leaf of 0 triangles)


def test_conv_shards_tile_the_file():
    """arx_group_conv_shard (host only): for any world size the ranks' output frames tile [0, n) in
    rank order; a rank owns whole one-second block pairs (2 sr frames each) of the file's
    ceil(floor(n / sr) / 2) pairs, the last rank with pairs also the tail past them; a file without a
    whole block belongs to rank 0."""
    import ctypes as C

    from audiorenderingv2_amd._lib import lib

    L = lib()
    for sr in (16000, 48000, 1100):
        for n in (0, 5, sr - 1, sr, 2 * sr, 2 * sr + 7, 16 * sr + 42, 807498, 17 * sr):
            S = n // sr
            P = (S + 1) // 2
            for W in (1, 2, 3, 4, 7, 8, 16):
                cursor = 0
                for r in range(W):
                    b, e = C.c_uint64(), C.c_uint64()
                    L.arx_group_conv_shard(sr, n, r, W, C.byref(b), C.byref(e))
                    b, e = b.value, e.value
                    assert b <= e and (b == cursor or b == e), (sr, n, W, r, b, e, cursor)
                    if e > b:
                        pb, pe = P * r // W, P * (r + 1) // W
                        if P == 0:
                            assert r == 0 and (b, e) == (0, n)
                        else:
                            assert b == (0 if pb == 0 else 2 * pb * sr)
                            assert e == (n if pe == P else 2 * pe * sr)
                    cursor = max(cursor, e)
                assert cursor == n, (sr, n, W)
