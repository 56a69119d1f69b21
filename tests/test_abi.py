"""The C-ABI library loads and exports every entry point include/orbx.h
declares (no compute calls: runs without a GPU)."""
import ctypes
import re
from pathlib import Path

import pytest

import orb_slam_amd as ox

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    text = (ROOT / "include" / "orbx.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(orbx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ["orbx_create", "orbx_extract", "orbx_dev_extract", "orbx_search_for_initialization",
                 "orbx_hamming_bf", "orbx_lba_solve", "orbx_window_search"]:
        assert must in names


def test_library_exports_all_declared_symbols():
    lib = ox.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_version_string():
    assert b"gfx950" in ox.lib().orbx_version()


def test_keypoint_layout_is_cv_keypoint():
    assert ox.KEYPOINT.itemsize == 28
    assert list(ox.KEYPOINT.names) == ["x", "y", "size", "angle", "response", "octave", "class_id"]


def test_descriptor_distance_host_entry():
    a = (ctypes.c_uint8 * 32)(*([0xFF] * 32))
    b = (ctypes.c_uint8 * 32)(*([0x0F] * 32))
    assert ox.lib().orbx_descriptor_distance(a, b) == 128


def test_context_setters_refuse_null_context():
    """The mode setters / getters validate their arguments before touching
    a device: a null context is ORBX_ERR_ARG (runs without a GPU)."""
    lib = ox.lib()
    err_arg = -1
    calls = [
        ("orbx_set_nth_pivot", (None, 1)),
        ("orbx_get_nth_pivot", (None,)),
        ("orbx_dev_set_split", (None, 3)),
        ("orbx_dev_set_async_match", (None, 1)),
        ("orbx_lba_run", (None, 5, 10, None)),
        ("orbx_set_launch_mode", (None, 1)),
        ("orbx_lba_set_workgroups", (None, 4)),
        ("orbx_lba_get_workgroups", (None,)),
        ("orbx_lba_last_workgroups", (None,)),
        ("orbx_debug_lba_split", (None, 1, 0, 0, -1)),
        ("orbx_pose_set_exact", (None, 1)),
        ("orbx_pose_get_exact", (None,)),
        ("orbx_get_launch_mode", (None,)),
        ("orbx_dev_upload_async", (None, 0, 1, None, 640, 480, 640)),
        ("orbx_dev_download_async", (None, 0, 1, None, None, None, None, None)),
        ("orbx_track_frame", (None, None)),
    ]
    for name, args in calls:
        assert getattr(lib, name)(*args) == err_arg, name


def test_abi_version_matches_header():
    """orbx_abi_version() equals the header's ORBX_ABI_VERSION (the adapter
    refuses a library of another revision)."""
    text = (ROOT / "include" / "orbx.h").read_text()
    want = int(re.search(r"#define ORBX_ABI_VERSION (\d+)", text).group(1))
    assert ox.lib().orbx_abi_version() == want


def test_host_alloc_refuses_bad_arguments():
    lib = ox.lib()
    out = ctypes.c_void_p()
    assert lib.orbx_host_alloc(0, ctypes.byref(out)) == -1
    assert lib.orbx_host_alloc(16, None) == -1
    lib.orbx_host_free(None)   # no-op
