"""CPU: the C-ABI library loads and exports every symbol include/*.h declares (no compute)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    for fn in os.listdir(os.path.join(ROOT, "include")):
        if not fn.endswith(".h"):
            continue
        txt = open(os.path.join(ROOT, "include", fn)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?\w+\s*\**\s*(lorb_\w+)\s*\(", txt, flags=re.M):
            syms.add(m.group(1))
    return syms


def test_header_declares_the_hot_path():
    s = declared_symbols()
    for must in ("lorb_bf_match", "lorb_bf_top2", "lorb_search_by_projection_frame",
                 "lorb_search_by_projection_local", "lorb_ba_pose_only", "lorb_ba_local",
                 "lorb_ba_plan_create", "lorb_is_in_frustum", "lorb_unproject_stereo"):
        assert must in s


def test_library_exports_every_declared_symbol():
    from lorb_slam_amd.runtime import LIB_PATH, lib
    lib()  # loads (raises if missing)
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = declared_symbols() - exported
    assert not missing, f"declared but not exported: {sorted(missing)}"


def test_abi_version_and_no_device_here():
    from lorb_slam_amd.runtime import lib
    L = lib()
    assert L.lorb_abi_version() == 1
    n = C.c_int(-1)
    L.lorb_device_count(C.byref(n))
    assert n.value >= 0


def test_null_args_rejected_without_device():
    from lorb_slam_amd.runtime import lib
    L = lib()
    assert L.lorb_bf_match(None, 0, None, None, None, None, None, None, None, None) != 0
    assert L.lorb_ba_local(None, 0, None, None, None, None, None) != 0
