"""CPU: the drop-in boundary compiles against the reference's UNCHANGED headers and callers.

SURVEY §4 item 5 / §8b: `integration/Simple_ORB_SLAM/{matcher,bundle_adjust,local_mapping}.cpp`
replace the reference's src files of the same names and must define exactly the members that
`include/matcher.h:15-36`, `include/bundle_adjust.h:12-21` and `include/local_mapping.h:15-46`
declare, so that `src/visual_odometry.cpp` (callers at :103,124,129,135,201,207,437) builds
unchanged.  OpenCV / Ceres are absent here, so every TU is run through `g++ -fsyntax-only` against
declaration-only stand-ins (tests/compile/shim).  The reference tree is read in place (never
copied into the repo); the test skips where it is absent (the GPU box).

A deliberately changed declaration in a scratch copy of matcher.h must make the drop-in fail.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.environ.get("LORB_REFERENCE", "/root/reference")
SHIM = os.path.join(ROOT, "tests", "compile", "shim")
INTEG = os.path.join(ROOT, "integration", "Simple_ORB_SLAM")
DROPINS = ("matcher.cpp", "bundle_adjust.cpp", "local_mapping.cpp")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "include")), reason="reference tree absent")


def gxx(src, inc_dir, *extra):
    cmd = ["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Wno-unused-variable", "-Wno-sign-compare",
           "-Wno-reorder", "-Wno-unused-but-set-variable", "-I", SHIM, "-I", os.path.join(ROOT, "include"),
           "-I", INTEG, "-I", inc_dir, *extra, src]
    return subprocess.run(cmd, capture_output=True, text=True, timeout=120)


def tree(tmp, include_src):
    """tmp/include -> headers, tmp/src/<drop-ins>: the layout the drop-ins expect
    (`#include "../include/matcher.h"`, as the reference's own src/*.cpp)."""
    inc = os.path.join(tmp, "include")
    if os.path.isdir(include_src) and include_src != inc:
        os.symlink(include_src, inc) if include_src == os.path.join(REF, "include") else shutil.copytree(include_src, inc)
    src = os.path.join(tmp, "src")
    os.makedirs(src, exist_ok=True)
    for f in DROPINS:
        shutil.copy(os.path.join(INTEG, f), src)
    return inc, src


@pytest.mark.parametrize("local_ba", [False, True])
def test_dropins_compile_against_unchanged_headers(tmp_path, local_ba):
    inc, src = tree(str(tmp_path), os.path.join(REF, "include"))
    for f in DROPINS:
        r = gxx(os.path.join(src, f), inc, *(["-DLORB_LOCAL_BA"] if local_ba else []))
        assert r.returncode == 0, f"{f}:\n{r.stderr[-4000:]}"


def test_reference_caller_compiles_unchanged():
    # the reference's own tracking thread, the caller of Matcher / BA / LocalMapping
    r = gxx(os.path.join(REF, "src", "visual_odometry.cpp"), os.path.join(REF, "include"))
    assert r.returncode == 0, r.stderr[-4000:]


def test_changed_signature_is_caught(tmp_path):
    mut = tmp_path / "include_mut"
    shutil.copytree(os.path.join(REF, "include"), mut)
    h = (mut / "matcher.h").read_text()
    h2 = h.replace("SearchByProjection(Frame* CurrentFrame, Frame* LastFrame, const float th);",
                   "SearchByProjection(Frame* CurrentFrame, Frame* LastFrame, const int th);", 1)
    assert h2 != h
    (mut / "matcher.h").write_text(h2)
    inc, src = tree(str(tmp_path / "t"), str(mut))
    r = gxx(os.path.join(src, "matcher.cpp"), inc)
    assert r.returncode != 0
    assert "SearchByProjection" in r.stderr


def test_friend_patched_headers_compile_the_row_adapters(tmp_path):
    """the §8f row 2/4 adapters read private Frame / MapPoint members and need
    two friend declarations; with them, every adapter instantiates on the reference's types."""
    inc = tmp_path / "include"
    shutil.copytree(os.path.join(REF, "include"), inc)
    fwd = "namespace lorb { template <class> struct FrameTraits; template <class> struct PointTraits; }\n"
    for name, cls, frd in (("frame.h", "Frame", "friend struct lorb::FrameTraits<Frame>;"),
                           ("map_point.h", "MapPoint", "friend struct lorb::PointTraits<MapPoint>;")):
        s = (inc / name).read_text()
        s = s.replace("namespace Simple_ORB_SLAM", fwd + "namespace Simple_ORB_SLAM", 1)
        s2 = re.sub(r"(class %s\s*\{\s*public:)" % cls, r"\1\n\t%s\npublic:" % frd, s, count=1)
        assert s2 != s, name
        (inc / name).write_text(s2)
    r = gxx(os.path.join(ROOT, "tests", "compile", "friends_tu.cpp"), str(inc), "-DLORB_REFERENCE_FRIENDS")
    assert r.returncode == 0, r.stderr[-4000:]
