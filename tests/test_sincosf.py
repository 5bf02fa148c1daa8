"""CPU: the device restatement of libm's cosf / sinf (lorb_slam_amd/csrc/lorb_sincosf.h, used by
the rBRIEF kernel) equals this machine's libm on every float angle the descriptor can form.

src/ORBextractor.cpp:114-115 computes `cos(angle)` with a float argument under `using namespace
std` (:69), i.e. std::cos(float) = cosf.  cosf is not the double cosine rounded to float: the two
differ on ~0.1 % of the angles, and a one-ulp change of a or b can move a cvRound at :121-122.
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sincosf_restatement_matches_libm_on_every_angle(tmp_path):
    exe = str(tmp_path / "sincosf_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-o", exe,
                    os.path.join(ROOT, "tests", "cpp", "sincosf_check.cpp")], check=True, timeout=300)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "mismatches 0" in r.stdout, r.stdout + r.stderr
    assert int(r.stdout.split()[1]) > 1_000_000_000
