"""GPU: the C++ host layer (include/lorb/adapters.hpp + local_mapping.hpp) driven like the
reference's VisualOdometry, checked against the oracle inside tests/cpp/test_adapters.cpp."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def test_cpp_host_layer():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "_build", "test_adapters")], capture_output=True,
                       text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0 and "RESULT PASS" in r.stdout, r.stdout + r.stderr
