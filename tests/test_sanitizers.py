"""CPU: sanitizer runs of the host code (SURVEY §5 "Race detection / sanitizers").

* ASan + UBSan: the C++ host layer (include/lorb/adapters.hpp, local_mapping.hpp) driven by
  tests/cpp/test_adapters.cpp, and every oracle entry point (tests/cpp/sanitize_oracle.c);
* TSan: the same host-layer test, whose LocalMapping queue runs on a mapper thread while the
  test thread inserts keyframes and polls it (the reference pops that queue without its lock,
  src/local_mapping.cpp:51-54).

The host layer calls the C-ABI; here it is linked against tests/cpp/abi_loopback.c, a test double
that forwards to the oracle (no GPU in this container; GPU sanitizers are unavailable on the pool).
"""
import fcntl
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")


def _build():
    # one make at a time: under pytest-xdist the three tests would otherwise build the same
    # targets concurrently and read half-written binaries
    os.makedirs(os.path.join(CPP, "_build"), exist_ok=True)
    with open(os.path.join(CPP, "_build", ".sanitize.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-j8", "-C", CPP, "sanitize"], check=True, capture_output=True, timeout=600)


def _run(binary, **env):
    e = dict(os.environ, **env)
    return subprocess.run([os.path.join(CPP, "_build", binary)], capture_output=True, text=True, timeout=600, env=e)


def test_host_layer_asan_ubsan():
    _build()
    # the test harness allocates frames it never frees: leaks are not what this run checks
    r = _run("adapters_asan", ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    assert r.returncode == 0 and "RESULT PASS" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_oracle_asan_ubsan():
    _build()
    r = _run("oracle_asan", ASAN_OPTIONS="detect_leaks=1:halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    assert r.returncode == 0 and "sanitize_oracle ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_host_layer_tsan():
    _build()
    r = _run("adapters_tsan", TSAN_OPTIONS="halt_on_error=1:exitcode=66")
    assert r.returncode == 0 and "RESULT PASS" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr
