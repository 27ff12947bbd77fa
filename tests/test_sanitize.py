"""CPU: host sanitizer runs ("host ASan/TSan builds of the C++
restatement").  No GPU is involved; the device code is not instrumented.

* AddressSanitizer + UndefinedBehaviorSanitizer: libbfrs_host_asan.so (the
  whole library, host code instrumented: make -C blockframe-rs_amd/csrc
  host-asan) and liboracle_asan.so (make -C oracle sanitize) under
  LD_PRELOAD of clang's ASan runtime, running the CPU suites that reach the
  host code -- the oracle, the integrity code (BLAKE3, Merkle, manifests),
  the C-ABI planner, the store and the malformed-manifest corpus.  UB aborts
  (-fno-sanitize-recover), so any finding fails the run.
* ThreadSanitizer: tools/tsan_host.cpp (threaded BLAKE3 + host_copy) and
  tools/tsan_oracle.c (oracle_batch workers, cold-start table init).
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "blockframe-rs_amd", "csrc")
HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
CLANG_RT = "/opt/rocm/lib/llvm/lib/clang"

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


def _asan_runtime():
    for ver in sorted(os.listdir(CLANG_RT), reverse=True) if os.path.isdir(CLANG_RT) else []:
        p = os.path.join(CLANG_RT, ver, "lib", "linux", "libclang_rt.asan-x86_64.so")
        if os.path.exists(p):
            return p
    pytest.skip("clang ASan runtime not found")


def _make(*args):
    subprocess.run(["make", "-s", "-j8", *args], check=True, capture_output=True, text=True)


@pytest.fixture(scope="module")
def sanitized_builds():
    _make("-C", CSRC, "host-asan", "host-tsan")
    _make("-C", os.path.join(ROOT, "oracle"), "sanitize")


def test_host_suites_under_asan_ubsan(sanitized_builds, tmp_path):
    logs = tmp_path / "san"
    logs.mkdir()
    env = dict(os.environ,
               LD_PRELOAD=_asan_runtime(),
               ASAN_OPTIONS=f"detect_leaks=0:abort_on_error=1:halt_on_error=1:log_path={logs}/asan",
               UBSAN_OPTIONS=f"halt_on_error=1:print_stacktrace=1:log_path={logs}/ubsan",
               BFRS_LIB="libbfrs_host_asan.so", ORACLE_LIB="liboracle_asan.so")
    tests = ["tests/test_oracle.py", "tests/test_integrity.py", "tests/test_abi.py",
             "tests/test_store.py", "tests/test_malformed.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu",
                        "-p", "no:cacheprovider", "--basetemp", str(tmp_path / "bt"), *tests],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=1500)
    out = r.stdout[-3000:] + r.stderr[-2000:]
    reports = "".join(p.read_text()[:6000] for p in sorted(logs.iterdir()))
    assert not reports, reports  # a sanitizer report (pytest's capture hides stderr)
    assert r.returncode == 0, out
    assert " passed" in r.stdout
    # the sanitized libraries were the ones loaded (the suites check LIB_PATH too)
    probe = subprocess.run(
        [sys.executable, "-c",
         "import sys; sys.path[:0] = ['blockframe-rs_amd', 'oracle']\n"
         "import bfrs, oracle; bfrs.lib(); oracle.lib()\n"
         "maps = open('/proc/self/maps').read()\n"
         "print('libbfrs_host_asan.so' in maps, 'liboracle_asan.so' in maps)"],
        cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert probe.stdout.split() == ["True", "True"], probe.stdout + probe.stderr


@pytest.mark.parametrize("binary,budget", [("blockframe-rs_amd/csrc/build/tsan_host", None),
                                           ("blockframe-rs_amd/csrc/build/tsan_host", "3"),
                                           ("oracle/_san/tsan_oracle", None)])
def test_threaded_host_code_under_tsan(sanitized_builds, binary, budget):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    if budget is not None:  # host_copy's process-wide helper budget (host_copy.cpp)
        env["BFRS_HOST_COPY_BUDGET"] = budget
    r = subprocess.run([os.path.join(ROOT, binary)], capture_output=True, text=True, timeout=600,
                       env=env)
    out = r.stdout + r.stderr[-4000:]
    assert "ThreadSanitizer" not in out, out
    assert r.returncode == 0 and " ok" in r.stdout, out
