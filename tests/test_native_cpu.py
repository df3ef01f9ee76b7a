"""Native runtime self-tests under sanitizers.

tests/native/test_mailbox.cpp drives a 4-rank loopback mesh of the C++ mailbox from
threads of one process.  It is compiled with ROCm's clang (its ThreadSanitizer runtime
intercepts pthread_cond_clockwait, which std::condition_variable::wait_for uses; GCC 11's
does not and reports false double-locks) and run under TSan and ASan+UBSan; any sanitizer
report fails the test.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "smdistributed_modelparallel_amd", "csrc", "runtime")
CXX = next((c for c in ("/opt/rocm/lib/llvm/bin/clang++", shutil.which("clang++")) if c and os.path.exists(c)), None)


@pytest.mark.skipif(CXX is None, reason="clang++ not available")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_mailbox_under_sanitizer(san, tmp_path):
    exe = str(tmp_path / "test_mailbox")
    srcs = [os.path.join(ROOT, "tests", "native", "test_mailbox.cpp"), os.path.join(RT, "mailbox.cpp")]
    subprocess.run([CXX, "-std=c++17", "-g", "-O1", f"-fsanitize={san}", "-fno-omit-frame-pointer",
                    "-I" + RT, *srcs, "-lpthread", "-o", exe], check=True, capture_output=True, text=True)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=180, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "ALL OK" in out
    assert "Sanitizer" not in out, out[-6000:]
