"""Host code of libwce.so under sanitizers (race detection /
sanitizers; no GPU involved): the 80-bit shared-state builder (F, the
reference's cofactor invF on a thread pool, the REF / TEXTBOOK / COV
covariances, the sinc table) driven by tools/sanitize_state.cpp, once under
AddressSanitizer + UndefinedBehaviorSanitizer (errors fatal) and once under
ThreadSanitizer."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def built():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "80211parallelestimation_amd", "csrc"), "san"])


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_state_builder_clean_under_sanitizer(built, kind):
    exe = os.path.join(REPO, "tools", f"sanitize_state_{kind}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "sanitize_state ok" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
