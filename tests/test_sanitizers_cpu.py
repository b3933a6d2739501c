"""ASan/UBSan and TSan runs of the host runtime (BFC allocator, shared-memory PS
with worker thread pools, HET cache) -- SURVEY §5.2.  The sanitizers
instrument standalone C++ binaries (csrc/tests/runtime_sanitize.cc) built from
the same sources as libhetu_runtime / libhetu_alloc."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, 'csrc', 'build')


@pytest.fixture(scope='module')
def binaries():
    r = subprocess.run(['make', '-C', os.path.join(ROOT, 'csrc'), 'sanitize'], capture_output=True, text=True,
                       timeout=600)
    if r.returncode != 0:
        pytest.fail('sanitizer build failed:\n' + r.stderr[-3000:])
    return os.path.join(BUILD, 'runtime_asan'), os.path.join(BUILD, 'runtime_tsan')


def _run(path, env):
    r = subprocess.run([path], capture_output=True, text=True, timeout=600, env=dict(os.environ, **env))
    assert r.returncode == 0 and 'OK' in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
    assert 'ERROR: AddressSanitizer' not in r.stderr and 'WARNING: ThreadSanitizer' not in r.stderr


def test_asan_ubsan_clean(binaries):
    _run(binaries[0], {'ASAN_OPTIONS': 'detect_leaks=0:abort_on_error=0', 'UBSAN_OPTIONS': 'print_stacktrace=1'})


def test_tsan_clean(binaries):
    _run(binaries[1], {'TSAN_OPTIONS': 'halt_on_error=1'})
