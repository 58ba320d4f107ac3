"""Race / memory-safety checks of the native host code (SURVEY §5 "race detection /
sanitizers"): the LMDB reader/writer (csrc/lmdb_io.cpp) built as a standalone program under
AddressSanitizer + UndefinedBehaviorSanitizer, round-tripped and fuzzed with corrupted files
(tests/native/lmdb_sanitize.cpp). GPU kernels are checked by their numerics tests; GPU ASan
is not available on the MI355X pool."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which('g++') is None, reason='no host C++ compiler')
def test_lmdb_asan_ubsan_round_trip_and_fuzz(tmp_path):
    exe = str(tmp_path / 'lmdb_sanitize')
    src = os.path.join(ROOT, 'tests', 'native', 'lmdb_sanitize.cpp')
    build = subprocess.run(['g++', '-std=c++17', '-O1', '-g', '-fno-omit-frame-pointer',
                            '-fsanitize=address,undefined', '-fno-sanitize-recover=all',
                            src, '-o', exe], capture_output=True, text=True, timeout=300)
    assert build.returncode == 0, build.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=1:abort_on_error=1',
               UBSAN_OPTIONS='print_stacktrace=1:halt_on_error=1')
    env.pop('LD_PRELOAD', None)
    scratch = tmp_path / 'scratch'
    scratch.mkdir()
    r = subprocess.run([exe, str(scratch), '1500'], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert 'round trips ok' in r.stdout
