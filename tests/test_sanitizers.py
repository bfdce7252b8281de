"""Host-side race / memory checking of the native runtime:
the transport stress test (6 producer threads on 4 contexts streaming
checksummed frames through a recycling slot allocator, plus concurrent
REQ/REP socket churn) built with ThreadSanitizer and AddressSanitizer.

TSan uses ROCm's clang: GCC 11's libtsan does not intercept
pthread_cond_clockwait (std::condition_variable::wait_until on the steady
clock) and reports bogus "double lock"s."""
import os
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SRCS = ['csrc/tests/stress_transport.cpp', 'csrc/transport/zmtp.cpp', 'csrc/codec/pickle_codec.cpp']
CLANG = '/opt/rocm/lib/llvm/bin/clang++'


@pytest.mark.slow
@pytest.mark.parametrize('san', ['thread', 'address'])
def test_transport_stress_sanitized(tmp_path, san, free_port):
    port = free_port  # 20 probed-free ports; the stress binds 6 of them
    cxx = CLANG if (san == 'thread' and os.path.exists(CLANG)) else 'g++'
    exe = tmp_path / f'stress_{san}'
    cmd = [cxx, '-std=c++17', '-O1', '-g', f'-fsanitize={san}', '-pthread', *[str(ROOT / s) for s in SRCS],
           '-o', str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS='halt_on_error=1 second_deadlock_stack=1',
               ASAN_OPTIONS='detect_leaks=0:halt_on_error=1')
    r = subprocess.run([str(exe), str(port), '--churn'], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert 'received=900 bad=0' in r.stdout
    assert 'WARNING: ThreadSanitizer' not in r.stderr


@pytest.mark.slow
@pytest.mark.parametrize('san', ['thread', 'address'])
def test_shmring_stress_sanitized(tmp_path, san):
    """Shared-memory frame ring under TSan/ASan: 4 producer threads x 3
    consumers with separate mappings, generation checks around every read,
    5% of descriptors dropped so the producers must recover slots through
    the lease."""
    cxx = CLANG if (san == 'thread' and os.path.exists(CLANG)) else 'g++'
    exe = tmp_path / f'stress_shm_{san}'
    cmd = [cxx, '-std=c++17', '-O1', '-g', f'-fsanitize={san}', '-pthread',
           str(ROOT / 'csrc/tests/stress_shmring.cpp'), str(ROOT / 'csrc/transport/shmring.cpp'), '-o', str(exe), '-lrt']
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, TSAN_OPTIONS='halt_on_error=1', ASAN_OPTIONS='detect_leaks=0:halt_on_error=1')
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert 'corrupt=0' in r.stdout and 'WARNING: ThreadSanitizer' not in r.stderr
    stats = dict(kv.split('=') for kv in r.stdout.split())
    assert int(stats['reclaimed']) > 0 and int(stats['verified']) > 1000


@pytest.mark.slow
def test_wire_fuzz_asan_ubsan(tmp_path, free_port):
    """Peer-controlled bytes under ASan + UBSan (csrc/tests/fuzz_wire.cpp):
    20k mutated pickles (wrapping 64-bit lengths, hostile shapes, truncation)
    never yield a payload range outside the frame, and hostile ZMTP peers
    (zero-size / overlong commands, 2^62-byte frames, garbage) cannot take the
    process down or stop a well-behaved peer's delivery."""
    exe = tmp_path / 'fuzz_wire'
    cmd = ['g++', '-std=c++17', '-O1', '-g', '-fsanitize=address,undefined', '-fno-sanitize-recover=undefined',
           '-pthread', str(ROOT / 'csrc/tests/fuzz_wire.cpp'), str(ROOT / 'csrc/transport/zmtp.cpp'),
           str(ROOT / 'csrc/codec/pickle_codec.cpp'), '-o', str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=0:halt_on_error=1', UBSAN_OPTIONS='halt_on_error=1')
    r = subprocess.run([str(exe), str(free_port)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert 'bad_ranges=0' in r.stdout and 'delivered=1' in r.stdout
