"""alphazero::nn::BatchQueue (cpp/include/alphazero/nn/batch_queue.h; reference
include/alphazero/nn/batch_queue.h:28-266, src/nn/batch_queue.cpp:61-363), driven by the C++ test
tests/native/batch_queue_host.cpp on the reference test's MockNeuralNetwork pattern
(tests/nn/batch_queue_test.cpp:11-52): configuration setters, answers equal to a direct evaluation
from several producer threads, priorities, drops, failures, adaptive batch targets, worker
restarts, destruction with pending requests -- plus a ThreadSanitizer build when clang is present.
The GPU case puts the queue in front of the device net (HipNeuralNetwork)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "alphazero-multi-game_amd")
BUILD = os.path.join(PKG, "build")
SRC = os.path.join(HERE, "native", "batch_queue_host.cpp")
INC = ["-I" + os.path.join(PKG, "cpp", "include"), "-I" + os.path.join(ROOT, "include")]


def _build(tmp, extra=(), name="bq"):
    if not os.path.exists(os.path.join(BUILD, "libalphazero_host.so")):
        pytest.skip("build the host library: make -C alphazero-multi-game_amd")
    out = str(tmp / name)
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", *INC, *extra, SRC, "-L" + BUILD, "-lalphazero_host",
                    "-laz_hip", "-Wl,-rpath," + BUILD, "-lpthread", "-o", out], check=True)
    return out


def test_batch_queue_mock(tmp_path):
    exe = _build(tmp_path)
    for _ in range(5):                        # timing-dependent paths: several runs
        r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert r.returncode == 0 and r.stdout.strip() == "OK", r.stderr


@pytest.mark.timeout(300)
def test_batch_queue_thread_sanitizer(tmp_path):
    clang = "/opt/rocm/lib/llvm/bin/clang++"
    if not os.path.exists(clang):
        clang = shutil.which("clang++")
    if not clang:
        pytest.skip("no clang++ (GCC 11's TSan misreads pthread_cond_clockwait)")
    out = str(tmp_path / "bq_tsan")
    srcs = [os.path.join(PKG, "cpp", "src", f) for f in ("batch_queue.cpp", "gomoku_state.cpp", "go_state.cpp")]
    subprocess.run([clang, "-std=c++17", "-O1", "-g", "-fsanitize=thread", *INC, SRC, *srcs, "-lpthread", "-o", out],
                   check=True)
    r = subprocess.run([out], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.strip() == "OK", r.stderr[-4000:]
    assert "ThreadSanitizer" not in r.stderr, r.stderr[-4000:]


@pytest.mark.gpu
def test_batch_queue_device_net(tmp_path):
    exe = _build(tmp_path, extra=["-DAZ_BQ_GPU"], name="bq_gpu")
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and r.stdout.startswith("OK gpu"), r.stdout + r.stderr
