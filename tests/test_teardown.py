"""The library's host thread pools: sized from the CPU quota and the devices of a call, and torn
down cleanly (CPU only, no GPU).

The pools are per device context (packing threads, lone-MSM tail helpers, pipelined-tail
threads); a call over a device list runs one host thread per device.  msm_test_pools reports the
sizes a call over `ndev` devices uses and starts them.  The sanitizer builds (make sanitize) run
the same pools under ASan and TSan and exit with and without msm_shutdown -- the teardown the
Python binding registers with atexit and the Node addon with napi_add_env_cleanup_hook.
"""
import ctypes
import os
import shutil
import subprocess

import pytest

import msm_amd as M

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "webgpu-msm_amd")


def _pools(ndev, run=0):
    out = (ctypes.c_int * 5)()
    assert M.load().msm_test_pools(ndev, run, out) == 0
    return {"budget": out[0], "pack": out[1], "tail": out[2], "horner": out[3], "total": out[4]}


def test_pool_sizes_follow_budget_and_devices():
    one = _pools(1)
    b = one["budget"]
    # one device: the measured defaults on a 16-CPU quota (8 packing, 3 tail helpers, 2 tail threads)
    assert one["pack"] == max(1, min(8, max(2, b) // 2))
    assert one["tail"] == min(3, max(2, b) // 4)
    assert one["horner"] == min(2, max(2, b) // 8)
    if b >= 16:
        assert (one["pack"], one["tail"], one["horner"]) == (8, 3, 2)
    prev = one
    for nd in (2, 4, 8):
        p = _pools(nd)
        assert p["pack"] <= prev["pack"] and p["tail"] <= prev["tail"] and p["horner"] <= prev["horner"]
        prev = p
    # an 8-device call stays within the quota (a floor of two threads per device: its host thread
    # and uploader); on the 16-CPU GPU boxes that is 15 threads
    eight = _pools(8)
    assert eight["total"] <= max(b, 2 * 8), eight
    assert (eight["pack"], eight["tail"], eight["horner"]) == ((1, 0, 0) if b <= 16 else (eight["pack"], eight["tail"], eight["horner"]))


def test_pools_start_and_stop():
    for nd in (1, 8, 1):
        _pools(nd, run=1)
    M.load().msm_shutdown()  # joins them; the library re-creates what a later call needs
    _pools(2, run=1)


def test_bad_device_count_rejected():
    out = (ctypes.c_int * 5)()
    assert M.load().msm_test_pools(0, 0, out) == -1


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc") and not shutil.which("hipcc"), reason="needs hipcc")
@pytest.mark.parametrize("san", ["asan", "tsan"])
def test_pool_teardown_under_sanitizers(san):
    subprocess.run(["make", "-s", "-C", PKG, "sanitize"], check=True, capture_output=True, timeout=900)
    exe = os.path.join(PKG, "build", f"teardown_{san}")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1", TSAN_OPTIONS="halt_on_error=1")
    for mode in ("0", "1"):  # with msm_shutdown, then exiting with the pools parked
        r = subprocess.run([exe, mode], capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "Sanitizer" not in r.stderr, r.stderr
        assert "devices 8:" in r.stdout
