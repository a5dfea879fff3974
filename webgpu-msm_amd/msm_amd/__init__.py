"""msm_amd — Python host binding of libmsm (MI355X Edwards-BLS12 MSM).

Mirrors the reference's public surface (src/submission/submission.ts:25-157):

    compute_msm(base_affine_points, scalars, window_size=None) -> (x, y)

with the same input shapes (BigIntPoint-like dicts / tuples, or U32ArrayPoint-like wire words),
the same output ({x, y} as ints, identity = (0, 1)), and the reference's helper entry points
(split_dynamic, point_add_affine, get_best_window_size).  All compute runs in libmsm's HIP
kernels; there is no CPU fallback: if the shared library or a gfx950 device is missing, calls
raise MsmError.
"""
from __future__ import annotations

import atexit
import ctypes
import os
from typing import Iterable, Optional, Sequence, Tuple, Union

import numpy as np

__all__ = [
    "MsmError", "MsmOpts", "load", "compute_msm", "compute_msm_wire", "compute_msm_device",
    "compute_msm_partial", "compute_msm_device_partial", "compute_msm_many_device", "compute_msm_many_device_partial",
    "compute_msm_shared_device", "compute_msm_many", "compute_msm_shared", "compute_msm_cpu", "MSM_FLAG_SERIAL",
    "combine_partials", "combine_partials_many", "point_add_affine",
    "split_dynamic", "get_best_window_size", "set_profiling", "last_profile", "device_count", "device_ordinals",
    "MSM_FLAG_DEVICES", "MSM_FLAG_WINDOWS", "MSM_FLAG_HALF_WINDOWS", "MSM_MAX_DEVICES", "window_count",
    "lib_path", "points_to_wire", "scalars_to_wire", "wire_to_int", "P",
]

P = 8444461749428370424248824938781546531375899335154063827935233455917409239041

_HERE = os.path.dirname(os.path.abspath(__file__))
# MSM_AMD_LIB selects an alternative in-tree build (kernel A/B experiments); default libmsm.so
_LIB = os.environ.get("MSM_AMD_LIB") or os.path.join(_HERE, "_lib", "libmsm.so")


class MsmError(RuntimeError):
    def __init__(self, code: int, where: str = ""):
        self.code = code
        msg = _strerror(code)
        super().__init__(f"libmsm error {code} ({msg}){' in ' + where if where else ''}")


class MsmOpts(ctypes.Structure):
    """include/msm.h msm_opts: the original four fields, then the device list (read by libmsm only
    when flags has MSM_FLAG_DEVICES), then the window range (MSM_FLAG_WINDOWS)."""
    _fields_ = [("window_bits", ctypes.c_uint32), ("run_length", ctypes.c_uint32),
                ("device", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("devices", ctypes.POINTER(ctypes.c_int32)), ("n_devices", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("window_lo", ctypes.c_uint32), ("window_hi", ctypes.c_uint32)]


class MsmProfile(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in (
        "prepare_points", "recode_count", "coarse_scan", "coarse_scatter", "fine_sort", "accumulate",
        "fixup", "bucket_reduce_1", "bucket_reduce_2", "readback", "device_total", "host_tail")] + [
        ("entries", ctypes.c_uint64), ("window_bits", ctypes.c_uint32), ("windows", ctypes.c_uint32),
        ("run_length", ctypes.c_uint32), ("chunk_len", ctypes.c_uint32),
        ("accumulate_sum", ctypes.c_double), ("device_total_sum", ctypes.c_double), ("profiled", ctypes.c_uint32),
        ("msms_per_launch", ctypes.c_uint32), ("accumulate_union_sum", ctypes.c_double)]

MSM_FLAG_SERIAL = 1  # pipelined entries: one launch in flight at a time
MSM_FLAG_DEVICES = 2  # msm_opts carries a device list (include/msm.h)
MSM_FLAG_WINDOWS = 4  # msm_opts carries a window range
MSM_FLAG_HALF_WINDOWS = 8  # with MSM_FLAG_WINDOWS: the range counts half windows
MSM_MAX_DEVICES = 16
MSM_STREAM_NULL = 1  # hip_stream value: order after the null (legacy default) stream


_lib: Optional[ctypes.CDLL] = None


def lib_path() -> str:
    return _LIB


def load() -> ctypes.CDLL:
    """Load libmsm.so (built in-tree by `make -C webgpu-msm_amd`).  Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB):
        raise MsmError(-6, f"libmsm.so not built at {_LIB} (run __graft_entry__.build())")
    # One HIP runtime per process: torch ships its own libamdhip64 (soname libamdhip64.so.7) that
    # its libraries NEED by the unversioned name.  Loading torch first lets libmsm bind to that
    # same runtime by soname; loading libmsm first would pull /opt/rocm's copy and torch would
    # then initialise a second runtime that sees no devices.
    # (MSM_AMD_NO_TORCH=1 skips this: libmsm then runs on /opt/rocm's runtime, as the Node addon and
    # C callers do -- for comparing the two runtimes)
    if not os.environ.get("MSM_AMD_NO_TORCH"):
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
    L = ctypes.CDLL(_LIB)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    vp = ctypes.c_void_p
    sz = ctypes.c_size_t
    optp = ctypes.POINTER(MsmOpts)
    sig = {
        "msm_init": ([], ctypes.c_int),
        "msm_shutdown": ([], None),
        "msm_device_count": ([], ctypes.c_int),
        "msm_device_ordinal": ([ctypes.c_int], ctypes.c_int),
        "msm_strerror": ([ctypes.c_int], ctypes.c_char_p),
        "msm_best_window": ([sz], ctypes.c_uint32),
        "msm_compute": ([vp, vp, sz, optp, u32p], ctypes.c_int),
        "msm_compute_partial": ([vp, vp, sz, optp, u32p], ctypes.c_int),
        "msm_compute_device": ([vp, vp, sz, optp, vp, u32p], ctypes.c_int),
        "msm_compute_device_partial": ([vp, vp, sz, optp, vp, u32p], ctypes.c_int),
        "msm_compute_batch_device": ([vp, vp, sz, sz, optp, vp, u32p], ctypes.c_int),
        "msm_compute_many_device": ([vp, vp, sz, sz, optp, vp, u32p], ctypes.c_int),
        "msm_compute_many_device_partial": ([vp, vp, sz, sz, optp, vp, u32p], ctypes.c_int),
        "msm_compute_shared_device": ([vp, vp, sz, sz, optp, vp, u32p], ctypes.c_int),
        "msm_compute_many": ([vp, vp, sz, sz, optp, u32p], ctypes.c_int),
        "msm_compute_shared": ([vp, vp, sz, sz, optp, u32p], ctypes.c_int),
        "msm_compute_cpu": ([vp, vp, sz, ctypes.c_uint32, ctypes.c_int, u32p], ctypes.c_int),
        "msm_compute_cocompute": ([vp, vp, sz, optp, ctypes.c_double, ctypes.c_int, u32p], ctypes.c_int),
        "msm_combine_partials": ([vp, sz, u32p], ctypes.c_int),
        "msm_combine_partials_many": ([vp, sz, sz, u32p], ctypes.c_int),
        "msm_point_add_affine": ([u32p, u32p, u32p], ctypes.c_int),
        "msm_split": ([ctypes.c_uint32, vp, sz, u32p], ctypes.c_int),
        "msm_split_windows": ([ctypes.c_uint32], ctypes.c_uint32),
        "msm_window_count": ([ctypes.c_uint32], ctypes.c_uint32),
        "msm_set_profiling": ([ctypes.c_int], ctypes.c_int),
        "msm_gen_points": ([u32p, ctypes.c_uint64, ctypes.c_uint64, sz, u32p], ctypes.c_int),
        "msm_gen_scalars": ([ctypes.c_uint64, sz, u32p], ctypes.c_int),
        "msm_last_profile": ([ctypes.POINTER(MsmProfile)], ctypes.c_int),
        "msm_test_field_op": ([ctypes.c_uint32, vp, vp, u32p, sz], ctypes.c_int),
        "msm_test_point_op": ([ctypes.c_uint32, vp, vp, u32p, sz], ctypes.c_int),
        "msm_test_shard_range": ([sz, sz, sz, ctypes.POINTER(sz), ctypes.POINTER(sz)], ctypes.c_int),
        "msm_test_sharded": ([ctypes.c_int, vp, vp, sz, optp, ctypes.POINTER(ctypes.c_int32), ctypes.c_uint32, vp,
                              u32p], ctypes.c_int),
        "msm_test_tail": ([sz, vp, ctypes.c_int, u32p, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "msm_test_tail_words": ([sz], sz),
        "msm_test_plan": ([sz, ctypes.c_uint32, ctypes.c_int, optp, u32p], ctypes.c_int),
        "msm_test_pack": ([vp, sz, ctypes.c_uint32, vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)],
                          ctypes.c_int),
        "msm_test_tail_batch": ([sz, ctypes.c_uint32, vp, ctypes.c_int, u32p, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "msm_test_peer_state": ([ctypes.c_int, ctypes.c_int], ctypes.c_int),
        "msm_test_host_timing": ([ctypes.c_int, sz, ctypes.POINTER(ctypes.c_double)], ctypes.c_int),
        "msm_test_pools": ([ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)], ctypes.c_int),
    }
    for name, (args, res) in sig.items():
        if name.startswith("msm_test_") and not hasattr(L, name):
            continue  # a test hook an older library variant (MSM_AMD_LIB A/B builds) predates
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    # Explicit teardown at interpreter exit (registered after torch's import, so it runs before
    # torch's own exit handlers): the library's streams, buffers and parked pool threads are released
    # and joined while the HIP runtime is still whole, not left to the shared objects' finalizers.
    atexit.register(_shutdown_at_exit)
    return L


def _shutdown_at_exit() -> None:
    if _lib is not None:
        _lib.msm_shutdown()


def _strerror(code: int) -> str:
    try:
        return load().msm_strerror(code).decode()
    except Exception:  # library itself missing
        return "libmsm unavailable"


def _check(rc: int, where: str) -> None:
    if rc != 0:
        raise MsmError(rc, where)


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.uint32)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p) if a.size else None


def _out(n: int) -> Tuple[np.ndarray, ctypes.POINTER(ctypes.c_uint32)]:
    o = np.zeros(n, dtype=np.uint32)
    return o, o.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))


def _opts(window_size: Optional[int], run_length: Optional[int] = None, device: int = -1, flags: int = 0,
          devices: Optional[Sequence[int]] = None, windows: Optional[Tuple[int, int]] = None):
    """A msm_opts by reference.  `devices` (a list of HIP ordinals) runs the call on several
    devices (MSM_FLAG_DEVICES); the array is kept alive by the returned object.  `windows` =
    (lo, hi) restricts the MSM to those signed-digit windows (MSM_FLAG_WINDOWS; needs an explicit
    window_size); (lo, hi, 2) counts the range in half windows (MSM_FLAG_HALF_WINDOWS: half window
    2w is window w's lower-half buckets, 2w + 1 its upper half)."""
    o = MsmOpts(int(window_size or 0), int(run_length or 0), int(device), int(flags))
    if windows is not None:
        o.window_lo, o.window_hi = int(windows[0]), int(windows[1])
        o.flags |= MSM_FLAG_WINDOWS
        if len(windows) > 2:
            if int(windows[2]) not in (1, 2):
                raise ValueError(f"window range unit 1/{windows[2]}: only whole (1) or half (2) windows")
            if int(windows[2]) == 2:
                o.flags |= MSM_FLAG_HALF_WINDOWS
    if devices is not None:
        arr = (ctypes.c_int32 * max(len(devices), 1))(*[int(d) for d in devices])
        o.devices = ctypes.cast(arr, ctypes.POINTER(ctypes.c_int32))
        o.n_devices = len(devices)
        o.flags |= MSM_FLAG_DEVICES
        o._keep = arr
    return ctypes.byref(o)


def wire_to_int(words: Iterable[int]) -> int:
    v = 0
    for w in words:
        v = (v << 32) | int(w)
    return v


def _int_be_words(v: int) -> bytes:
    if v < 0 or v >= 1 << 256:
        raise ValueError("value does not fit 256 bits")
    return int(v).to_bytes(32, "big")


def points_to_wire(points) -> np.ndarray:
    """BigIntPoint[] ({x,y,t,z} ints or (x,y,t,z) tuples) or U32ArrayPoint[] -> wire [n, 32] u32.

    Same layout as submission.ts:35-86 / convert_worker.ts:8-57: x|y|t|z, each 8 BE words.
    A numpy array of shape [n, 32] is taken as already-marshalled wire data.
    """
    if isinstance(points, np.ndarray):
        return _u32(points).reshape(-1, 32)
    pts = list(points)
    if not pts:
        return np.zeros((0, 32), dtype=np.uint32)
    first = pts[0]
    keys = ("x", "y", "t", "z")
    if isinstance(first, dict):
        get = lambda p, k: p[k]  # noqa: E731
    elif hasattr(first, "x"):
        get = lambda p, k: getattr(p, k)  # noqa: E731
    else:
        get = lambda p, k: p[keys.index(k)]  # noqa: E731
    sample = get(first, "x")
    if isinstance(sample, (int, np.integer)):
        buf = b"".join(_int_be_words(int(get(p, k))) for p in pts for k in keys)
        return np.frombuffer(buf, dtype=">u4").astype(np.uint32).reshape(-1, 32)
    out = np.empty((len(pts), 32), dtype=np.uint32)
    for i, p in enumerate(pts):  # U32ArrayPoint: four BE u32[8]
        for j, k in enumerate(keys):
            out[i, 8 * j: 8 * j + 8] = np.asarray(get(p, k), dtype=np.uint32)
    return out


def scalars_to_wire(scalars) -> np.ndarray:
    """bigint[] or Uint32Array[] (BE u32[8]) -> [n, 8] u32."""
    if isinstance(scalars, np.ndarray):
        return _u32(scalars).reshape(-1, 8)
    sc = list(scalars)
    if not sc:
        return np.zeros((0, 8), dtype=np.uint32)
    if isinstance(sc[0], (int, np.integer)):
        buf = b"".join(_int_be_words(int(s)) for s in sc)
        return np.frombuffer(buf, dtype=">u4").astype(np.uint32).reshape(-1, 8)
    return np.stack([np.asarray(s, dtype=np.uint32).reshape(8) for s in sc])


def _xy(o: np.ndarray) -> Tuple[int, int]:
    return wire_to_int(o[:8]), wire_to_int(o[8:16])


def get_best_window_size(n: int) -> int:
    """getBestWindowSize (submission.ts:18-23), retuned for the signed-digit GPU pipeline."""
    return int(load().msm_best_window(n))


def compute_msm_wire(points_wire: np.ndarray, scalars_wire: np.ndarray, window_size: Optional[int] = None,
                     run_length: Optional[int] = None, device: int = -1,
                     devices: Optional[Sequence[int]] = None, cpu_work_ratio: float = 0.0,
                     cpu_threads: int = 0) -> Tuple[int, int]:
    """msm_compute on host wire arrays; `devices` shards the points over those HIP ordinals.
    cpu_work_ratio > 0 is the reference's CPU/GPU co-compute (?cpuWorkRatio, submission.ts:94-154):
    the first floor(ratio n) points on the host Pippenger (cpu_threads threads, 0 = all) beside the
    GPU share, joined with one EC add (msm_compute_cocompute)."""
    L = load()
    pts = _u32(points_wire).reshape(-1, 32)
    sc = _u32(scalars_wire).reshape(-1, 8)
    n = min(pts.shape[0], sc.shape[0])  # the oracle zips to the shorter length
    pts, sc = np.ascontiguousarray(pts[:n]), np.ascontiguousarray(sc[:n])
    o, op = _out(16)
    opts = _opts(window_size, run_length, device, devices=devices)
    if cpu_work_ratio:
        _check(L.msm_compute_cocompute(_ptr(pts), _ptr(sc), n, opts, float(cpu_work_ratio), int(cpu_threads), op),
               "msm_compute_cocompute")
    else:
        _check(L.msm_compute(_ptr(pts), _ptr(sc), n, opts, op), "msm_compute")
    return _xy(o)


def compute_msm(base_affine_points, scalars, window_size: Optional[int] = None,
                run_length: Optional[int] = None, device: int = -1,
                devices: Optional[Sequence[int]] = None, cpu_work_ratio: float = 0.0) -> Tuple[int, int]:
    """compute_msm (submission.ts:25-157): MSM of BigIntPoint[]/U32ArrayPoint[] with bigint[]/Uint32Array[];
    cpu_work_ratio as the reference's ?cpuWorkRatio (compute_msm_wire)."""
    return compute_msm_wire(points_to_wire(base_affine_points), scalars_to_wire(scalars), window_size,
                            run_length, device, devices, cpu_work_ratio)


def compute_msm_partial(points_wire: np.ndarray, scalars_wire: np.ndarray, window_size: Optional[int] = None,
                        device: int = -1, devices: Optional[Sequence[int]] = None,
                        windows: Optional[Tuple[int, int]] = None) -> np.ndarray:
    L = load()
    pts = _u32(points_wire).reshape(-1, 32)
    sc = _u32(scalars_wire).reshape(-1, 8)
    n = min(pts.shape[0], sc.shape[0])
    pts, sc = np.ascontiguousarray(pts[:n]), np.ascontiguousarray(sc[:n])
    o, op = _out(32)
    _check(L.msm_compute_partial(_ptr(pts), _ptr(sc), n,
                                 _opts(window_size, None, device, devices=devices, windows=windows), op),
           "msm_compute_partial")
    return o


def launch_plan(n: int, nm: int = 1, pipelined: bool = False, window_size: Optional[int] = None,
                run_length: Optional[int] = None, windows: Optional[Tuple[int, int]] = None) -> dict:
    """The launch plan libmsm builds for n points and nm MSMs per launch (msm_test_plan; default
    device shape): window width c, windows per MSM in the launch, run length K, reduction chunk L,
    coarse bins per window and the skew floor of K.  No GPU needed."""
    out = np.zeros(7, np.uint32)
    _check(load().msm_test_plan(n, nm, int(pipelined), _opts(window_size, run_length, windows=windows),
                                out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))), "msm_test_plan")
    return dict(zip(("c", "windows", "run_length", "chunk_len", "msms_per_launch", "coarse_bins", "skew_floor"),
                    (int(v) for v in out)))


def pack_points(points_wire, xyz: bool = False) -> Tuple[np.ndarray, bool, bool]:
    """The packed uploads' host packing (msm_test_pack): wire records -> x|y (or x|y|z) words,
    whether every z is 1, whether some t >= p.  No GPU needed."""
    pts = np.ascontiguousarray(_u32(points_wire).reshape(-1, 32))
    n = pts.shape[0]
    w = 24 if xyz else 16
    out = np.zeros((n, w), np.uint32)
    z1, tb = ctypes.c_int(0), ctypes.c_int(0)
    _check(load().msm_test_pack(_ptr(pts), n, 2 if xyz else 1, _ptr(out), ctypes.byref(z1), ctypes.byref(tb)),
           "msm_test_pack")
    return out, bool(z1.value), bool(tb.value)


def window_count(window_size: int) -> int:
    """Signed-digit windows of an MSM at window width c, overflow window included
    (msm_window_count): the index space of the `windows=(lo, hi)` ranges."""
    return int(load().msm_window_count(int(window_size)))


def _dev_ptr(t) -> int:
    return int(t.data_ptr()) if hasattr(t, "data_ptr") else int(t)


def _stream(stream: Optional[int], *tensors) -> Optional[int]:
    """The stream libmsm orders its work after: the caller's, or -- when any input is a torch
    tensor -- torch's current stream on that tensor's device (so inputs written by kernels just
    enqueued there are complete before libmsm reads them).  Raw device pointers with no stream
    leave the ordering to the caller (None)."""
    if stream:
        return stream
    for t in tensors:
        if hasattr(t, "is_cuda") and t.is_cuda:
            import torch

            return torch.cuda.current_stream(t.device).cuda_stream or MSM_STREAM_NULL
    return None


def _first(xs):
    return xs[0] if len(xs) else None


def compute_msm_device(d_points, d_scalars, n: int, window_size: Optional[int] = None,
                       run_length: Optional[int] = None, device: int = -1, stream: int = 0,
                       devices: Optional[Sequence[int]] = None) -> Tuple[int, int]:
    """Inputs already in HBM (torch tensors or raw device pointers, wire layout).  With `devices`
    the listed devices other than the inputs' own copy their shard over xGMI and reduce it."""
    L = load()
    o, op = _out(16)
    _check(L.msm_compute_device(_dev_ptr(d_points), _dev_ptr(d_scalars), n,
                                _opts(window_size, run_length, device, devices=devices),
                                _stream(stream, d_points, d_scalars), op), "msm_compute_device")
    return _xy(o)


def compute_msm_device_partial(d_points, d_scalars, n: int, window_size: Optional[int] = None,
                               device: int = -1, stream: int = 0,
                               devices: Optional[Sequence[int]] = None,
                               windows: Optional[Tuple[int, int]] = None) -> np.ndarray:
    L = load()
    o, op = _out(32)
    _check(L.msm_compute_device_partial(_dev_ptr(d_points), _dev_ptr(d_scalars), n,
                                        _opts(window_size, None, device, devices=devices, windows=windows),
                                        _stream(stream, d_points, d_scalars), op), "msm_compute_device_partial")
    return o


def compute_msm_batch_device(d_points, d_scalars, n: int, count: int, window_size: Optional[int] = None,
                             device: int = -1, stream: int = 0) -> np.ndarray:
    L = load()
    o, op = _out(16 * count)
    _check(L.msm_compute_batch_device(_dev_ptr(d_points), _dev_ptr(d_scalars), n, count,
                                      _opts(window_size, None, device), _stream(stream, d_points, d_scalars), op),
           "msm_compute_batch_device")
    return o.reshape(count, 16)


def compute_msm_many_device(points_list, scalars_list, n: int, window_size: Optional[int] = None,
                            run_length: Optional[int] = None, device: int = -1, stream: int = 0,
                            flags: int = 0) -> np.ndarray:
    """len(points_list) independent n-point MSMs on device-resident inputs (torch tensors or raw
    device pointers), pipelined inside libmsm: the device runs MSM b+1 while the host finishes
    MSM b.  Returns [count][16] BE words (x | y)."""
    L = load()
    count = len(points_list)
    if len(scalars_list) != count:
        raise ValueError("points_list and scalars_list differ in length")
    pp = (ctypes.c_void_p * max(count, 1))(*[_dev_ptr(t) for t in points_list])
    ss = (ctypes.c_void_p * max(count, 1))(*[_dev_ptr(t) for t in scalars_list])
    o, op = _out(16 * max(count, 1))
    _check(L.msm_compute_many_device(ctypes.cast(pp, ctypes.c_void_p), ctypes.cast(ss, ctypes.c_void_p), n, count,
                                     _opts(window_size, run_length, device, flags),
                                     _stream(stream, _first(points_list), _first(scalars_list)), op),
           "msm_compute_many_device")
    return o[:16 * count].reshape(count, 16)


def compute_msm_shared_device(d_points, scalars_list, n: int, window_size: Optional[int] = None,
                              run_length: Optional[int] = None, device: int = -1, stream: int = 0,
                              flags: int = 0) -> np.ndarray:
    """Prover batch: len(scalars_list) MSMs over ONE device-resident base vector (prepared once
    per call).  Returns [count][16] BE words."""
    L = load()
    count = len(scalars_list)
    ss = (ctypes.c_void_p * max(count, 1))(*[_dev_ptr(t) for t in scalars_list])
    o, op = _out(16 * max(count, 1))
    _check(L.msm_compute_shared_device(_dev_ptr(d_points), ctypes.cast(ss, ctypes.c_void_p), n, count,
                                       _opts(window_size, run_length, device, flags),
                                       _stream(stream, d_points, _first(scalars_list)), op),
           "msm_compute_shared_device")
    return o[:16 * count].reshape(count, 16)


def _host_list(arrs, words: int):
    keep = [np.ascontiguousarray(_u32(a).reshape(-1, words)) for a in arrs]
    ptrs = (ctypes.c_void_p * max(len(keep), 1))(*[a.ctypes.data for a in keep])
    return keep, ptrs


def compute_msm_many(points_list, scalars_list, n: int, window_size: Optional[int] = None,
                     run_length: Optional[int] = None, device: int = -1, flags: int = 0,
                     devices: Optional[Sequence[int]] = None) -> np.ndarray:
    """len(points_list) independent n-point MSMs of HOST arrays (wire [n, 32] / [n, 8] each),
    uploaded into libmsm's in-flight launch slots while the others compute.  [count][16]."""
    L = load()
    count = len(points_list)
    if len(scalars_list) != count:
        raise ValueError("points_list and scalars_list differ in length")
    kp, pp = _host_list(points_list, 32)
    ks, ss = _host_list(scalars_list, 8)
    for a, b in zip(kp, ks):
        if a.shape[0] < n or b.shape[0] < n:
            raise ValueError("an input holds fewer than n points/scalars")
    o, op = _out(16 * max(count, 1))
    _check(L.msm_compute_many(ctypes.cast(pp, ctypes.c_void_p), ctypes.cast(ss, ctypes.c_void_p), n, count,
                              _opts(window_size, run_length, device, flags, devices), op), "msm_compute_many")
    return o[:16 * count].reshape(count, 16)


def compute_msm_shared(points_wire, scalars_list, n: Optional[int] = None, window_size: Optional[int] = None,
                       run_length: Optional[int] = None, device: int = -1, flags: int = 0,
                       devices: Optional[Sequence[int]] = None) -> np.ndarray:
    """Prover batch of HOST arrays: one base vector [n, 32], len(scalars_list) scalar vectors
    [n, 8]; the base vector is uploaded and prepared once.  [count][16]."""
    L = load()
    pts = np.ascontiguousarray(_u32(points_wire).reshape(-1, 32))
    n = pts.shape[0] if n is None else n
    ks, ss = _host_list(scalars_list, 8)
    if pts.shape[0] < n or any(b.shape[0] < n for b in ks):
        raise ValueError("an input holds fewer than n points/scalars")
    count = len(ks)
    o, op = _out(16 * max(count, 1))
    _check(L.msm_compute_shared(_ptr(pts), ctypes.cast(ss, ctypes.c_void_p), n, count,
                                _opts(window_size, run_length, device, flags, devices), op), "msm_compute_shared")
    return o[:16 * count].reshape(count, 16)


def compute_msm_cpu(points_wire, scalars_wire, window_size: Optional[int] = None,
                    threads: int = 0) -> Tuple[int, int]:
    """The reference's CPU-only path (cpuWorkRatio = 1, msm_end_to_end lib.rs:106-121) as
    libmsm's own multithreaded host Pippenger (msm_compute_cpu).  Explicit; never a fallback."""
    L = load()
    pts = _u32(points_wire).reshape(-1, 32)
    sc = _u32(scalars_wire).reshape(-1, 8)
    n = min(pts.shape[0], sc.shape[0])
    pts, sc = np.ascontiguousarray(pts[:n]), np.ascontiguousarray(sc[:n])
    o, op = _out(16)
    _check(L.msm_compute_cpu(_ptr(pts), _ptr(sc), n, int(window_size or 0), int(threads), op), "msm_compute_cpu")
    return _xy(o)


def compute_msm_many_device_partial(points_list, scalars_list, n: int, window_size: Optional[int] = None,
                                    run_length: Optional[int] = None, device: int = -1,
                                    stream: int = 0, flags: int = 0,
                                    windows: Optional[Tuple[int, int]] = None) -> np.ndarray:
    """compute_msm_many_device, each result as a projective X|Y|T|Z partial: [count][32] BE words."""
    L = load()
    count = len(points_list)
    if len(scalars_list) != count:
        raise ValueError("points_list and scalars_list differ in length")
    pp = (ctypes.c_void_p * max(count, 1))(*[_dev_ptr(t) for t in points_list])
    ss = (ctypes.c_void_p * max(count, 1))(*[_dev_ptr(t) for t in scalars_list])
    o, op = _out(32 * max(count, 1))
    _check(L.msm_compute_many_device_partial(ctypes.cast(pp, ctypes.c_void_p), ctypes.cast(ss, ctypes.c_void_p), n,
                                             count, _opts(window_size, run_length, device, flags, windows=windows),
                                             _stream(stream, _first(points_list), _first(scalars_list)), op),
           "msm_compute_many_device_partial")
    return o[:32 * count].reshape(count, 32)


def combine_partials(partials: np.ndarray) -> Tuple[int, int]:
    L = load()
    p = _u32(partials).reshape(-1, 32)
    o, op = _out(16)
    _check(L.msm_combine_partials(_ptr(p), p.shape[0], op), "msm_combine_partials")
    return _xy(o)


def combine_partials_many(parts: np.ndarray):
    """parts [world, K, 32] (an all_gather of K partials per rank) -> the K joined affine results."""
    L = load()
    p = np.ascontiguousarray(_u32(parts))
    world, count = p.shape[0], p.shape[1]
    o, op = _out(16 * max(count, 1))
    _check(L.msm_combine_partials_many(_ptr(p.reshape(-1)), world, count, op), "msm_combine_partials_many")
    return [_xy(o[16 * k: 16 * k + 16]) for k in range(count)]


def point_add_affine(a: Tuple[int, int], b: Tuple[int, int]) -> Tuple[int, int]:
    """point_add_affine (lib.rs:240-253)."""
    L = load()
    aw = np.frombuffer(_int_be_words(a[0]) + _int_be_words(a[1]), dtype=">u4").astype(np.uint32)
    bw = np.frombuffer(_int_be_words(b[0]) + _int_be_words(b[1]), dtype=">u4").astype(np.uint32)
    o, op = _out(16)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    _check(L.msm_point_add_affine(aw.ctypes.data_as(u32p), bw.ctypes.data_as(u32p), op), "msm_point_add_affine")
    return _xy(o)


def split_dynamic(window_size: int, scalars_wire: np.ndarray) -> np.ndarray:
    """split_dynamic (lib.rs:196-202): [n_windows * n] u32, window 0 most significant."""
    L = load()
    sc = _u32(scalars_wire).reshape(-1, 8)
    nw = L.msm_split_windows(window_size)
    o, op = _out(max(nw * sc.shape[0], 1))
    _check(L.msm_split(window_size, _ptr(sc), sc.shape[0], op), "msm_split")
    return o[: nw * sc.shape[0]]


BENCH_G = (2796670805570508460920584878396618987767121022598342527208237783066948667246,
           8134280397689638111748378379571739274369602049665521098046934931245960532166)
XORSHIFT_SEED = 0x9E3779B97F4A7C15


def gen_points(n: int, k0: int = 1, step: int = 1, base: Tuple[int, int] = BENCH_G) -> np.ndarray:
    """Wire points [n, 32]: (k0 + i*step) * base (the benchmark page's fixed base, AllBenchmarks.tsx:111-119)."""
    L = load()
    g = np.frombuffer(_int_be_words(base[0]) + _int_be_words(base[1]), dtype=">u4").astype(np.uint32)
    o, op = _out(max(n, 1) * 32)
    _check(L.msm_gen_points(g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), k0, step, n, op), "msm_gen_points")
    return o[: n * 32].reshape(n, 32)


def gen_scalars(n: int, seed: int = XORSHIFT_SEED) -> np.ndarray:
    """Scalars [n, 8] BE: xorshift64(13,7,17), 4 words each (first most significant), mod p."""
    L = load()
    o, op = _out(max(n, 1) * 8)
    _check(L.msm_gen_scalars(seed, n, op), "msm_gen_scalars")
    return o[: n * 8].reshape(n, 8)


def set_profiling(enable=True) -> None:
    """0/False: off.  1/True: hipEvents between every phase (eager launches).  2: k_accumulate and
    the device total only, keeping the captured-graph replay (what bench.py times)."""
    mode = int(enable) if not isinstance(enable, bool) else (1 if enable else 0)
    _check(load().msm_set_profiling(mode), "msm_set_profiling")


def last_profile() -> dict:
    prof = MsmProfile()
    _check(load().msm_last_profile(ctypes.byref(prof)), "msm_last_profile")
    return {name: getattr(prof, name) for name, _ in MsmProfile._fields_}


def device_count() -> int:
    return int(load().msm_device_count())


def device_ordinals() -> list:
    """HIP ordinals of the visible gfx950 devices (msm_device_ordinal)."""
    L = load()
    return [int(L.msm_device_ordinal(i)) for i in range(int(L.msm_device_count()))]


def _test_field_op(op: int, a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Device field op on canonical little-endian word arrays [n, 8] (test hook)."""
    L = load()
    a = _u32(a).reshape(-1, 8)
    b = _u32(b).reshape(-1, 8)
    o, op_ = _out(a.size)
    _check(L.msm_test_field_op(op, _ptr(a), _ptr(b), op_, a.shape[0]), "msm_test_field_op")
    return o.reshape(-1, 8)


def _test_point_op(op: int, p: np.ndarray, q: np.ndarray) -> np.ndarray:
    """Device point op on affine LE word arrays [n, 16] -> projective std LE words [n, 32] (test hook)."""
    L = load()
    p = _u32(p).reshape(-1, 16)
    q = _u32(q).reshape(-1, 16)
    o, op_ = _out(p.shape[0] * 32)
    _check(L.msm_test_point_op(op, _ptr(p), _ptr(q), op_, p.shape[0]), "msm_test_point_op")
    return o.reshape(-1, 32)


def _test_sharded(mode: int, points, scalars, n: int, devices: Sequence[int], window_size: Optional[int] = None,
                  stream: int = 0) -> Tuple[int, int]:
    """Test hook: the device-list shard/join paths with a list that may repeat a device (mode 0:
    host wire arrays as msm_compute, 1: device-resident inputs as msm_compute_device)."""
    L = load()
    arr = (ctypes.c_int32 * len(devices))(*devices)
    o, op = _out(16)
    if mode == 0:
        pts = np.ascontiguousarray(_u32(points).reshape(-1, 32)[:n])
        sc = np.ascontiguousarray(_u32(scalars).reshape(-1, 8)[:n])
        pp, sp, st = _ptr(pts), _ptr(sc), None
    else:
        pp, sp, st = _dev_ptr(points), _dev_ptr(scalars), _stream(stream, points, scalars)
    _check(L.msm_test_sharded(mode, pp, sp, n, _opts(window_size), arr, len(devices), st, op), "msm_test_sharded")
    return _xy(o)
