"""C-ABI boundary checks that need no GPU: every symbol include/msm.h declares is exported by
libmsm.so, and the host-side entry points (split, point_add_affine, combine, generators) agree
with the oracle."""
import ctypes
import json
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import msm_amd as M
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "msm.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(msm_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ("msm_init", "msm_compute", "msm_compute_device", "msm_point_add_affine", "msm_split",
                 "msm_best_window", "msm_combine_partials", "msm_compute_batch_device"):
        assert must in names


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", M.lib_path()], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    L = M.load()
    for n in declared_functions():
        assert isinstance(getattr(L, n), ctypes._CFuncPtr)


def test_addon_exports():
    addon = os.path.join(ROOT, "webgpu-msm_amd", "js", "msm_napi.node")
    assert os.path.exists(addon)
    out = subprocess.run(["nm", "-D", addon], capture_output=True, text=True, check=True).stdout
    assert "napi_module_register" in out  # NAPI_MODULE registers through a static constructor
    node = shutil.which("node")
    if node:
        script = f"const a = require({addon!r}); console.log(Object.keys(a).sort().join(','))"
        keys = subprocess.run([node, "-e", script], capture_output=True, text=True, check=True).stdout.strip()
        assert keys.split(",") == sorted(["computeMsmU32", "computeMsmBigInt", "pointAddAffine", "split",
                                          "bestWindowSize", "init", "deviceCount", "deviceOrdinals", "strerror",
                                          "flattenU32"])


def test_addon_native_flatten_matches_js():
    # the native flatten (measured slower than the JS loop, tools/node_flatten_ab.mjs) writes the
    # same wire words, and rejects coordinates that are not 8-word Uint32Arrays
    node = shutil.which("node")
    if not node:
        pytest.skip("node not installed")
    js = os.path.join(ROOT, "webgpu-msm_amd", "js", "submission.mjs")
    addon = os.path.join(ROOT, "webgpu-msm_amd", "js", "msm_napi.node")
    script = f"""
import {{ createRequire }} from "module";
import {{ flattenU32 }} from {js!r};
const a = createRequire({addon!r})({addon!r});
const mk = (k) => Uint32Array.from({{length: 8}}, (_, i) => (k * 8 + i) * 2654435761 >>> 0);
const pts = [], sc = [];
for (let i = 0; i < 37; i++) {{ pts.push({{x: mk(4 * i), y: mk(4 * i + 1), t: mk(4 * i + 2), z: mk(4 * i + 3)}}); sc.push(mk(999 + i)); }}
const [pb, sb] = flattenU32(pts, sc);
const pw = new Uint32Array(37 * 32), sw = new Uint32Array(37 * 8);
const n = a.flattenU32(pts, sc, pw, sw);
let bad = 0;
try {{ a.flattenU32([{{x: [1], y: mk(0), t: mk(0), z: mk(0)}}], [mk(1)], pw, sw); }} catch (e) {{ bad = 1; }}
console.log(JSON.stringify({{n, same: pb.every((v, i) => v === pw[i]) && sb.every((v, i) => v === sw[i]), bad}}));
"""
    r = subprocess.run([node, "--input-type=module", "-e", script], capture_output=True, text=True, check=True)
    assert json.loads(r.stdout) == {"n": 37, "same": True, "bad": 1}


def test_addon_bigint_marshalling_errors():
    """computeMsmBigInt checks every coordinate while marshalling (in blocks of 1,024 points, each
    in its own handle scope): a bad element past the first block is still reported synchronously
    with the reference's error class, and a throwing getter's own exception propagates."""
    node = shutil.which("node")
    if not node:
        pytest.skip("node not installed")
    addon = os.path.join(ROOT, "webgpu-msm_amd", "js", "msm_napi.node")
    script = f"""
const a = require({addon!r});
const n = 3000;
const pts = Array.from({{length: n}}, () => ({{x: 1n, y: 2n, t: 3n, z: 1n}}));
const sc = Array.from({{length: n}}, () => 5n);
const out = [];
const tryit = (f) => {{ try {{ f(); return 'ok'; }} catch (e) {{ return e.constructor.name + ':' + e.message; }} }};
const p1 = pts.slice(); p1[2500] = {{x: -1n, y: 2n, t: 3n, z: 1n}};
out.push(tryit(() => a.computeMsmBigInt(p1, sc)));
const s1 = sc.slice(); s1[1500] = 1n << 256n;
out.push(tryit(() => a.computeMsmBigInt(pts, s1)));
const p2 = pts.slice(); p2[2048] = {{get x() {{ throw new Error('getter'); }}, y: 2n, t: 3n, z: 1n}};
out.push(tryit(() => a.computeMsmBigInt(p2, sc)));
out.push(tryit(() => a.computeMsmBigInt(5, sc)));
console.log(JSON.stringify(out));
"""
    got = json.loads(subprocess.run([node, "-e", script], capture_output=True, text=True, check=True).stdout)
    assert got[0] == "RangeError:point coordinate must be a bigint in [0, 2^256)"
    assert got[1] == "RangeError:scalar must be a bigint in [0, 2^256)"
    assert got[2] == "Error:getter"
    assert got[3].startswith("TypeError:")


def test_init_reports_device_state():
    rc = M.load().msm_init()
    assert rc in (0, -6)
    if rc == -6:  # no GPU here: every compute entry must fail loudly (no CPU fallback)
        with pytest.raises(M.MsmError) as e:
            M.compute_msm_wire(O.gen_points(3), O.ints_to_be_words([1, 2, 3]))
        assert e.value.code == -6
        for ratio in (0.5, 1.0):  # the co-compute entry too, even when the host would take every point
            with pytest.raises(M.MsmError) as e:
                M.compute_msm_wire(O.gen_points(3), O.ints_to_be_words([1, 2, 3]), cpu_work_ratio=ratio)
            assert e.value.code == -6


@pytest.mark.parametrize("ratio", [-0.5, float("nan"), float("-inf")])
def test_cocompute_rejects_bad_ratio(ratio):
    """msm_compute_cocompute checks cpu_work_ratio before anything else (no GPU needed)."""
    with pytest.raises(M.MsmError) as e:
        M.compute_msm_wire(O.gen_points(3), O.ints_to_be_words([1, 2, 3]), cpu_work_ratio=ratio)
    assert e.value.code == -1


@pytest.mark.parametrize("ratio", [0.0, 0.5, 1.0])
def test_cocompute_rejects_window_range(ratio):
    """A window range (MSM_FLAG_WINDOWS) has no host counterpart: msm_compute_cocompute rejects it
    before touching a device, at every ratio."""
    L = M.load()
    pts, sc = O.gen_points(3), O.ints_to_be_words([1, 2, 3])
    o = np.zeros(16, np.uint32)
    opts = M._opts(15, windows=(0, 8))
    rc = L.msm_compute_cocompute(M._ptr(np.ascontiguousarray(pts, np.uint32)), M._ptr(np.ascontiguousarray(sc, np.uint32)),
                                 3, opts, float(ratio), 1, o.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    assert rc == -1


def test_strerror_and_best_window():
    assert M.load().msm_strerror(0) == b"ok"
    assert M.load().msm_strerror(-3) == b"coordinate not in [0, p)"
    for n in (1, 1 << 10, 1 << 16, 1 << 20, 1 << 24):
        c = M.get_best_window_size(n)
        assert 8 <= c <= 16
    assert M.get_best_window_size(1 << 20) >= M.get_best_window_size(1 << 12)


@pytest.mark.parametrize("c", [8, 9, 10, 11, 12, 13, 14, 15, 16, 20])
def test_split_dynamic_matches_oracle(c):
    rng = np.random.default_rng(c)
    sc = rng.integers(0, 2**32, size=(37, 8), dtype=np.uint64).astype(np.uint32)
    sc[0] = 0xFFFFFFFF
    sc[1] = 0
    assert np.array_equal(M.split_dynamic(c, sc), O.split(c, sc))


def test_split_rejects_bad_window():
    with pytest.raises(M.MsmError):
        M.split_dynamic(0, np.zeros((1, 8), np.uint32))


def test_point_add_affine_matches_oracle(golden):
    for a, b, exp in golden["kats"]["add_points_x"]["cases"]:
        pa, pb = O.point_from_x(int(a)), O.point_from_x(int(b))
        got = M.point_add_affine(pa, pb)
        assert got == O.aff_add(pa, pb)
        assert got[0] == int(exp)
    assert M.point_add_affine(O.G, O.IDENTITY) == O.G
    assert M.point_add_affine(O.G, O.aff_neg(O.G)) == O.IDENTITY
    with pytest.raises(M.MsmError):
        M.point_add_affine((O.P, 1), O.G)


def test_combine_partials():
    pts = [O.scalar_mul(O.G, k) for k in (3, 10, 77, 1000)]
    parts = np.zeros((4, 32), np.uint32)
    for i, (x, y) in enumerate(pts):
        z = 5 + i  # projective, z != 1
        X, Y, T = x * z % O.P, y * z % O.P, x * y % O.P * z % O.P
        for j, v in enumerate((X, Y, T, z)):
            parts[i, 8 * j: 8 * j + 8] = O.int_to_be_words(v)
    assert M.combine_partials(parts) == O.scalar_mul(O.G, 3 + 10 + 77 + 1000)
    assert M.combine_partials(np.zeros((0, 32), np.uint32)) == O.IDENTITY


def test_generators_match_oracle():
    assert np.array_equal(M.gen_points(300, k0=5, step=9), O.gen_points(300, k0=5, step=9))
    assert np.array_equal(M.gen_points(5000), O.gen_points(5000))
    assert np.array_equal(M.gen_scalars(777, seed=3), O.xorshift_scalars_np(777, seed=3))


def test_opts_struct_layout_matches_header():
    """msm_opts: the original 16-byte layout, then the device list (include/msm.h)."""
    src = open(HEADER).read()
    body = src[src.index("typedef struct msm_opts {"):src.index("} msm_opts;")]
    names = []
    for decl in re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\s*\*?\s*([a-z_][a-z_, ]*);", body, flags=re.M):
        names += [x.strip() for x in decl.split(",")]
    assert names == [n for n, _ in M.MsmOpts._fields_]
    assert ctypes.sizeof(M.MsmOpts) == 40
    assert M.MsmOpts.devices.offset == 16 and M.MsmOpts.n_devices.offset == 24
    assert M.MsmOpts.window_lo.offset == 32 and M.MsmOpts.window_hi.offset == 36
    flags = dict(re.findall(r"#define (MSM_FLAG_[A-Z_]+) (\d+)u", src))
    assert int(flags["MSM_FLAG_SERIAL"]) == M.MSM_FLAG_SERIAL and int(flags["MSM_FLAG_DEVICES"]) == M.MSM_FLAG_DEVICES
    assert int(flags["MSM_FLAG_WINDOWS"]) == M.MSM_FLAG_WINDOWS
    assert int(flags["MSM_FLAG_HALF_WINDOWS"]) == M.MSM_FLAG_HALF_WINDOWS
    assert len(set(flags.values())) == len(flags)  # distinct bits
    assert int(re.search(r"#define MSM_MAX_DEVICES (\d+)", src).group(1)) == M.MSM_MAX_DEVICES


@pytest.mark.parametrize("devices", [[], [0, 0], [-1], [1, 2, 1], list(range(17))])
def test_bad_device_lists_rejected_before_any_device_work(devices):
    """Shape errors in a device list are MSM_ERR_INVALID_ARG whether or not a GPU is present."""
    pts, sc = O.gen_points(4), O.ints_to_be_words([1, 2, 3, 4])
    for call in (lambda: M.compute_msm_wire(pts, sc, devices=devices),
                 lambda: M.compute_msm_partial(pts, sc, devices=devices),
                 lambda: M.compute_msm_many([pts], [sc], 4, devices=devices),
                 lambda: M.compute_msm_shared(pts, [sc], 4, devices=devices)):
        with pytest.raises(M.MsmError) as e:
            call()
        assert e.value.code == -1


def test_null_device_list_rejected():
    L = M.load()
    o = M.MsmOpts(0, 0, -1, M.MSM_FLAG_DEVICES)
    o.n_devices = 2  # devices left NULL
    out = (ctypes.c_uint32 * 16)()
    pts, sc = O.gen_points(2), O.ints_to_be_words([1, 2])
    assert L.msm_compute(pts.ctypes.data, sc.ctypes.data, 2, ctypes.byref(o), out) == -1


def test_device_ordinals_consistent():
    L = M.load()
    n = L.msm_device_count()
    assert M.device_ordinals() == [L.msm_device_ordinal(i) for i in range(n)]
    assert L.msm_device_ordinal(-1) == -1 and L.msm_device_ordinal(n) == -1
    if n == 0:  # no GPU here: a well-formed list fails loudly with MSM_ERR_NO_DEVICE
        with pytest.raises(M.MsmError) as e:
            M.compute_msm_wire(O.gen_points(3), O.ints_to_be_words([1, 2, 3]), devices=[0])
        assert e.value.code == -6


def test_window_count():
    """msm_window_count: balanced main windows over scalar bits [0, 254) plus the overflow window
    (DESIGN.md §2); 0 for an unsupported width."""
    L = M.load()
    for c in range(4, 21):
        assert L.msm_window_count(c) == -(-254 // c) + 1 == M.window_count(c)
    assert L.msm_window_count(16) == 17 and L.msm_window_count(0) == 0 and L.msm_window_count(21) == 0
