"""Several devices behind the product boundary (msm_opts MSM_FLAG_DEVICES, include/msm.h): the
MSM sharded over a device list inside ONE call -- the reference's CPU/GPU split of compute_msm
(src/submission/submission.ts:116-154, gpu_worker.ts:9-18, joined by point_add_affine
msm-wasm/src/lib.rs:240-253) generalised to gfx950 devices.

The box these tests run on has one GPU, so the lists hold every visible device (one), and the
shard/join machinery with several shards runs through the test hook msm_test_sharded, which may
list the one device repeatedly (its later shards of device-resident inputs then take the xGMI
peer-copy path: a device-to-device copy).  Every result is compared with the closed form."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

import msm_amd as M
from _closed_form import closed_form

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JS = os.path.join(ROOT, "webgpu-msm_amd", "js", "submission.mjs")
NODE = shutil.which("node")


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32)).cuda()


@pytest.fixture(scope="module")
def devices():
    d = M.device_ordinals()
    assert d, "no gfx950 device"
    return d


@pytest.mark.parametrize("n", [1, 1000, (1 << 18) + 3])
def test_host_entry_every_device(devices, n):
    pts = M.gen_points(n, k0=11, step=7)
    sc = M.gen_scalars(n, seed=5 + n % 3)
    exp = closed_form(11, 7, sc)
    assert M.compute_msm_wire(pts, sc, devices=devices) == exp
    part = M.compute_msm_partial(pts, sc, devices=devices)
    assert M.combine_partials(np.asarray(part, np.uint32).reshape(1, 32)) == exp


def test_device_entry_every_device(devices):
    n = 70001
    pts = M.gen_points(n, k0=2, step=9)
    sc = M.gen_scalars(n, seed=8)
    exp = closed_form(2, 9, sc)
    dp, ds = _dev(pts), _dev(sc)
    assert M.compute_msm_device(dp, ds, n, devices=devices) == exp
    part = M.compute_msm_device_partial(dp, ds, n, devices=devices)
    assert M.combine_partials(np.asarray(part, np.uint32).reshape(1, 32)) == exp


def test_host_batches_every_device(devices):
    n, count = 5000, 5
    pts = [M.gen_points(n, k0=1 + b, step=3) for b in range(count)]
    sc = [M.gen_scalars(n, seed=100 + b) for b in range(count)]
    out = M.compute_msm_many(pts, sc, n, devices=devices)
    for b in range(count):
        assert (M.wire_to_int(out[b, :8]), M.wire_to_int(out[b, 8:])) == closed_form(1 + b, 3, sc[b])
    shared = M.compute_msm_shared(pts[0], sc, n, devices=devices)
    for b in range(count):
        assert (M.wire_to_int(shared[b, :8]), M.wire_to_int(shared[b, 8:])) == closed_form(1, 3, sc[b])


@pytest.mark.parametrize("shards", [2, 3, 8])
@pytest.mark.parametrize("n", [5, 100003, (1 << 19) + 1])
def test_shard_join_paths(devices, shards, n):
    """Several shards (the one device repeated through the test hook): host-array shards, each
    uploaded and reduced on its own thread, and device-resident shards, the later ones copied by
    the peer-copy path; joined with one EC add each."""
    pts = M.gen_points(n, k0=4, step=11)
    sc = M.gen_scalars(n, seed=3 + shards)
    exp = closed_form(4, 11, sc)
    lst = [devices[0]] * shards
    assert M._test_sharded(0, pts, sc, n, lst) == exp
    assert M._test_sharded(1, _dev(pts), _dev(sc), n, lst) == exp


def test_invalid_and_repeated_ordinals_rejected(devices):
    pts, sc = M.gen_points(8), M.gen_scalars(8)
    for bad in ([devices[0], devices[0]], [99], [devices[0], 99], []):
        with pytest.raises(M.MsmError) as e:
            M.compute_msm_wire(pts, sc, devices=bad)
        assert e.value.code == -1, bad
        with pytest.raises(M.MsmError):
            M.compute_msm_device(_dev(pts), _dev(sc), 8, devices=bad)
    # device batches take one device
    import ctypes
    L = M.load()
    out = (ctypes.c_uint32 * 16)()
    pp = (ctypes.c_void_p * 1)(_dev(pts).data_ptr())
    ss = (ctypes.c_void_p * 1)(_dev(sc).data_ptr())
    rc = L.msm_compute_many_device(ctypes.cast(pp, ctypes.c_void_p), ctypes.cast(ss, ctypes.c_void_p), 8, 1,
                                   M._opts(None, devices=devices), None, out)
    assert rc == -1


@pytest.mark.skipif(NODE is None, reason="node not installed")
def test_js_compute_msm_devices_option(devices, tmp_path):
    """compute_msm(points, scalars, { devices }) with flat buffers over a SharedArrayBuffer (read
    in place) and over a plain ArrayBuffer (copied by the addon first), and U32ArrayPoint[]."""
    n = 300
    pts = M.gen_points(n, k0=6, step=5)
    sc = M.gen_scalars(n, seed=21)
    exp = closed_form(6, 5, sc)
    pts_f, sc_f = tmp_path / "p.bin", tmp_path / "s.bin"
    pts.astype(np.uint32).tofile(pts_f)
    sc.astype(np.uint32).tofile(sc_f)
    script = f"""
import * as m from {json.dumps(JS)};
import fs from "fs";
const plainP = new Uint32Array(fs.readFileSync({json.dumps(str(pts_f))}).buffer.slice(0));
const plainS = new Uint32Array(fs.readFileSync({json.dumps(str(sc_f))}).buffer.slice(0));
const sabP = new Uint32Array(new SharedArrayBuffer(plainP.length * 4)); sabP.set(plainP);
const sabS = new Uint32Array(new SharedArrayBuffer(plainS.length * 4)); sabS.set(plainS);
const objs = []; const scs = [];
for (let i = 0; i < {n}; i++) {{
  const w = (k) => plainP.slice(32 * i + 8 * k, 32 * i + 8 * k + 8);
  objs.push({{x: w(0), y: w(1), t: w(2), z: w(3)}}); scs.push(plainS.slice(8 * i, 8 * i + 8));
}}
(async () => {{  // Node 12: no top-level await
  const devices = m.deviceOrdinals();
  const out = [];
  out.push(await m.compute_msm(sabP, sabS, {{ devices }}));
  out.push(await m.compute_msm(plainP, plainS, {{ devices }}));
  out.push(await m.compute_msm(objs, scs, {{ devices }}));
  let rejected = false;
  try {{ await m.compute_msm(sabP, sabS, {{ devices: [devices[0], devices[0]] }}); }} catch (e) {{ rejected = e.code === -1; }}
  console.log(JSON.stringify({{ res: out.map((r) => [r.x.toString(), r.y.toString()]), rejected }}));
}})().catch((e) => {{ console.error(e); process.exit(3); }});
"""
    path = tmp_path / "run_dev.mjs"
    path.write_text(script)
    r = subprocess.run([NODE, str(path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout.strip().splitlines()[-1])
    assert all((int(x), int(y)) == exp for x, y in got["res"])
    assert got["rejected"]
