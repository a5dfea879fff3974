"""bench.py's N-GPU modes and the RCCL join, on the one-GPU box.

- `bench.py --gpus N` without torchrun measures N devices in ONE process (devices_bench: a host
  thread per device, resident shards, libmsm's pipelined partial entry, host join).  At N = 1 the
  path runs for real (every timed result checked against its closed form); asking for more devices
  than are visible must fail, never report a one-GPU number as N.
- The torch.distributed "nccl" (= RCCL) code path of msm_amd.dist -- device tensors through
  gather_partials and sharded_msm_many_device -- on a world-size-1 process group on the one GPU
  (the driver's 8-GPU run uses the same calls over 8 ranks).
"""
import json
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT, env=dict(os.environ, WORLD_SIZE="1"))
    return r


def test_devices_mode_one_gpu_2_20():
    r = _bench("--gpus", "1", "--mode", "devices", "--steps", "6", "--warmup", "2", "--no-extras",
               "--no-cpu-baseline")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["results_checked"] == 6 and out["correct"] is True
    assert out["config"]["n_points"] == 1 << 20
    assert out["roofline"]["kernel_ms"] > 0


def test_devices_mode_with_extras_2_18():
    # the lone-MSM latency over the resident shards and the multi-device host-array pass, checked
    r = _bench("--gpus", "1", "--mode", "devices", "--n", str(1 << 18), "--steps", "4", "--warmup", "1",
               "--no-cpu-baseline")
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["correct"] is True and out["latency_ms"] > 0
    assert out["multi_device"]["correct"] is True


def test_more_gpus_than_visible_fails():
    import msm_amd as M

    n = len(M.device_ordinals())
    r = _bench("--gpus", str(n + 1), "--steps", "2", "--warmup", "1", "--no-extras", "--no-cpu-baseline", timeout=120)
    assert r.returncode != 0
    assert "gfx950 device(s) visible" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


RCCL_SCRIPT = textwrap.dedent("""
    import json, os, sys
    sys.path[:0] = [{root!r}, os.path.join({root!r}, "webgpu-msm_amd"), os.path.join({root!r}, "tests")]
    import numpy as np
    import torch
    import torch.distributed as dist
    import msm_amd as M
    from msm_amd.dist import gather_partials, sharded_msm_device, sharded_msm_many_device
    from _closed_form import closed_form

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    assert dist.get_backend() == "nccl"
    n, k = 70001, 5
    pts = M.gen_points(n, k0=3, step=5)
    d_pts = torch.from_numpy(pts.view(np.int32)).to(dev)
    scs = [M.gen_scalars(n, seed=40 + j) for j in range(k)]
    d_scs = [torch.from_numpy(s.view(np.int32)).to(dev) for s in scs]
    torch.cuda.synchronize()
    exp = [closed_form(3, 5, s) for s in scs]
    got = sharded_msm_many_device([d_pts] * k, d_scs, n, 0, device=dev)
    one = sharded_msm_device(d_pts, d_scs[0], n, 0, device=dev)
    parts = M.compute_msm_many_device_partial([d_pts] * k, d_scs, n)
    g = gather_partials(parts, device=dev)
    dist.destroy_process_group()
    print(json.dumps({{"many": [tuple(r) == tuple(e) for r, e in zip(got, exp)],
                      "one": tuple(one) == tuple(exp[0]), "shape": list(g.shape),
                      "same": bool((g[0] == parts).all())}}))
""")


def test_rccl_world_size_1_join(tmp_path):
    script = tmp_path / "rccl1.py"
    script.write_text(RCCL_SCRIPT.format(root=ROOT))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29600 + os.getpid() % 1000), RANK="0",
               WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["many"] == [True] * 5 and out["one"] is True
    assert out["shape"] == [1, 5, 32] and out["same"] is True


def test_peer_access_state():
    # the device-list peer copies enable peer access first; a device with itself is always "enabled",
    # an unknown ordinal is rejected
    import msm_amd as M

    L = M.load()
    devs = M.device_ordinals()
    for a in devs:
        for b in devs:
            assert L.msm_test_peer_state(a, b) in (0, 1)
        assert L.msm_test_peer_state(a, a) == 1
    assert L.msm_test_peer_state(devs[0], 999) == -1
