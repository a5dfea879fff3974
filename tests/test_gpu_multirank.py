"""The multi-GPU configurations' code paths on the HIP kernels (BASELINE configs[3] and [4]).

No 8-GPU node is available to these tests, so each runs bench.py itself under torchrun with two
ranks that share GPU 0 over the gloo backend (MSM_DIST_BACKEND=gloo): the same shard split,
pipelined per-rank partials, one all_gather per K steps and rank-0 join (configs[3]), and the
same replica dealing of a shared-base prover batch (configs[4]) that the driver's 8-GPU run
exercises over RCCL.  bench.py checks every result against its closed form
(tests/golden/bench_expected.json) and prints "correct".
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _torchrun(nproc, *bench_args, timeout=240):
    env = dict(os.environ, MSM_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 2000),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), *bench_args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_point_sharded_2_ranks_2_20():
    # configs[3] shape on 2 ranks: each rank pipelines 2^19-point partials; distinct scalar sets
    # per step; every joined result checked
    out = _torchrun(2, "--points", str(1 << 20), "--steps", "6", "--warmup", "2", "--no-extras", "--no-cpu-baseline")
    assert out["n_gpus"] == 2 and out["results_checked"] == 6
    assert out["correct"] is True


def test_point_sharded_3_ranks_uneven():
    # uneven shards (2^16 over 3 ranks)
    out = _torchrun(3, "--points", str(1 << 16), "--steps", "5", "--warmup", "1", "--no-extras", "--no-cpu-baseline")
    assert out["results_checked"] == 5 and out["correct"] is True


def test_prover_batch_replicas_2_ranks():
    # configs[4] code path: 16 distinct-seed 2^18-point MSMs over one base vector, dealt to 2 ranks
    out = _torchrun(2, "--batch", "16", "--points", str(1 << 18), "--steps", "2", "--warmup", "1")
    assert out["results_checked"] == 32
    assert out["correct"] is True


def test_point_sharded_8_ranks_configs3_shape():
    # configs[3] at its real shape: 8 ranks, 2^17-point shards (the throughput window and four
    # MSMs per launch), the 8-way batched join on rank 0
    out = _torchrun(8, "--points", str(1 << 20), "--steps", "4", "--warmup", "1", "--no-extras", "--no-cpu-baseline",
                    timeout=420)
    assert out["n_gpus"] == 8 and out["results_checked"] == 4
    assert out["correct"] is True


def test_prover_batch_64_replicas_configs4_shape():
    # configs[4] at its real shape: 64 distinct-seed 2^18-point MSMs over one base vector, dealt
    # to 2 ranks; every one of the 64 results checked against its closed form
    out = _torchrun(2, "--batch", "64", "--points", str(1 << 18), "--steps", "1", "--warmup", "1", timeout=300)
    assert out["results_checked"] == 64
    assert out["correct"] is True
