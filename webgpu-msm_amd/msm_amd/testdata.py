"""The reference's on-disk test-case format (src/test-data/testCases.ts:34-52).

    points file : one JSON object per line, {"x": "<dec>", "y": "<dec>", "t": "<dec>", "z": "<dec>"}
                  (every string is parsed as a BigInt, testCases.ts:38-43)
    scalars file: one decimal integer per line (testCases.ts:45-48)

The reference ships these for 2^16..2^20 as Git-LFS objects (public/test-data/**) together with
their expected results (testCases.ts:11-32, `EXPECTED_POWERS` below).  `load_test_case` returns
wire buffers ready for `compute_msm_wire`; `write_test_case` produces files in the same format.
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional, Sequence, Tuple

import numpy as np

# testCases.ts:11-32 (getExpectedResult)
EXPECTED_POWERS: Dict[int, Tuple[int, int]] = {
    16: (4490298471131273381350715833932091894064554978284853693957586604825823442429,
         207233051598812890797414182362695316831408959017076683749810755208551572458),
    17: (405755281347735151880827575059343698498813029460786026451708154294960743560,
         7112985356832152643523650125935205310677117771129806490701829425450717492869),
    18: (4020134989704514076121556080357844499902614818105934254331815581426895427831,
         2694327822589008080344499645494473764166611881342421427746308662023437975766),
    19: (3856727778963570638772781884183843350150969534777451295534564482755471873113,
         1398750101296346671684024297455637342909036274728274942667983346895370713922),
    20: (5201851187583570844529445080011852189038251929148722905178398320328749074909,
         3586360219804356686204324370397321114669962278596135149389460948678051407803),
}

_LFS_MAGIC = "version https://git-lfs.github.com/spec/v1"


def _words(v: int) -> np.ndarray:
    """Unsigned integer < 2^256 -> 8 big-endian u32 words (webgpu/utils.test.ts:4-41 order)."""
    if v < 0 or v >> 256:
        raise ValueError(f"value out of range for 256 bits: {v}")
    return np.frombuffer(v.to_bytes(32, "big"), dtype=">u4").astype(np.uint32)


def is_lfs_pointer(path: str) -> bool:
    """True when `path` is a Git-LFS pointer stub instead of the data (as in the reference tree)."""
    with open(path, "r", errors="replace") as f:
        return f.readline().strip() == _LFS_MAGIC


def load_points(path: str, limit: Optional[int] = None) -> np.ndarray:
    """JSON-lines points -> [n][32] u32 wire words (x|y|t|z, BE)."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            obj = json.loads(line)
            rows.append(np.concatenate([_words(int(obj[k])) for k in ("x", "y", "t", "z")]))
            if limit is not None and len(rows) >= limit:
                break
    return np.stack(rows) if rows else np.zeros((0, 32), np.uint32)


def load_scalars(path: str, limit: Optional[int] = None) -> np.ndarray:
    """One decimal per line -> [n][8] u32 wire words (BE)."""
    rows = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            rows.append(_words(int(line)))
            if limit is not None and len(rows) >= limit:
                break
    return np.stack(rows) if rows else np.zeros((0, 8), np.uint32)


def load_test_case(points_path: str, scalars_path: str, limit: Optional[int] = None):
    """loadTestCase (testCases.ts:34-52) for explicit paths: (points [n][32], scalars [n][8])."""
    for p in (points_path, scalars_path):
        if is_lfs_pointer(p):
            raise FileNotFoundError(f"{p} is a Git-LFS pointer stub, not the test data")
    return load_points(points_path, limit), load_scalars(scalars_path, limit)


def load_powers_case(test_data_dir: str, power: int):
    """The reference's `public/test-data` layout: returns (points, scalars, expected (x, y))."""
    pts = os.path.join(test_data_dir, "points", f"{power}-power-points.txt")
    scs = os.path.join(test_data_dir, "scalars", f"{power}-power-scalars.txt")
    p, s = load_test_case(pts, scs)
    return p, s, EXPECTED_POWERS[power]


def write_test_case(points_path: str, scalars_path: str, points: Sequence[Tuple[int, int, int, int]],
                    scalars: Sequence[int]) -> None:
    """Write (x, y, t, z) points and scalars in the reference's format."""
    with open(points_path, "w") as f:
        for x, y, t, z in points:
            f.write(json.dumps({"x": str(x), "y": str(y), "t": str(t), "z": str(z)}, separators=(",", ":")) + "\n")
    with open(scalars_path, "w") as f:
        for s in scalars:
            f.write(f"{int(s)}\n")
