"""The oracle itself, pinned against the reference's own known-answer vectors (CPU only).

Vectors: tests/golden/reference_kats.json (transcribed from wasmFunctions.test.ts,
FieldMath.test.ts, webgpu/utils.test.ts) and tests/golden/msm_vectors.json (closed form,
re-derived survey rows that the Aleo wasm confirmed: SURVEY.md §8c).
"""
import numpy as np
import pytest

from oracle import oracle as O


def test_field_kats(golden):
    k = golden["kats"]
    for a, b, exp in k["add_fields"]["cases"]:
        assert (int(a) + int(b)) % O.P == int(exp)
        assert O.c_field_op(1, int(a), int(b)) == int(exp)
    for a, exp in k["double_field"]["cases"]:
        assert O.c_field_op(4, int(a)) == int(exp)


def test_get_point_from_x_kats(golden):
    for x, y in golden["kats"]["get_point_from_x"]["cases"]:
        assert O.point_from_x(int(x)) == (int(x), int(y))
        assert O.c_point_from_x(int(x)) == int(y)


def test_add_points_kats(golden):
    # Aleo "group" strings are x-coordinates of subgroup points (wasmFunctions.test.ts:31-37)
    for a, b, exp in golden["kats"]["add_points_x"]["cases"]:
        pa, pb = O.point_from_x(int(a)), O.point_from_x(int(b))
        assert O.aff_add(pa, pb)[0] == int(exp)
        assert O.c_point_add(pa, pb)[0] == int(exp)
        if a == b:
            assert O.c_point_double(pa)[0] == int(exp)


def test_group_scalar_mul_kats(golden):
    for x, s, exp in golden["kats"]["group_scalar_mul_x"]["cases"]:
        pt = O.point_from_x(int(x))
        assert O.scalar_mul(pt, int(s))[0] == int(exp)
        assert O.c_scalar_mul(pt, int(s))[0] == int(exp)


def test_fieldmath_multiply_kats(golden):
    for (x, y), s, (ex, ey) in golden["kats"]["fieldmath_multiply"]["cases"]:
        assert O.scalar_mul((int(x), int(y)), int(s)) == (int(ex), int(ey))
        assert O.c_scalar_mul((int(x), int(y)), int(s)) == (int(ex), int(ey))


def test_be_limb_order_kats(golden):
    for v, words in golden["kats"]["be_limbs"]["cases"]:
        assert O.int_to_be_words(int(v)) == words
        assert O.be_words_to_int(words) == int(v)
    vals = [int(v) for v, _ in golden["kats"]["be_limbs"]["cases"]]
    arr = O.ints_to_be_words(vals)
    assert arr.tolist() == [w for _, w in golden["kats"]["be_limbs"]["cases"]]
    assert O.be_words_to_ints(arr) == vals


def test_benchmark_point(golden):
    bp = golden["kats"]["benchmark_point"]
    x, y, t = int(bp["x"]), int(bp["y"]), int(bp["t"])
    assert (x, y) == O.G and O.on_curve(O.G)
    assert x * y % O.P == t
    assert O.scalar_mul(O.G, O.R_ORDER) == O.IDENTITY


def test_split_matches_macro_definition():
    # msm-macro/src/lib.rs:90-176: window i = bits [c i, c i + c), emitted MSB window first
    rng = np.random.default_rng(1)
    vals = [int(rng.integers(0, 2**63)) << 193 | int(rng.integers(0, 2**63)) for _ in range(20)] + [(1 << 256) - 1, 0]
    sc = O.ints_to_be_words(vals)
    for c in (8, 11, 13, 16, 20):
        nw = (256 + c - 1) // c
        out = O.split(c, sc).reshape(nw, len(vals))
        for j, v in enumerate(vals):
            for i in range(nw):
                assert out[nw - 1 - i, j] == (v >> (c * i)) & ((1 << c) - 1)


def test_small_vectors_c_oracle(golden):
    # every small fixture through the C restatement of lib.rs's Pippenger at several windows
    for case in golden["msm"]["small"]:
        ks = [int(k) for k in case["ks"]]
        ss = [int(s, 16) for s in case["scalars"]]
        pts = O.affine_to_wire([O.scalar_mul(O.G, k % O.R_ORDER) for k in ks])
        for c in (9, 13):
            assert O.msm(pts, O.ints_to_be_words(ss), window=c) == (int(case["x"]), int(case["y"])), case["name"]


def test_survey_rows_closed_form(golden):
    rows = {r["n"]: r for r in golden["msm"]["survey"]}
    r = rows[1 << 12]
    ss = O.xorshift_scalars(1 << 12)
    assert O.closed_form_msm(range(1, (1 << 12) + 1), ss) == (int(r["x"]), int(r["y"]))
    assert r["x"] == r["aleo_wasm_confirmed_x"]


def test_closed_form_rows_match_c_oracle(golden):
    # the 2^17 bench row: closed form == the C restatement of the reference's Pippenger
    r = {r["n"]: r for r in golden["msm"]["closed_form"]}[1 << 17]
    pts = O.gen_points(1 << 17)
    sc = O.xorshift_scalars_np(1 << 17)
    assert O.msm(pts, sc, window=12, threads=8) == (int(r["x"]), int(r["y"]))


def test_c_oracle_matches_survey_2_12(golden):
    r = {r["n"]: r for r in golden["msm"]["survey"]}[1 << 12]
    pts = O.gen_points(1 << 12)
    sc = O.xorshift_scalars_np(1 << 12)
    assert O.msm(pts, sc, window=11, threads=4) == (int(r["x"]), int(r["y"]))


def test_gen_points_match_python():
    pts = O.gen_points(5, k0=3, step=4)
    for i in range(5):
        exp = O.scalar_mul(O.G, 3 + 4 * i)
        assert O.be_words_to_int(pts[i, :8]) == exp[0]
        assert O.be_words_to_int(pts[i, 8:16]) == exp[1]
        assert O.be_words_to_int(pts[i, 16:24]) == exp[0] * exp[1] % O.P
        assert O.be_words_to_int(pts[i, 24:32]) == 1


def test_oracle_rejects_out_of_range_coordinate():
    pts = O.gen_points(2)
    pts[1, :8] = O.int_to_be_words(O.P)  # x = p: bytes.rs:19 panics
    with pytest.raises(ValueError):
        O.msm(pts, O.ints_to_be_words([1, 2]))
