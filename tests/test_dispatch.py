"""The build's datatype/op dispatch against the reference's OWN generator output (CPU, no GPU).

tests/golden/dispatch.json was produced by running the reference's src/device/generate.py unmodified
(tests/golden/make_dispatch_golden.py, in the build container). For every reduction row on the
RING and TREE schedules it records the functor and C++ element type the reference instantiates, and
the compile guard on it. These tests hold the build to those decisions:

- the datatype and device-op enumerations are in the generator's order (it indexes tables by them);
- nexrReduceCopy accepts exactly the (op, datatype) pairs the fork compiles: a row must exist and its
  guard must not need __CUDA_ARCH__ >= 900, which the fork's g++ device build never defines
  (src/device/Makefile COMPILE.cc);
- where the generator folds a signed integer row onto the unsigned instantiation
  (equivalent_primary, generate.py:128-136) for Sum/Prod/PreMulSum/SumPostDiv, the oracle the GPU
  kernel is checked against gives the same bytes at the signed and the unsigned datatype;
- signed MinMax is also folded onto the unsigned instantiation in the fork, whose FuncMinMax ignores
  the xormask: the build deliberately compares at the user's signedness (deviation 2),
  and the test shows both results side by side.
"""
import ctypes
import json
import os

import numpy as np
import pytest

import make_golden as mg
from conftest import GOLDEN

TY_IDS = {"i8": 0, "u8": 1, "i32": 2, "u32": 3, "i64": 4, "u64": 5, "f16": 6, "f32": 7, "f64": 8, "bf16": 9,
          "f8e4m3": 10, "f8e5m2": 11}
REDOP_IDS = {"Sum": 0, "Prod": 1, "MinMax": 2, "PreMulSum": 3, "SumPostDiv": 4}
CTYPE_UNSIGNED = {"uint8_t": 1, "uint32_t": 3, "uint64_t": 5}


@pytest.fixture(scope="module")
def dispatch():
    with open(os.path.join(GOLDEN, "dispatch.json")) as f:
        return json.load(f)


def _row(dispatch, coll, redop, ty, algo, proto):
    for r in dispatch["rows"]:
        if (r["coll"], r["redop"], r["ty"], r["algo"], r["proto"]) == (coll, redop, ty, algo, proto):
            return r
    return None


def _compiled_in_fork(row) -> bool:
    return row is not None and row["id"] >= 0 and "__CUDA_ARCH__ >= 900" not in (row.get("guard") or "")


def test_enumeration_order_matches_generator(nexr, dispatch):
    order = dispatch["order"]
    assert [TY_IDS[t] for t in order["all_tys"]] == list(range(12))
    assert [int(nexr.DataType[n]) for n in ("Int8", "Uint8", "Int32", "Uint32", "Int64", "Uint64", "Float16",
                                            "Float32", "Float64", "Bfloat16")] == list(range(10))
    assert [REDOP_IDS[o] for o in order["all_redops"]] == [int(o) for o in nexr.DevRedOp]


@pytest.mark.parametrize("redop", sorted(REDOP_IDS))
@pytest.mark.parametrize("ty", sorted(TY_IDS))
def test_validation_accepts_exactly_what_the_fork_compiles(nexr, dispatch, redop, ty):
    L = nexr.lib()
    sa = (ctypes.c_void_p * 2)(0x1000, 0x2000)
    da = (ctypes.c_void_p * 1)(0x3000)
    pre = (ctypes.c_uint64 * 2)(0, 0)
    for proto in ("SIMPLE", "LL", "LL128"):
        for algo in ("RING", "TREE"):
            row = _row(dispatch, "AllReduce", redop, ty, algo, proto)
            assert _compiled_in_fork(row) == _compiled_in_fork(_row(dispatch, "AllReduce", redop, ty, "RING",
                                                                      "SIMPLE")), (algo, proto)
    want = _compiled_in_fork(_row(dispatch, "AllReduce", redop, ty, "RING", "SIMPLE"))
    arg = (2 << 1) if redop == "SumPostDiv" else 0
    # nElts = 0: full validation, then a no-op (no device needed)
    rc = L.nexrReduceCopy(2, sa, 1, da, 0, TY_IDS[ty], REDOP_IDS[redop], arg, 0, pre, 0, None)
    assert rc == (0 if want else 4), (redop, ty)


@pytest.mark.parametrize("redop", ["Sum", "Prod", "PreMulSum", "SumPostDiv", "MinMax"])
@pytest.mark.parametrize("ty", ["i8", "i32", "i64"])
def test_signed_rows_use_the_unsigned_instantiation(dispatch, redop, ty):
    for coll in ("AllReduce", "Reduce", "ReduceScatter"):
        row = _row(dispatch, coll, redop, ty, "RING", "SIMPLE")
        assert row is not None and row["functor"] == "Func" + redop
        assert row["ctype"] == "uint" + ty[1:] + "_t", (coll, row)


@pytest.mark.parametrize("redop", ["Sum", "Prod", "PreMulSum", "SumPostDiv"])
@pytest.mark.parametrize("ty", ["i8", "i32", "i64"])
def test_signed_equals_unsigned_where_the_fork_folds_them(oracle, redop, ty):
    """equivalent_primary maps these signed rows onto the unsigned function; the build's arithmetic at
    the signed datatype (the oracle the GPU kernel is pinned to) must give the unsigned bytes."""
    dt_s = TY_IDS[ty]
    dt_u = dt_s + 1
    k, n = 4, 4099
    srcs = mg.gen_inputs(dt_s, k, n, 11, special=True)
    op = REDOP_IDS[redop]
    pre = None
    arg = 0
    post = False
    if redop == "PreMulSum":
        pre = [3, 0xFF, 7, 1]  # raw scalar bits per source
    if redop == "SumPostDiv":
        arg = (3 << 1) | 1  # nRanks = 3, signed (hostToDevRedOp, enqueue.cc:2225-2240)
        post = True
    a = oracle.reduce_copy(srcs, 1, dt_s, op, arg, pre, post)[0]
    b = oracle.reduce_copy(srcs, 1, dt_u, op, arg, pre, post)[0]
    assert a.tobytes() == b.tobytes()


@pytest.mark.parametrize("ty,lo,hi", [("i8", -5, 3), ("i32", -5, 3), ("i64", -5, 3)])
def test_signed_minmax_deviation_is_the_documented_one(oracle, dispatch, ty, lo, hi):
    """The fork instantiates signed MinMax at the unsigned type (fixture) and its FuncMinMax never
    applies the xormask, so min(-5, 3) there is 3 (SURVEY §0 probe). The build returns -5, upstream
    NCCL's answer; at the unsigned datatype both agree on the unsigned comparison."""
    assert _row(dispatch, "AllReduce", "MinMax", ty, "RING", "SIMPLE")["ctype"] == "uint" + ty[1:] + "_t"
    dt_s = TY_IDS[ty]
    st = mg.STORE[dt_s]
    sg = mg.SIGNED[dt_s]
    srcs = [np.array([lo], dtype=sg).view(st), np.array([hi], dtype=sg).view(st)]
    min_arg = mg.minmax_arg(dt_s, False)
    build = oracle.reduce_copy(srcs, 1, dt_s, 2, min_arg)[0].view(sg)[0]
    fork = oracle.reduce_copy(srcs, 1, dt_s + 1, 2, 0)[0].view(sg)[0]  # the uint kernel: unsigned compare
    assert build == lo
    assert fork == hi


def test_fp8_rows_need_sm90_and_sumpostdiv_floats_do_not_exist(dispatch):
    for ty in ("f8e4m3", "f8e5m2"):
        for redop in REDOP_IDS:
            row = _row(dispatch, "AllReduce", redop, ty, "RING", "SIMPLE")
            if redop == "SumPostDiv":
                assert row is None
            else:
                assert "__CUDA_ARCH__ >= 900" in row["guard"]
    for ty in ("f16", "f32", "f64", "bf16"):
        assert _row(dispatch, "AllReduce", "SumPostDiv", ty, "RING", "SIMPLE") is None
