#!/usr/bin/env python3
"""Generate tests/golden/manifest.json — golden reduce-copy vectors.

TEST INFRASTRUCTURE. The expected outputs here come from an INDEPENDENT numpy restatement of the
reference semantics (not from oracle/nexr_oracle.c, which the tests check against these vectors):

  * element loop / fold order: reference src/device/common_kernel.h:141-237 (acc = src0, then
    acc = op(acc, src_s) for s = 1..K-1, pre-op per src, post-op at the end);
  * per-type arithmetic: src/device/reduce_kernel.h:238-539 with SKIP_COMP (:432) removed;
    integer sum/prod wrap in the unsigned type (generate.py:128-136), min/max at the user's
    signedness (upstream NCCL; DESIGN.md "Deviations");
  * half: numpy's IEEE binary16 conversion (round-to-nearest-even), every NaN -> 0x7fff
    (CUDA 12.8 cuda_fp16.hpp host __float2half, a third-party algorithm the reference calls);
  * bfloat16: torch's float32 -> bfloat16 conversion (round-to-nearest-even), every NaN -> 0x7fff
    (CUDA 12.8 cuda_bf16.hpp host __float2bfloat16_rn).

Inputs are regenerated deterministically from seeds by ``gen_inputs`` (splitmix64), so the
manifest stores parameters + the expected output (hex for tiny cases, sha256 otherwise).

    python tests/golden/make_golden.py          # rewrites tests/golden/manifest.json
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# datatype ids = ncclDataType_t (src/nccl.h.in:278-290)
I8, U8, I32, U32, I64, U64, F16, F32, F64, BF16 = 0, 1, 2, 3, 4, 5, 6, 7, 8, 9
DT_NAMES = {I8: "i8", U8: "u8", I32: "i32", U32: "u32", I64: "i64", U64: "u64", F16: "f16", F32: "f32",
            F64: "f64", BF16: "bf16"}
# storage numpy dtype per datatype (unsigned storage for integers and 16-bit floats)
STORE = {I8: np.uint8, U8: np.uint8, I32: np.uint32, U32: np.uint32, I64: np.uint64, U64: np.uint64,
         F16: np.uint16, F32: np.float32, F64: np.float64, BF16: np.uint16}
SIGNED = {I8: np.int8, I32: np.int32, I64: np.int64}
INTS = (I8, U8, I32, U32, I64, U64)
# ncclDevRedOp_t (src/include/device.h:683-687)
SUM, PROD, MINMAX, PREMULSUM, SUMPOSTDIV = 0, 1, 2, 3, 4

M64 = (1 << 64) - 1


def _splitmix64_into(z: np.ndarray, seed: int, first: int, tmp: np.ndarray) -> None:
    """z[j] = output first + j of splitmix64 from `seed`, computed in place (wrapping uint64)."""
    gamma, c1, c2 = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xBF58476D1CE4E5B9), np.uint64(0x94D049BB133111EB)
    with np.errstate(over="ignore"):
        z[:] = np.arange(first + 1, first + 1 + z.size, dtype=np.uint64)
        np.multiply(z, gamma, out=z)
        np.add(z, np.uint64(seed & M64), out=z)
        for shift, mul in ((30, c1), (27, c2), (31, None)):
            np.right_shift(z, np.uint64(shift), out=tmp)
            np.bitwise_xor(z, tmp, out=z)
            if mul is not None:
                np.multiply(z, mul, out=z)


def splitmix64(seed: int, n: int, chunk: int = 1 << 18) -> np.ndarray:
    """n outputs of splitmix64 starting from `seed` (vectorised, wrapping uint64 arithmetic), in
    cache-sized chunks with in-place steps."""
    out = np.empty(n, dtype=np.uint64)
    tmp = np.empty(min(n, chunk), dtype=np.uint64)
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        _splitmix64_into(out[a:b], seed, a, tmp[:b - a])
    return out


def f32_to_f16_bits(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore", invalid="ignore"):
        h = x.astype(np.float32).astype(np.float16).view(np.uint16).copy()
    h[np.isnan(x)] = 0x7FFF
    return h


def f16_bits_to_f32(h: np.ndarray) -> np.ndarray:
    return h.view(np.float16).astype(np.float32)


def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    import torch
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(torch.bfloat16)
    b = t.view(torch.int16).numpy().view(np.uint16).copy()
    b[np.isnan(x)] = 0x7FFF
    return b


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << np.uint32(16)).view(np.float32)


SPECIAL_F32 = np.array([np.nan, np.inf, -np.inf, 0.0, -0.0, 1e-45, -1e-45, 1.1754942e-38, 3.4028235e38,
                        -3.4028235e38, 1.0, -1.0, 65504.0, 65520.0, 6.1e-5, 5.96e-8, 2.98e-8, 1.00390625,
                        1.005859375, 0.5, -2.0, 3.0], dtype=np.float32)


def _gen_chunk(dt: int, r: np.ndarray, special: bool) -> np.ndarray:
    """One stretch of an input buffer from its splitmix64 outputs `r` (every element depends only
    on its own r[i], so any split into stretches gives the same buffer)."""
    if dt in INTS:
        a = r.astype(STORE[dt])  # full-range uniform bits (truncating cast)
        if special:
            bits = np.dtype(STORE[dt]).itemsize * 8
            ext = np.array([0, 1, (1 << bits) - 1, 1 << (bits - 1), (1 << (bits - 1)) - 1, 2, 3],
                           dtype=np.uint64).astype(STORE[dt])
            pick = (r >> np.uint64(59)) < np.uint64(6)
            a[pick] = ext[(r[pick] >> np.uint64(8)) % np.uint64(len(ext))]
        return a
    # uniform [-1, 1); r >> 40 < 2^24, so the int64 view converts exactly (and faster than uint64)
    u = ((r >> np.uint64(40)).view(np.int64).astype(np.float64) * 2.0 ** -24 * 2.0 - 1.0)
    f = u.astype(np.float32)
    if special:
        pick = (r >> np.uint64(58)) < np.uint64(10)
        f[pick] = SPECIAL_F32[((r[pick] >> np.uint64(8)) % np.uint64(len(SPECIAL_F32))).astype(np.int64)]
    if dt == F32:
        return f
    if dt == F64:
        a = u.copy()
        if special:
            a[pick] = f[pick].astype(np.float64)
        return a
    if dt == F16:
        a = f32_to_f16_bits(f)
        raw = np.array([0x7E01, 0xFC00, 0x0001, 0x8001, 0x03FF, 0x7BFF, 0x3C00], dtype=np.uint16)
    else:  # BF16
        a = f32_to_bf16_bits(f)
        raw = np.array([0x7FC1, 0xFF80, 0x0001, 0x8001, 0x7F7F, 0x3F80, 0x3BC0], dtype=np.uint16)
    if special:  # raw 16-bit specials incl. NaN payloads and subnormals
        p2 = (r >> np.uint64(61)) == np.uint64(0)
        a[p2] = raw[((r[p2] >> np.uint64(16)) % np.uint64(len(raw))).astype(np.int64)]
    return a


GEN_CHUNK = 1 << 18


def gen_inputs(dt: int, k: int, n: int, seed: int, special: bool) -> list:
    """K input buffers (storage dtype) for one case; buffer s uses seed + s.
    Large buffers are built in stretches of GEN_CHUNK elements on a thread pool (numpy releases the
    GIL in its loops; every element depends only on its own splitmix64 output, so the bytes are the
    same as one whole-buffer pass): the GPU suite's 100+ MiB buffers in seconds, not minutes."""
    out = []
    for s in range(k):
        a = np.empty(n, dtype=STORE[dt])

        def fill(lo, s=s, a=a):
            hi = min(n, lo + GEN_CHUNK)
            r = np.empty(hi - lo, dtype=np.uint64)
            _splitmix64_into(r, seed + s, lo, np.empty_like(r))
            a[lo:hi] = _gen_chunk(dt, r, special)

        starts = range(0, n, GEN_CHUNK)
        if n <= 4 * GEN_CHUNK:
            for lo in starts:
                fill(lo)
        else:
            for _ in _pool().map(fill, starts):
                pass
        out.append(a)
    return out


_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4))
    return _POOL


# ---- the independent restatement --------------------------------------------------------------
def _float_step(dt, op, is_min, c, v):
    """One step in float32/float64 then back to T (per reduce_kernel.h:329-367, :470-473)."""
    if dt in (F16, BF16):
        to_f = f16_bits_to_f32 if dt == F16 else bf16_bits_to_f32
        from_f = f32_to_f16_bits if dt == F16 else f32_to_bf16_bits
        fc, fv = to_f(c), to_f(v)
    else:
        fc, fv = c, v
    with np.errstate(all="ignore"):
        if op == PROD:
            r = fc * fv
        elif op == MINMAX:
            r = np.where(fv < fc, fv, fc) if is_min else np.where(fv > fc, fv, fc)
        else:
            r = fc + fv
    if dt in (F16, BF16):
        return from_f(np.asarray(r, dtype=np.float32))
    return np.asarray(r, dtype=STORE[dt])


def _int_step(dt, op, is_min, c, v):
    if op == PROD:
        return (c * v).astype(STORE[dt])
    if op == MINMAX:
        if dt in SIGNED:
            sc, sv = c.view(SIGNED[dt]), v.view(SIGNED[dt])
            r = np.where(sv < sc, sv, sc) if is_min else np.where(sv > sc, sv, sc)
            return r.view(STORE[dt])
        return np.where(v < c, v, c) if is_min else np.where(v > c, v, c)
    return (c + v).astype(STORE[dt])


def _preop(dt, x, raw):
    """x * ncclDecodeScalar<T>(raw) (reduce_kernel.h:498-518)."""
    if dt in INTS:
        bits = np.dtype(STORE[dt]).itemsize * 8
        f = np.array(raw & ((1 << bits) - 1), dtype=STORE[dt])
        with np.errstate(over="ignore"):
            return (x * f).astype(STORE[dt])
    if dt == F32:
        return (x * np.array([raw & 0xFFFFFFFF], dtype=np.uint32).view(np.float32)[0]).astype(np.float32)
    if dt == F64:
        return x * np.array([raw & M64], dtype=np.uint64).view(np.float64)[0]
    return _float_step(dt, PROD, True, x, np.full(x.shape, raw & 0xFFFF, dtype=np.uint16))


def _postdiv(dt, x, arg):
    """FuncSumPostDiv::divide (reduce_kernel.h:74-98)."""
    divisor = (arg >> 1) & 0xFFFFFFFF
    if divisor == 0:
        divisor = 1
    is_signed = (arg & 1) != 0
    bits = np.dtype(STORE[dt]).itemsize * 8
    if not is_signed:
        return (x.astype(np.uint64) // np.uint64(divisor)).astype(STORE[dt])
    d = int(np.array(divisor, dtype=np.uint64).astype(np.dtype(f"u{bits // 8}")).view(np.dtype(f"i{bits // 8}")))
    s = [int(v) for v in x.view(np.dtype(f"i{bits // 8}"))]
    q = []
    for v in s:
        if d == -1:
            r = -v
        else:
            r = abs(v) // abs(d)
            if (v < 0) != (d < 0):
                r = -r
        q.append(r & ((1 << bits) - 1))
    return np.array(q, dtype=np.uint64).astype(STORE[dt])


def reference_reduce(dt, op, arg, srcs, pre=None, post=False):
    pre = pre or []
    is_min = (arg & 1) == 0
    step = _int_step if dt in INTS else _float_step
    acc = srcs[0].copy()
    if op == PREMULSUM and len(pre) > 0:
        acc = _preop(dt, acc, pre[0])
    for s in range(1, len(srcs)):
        v = srcs[s]
        if op == PREMULSUM and s < len(pre):
            v = _preop(dt, v, pre[s])
        with np.errstate(over="ignore"):
            acc = step(dt, op, is_min, acc, v)
    if op == SUMPOSTDIV and post:
        acc = _postdiv(dt, acc, arg)
    return np.ascontiguousarray(acc)


def minmax_arg(dt, is_max):
    """hostToDevRedOp's xormask (src/enqueue.cc:2207-2216)."""
    bits = np.dtype(STORE[dt]).itemsize * 8
    all_bits = (1 << bits) - 1
    sign = all_bits ^ (all_bits >> 1)
    a = sign if dt in (I8, I32, I64) else 0
    return a ^ (all_bits if is_max else 0)


def float_scalar_bits(dt, value):
    if dt == F32:
        return int(np.array([value], dtype=np.float32).view(np.uint32)[0])
    if dt == F64:
        return int(np.array([value], dtype=np.float64).view(np.uint64)[0])
    if dt == F16:
        return int(f32_to_f16_bits(np.array([value], dtype=np.float32))[0])
    if dt == BF16:
        return int(f32_to_bf16_bits(np.array([value], dtype=np.float32))[0])
    bits = np.dtype(STORE[dt]).itemsize * 8
    return int(value) & ((1 << bits) - 1)


def case_list():
    cases = []
    seed = 0x5EED0000
    for dt in DT_NAMES:
        ops = [("sum", SUM, 0), ("prod", PROD, 0), ("min", MINMAX, minmax_arg(dt, False)),
               ("max", MINMAX, minmax_arg(dt, True)), ("premulsum", PREMULSUM, 0)]
        if dt in INTS:
            ops.append(("sumpostdiv", SUMPOSTDIV, None))
        for name, op, arg in ops:
            for k in (1, 2, 3, 4, 8):
                for n in (1, 3, 17, 4099, 65537):
                    if n == 65537 and k not in (2, 8):
                        continue
                    for special in (False, True):
                        if special and n < 17:
                            continue
                        c = dict(dt=dt, op=op, name=name, k=k, n=n, special=special, seed=seed,
                                 pre=[], post=False, arg=0)
                        seed += 16
                        if op == MINMAX:
                            c["arg"] = arg
                        if op == PREMULSUM:
                            scal = [0.5, -1.25, 3.0, 0.125, 1.0, -0.75, 2.0, 0.3333333]
                            npre = k if k != 3 else 1
                            c["pre"] = [float_scalar_bits(dt, scal[s] if dt not in INTS else (s * 7 + 3))
                                        for s in range(npre)]
                            c["post"] = True
                        if op == SUMPOSTDIV:
                            signed = dt in (I8, I32, I64)
                            c["arg"] = (k << 1) | int(signed)
                            c["post"] = True
                        cases.append(c)
    return cases


def canon_bytes(dt, arr: np.ndarray) -> bytes:
    """Bytes used for the digest: float32/float64 NaNs compared by class (a NaN's sign/payload
    from x86 or the GPU is not specified by the reference), everything else bit-exact."""
    if dt in (F32, F64):
        a = np.array(arr, copy=True)
        a[np.isnan(a)] = np.nan
        return a.tobytes()
    return np.asarray(arr).tobytes()


def expected_for(c):
    srcs = gen_inputs(c["dt"], c["k"], c["n"], c["seed"], c["special"])
    return reference_reduce(c["dt"], c["op"], c["arg"], srcs, c["pre"], c["post"])


def main():
    cases = case_list()
    out = []
    for c in cases:
        exp = expected_for(c)
        rec = dict(c)
        raw = exp.tobytes()
        rec["sha256"] = hashlib.sha256(canon_bytes(c["dt"], exp)).hexdigest()
        if c["n"] <= 17:
            rec["expected_hex"] = raw.hex()
        out.append(rec)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_golden.py", "n_cases": len(out), "cases": out}, f, indent=0)
    print(f"wrote {len(out)} cases")


if __name__ == "__main__":
    sys.exit(main())
