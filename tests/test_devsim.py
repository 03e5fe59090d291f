"""Device arithmetic (csrc/device/dev_field.h) compiled for the host and
checked against Python integers and the CPU oracle: radix-2^25.5 field
multiply/square at the worst-case limb bounds the point formulas rely on,
canonical encoding, scalar Montgomery ops, and every point-formula variant
(extended, cached, T-less doubling) against oracle point arithmetic."""
import ctypes
import os
import random
import subprocess

import pytest

from conftest import ROOT

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
W = [26, 25] * 5
POS = [sum(W[:i]) for i in range(10)]
SO = os.path.join(ROOT, "tests", "devsim", "_build", "devsim.so")


@pytest.fixture(scope="module")
def sim():
    src = os.path.join(ROOT, "tests", "devsim", "devsim.cpp")
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(
            os.path.getmtime(src),
            os.path.getmtime(os.path.join(ROOT, "bulletproof-gadgets_amd", "csrc", "device", "dev_field.h"))):
        subprocess.check_call(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", SO, src])
    return ctypes.CDLL(SO)


def limbs_val(l):
    return sum(x << POS[i] for i, x in enumerate(l))


def arr(vals, n=10):
    return (ctypes.c_uint32 * n)(*vals)


def words(x):
    return arr([(x >> (32 * i)) & 0xffffffff for i in range(8)], 8)


def from_words(w):
    return sum(w[i] << (32 * i) for i in range(8))


def tight_max():
    return [(1 << w) - 1 + (1 << 17) for w in W]


def rand_bounded(rnd, factor):
    return [rnd.randrange(0, int(factor * m) + 1) for m in tight_max()]


def test_mul_sq_at_bounds(sim):
    rnd = random.Random(7)
    cases = []
    for fa, gb in [(1, 1), (2, 2), (3, 3), (5, 1), (5, 2), (5, 3), (6, 2), (3, 2), (2, 3)]:
        cases.append(([int(fa * m) for m in tight_max()], [int(gb * m) for m in tight_max()]))  # all-max
        for _ in range(40):
            cases.append((rand_bounded(rnd, fa), rand_bounded(rnd, gb)))
    out = arr([0] * 10)
    for f, g in cases:
        sim.sim_fe_mul_limbs(arr(f), arr(g), out)
        r = list(out)
        assert all(x <= m for x, m in zip(r, tight_max())), r
        assert limbs_val(r) % P == limbs_val(f) * limbs_val(g) % P
    for fa in (1, 2, 3):
        for _ in range(60):
            f = rand_bounded(rnd, fa)
            sim.sim_fe_sq_limbs(arr(f), out)
            assert limbs_val(list(out)) % P == limbs_val(f) ** 2 % P
        f = [int(fa * m) for m in tight_max()]
        sim.sim_fe_sq_limbs(arr(f), out)
        assert limbs_val(list(out)) % P == limbs_val(f) ** 2 % P


def test_carry_and_canonical(sim):
    rnd = random.Random(8)
    out = arr([0] * 10)
    w = (ctypes.c_uint32 * 8)()
    specials = [P - 1, P, P + 1, 2 * P - 1, 2**255 - 1, 2**255, 0, 18, 19, 2**255 + 18]
    # limbs at width, the top limb takes the rest (values up to 2^256)
    vals = [[(v >> POS[i]) & ((1 << W[i]) - 1) if i < 9 else v >> POS[9] for i in range(10)] for v in specials]
    for _ in range(200):
        vals.append(rand_bounded(rnd, rnd.choice([1, 2, 5, 6])))
    for l in vals:
        v = limbs_val(l)
        sim.sim_fe_carry_limbs(arr(l), out)
        r = list(out)
        assert limbs_val(r) % P == v % P and all(x <= m for x, m in zip(r, tight_max()))
        sim.sim_fe_canon_limbs(arr(l), out)
        assert limbs_val(list(out)) == v % P
        sim.sim_fe_tow_limbs(arr(l), w)
        assert from_words(w) == v % P


def test_field_word_ops(sim):
    rnd = random.Random(9)
    r = (ctypes.c_uint32 * 8)()
    for _ in range(100):
        a, b = rnd.randrange(P), rnd.randrange(P)
        sim.sim_fe_mul(words(a), words(b), r); assert from_words(r) == a * b % P
        sim.sim_fe_sq(words(a), r); assert from_words(r) == a * a % P
        sim.sim_fe_add(words(a), words(b), r); assert from_words(r) == (a + b) % P
        sim.sim_fe_sub(words(a), words(b), r); assert from_words(r) == (a - b) % P
    for a in (1, 2, P - 1, rnd.randrange(P)):
        sim.sim_fe_invert(words(a), r)
        assert from_words(r) == pow(a, P - 2, P)


def test_scalar_ops(sim):
    rnd = random.Random(10)
    r = (ctypes.c_uint32 * 8)()
    Rinv = pow(2**256, -1, L)
    for _ in range(100):
        a, b = rnd.randrange(L), rnd.randrange(L)
        sim.sim_sc_montmul(words(a), words(b), r); assert from_words(r) == a * b * Rinv % L
        sim.sim_sc_add(words(a), words(b), r); assert from_words(r) == (a + b) % L
        sim.sim_sc_sub(words(a), words(b), r); assert from_words(r) == (a - b) % L
        x = rnd.randrange(2**256)
        sim.sim_sc_reduce(words(x), r); assert from_words(r) == x % L


def test_point_formulas_vs_oracle(sim):
    import oracle as O
    rnd = random.Random(11)
    r = (ctypes.c_uint32 * 8)()
    B, _ = O.pedersen_gens()
    pts = [O.point_mul(rnd.randrange(L).to_bytes(32, "little"), B) for _ in range(6)]
    pts.append(B)
    neg1 = (L - 1).to_bytes(32, "little")
    two = (2).to_bytes(32, "little")
    for i in range(len(pts)):
        a, b = pts[i], pts[(i + 1) % len(pts)]
        wa, wb = (ctypes.c_uint32 * 8).from_buffer_copy(a), (ctypes.c_uint32 * 8).from_buffer_copy(b)
        add = O.point_add(a, b)
        sub = O.point_add(a, O.point_mul(neg1, b))
        dbl = O.point_mul(two, a)
        four_plus = O.point_add(O.point_mul((4).to_bytes(32, "little"), a), b)
        two_add_plus = O.point_add(O.point_mul(two, add), b)      # 2(a + b) + b
        two_sub_plus = O.point_add(O.point_mul(two, sub), b)      # 2(a - b) + b
        for op, want in [(0, add), (1, sub), (2, add), (3, sub), (4, dbl), (5, four_plus), (6, add), (7, sub),
                         (8, add), (9, add), (10, sub), (11, add), (12, sub), (13, two_add_plus), (14, two_sub_plus)]:
            assert sim.sim_pt_op(op, wa, wb, r) == 0
            assert bytes(r) == want, (op, i)


def test_elligator_vs_oracle(sim):
    import oracle as O
    rnd = random.Random(12)
    r = (ctypes.c_uint32 * 8)()
    for _ in range(20):
        u = bytes(rnd.getrandbits(8) for _ in range(64))
        sim.sim_from_uniform((ctypes.c_uint32 * 16).from_buffer_copy(u), r)
        assert bytes(r) == O.from_uniform(u)
