"""ctypes wrapper around oracle/_build/liboracle.so (the CPU restatement).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg; never by the product package.
"""
import ctypes
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


class R1csView(ctypes.Structure):
    """Mirror of `bpg_r1cs_view` (include/bpg.h)."""
    _fields_ = [
        ("n", ctypes.c_uint32), ("m", ctypes.c_uint32), ("q", ctypes.c_uint32), ("nnz", ctypes.c_uint32),
        ("a_L", ctypes.c_void_p), ("a_R", ctypes.c_void_p), ("a_O", ctypes.c_void_p),
        ("v", ctypes.c_void_p), ("v_blinding", ctypes.c_void_p),
        ("row_ptr", ctypes.c_void_p), ("term_var", ctypes.c_void_p), ("term_coeff", ctypes.c_void_p),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        vp, sz, u32, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64
        L.oracle_r1cs_prove.argtypes = [vp, sz, ctypes.POINTER(R1csView), vp, vp, sz, ctypes.POINTER(sz), vp]
        L.oracle_r1cs_verify.argtypes = [vp, sz, ctypes.POINTER(R1csView), vp, vp, sz, vp]
        L.oracle_msm.argtypes = [vp, vp, u32, vp]
        L.oracle_generators.argtypes = [u32, vp, vp]
        L.oracle_seed_stream.argtypes = [u64, u64, vp, sz]
        L.oracle_merlin_test.argtypes = [vp, sz, ctypes.c_char_p, vp, sz, ctypes.c_char_p, vp, sz]
        L.oracle_shake256.argtypes = [vp, sz, vp, sz]
        L.oracle_sha3_512.argtypes = [vp, vp, sz]
        L.oracle_from_uniform.argtypes = [vp, vp]
        L.oracle_point_add.argtypes = [vp, vp, vp]
        L.oracle_point_mul.argtypes = [vp, vp, vp]
        L.oracle_pedersen_commit.argtypes = [vp, vp, vp]
        L.oracle_pedersen_gens.argtypes = [vp, vp]
        L.oracle_decompress_ok.argtypes = [vp]
        for f in ("oracle_sc_mul", "oracle_sc_add"):
            getattr(L, f).argtypes = [vp, vp, vp]
        L.oracle_sc_invert.argtypes = [vp, vp]
        L.oracle_sc_wide.argtypes = [vp, vp]
        _lib = L
    return _lib


def _buf(n):
    return ctypes.create_string_buffer(max(n, 1))


def _p(b):
    return ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p) if b is not None else None


def from_uniform(b64):
    out = _buf(32)
    lib().oracle_from_uniform(b64, out)
    return out.raw[:32]


def point_add(a, b):
    out = _buf(32)
    if lib().oracle_point_add(a, b, out) != 0:
        raise ValueError("bad point")
    return out.raw[:32]


def point_mul(s, a):
    out = _buf(32)
    if lib().oracle_point_mul(s, a, out) != 0:
        raise ValueError("bad point")
    return out.raw[:32]


def decompress_ok(a):
    return bool(lib().oracle_decompress_ok(a))


def msm(scalars, points):
    n = len(scalars)
    out = _buf(32)
    rc = lib().oracle_msm(b"".join(scalars), b"".join(points), n, out)
    if rc != 0:
        raise ValueError("bad point")
    return out.raw[:32]


def generators(n):
    G, H = _buf(32 * n), _buf(32 * n)
    lib().oracle_generators(n, G, H)
    return [G.raw[32 * i:32 * i + 32] for i in range(n)], [H.raw[32 * i:32 * i + 32] for i in range(n)]


def pedersen_gens():
    B, Bb = _buf(32), _buf(32)
    lib().oracle_pedersen_gens(B, Bb)
    return B.raw[:32], Bb.raw[:32]


def pedersen_commit(v, vb):
    out = _buf(32)
    lib().oracle_pedersen_commit(v, vb, out)
    return out.raw[:32]


def seed_stream(seed, offset, n):
    out = _buf(n)
    lib().oracle_seed_stream(seed, offset, out, n)
    return out.raw[:n]


def merlin_test(proto, l1, m1, l2, n):
    out = _buf(n)
    lib().oracle_merlin_test(proto, len(proto), l1, m1, len(m1), l2, out, n)
    return out.raw[:n]


def shake256(data, n):
    out = _buf(n)
    lib().oracle_shake256(data, len(data), out, n)
    return out.raw[:n]


def sha3_512(data):
    out = _buf(64)
    lib().oracle_sha3_512(out, data, len(data))
    return out.raw[:64]


def sc_mul(a, b):
    out = _buf(32); lib().oracle_sc_mul(a, b, out); return out.raw[:32]


def sc_add(a, b):
    out = _buf(32); lib().oracle_sc_add(a, b, out); return out.raw[:32]


def sc_invert(a):
    out = _buf(32); lib().oracle_sc_invert(a, out); return out.raw[:32]


def sc_wide(a):
    out = _buf(32); lib().oracle_sc_wide(a, out); return out.raw[:32]


class FlatCS:
    """A flattened constraint system (bpg_r1cs_view) held in Python bytes."""

    def __init__(self, n, m, a_L, a_R, a_O, v, v_blinding, rows):
        # rows: list of lists of (var_code, coeff_bytes32)
        self.n, self.m = n, m
        self.a_L, self.a_R, self.a_O = a_L, a_R, a_O
        self.v, self.v_blinding = v, v_blinding
        self.rows = rows
        rp = [0]
        tv, tc = [], []
        for r in rows:
            for var, c in r:
                tv.append(var)
                tc.append(c)
            rp.append(len(tv))
        self.row_ptr = (ctypes.c_uint32 * len(rp))(*rp)
        self.term_var = (ctypes.c_uint32 * max(len(tv), 1))(*tv)
        self.term_coeff = b"".join(tc) or b"\0" * 32
        self.q, self.nnz = len(rows), len(tv)
        self._keep = [b"".join(a_L) or b"\0", b"".join(a_R) or b"\0", b"".join(a_O) or b"\0",
                      b"".join(v) or b"\0", b"".join(v_blinding) or b"\0", self.term_coeff]

    def view(self, secrets=True):
        k = self._keep
        cv = lambda b: ctypes.cast(ctypes.c_char_p(b), ctypes.c_void_p)
        return R1csView(self.n, self.m, self.q, self.nnz,
                        cv(k[0]) if secrets else None, cv(k[1]) if secrets else None,
                        cv(k[2]) if secrets else None, cv(k[3]) if secrets else None,
                        cv(k[4]) if secrets else None,
                        ctypes.cast(self.row_ptr, ctypes.c_void_p), ctypes.cast(self.term_var, ctypes.c_void_p),
                        cv(self.term_coeff))


def r1cs_prove(label, cs, entropy):
    view = cs.view()
    out = _buf(417 + 64 * 31)
    plen = ctypes.c_size_t(0)
    V = _buf(32 * max(cs.m, 1))
    rc = lib().oracle_r1cs_prove(label, len(label), ctypes.byref(view), entropy, out, 417 + 64 * 31,
                                 ctypes.byref(plen), V)
    if rc != 0:
        raise RuntimeError("oracle prove failed: %d" % rc)
    return out.raw[:plen.value], [V.raw[32 * i:32 * i + 32] for i in range(cs.m)]


def r1cs_verify(label, cs, V, proof, entropy=b"\x07" * 32):
    view = cs.view(secrets=False)
    Vb = b"".join(V) or b"\0" * 32
    return lib().oracle_r1cs_verify(label, len(label), ctypes.byref(view), Vb, proof, len(proof), entropy)
