"""The Gadget-API boundary (bpg_cs_*, the ProverBuffer / VerifierBuffer cut
of src/cs_buffer.rs:22-199) against the oracle's Gadget-API mirror
(oracle/synth.py Cs + gadgets), on the CPU: the flattened systems must be
byte-identical. Device proofs over these views are in test_gpu_fullsize.py
(merkle512) and test_gpu_reference_matrix.py.
"""
import ctypes
import os

import pytest

import synth as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# merkle_tree_gadget.rs test constants (W2, W12..W15 and the root W1 of
# test_merkle_tree_gadget_6, :433-471), via tests/golden/reference_cases.json
W1 = bytes.fromhex("0522a64d7b931e21760cf955a15fcc793e8a52b42a56ab03afddec8beb668749")


@pytest.fixture(scope="module")
def bpg():
    import workloads
    return workloads._bpg()


def view_tuple(v):
    """(n, m, q, a_L, a_R, a_O, v, v_blinding, row_ptr, term_var, term_coeff)
    of any bpg_r1cs_view mirror."""
    def raw(p, k):
        return ctypes.string_at(p, k) if k and p else b""
    out = [v.n, v.m, v.q]
    for f in ("a_L", "a_R", "a_O"):
        out.append(raw(getattr(v, f), 32 * v.n))
    for f in ("v", "v_blinding"):
        out.append(raw(getattr(v, f), 32 * v.m))
    out.append(raw(v.row_ptr, 4 * (v.q + 1)))
    out.append(raw(v.term_var, 4 * v.nnz))
    out.append(raw(v.term_coeff, 32 * v.nnz))
    return tuple(out)


def oracle_merkle(leaves, pattern, inst=(), seed=11):
    rng = S.Rng(seed)
    cs = S.Cs(True)
    vs = [cs.commit(S.be_to_scalar(x), rng.scalar()) for x in leaves]
    S.Merkle(S.lc_const(S.be_to_scalar(W1)), [S.lc_const(S.be_to_scalar(i)) for i in inst],
             [S.lc_var(v) for v in vs], pattern).assemble(cs, [], [])
    return cs


def product_merkle(bpg, leaves, pattern, inst=(), seed=11):
    rng = S.Rng(seed)
    cs = bpg.GadgetCS(prover=True)
    vs = [cs.commit(int.from_bytes(x, "big"), rng.scalar()) for x in leaves]
    cs.merkle_tree([(bpg.ONE, int.from_bytes(W1, "big"))], [[(bpg.ONE, int.from_bytes(i, "big"))] for i in inst],
                   [[(v, 1)] for v in vs], bpg.pattern_str(pattern))
    return cs


def leaves(k, seed=3):
    import random
    r = random.Random(seed)
    return [bytes([r.getrandbits(6)]) + bytes(r.getrandbits(8) for _ in range(31)) for _ in range(k)]


H = lambda a, b: ("H", a, b)  # noqa: E731
Wp, Ip = ("W",), ("I",)


@pytest.mark.parametrize("pattern,nw,ni", [
    (H(Wp, H(H(Wp, Wp), H(Wp, Wp))), 5, 0),                     # test_merkle_tree_gadget_6 shape
    (H(H(H(Wp, Wp), H(Ip, Wp)), H(H(Ip, Wp), H(Wp, Ip))), 5, 3),  # _2 shape (instance leaves)
    (H(H(H(Wp, Wp), H(Wp, Wp)), Wp), 5, 0),                     # _4 shape
])
def test_merkle_recorder_matches_oracle(bpg, pattern, nw, ni):
    lv = leaves(nw + ni)
    w, i = lv[:nw], lv[nw:]
    o = oracle_merkle(w, pattern, i).to_flat()
    p = product_merkle(bpg, w, pattern, i)
    assert view_tuple(p.view) == view_tuple(o.view())


def test_ops_replay_matches_oracle(bpg):
    """A Rust caller replays its ProverBuffer op list (cs_buffer.rs:89-116:
    commit, multiply, constrain in program order) into the recorder; the
    result is the oracle's flattened system, byte for byte."""
    pattern = H(H(Wp, Wp), H(Wp, Wp))
    ocs = oracle_merkle(leaves(4), pattern)
    rng = S.Rng(11)
    cs = bpg.GadgetCS(prover=True)
    for x in leaves(4):
        cs.commit(int.from_bytes(x, "big"), rng.scalar())
    for op in ocs.ops[0]:
        if op[0] == "mul":
            l, r, o = cs.multiply(op[1], op[2])
            assert (l, r) == (op[3], op[4])
        else:
            cs.constrain(op[1])
    assert view_tuple(cs.view) == view_tuple(ocs.to_flat().view())


@pytest.mark.parametrize("value,bits", [(0x0522a64d7b931e, 56), (0, 8), ((1 << 64) - 1, 64)])
def test_range_proof_recorder(bpg, value, bits):
    """utils.rs:5 range_proof through the recorder vs the oracle's."""
    ocs = S.Cs(True)
    S.range_proof(ocs, S.lc_const(value), bits, value)
    cs = bpg.GadgetCS(prover=True)
    cs.range_proof([(bpg.ONE, value)], bits, value)
    assert view_tuple(cs.view) == view_tuple(ocs.to_flat().view())


def test_verifier_side_recorder(bpg):
    """VerifierBuffer side: points committed, no assignments; the constraint
    matrix equals the prover side's."""
    pattern = H(H(Wp, Wp), H(Wp, Wp))
    p = product_merkle(bpg, leaves(4), pattern)
    pv = view_tuple(p.view)
    cs = bpg.GadgetCS(prover=False)
    pts = [bytes([k + 1]) * 32 for k in range(4)]
    vs = [cs.commit(P) for P in pts]
    cs.merkle_tree([(bpg.ONE, int.from_bytes(W1, "big"))], [], [[(v, 1)] for v in vs], bpg.pattern_str(pattern))
    vv = view_tuple(cs.view)
    assert vv[:3] == pv[:3]
    assert vv[-3:] == pv[-3:]
    assert vv[3] == b""
    assert ctypes.string_at(bpg.lib().bpg_cs_V(cs.h), 128) == b"".join(pts)


def test_recorder_rejects_bad_input(bpg):
    cs = bpg.GadgetCS(prover=True)
    with pytest.raises(bpg.BpgError):
        cs.multiply([(bpg.lib and (4 << 28) | 3, 1)], [(0, 1)])    # commitment 3 does not exist
    with pytest.raises(bpg.BpgError):
        cs.merkle_tree([(0, 1)], [], [], "H(W W)")                 # too few leaves for the pattern
    with pytest.raises(bpg.BpgError):
        cs.merkle_tree([(0, 1)], [], [], "H(W")                    # malformed pattern
    with pytest.raises(bpg.BpgError):
        cs.allocate_multiplier(None)                               # prover side needs an assignment
