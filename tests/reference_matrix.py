"""The reference's accept/reject matrix: every round-trip test of
the reference crate (27 `is_ok` + 11 `is_err` in src/, plus
tests/combine_gadgets.rs) restated as a Gadget-API circuit over the oracle's
Gadget mirror (oracle/synth.py), with the inputs and the expected verdicts
read from tests/golden/reference_cases.json (extracted from the reference by
tests/golden/extract_reference_cases.py).

TEST INFRASTRUCTURE: each case builds a prover-side and a verifier-side
flattened system (oracle.FlatCS) the way the reference test drives
Prover / Verifier: commit / commit_single / commit_all_single
(commitments.rs:9-47), Gadget::setup / prove / verify (gadget.rs:7-60),
ProverBuffer + or() for the OR test (or_conjunction.rs:4-38). Blindings come
from one seeded stream (deterministic mode), so every proof is reproducible.
"""
import json
import os

import oracle as O
import synth as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_cases.json")))


class Side:
    """One side of a reference test: the prover (values, seeded blindings) or
    the verifier (the prover's commitments, in the same order)."""

    def __init__(self, prover, rng=None, V=None, derived_counts=None):
        self.prover = prover
        self.cs = S.Cs(prover)
        self.rng = rng
        self.V = list(V or [])
        self.derived_counts = list(derived_counts or [])
        self.counts = []

    def commit(self, s):
        if self.prover:
            return self.cs.commit(s, self.rng.scalar())
        return self.cs.commit(V=self.V.pop(0))

    # commitments.rs:9-47
    def commit_single(self, data):
        assert len(data) <= 32
        s = S.be_to_scalar(data)
        return s, self.commit(s)

    def commit_multi(self, data):
        ss = S.be_to_scalars(data)
        return ss, [self.commit(s) for s in ss]

    # gadget.rs:19-42: preprocess -> one commitment per derived scalar
    def setup(self, derive):
        if self.prover:
            ds = derive()
            self.counts.append(len(ds))
            return [(s, self.commit(s)) for s in ds]
        k = self.derived_counts.pop(0)
        return [(None, self.commit(None)) for _ in range(k)]


def _case_data(fn):
    for f, v in CASES.items():
        for t in v["tests"]:
            if t["fn"] == fn:
                return f, v["consts"], t
    raise KeyError(fn)


def _b(consts, tok):
    return bytes.fromhex(consts[tok]) if tok in consts else bytes.fromhex(tok)


def _pattern(s):
    """hash!(a,b) / W / I (whitespace stripped) -> ('H', l, r) tuples."""
    pos = 0

    def rec():
        nonlocal pos
        if s.startswith("hash!(", pos):
            pos += 6
            left = rec()
            assert s[pos] == ","
            pos += 1
            right = rec()
            assert s[pos] == ")"
            pos += 1
            return ("H", left, right)
        c = s[pos]
        pos += 1
        return (c,)
    p = rec()
    assert pos == len(s)
    return p


def build(fn, P):
    """Run reference test `fn` on side P (Side)."""
    f, consts, t = _case_data(fn)
    lets = t["lets"]
    one = lambda name: _b(consts, lets[name][0])  # noqa: E731
    cs = P.cs
    if "bounds_check" in f:
        ss, vs = P.commit_multi(one("witness"))
        g = S.BoundsCheck(one("min"), one("max"))
        g.assemble(cs, vs, P.setup(lambda: g.preprocess(ss)))
    elif f.startswith("src/equality/"):
        k = int(fn.rsplit("_", 1)[1])
        rb = one("right")
        right = [S.lc_const(S.be_to_scalar(rb))] if k in (1, 2) else [S.lc_const(x) for x in S.be_to_scalars(rb)]
        ss, vs = P.commit_multi(one("left"))
        d = P.setup(lambda: []) if k != 4 else []          # Equality::preprocess derives nothing
        S.Equality(right).assemble(cs, vs, d)
    elif "inequality" in f:
        rb = one("right") if "right" in lets else one("value")
        lb = one("left_assignment") if "left_assignment" in lets else one("value")
        ra = S.be_to_scalars(rb)
        g = S.Inequality([S.lc_const(x) for x in ra], ra)
        ss, vs = P.commit_multi(lb)
        g.assemble(cs, vs, P.setup(lambda: g.preprocess(ss)))
    elif "less_than" in f:
        la, ra = S.be_to_scalar(one("left")), S.be_to_scalar(one("right"))
        g = S.LessThan(S.lc_const(la), la, S.lc_const(ra), ra)
        g.assemble(cs, [], P.setup(lambda: g.preprocess([])))
    elif "merkle_tree" in f:
        root = S.be_to_scalar(one("root"))
        wit = [S.lc_var(P.commit_single(bytes.fromhex(consts[c]))[1]) for tgt, c in t["refs"] if tgt == "witnesses"]
        inst = [S.lc_const(S.be_to_scalar(bytes.fromhex(consts[c]))) for tgt, c in t["refs"] if tgt == "instance_vars"]
        S.Merkle(S.lc_const(root), inst, wit, _pattern(t["patterns"][0])).assemble(cs, [], [])
    elif "mimc_hash_gadget" in f:
        g = S.MimcHash(S.lc_const(S.be_to_scalar(one("image"))))
        ss, vs = P.commit_multi(one("preimage"))
        g.assemble(cs, vs, P.setup(lambda: g.preprocess(ss)))
    elif "or_conjunction" in f:
        cache = []
        cs.ops.append([])                                   # ProverBuffer / VerifierBuffer
        for k in (1, 2, 3):
            g = S.MimcHash(S.lc_const(S.be_to_scalar(one("image_%d" % k))))
            ss, vs = P.commit_multi(one("preimage_%d" % k))
            d = P.setup(lambda: g.preprocess(ss))
            g.assemble(cs, vs, d)                           # gadget.prove(prover_buffer, ...)
            cache.append(cs.ops[-1])                        # prover_buffer.rewind()
            cs.ops[-1] = []
        cs.ops.pop()
        S.or_block(cs, cache)                               # or(&mut prover_main, &prover_buffer)
    elif "set_membership" in f:
        va, vv = P.commit_single(one("witness_value"))
        inst_a = [S.be_to_scalar(_b(consts, x)) for x in lets["instance_set"]]
        g = S.SetMembership(S.lc_var(vv), va, [S.lc_const(x) for x in inst_a], inst_a)
        ws = [P.commit_single(_b(consts, x)) for x in lets.get("witness_set", [])]
        d = P.setup(lambda: g.preprocess([a for a, _ in ws]))
        g.assemble(cs, [v for _, v in ws], d)
    elif "utils.rs" in f:
        x = S.be_to_scalar(one("x_assignment"))
        S.range_proof(cs, S.lc_const(x), t["ints"][0], x if P.prover else None)
    elif "combine_gadgets" in f:
        w1s, w1v = P.commit_multi(one("val"))
        _, w2v = P.commit_single(one("image"))
        b = S.BoundsCheck(one("min"), one("max"))
        b.assemble(cs, w1v, P.setup(lambda: b.preprocess(w1s)))
        h = S.MimcHash(S.lc_var(w2v))
        h.assemble(cs, w1v, P.setup(lambda: h.preprocess(w1s)))
        leaf = S.lc_const(S.be_to_scalar(one("merkle_leaf")))
        S.Merkle(S.lc_const(S.be_to_scalar(one("root"))), [leaf], [S.lc_var(w2v)],
                 _pattern(t["patterns"][0])).assemble(cs, [], [])
    else:
        raise KeyError(f)


def cases():
    """[(fn, label, expected verdict 'ok'|'err', file:line)] of the matrix,
    merkle512 excluded (it is the full-size golden of test_gpu_fullsize)."""
    out = []
    for f, v in CASES.items():
        for t in v["tests"]:
            if t["fn"] == "test_merkle_tree_gadget_512":
                continue
            out.append((t["fn"], t["label"], t["verdict"], "%s:%d" % (f, t["verdict_line"])))
    return out


def make(fn, seed=777):
    """-> (label, prover FlatCS, verifier FlatCS builder, entropy).
    The verifier side needs the prover's commitments, so it is returned as
    a function of V."""
    _, _, t = _case_data(fn)
    rng = S.Rng(seed)
    P = Side(True, rng=rng)
    build(fn, P)
    ent = rng.bytes(32)

    def verifier(V):
        Q = Side(False, V=V, derived_counts=P.counts)
        build(fn, Q)
        return Q.cs.to_flat()
    return t["label"].encode(), P.cs.to_flat(), verifier, ent


def oracle_verdict(fn, seed=777):
    label, pf, verifier, ent = make(fn, seed)
    proof, V = O.r1cs_prove(label, pf, ent)
    vf = verifier(V)
    return O.r1cs_verify(label, vf, V, proof) == 1, proof, V, pf, vf, label, ent
