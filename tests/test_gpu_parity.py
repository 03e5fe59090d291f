"""Device parity tests (MI355X): HIP path through the C-ABI vs the CPU oracle.

All comparisons are bit-exact (integer/byte work). Sizes here keep the oracle
within seconds; full-size properties are in test_gpu_scale.py.
"""
import os
import random

import pytest

import oracle as O
import synth as S
from conftest import read_fixture

pytestmark = pytest.mark.gpu

L = S.L


@pytest.fixture(scope="module")
def bpg():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bpg", os.path.join(root, "bulletproof-gadgets_amd", "bpg.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="module")
def ctx(bpg):
    return bpg.Context(0)


def rand_points(rnd, k):
    return [O.from_uniform(bytes(rnd.getrandbits(8) for _ in range(64))) for _ in range(k)]


@pytest.mark.parametrize("n", [1, 2, 7, 64, 191, 1000, 5000])
def test_msm_random(ctx, n):
    rnd = random.Random(n)
    pts = rand_points(rnd, min(n, 64))
    pts = [pts[i % len(pts)] for i in range(n)]
    sc = [rnd.randrange(L).to_bytes(32, "little") for _ in range(n)]
    assert ctx.msm(sc, pts) == O.msm(sc, pts)


def test_msm_structured_scalars(ctx):
    # bits / small values / zeros / l-1 / non-canonical inputs: skewed buckets
    rnd = random.Random(3)
    n = 3000
    pts = rand_points(rnd, 50)
    pts = [pts[i % 50] for i in range(n)]
    vals = []
    for i in range(n):
        k = i % 6
        v = [0, 1, rnd.randrange(2), L - 1, rnd.randrange(1 << 64), (1 << 256) - 1 - i][k]
        vals.append(v.to_bytes(32, "little"))
    assert ctx.msm(vals, pts) == O.msm(vals, pts)
    ones = [(1).to_bytes(32, "little")] * 4096
    same = [pts[0]] * 4096
    assert ctx.msm(ones, same) == O.msm(ones, same)


def test_msm_large_structured(ctx):
    """A job big enough for 16-bit windows (2^18 + 5 points: the two-digit
    radix sort and the run merges at their full depth) with a quarter of the
    scalars equal to 1 (one bucket of 65K entries: runs far longer than any
    sort tile or reduction chunk), a quarter small, the rest random."""
    rnd = random.Random(18)
    n = (1 << 18) + 5
    pts = rand_points(rnd, 97)
    pts = [pts[i % 97] for i in range(n)]
    vals = []
    for i in range(n):
        k = i % 4
        v = [1, rnd.randrange(1 << 20), rnd.randrange(L), L - 1 - i][k]
        vals.append(v.to_bytes(32, "little"))
    assert ctx.msm(vals, pts) == O.msm(vals, pts)


def test_msm_identity_and_invalid(ctx, bpg):
    assert ctx.msm([b"\0" * 32], [O.pedersen_gens()[0]]) == b"\0" * 32
    with pytest.raises(bpg.BpgError):
        ctx.msm([b"\1" + b"\0" * 31], [b"\xff" * 32])


def test_pedersen(ctx):
    rnd = random.Random(11)
    v = [rnd.getrandbits(255).to_bytes(32, "little") for _ in range(70)]    # from_bits: may exceed l
    vb = [rnd.randrange(L).to_bytes(32, "little") for _ in range(70)]
    got = ctx.pedersen(v, vb)
    for a, b, g in zip(v, vb, got):
        assert g == O.pedersen_commit(a, b)


def test_range_proof_inner_abi(ctx):
    x = S.be_to_scalar(bytes([0x05, 0x22, 0xa6, 0x4d, 0x7b, 0x93, 0x1e]))
    for n, ok in [(56, True), (48, False)]:
        cs = S.Cs(True)
        S.range_proof(cs, S.lc_const(x), n, x)
        flat = cs.to_flat()
        ent = bytes(range(32))
        proof, _ = ctx.r1cs_prove(b"RangeProof", flat.view(), ent)
        o_proof, _ = O.r1cs_prove(b"RangeProof", flat, ent)
        assert proof == o_proof
        vcs = S.Cs(False)
        S.range_proof(vcs, S.lc_const(x), n, None)
        vflat = vcs.to_flat()
        assert ctx.r1cs_verify(b"RangeProof", vflat.view(secrets=False), [], proof) == ok
        assert O.r1cs_verify(b"RangeProof", vflat, [], proof) == (1 if ok else 0)


FIXTURES = ["bounds_check", "equality", "inequality", "less_than", "or3", "or5", "or", "example"]


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_bit_exact(bpg, resources, name):
    fx = read_fixture(os.path.join(resources, name))
    seed = 77 + len(name)
    bpg.set_seed(seed)
    proof, coms = bpg.prove(name, fx["inst"], fx["wtns"], fx["gadgets"])
    o_proof, o_coms, flat = S.prove_statement(name.encode(), fx["inst"], fx["wtns"], fx["gadgets"], seed)
    assert coms == o_coms
    assert proof == o_proof
    assert bpg.verify(name, fx["inst"], proof, coms, fx["gadgets"])
    assert S.verify_statement(name.encode(), fx["inst"], proof, coms, fx["gadgets"])


@pytest.mark.parametrize("tables,pairs,tail", [(0, 0, -1), (1, 0, -1), (0, 1, -1), (1, 1, -1), (-1, -1, -1),
                                               (1, 2, 4), (0, 2, 4), (1, 1, 4), (0, 2, 16), (-1, -1, 8)])
@pytest.mark.parametrize("name", ["bounds_check", "less_than", "example", "inequality", "or5"])
def test_fold_strategy_bit_exact(bpg, resources, name, tables, pairs, tail):
    """Every IPP fold strategy of a context (per-round variable-base fold;
    comb-table pass for rounds 0-1 with a lazily expanded round-1 MSM; round
    pairs folded by the three-scalar Straus pass with lazily expanded
    odd-round MSMs; round triples folded by the seven-scalar Straus pass with
    bases expanded two levels deep; the default) gives the oracle's bytes
    through the inner ABI (bpg_r1cs_prove). A small IPP tail threshold makes
    the fold passes run on these small circuits (the default tail would take
    over right after the comb pass). The fixtures put n - N/2 on both sides
    of N/4, so every lane class of the two-round passes occurs."""
    fx = read_fixture(os.path.join(resources, name))
    seed = 900 + len(name)
    st = S.synthesize_prover(fx["inst"], fx["wtns"], fx["gadgets"], seed)
    flat = st.cs.to_flat()
    ent = S.entropy_for(st)
    o_proof, o_V = O.r1cs_prove(name.encode(), flat, ent)
    c = bpg.Context(0)
    c.set_strategy(tables, pairs, tail)
    proof, V = c.r1cs_prove(name.encode(), flat.view(), ent)
    assert V == o_V
    assert proof == o_proof


@pytest.mark.parametrize("msm_tables,tail", [(0, -1), (1, -1), (1, 8), (0, 8)])
@pytest.mark.parametrize("name", ["bounds_check", "example", "or5"])
def test_msm_tables_bit_exact(bpg, resources, name, msm_tables, tail):
    """Fixed-base generator tables (bpg_ctx_set_msm_tables: 13 windows of
    2^(20w) G_i / H_i, one bucket row per MSM, keys sorted in three radix
    passes) for the commitment and IPP round-0/1 jobs (on), or the ordinary
    windowed jobs (off, and the default): the oracle's bytes either way, with
    the default and a small IPP tail threshold."""
    fx = read_fixture(os.path.join(resources, name))
    seed = 700 + len(name)
    st = S.synthesize_prover(fx["inst"], fx["wtns"], fx["gadgets"], seed)
    flat = st.cs.to_flat()
    ent = S.entropy_for(st)
    o_proof, o_V = O.r1cs_prove(name.encode(), flat, ent)
    c = bpg.Context(0)
    c.set_strategy(ipp_tail=tail, msm_tables=msm_tables)
    proof, V = c.r1cs_prove(name.encode(), flat.view(), ent)
    assert V == o_V
    assert proof == o_proof
    if msm_tables:
        assert c.setup_stats()["msm_table_bytes"] > 0


@pytest.mark.parametrize("name", ["bounds_check", "less_than", "example"])
def test_fixture_rejects(bpg, resources, name):
    fx = read_fixture(os.path.join(resources, name))
    bpg.set_seed(5)
    proof, coms = bpg.prove(name, fx["inst"], fx["wtns"], fx["gadgets"])
    assert not bpg.verify(name + "x", fx["inst"], proof, coms, fx["gadgets"])        # label is bound
    for pos in (1, 100, 300, len(proof) - 70, len(proof) - 1):
        bad = bytearray(proof)
        bad[pos] ^= 0x10
        assert not bpg.verify(name, fx["inst"], bytes(bad), coms, fx["gadgets"])
    assert not bpg.verify(name, fx["inst"], proof[:-32], coms, fx["gadgets"])
    lines = coms.splitlines()
    lines[0], lines[1] = lines[1], lines[0]
    assert not bpg.verify(name, fx["inst"], proof, "\n".join(lines) + "\n", fx["gadgets"])


@pytest.mark.slow
@pytest.mark.parametrize("name", ["mimc_hash", "merkle_tree", "set_membership", "or2", "or4"])
def test_fixture_bit_exact_large(bpg, resources, name):
    test_fixture_bit_exact(bpg, resources, name)


def test_unsatisfied_statement_rejected(bpg, resources):
    # less_than.wtns witnesses with the operands swapped: the circuit is not
    # satisfied, the proof must not verify (reference less_than tests)
    fx = read_fixture(os.path.join(resources, "less_than"))
    g = fx["gadgets"].splitlines()
    swapped = []
    for line in g:
        t = line.split()
        swapped.append(" ".join([t[0], t[2], t[1]]) if t and t[0] == "LESS_THAN" else line)
    gad = "\n".join(swapped)
    bpg.set_seed(1)
    proof, coms = bpg.prove("lt", fx["inst"], fx["wtns"], gad)
    assert not bpg.verify("lt", fx["inst"], proof, coms, gad)


def test_prepared_batch_matches_single(bpg, ctx, resources):
    fx = read_fixture(os.path.join(resources, "or5"))
    bpg.set_seed(2)
    syn = bpg.Synth(fx["inst"], fx["wtns"], fx["gadgets"])
    prep = ctx.prepare(syn.view)
    ents = [bytes([k]) * 32 for k in range(6)]
    proofs = prep.prove_batch(b"batch", ents, threads=3)
    for k, p in enumerate(proofs):
        single, _ = ctx.r1cs_prove(b"batch", syn.view, ents[k])
        assert p == single
    assert len(set(proofs)) == 6


@pytest.mark.parametrize("producers,lockstep", [(1, 1), (2, 2), (1, 3), (3, 4)])
def test_batch_layouts_bit_exact(bpg, resources, producers, lockstep):
    """The batched prover's pipeline layout (bpg_ctx_set_pipeline: RNG
    producers, proofs per consumer step) never changes proof bytes: 11 proofs
    (a partial RNG group of 8 and partial lockstep steps) equal single proofs,
    and bpg_last_batch_stats reports the layout that ran."""
    fx = read_fixture(os.path.join(resources, "or5"))
    bpg.set_seed(2)
    syn = bpg.Synth(fx["inst"], fx["wtns"], fx["gadgets"])
    c = bpg.Context(0)
    c.set_pipeline(producers=producers, lockstep=lockstep)
    prep = c.prepare(syn.view)
    ents = [bytes([k + 40]) * 32 for k in range(11)]
    proofs = prep.prove_batch(b"layout", ents, threads=producers + 3)
    st = bpg.last_batch_stats()
    # 11 proofs are two RNG groups of 8: at most two producers have work
    assert st["producers"] == min(producers, 2) and st["lockstep"] == lockstep and st["consumers"] >= 1
    assert st["wall_ms"] > 0 and st["producer_draw_ms"] > 0 and st["consumer_prove_ms"] > 0
    for k in (0, 5, 10):
        assert proofs[k] == c.r1cs_prove(b"layout", syn.view, ents[k])[0]
    assert len(set(proofs)) == 11
    with pytest.raises(bpg.BpgError):
        c.set_pipeline(producers=9)


def test_verify_batch(bpg, ctx, resources):
    """bpg_verify_batch (config 5's batch verification: chunks of proofs
    checked by one random-linear-combination MSM each): every valid proof of
    a batch accepted, each tampered one rejected, same verdicts as the single
    verifier, whatever the thread count."""
    fx = read_fixture(os.path.join(resources, "or5"))
    bpg.set_seed(3)
    syn = bpg.Synth(fx["inst"], fx["wtns"], fx["gadgets"])
    prep = ctx.prepare(syn.view)
    proofs = prep.prove_batch(b"vb", [bytes([k + 1]) * 32 for k in range(6)], threads=2)
    V = ctx.pedersen(syn.vec("v", syn.m), syn.vec("v_blinding", syn.m))
    bad = []
    for k, p in enumerate(proofs[:3]):
        b = bytearray(p)
        b[[1, 300, len(b) - 1][k]] ^= 4     # A_I1 point, t_x_blinding, IPP b scalar
        bad.append(bytes(b))
    batch = proofs + bad + [proofs[0][:-32]]
    want = [True] * 6 + [False] * 4
    vprep = ctx.prepare(syn.view, verifier=True)
    for threads in (1, 4):
        assert vprep.verify_batch(b"vb", V, batch, threads) == want
    assert [ctx.r1cs_verify(b"vb", syn.view, V, p) for p in batch] == want
    assert vprep.verify_batch(b"other label", V, proofs[:2], 2) == [False, False]
    with pytest.raises(bpg.BpgError):
        prep.verify_batch(b"vb", V, proofs[:1], 1)   # prover layout
    # one chunk checked by a single random-linear-combination MSM: all valid
    # -> accepted at once; one canonical-but-wrong proof inside -> the chunk
    # fails and is re-verified proof by proof
    many = prep.prove_batch(b"vb", [bytes([k + 40]) * 32 for k in range(20)], threads=2)
    assert vprep.verify_batch(b"vb", V, many, 1) == [True] * 20
    mixed = list(many)
    b = bytearray(mixed[13]); b[300] ^= 4; mixed[13] = bytes(b)
    assert vprep.verify_batch(b"vb", V, mixed, 1) == [k != 13 for k in range(20)]
    assert vprep.verify_batch(b"vb", V, mixed, 3) == [k != 13 for k in range(20)]
