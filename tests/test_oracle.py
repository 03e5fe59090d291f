"""The CPU oracle pinned against independent implementations and the
reference's own known answers."""
import ctypes
import hashlib
import os
import random

import pytest

import oracle as O
import synth as S
from conftest import read_fixture

L = S.L
SODIUM = "/opt/conda/lib/libsodium.so"


def test_keccak_against_hashlib():
    for data in [b"", b"abc", bytes(range(256)) * 3]:
        assert O.sha3_512(data) == hashlib.sha3_512(data).digest()
        assert O.shake256(data, 500) == hashlib.shake_256(data).digest(500)


def test_merlin_conformance_vector():
    # merlin 2.0.1 tests: Transcript::new("test protocol"), append_message,
    # challenge_bytes("challenge", 32)
    c = O.merlin_test(b"test protocol", b"some label", b"some data", b"challenge", 32)
    assert c.hex() == "d5a21972d0d5fe320c0d263fac7fffb8145aa640af6e9bca177c03c7efcf0615"


def test_pedersen_gens():
    B, Bb = O.pedersen_gens()
    assert B.hex() == "e2f2ae0a6abc4e71a884a961c500515f58e30b6aa582dd8db6a65945e08d2d76"
    assert Bb.hex() == "8c9240b456a9e6dc65c377a1048d745f94a08cdb7f44cbcd7b46f34048871134"


def test_generator_chain_mechanism():
    G, H = O.generators(3)
    g = hashlib.shake_256(b"GeneratorsChain" + b"G" + b"\0" * 4).digest(192)
    h = hashlib.shake_256(b"GeneratorsChain" + b"H" + b"\0" * 4).digest(192)
    for i in range(3):
        assert G[i] == O.from_uniform(g[64 * i:64 * i + 64])
        assert H[i] == O.from_uniform(h[64 * i:64 * i + 64])
    assert G[0].hex() == "fc3b25801422672a6a8d3adb5d8457d4301fe92324b4fc56ae934c8713ddfe2d"


@pytest.mark.skipif(not os.path.exists(SODIUM), reason="libsodium not present")
def test_ristretto_against_libsodium():
    so = ctypes.CDLL(SODIUM)
    so.sodium_init()
    rnd = random.Random(5)
    out = ctypes.create_string_buffer(32)
    for _ in range(40):
        h = bytes(rnd.getrandbits(8) for _ in range(64))
        so.crypto_core_ristretto255_from_hash(out, h)
        assert out.raw == O.from_uniform(h)
    for _ in range(10):
        a = O.from_uniform(bytes(rnd.getrandbits(8) for _ in range(64)))
        b = O.from_uniform(bytes(rnd.getrandbits(8) for _ in range(64)))
        so.crypto_core_ristretto255_add(out, a, b)
        assert out.raw == O.point_add(a, b)
        s = rnd.getrandbits(252).to_bytes(32, "little")
        so.crypto_scalarmult_ristretto255(out, s, a)
        assert out.raw == O.point_mul(s, a)


def test_scalar_arithmetic():
    rnd = random.Random(6)
    for _ in range(200):
        a, b, w = rnd.getrandbits(256), rnd.getrandbits(256), rnd.getrandbits(512)
        ab, bb = a.to_bytes(32, "little"), b.to_bytes(32, "little")
        assert int.from_bytes(O.sc_mul(ab, bb), "little") == a * b % L
        assert int.from_bytes(O.sc_add(ab, bb), "little") == (a + b) % L
        assert int.from_bytes(O.sc_wide(w.to_bytes(64, "little")), "little") == w % L
    assert O.sc_invert(b"\0" * 32) == b"\0" * 32


def test_msm_matches_sum_of_products():
    rnd = random.Random(7)
    pts = [O.from_uniform(bytes(rnd.getrandbits(8) for _ in range(64))) for _ in range(220)]
    sc = [rnd.getrandbits(253).to_bytes(32, "little") for _ in range(220)]
    acc = None
    for s, p in zip(sc, pts):
        t = O.point_mul(s, p)
        acc = t if acc is None else O.point_add(acc, t)
    assert O.msm(sc, pts) == acc          # Pippenger path (>190)


def test_mimc_known_answers():
    # src/mimc_hash/mimc.rs:104-143
    pre1 = bytes([0x38, 0x53, 0x54, 0x50, 0x43, 0x30, 0x43, 0x54, 0x6f, 0x31, 0x38, 0x77, 0x61, 0x5a, 0x6a, 0x42, 0x36, 0x63])
    assert S.scalar_to_be(S.mimc_hash(pre1)).hex() == "0d2203069ac15f58172bae1b3af98d8982deef9df37482c1a920b8832ee813a4"
    pre2 = b"The quick brown fox jumps over t"
    assert S.scalar_to_be(S.mimc_hash(pre2)).hex() == "01245409f28ae2f076077d4a40bd91551b3a03b1ad8adb2b1da116d29c60a85c"


def test_merkle_golden_roots():
    # merkle_tree_gadget.rs:476-503: 9 intermediate roots of the 512-leaf tree
    w1 = bytes([0x05, 0x22, 0xa6, 0x4d, 0x7b, 0x93, 0x1e, 0x21, 0x76, 0x0c, 0xf9, 0x55, 0xa1, 0x5f, 0xcc, 0x79,
                0x3e, 0x8a, 0x52, 0xb4, 0x2a, 0x56, 0xab, 0x03, 0xaf, 0xdd, 0xec, 0x8b, 0xeb, 0x66, 0x87, 0x49])
    expect = ["0b79280bd08952b2f43c000fa7ee45d0f73c0242a34033e9fde3cac80deaff7c",
              "0f06bee0afba3bfe751787721eafd769e993e1700cde9b7b2146fc508efc54e5",
              "04af68c673b12851f92603154c51a9ea1714a855686f275b54539a8696d6ce60",
              "004ce529f3e16d7c7d40fd72033ccdb351b710d0aab96ab350fb206202a0328b",
              "0fe33807557b26124c6f60abede601a601298794 41c08d8ea940cf45086e1cce".replace(" ", ""),
              "0a3bcac677f47d10383e7efd397d0f71b951704504b7a9ad81848fdc29855f3a",
              "049057939c976063cfaed9e15fc02c8dbd997e12f9b919a97781870ad689bd41",
              "0c61fcdd0add4eb6d44de2be6ef2353871696ed586af8aa5fd1b54478c989fe1",
              "038c137beec8e2edfb5c48cbd063f04e569139d2221a4eb7befb85aa1bf8ba40"]
    # leaves are the raw scalars (merkle gadget test commits W1 directly)
    node = S.be_to_scalar(w1)

    def sponge2(a, b):
        state = 0
        for blk in (a, b):
            state = (state + blk) % L
            for c in S.mimc_constants():
                t = (state + c) % L
                state = t * t % L * t % L
        return state
    for e in expect:
        node = sponge2(node, node)
        assert S.scalar_to_be(node).hex() == e


def test_fixture_images_match_reference(resources):
    # tests/resources/merkle_tree.inst I0 = H(H("John"), H("John")) etc.
    fx = read_fixture(os.path.join(resources, "mimc_hash"))
    inst = dict(S.parse_var_line(l) for l in fx["inst"].splitlines())
    wit = dict(S.parse_var_line(l) for l in fx["wtns"].splitlines())
    assert S.scalar_to_be(S.mimc_hash(wit["W1"])) == wit["W0"].rjust(32, b"\0")
    assert S.scalar_to_be(S.mimc_hash(wit["W2"])) == inst["I0"].rjust(32, b"\0")


@pytest.mark.parametrize("name,n,q,m", [
    ("bounds_check", 1440, 2889, 9), ("equality", 0, 9, 12), ("inequality", 24, 63, 36),
    ("less_than", 1137, 2289, 12), ("or3", 3, 9, 3), ("or5", 4721, 10531, 29),
])
def test_fixture_round_trip(resources, name, n, q, m):
    fx = read_fixture(os.path.join(resources, name))
    proof, coms, flat = S.prove_statement(name.encode(), fx["inst"], fx["wtns"], fx["gadgets"], seed=3)
    assert (flat.n, flat.q, flat.m) == (n, q, m)
    N = 1
    while N < n:
        N *= 2
    assert len(proof) == 417 + 64 * (N.bit_length() - 1)
    assert S.verify_statement(name.encode(), fx["inst"], proof, coms, fx["gadgets"])
    # wrong label, tampered proof and tampered commitment are rejected
    assert not S.verify_statement(b"other", fx["inst"], proof, coms, fx["gadgets"])
    bad = bytearray(proof)
    bad[-40] ^= 1
    assert not S.verify_statement(name.encode(), fx["inst"], bytes(bad), coms, fx["gadgets"])


def test_mimc_gadget_constraint_count():
    # or_conjunction.rs:85 "HASH GADGET: 1946 Constraints" (one block, padded)
    cs = S.Cs(True)
    w = [S.be_to_scalar(b"\x43")]
    vars_ = [cs.commit(w[0], 1)]
    g = S.MimcHash(S.lc_const(S.mimc_hash(b"\x43")))
    d = S.setup(cs, g.preprocess(w), S.Rng(1))
    g.assemble(cs, vars_, d)
    assert len(cs.flat_rows()) == 1946 and cs.nvars == 972


def test_range_proof_accept_reject():
    # utils.rs:45-90
    x = S.be_to_scalar(bytes([0x05, 0x22, 0xa6, 0x4d, 0x7b, 0x93, 0x1e]))
    for n, ok in [(56, 1), (48, 0)]:
        cs = S.Cs(True)
        S.range_proof(cs, S.lc_const(x), n, x)
        proof, _ = O.r1cs_prove(b"RangeProof", cs.to_flat(), b"\x01" * 32)
        vcs = S.Cs(False)
        S.range_proof(vcs, S.lc_const(x), n, None)
        assert O.r1cs_verify(b"RangeProof", vcs.to_flat(), [], proof) == ok


def test_deterministic_seed_gives_identical_bytes(resources):
    fx = read_fixture(os.path.join(resources, "inequality"))
    a = S.prove_statement(b"x", fx["inst"], fx["wtns"], fx["gadgets"], seed=11)
    b = S.prove_statement(b"x", fx["inst"], fx["wtns"], fx["gadgets"], seed=11)
    c = S.prove_statement(b"x", fx["inst"], fx["wtns"], fx["gadgets"], seed=12)
    assert a[0] == b[0] and a[1] == b[1]
    assert a[0] != c[0]
