"""Full-size byte parity (BASELINE.json configs 4 and 5, and the reference's
own 2^20 circuit) against committed oracle proofs.

tests/golden/fullsize.json was written in the CPU container by
tests/golden/make_fullsize.py: the Python statement layer (oracle/synth.py)
synthesised each statement under deterministic mode and the C oracle
(oracle/bpg_oracle.c) proved it (minutes per statement). Here the device
proves the same statements through every production entry point and must
reproduce those bytes exactly:

* c_prove (the reference's iOS C-ABI, prove.rs:37) with the same seed;
* bpg_r1cs_prove (the inner ABI, prove.rs:79) with the default strategy;
* bpg_prepare + bpg_prove_batch (the bench's path: lockstep TranscriptRng
  producers, one HIP stream per consumer thread);
* for merkle512 (merkle_tree_gadget.rs:473-545, n = 993,384, N = 2^20), the
  Gadget-API recorder (bpg_cs_*, the ProverBuffer cut of cs_buffer.rs) builds
  the circuit natively.
"""
import hashlib
import json
import os

import pytest

import synth as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "fullsize.json")))

# merkle_tree_gadget.rs:126-131 (W1) and :475 (the hash_512 root)
W1 = bytes.fromhex("0522a64d7b931e21760cf955a15fcc793e8a52b42a56ab03afddec8beb668749")
ROOT512 = bytes.fromhex("038c137beec8e2edfb5c48cbd063f04e569139d2221a4eb7befb85aa1bf8ba40")


@pytest.fixture(scope="module")
def W():
    import workloads
    return workloads


@pytest.fixture(scope="module")
def bpg(W):
    return W._bpg()


@pytest.fixture(scope="module")
def ctx(bpg):
    return bpg.Context(0)


def _statement(W, name):
    inst, wit, gad = W.CONFIGS[int(name[-1])]()
    g = GOLDEN[name]
    assert hashlib.sha256((inst + "\0" + wit + "\0" + gad).encode()).hexdigest() == g["statement_sha256"], \
        "workloads.py no longer generates the statement the golden proof was made for"
    return inst, wit, gad, g


@pytest.mark.parametrize("name", ["config4", "config5"])
def test_c_prove_matches_oracle(bpg, W, name):
    inst, wit, gad, g = _statement(W, name)
    bpg.set_seed(g["seed"])
    proof, coms = bpg.prove(g["label"], inst, wit, gad)
    assert hashlib.sha256(coms.encode()).hexdigest() == g["coms_sha256"]
    assert proof.hex() == g["proof"]
    assert bpg.verify(g["label"], inst, proof, coms, gad)


@pytest.mark.parametrize("name", ["config4", "config5"])
def test_inner_abi_and_batch_match_oracle(bpg, ctx, W, name):
    inst, wit, gad, g = _statement(W, name)
    bpg.set_seed(g["seed"])                     # the same blindings as c_prove's synthesis
    syn = bpg.Synth(inst, wit, gad)
    assert (syn.n, syn.m, syn.q) == (g["n"], g["m"], g["q"])
    ent = bytes.fromhex(g["entropy"])
    label = g["label"].encode()
    proof, V = ctx.r1cs_prove(label, syn.view, ent)
    assert proof.hex() == g["proof"]
    assert V[0].hex() == g["V0"]
    prep = ctx.prepare(syn.view)
    other = bytes(32)
    batch = prep.prove_batch(label, [other, ent, other, ent], threads=3)
    assert batch[1].hex() == g["proof"] and batch[3].hex() == g["proof"]
    assert batch[0] == batch[2] != batch[1]


def test_merkle512_gadget_api_matches_oracle(bpg, ctx):
    """test_merkle_tree_gadget_512 (#[ignore] in the reference: minutes of
    single-core dalek) through the Gadget-API recorder: commit_all_single of
    512 copies of W1 (blindings from the same seeded stream as the oracle),
    MerkleTree256 over hash_512, prove on the device, verify on the device."""
    g = GOLDEN["merkle512"]
    rng = S.Rng(g["seed"])
    cs = bpg.GadgetCS(prover=True)
    w = int.from_bytes(W1, "big")
    variables = [cs.commit(w, rng.scalar()) for _ in range(512)]
    pattern = ("W",)
    for _ in range(9):
        pattern = ("H", pattern, pattern)
    cs.merkle_tree([(bpg.ONE, int.from_bytes(ROOT512, "big"))], [], [[(v, 1)] for v in variables],
                   bpg.pattern_str(pattern))
    view = cs.view
    assert (view.n, view.m, view.q) == (g["n"], g["m"], g["q"])
    ent = rng.bytes(32)
    assert ent.hex() == g["entropy"]
    proof, V = ctx.r1cs_prove(g["label"].encode(), view, ent)
    assert hashlib.sha256(b"".join(V)).hexdigest() == g["coms_sha256"]
    assert proof.hex() == g["proof"]
    assert ctx.r1cs_verify(g["label"].encode(), view, V, proof)
    bad = bytearray(proof)
    bad[-40] ^= 1
    assert not ctx.r1cs_verify(g["label"].encode(), view, V, bytes(bad))
