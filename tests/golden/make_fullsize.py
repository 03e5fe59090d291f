#!/usr/bin/env python3
"""Generate the full-size golden proofs (tests/golden/fullsize.json).

Runs in the CPU container only (minutes of oracle work per statement); the GPU
tests (tests/test_gpu_fullsize.py) read the committed JSON and never run this.

For each statement the Python statement-layer restatement (oracle/synth.py)
synthesises the circuit under deterministic mode (seeded ChaCha20 for the
commitment blindings and the TranscriptRng finalize entropy)
and the C oracle (oracle/bpg_oracle.c) proves it. Recorded per statement:
sizes, the sha256 of the statement text (so a drifting generator is caught),
the full proof bytes, the sha256 of the `.coms` text (or, for the Gadget-API
circuit, of the concatenated commitments), and the finalize entropy.

Statements:
  config4    workloads.config4()  4 x depth-32 MERKLE paths, N = 2^18
  config5    workloads.config5()  the bench's own statement, N = 2^20
  merkle512  the reference's Gadget-API test test_merkle_tree_gadget_512
             (src/merkle_tree/merkle_tree_gadget.rs:473-545): 512 committed
             copies of W1 (:126-131) under hash_512, root at :475, transcript
             label "MerkleTree", BulletproofGens::new(1048576, 1) -> N = 2^20,
             n = 993,384. Built with the Gadget-API mirror synth.Cs +
             synth.Merkle (commit_all_single = commitments.rs:9-31).

usage: python tests/golden/make_fullsize.py [name ...]
"""
import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402
import synth  # noqa: E402

# merkle_tree_gadget.rs:126-131 (W1) and :475 (root of hash_512)
W1 = bytes.fromhex("0522a64d7b931e21760cf955a15fcc793e8a52b42a56ab03afddec8beb668749")
ROOT512 = bytes.fromhex("038c137beec8e2edfb5c48cbd063f04e569139d2221a4eb7befb85aa1bf8ba40")

SEEDS = {"config4": 404, "config5": 505, "merkle512": 512}
LABELS = {"config4": b"cfg4", "config5": b"cfg5", "merkle512": b"MerkleTree"}


def pattern(levels):
    """hash!(p, p) nested `levels` deep over W leaves (hash_2 .. hash_512)."""
    p = ("W",)
    for _ in range(levels):
        p = ("H", p, p)
    return p


def merkle512_cs(seed, leaves=512):
    """test_merkle_tree_gadget_512 through the Gadget API: commit_all_single
    (one Prover::commit per 32-byte witness, blinding from the seeded stream in
    program order), then MerkleTree256::assemble. Returns (Cs, rng)."""
    rng = synth.Rng(seed)
    cs = synth.Cs(True)
    s = synth.be_to_scalar(W1)
    variables = [cs.commit(s, rng.scalar()) for _ in range(leaves)]
    levels = leaves.bit_length() - 1
    root = synth.lc_const(synth.be_to_scalar(ROOT512))
    synth.Merkle(root, [], [synth.lc_var(v) for v in variables], pattern(levels)).assemble(cs, [], [])
    return cs, rng


def make(name):
    import workloads as W
    t0 = time.time()
    seed, label = SEEDS[name], LABELS[name]
    if name == "merkle512":
        cs, rng = merkle512_cs(seed)
        flat = cs.to_flat()
        ent = rng.bytes(32)
        proof, V = O.r1cs_prove(label, flat, ent)
        coms_sha = hashlib.sha256(b"".join(V)).hexdigest()
        stmt_sha = hashlib.sha256(W1 + ROOT512).hexdigest()
    else:
        inst, wit, gad = W.CONFIGS[int(name[-1])]()
        st = synth.synthesize_prover(inst, wit, gad, seed)
        flat = st.cs.to_flat()
        ent = synth.entropy_for(st)
        proof, V = O.r1cs_prove(label, flat, ent)
        coms = "".join("%s = 0x%s\n" % (nm, V[i].hex()) for i, nm in enumerate(st.com_order))
        coms_sha = hashlib.sha256(coms.encode()).hexdigest()
        stmt_sha = hashlib.sha256((inst + "\0" + wit + "\0" + gad).encode()).hexdigest()
    t_prove = time.time() - t0
    # the oracle verifier must accept its own proof
    ok = O.r1cs_verify(label, flat, V, proof) == 1
    assert ok, "oracle rejected its own %s proof" % name
    N = 1
    while N < flat.n:
        N *= 2
    return {"label": label.decode(), "seed": seed, "n": flat.n, "m": flat.m, "q": flat.q, "N": N,
            "statement_sha256": stmt_sha, "entropy": ent.hex(), "proof": proof.hex(),
            "coms_sha256": coms_sha, "V0": V[0].hex() if V else None,
            "oracle_seconds": round(t_prove, 1)}


def main():
    path = os.path.join(HERE, "fullsize.json")
    data = json.load(open(path)) if os.path.exists(path) else {}
    for name in sys.argv[1:] or list(SEEDS):
        print("generating %s ..." % name, flush=True)
        data[name] = make(name)
        print("  n=%d q=%d N=%d in %.0f s" % (data[name]["n"], data[name]["q"], data[name]["N"],
                                              data[name]["oracle_seconds"]), flush=True)
        json.dump(data, open(path, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
