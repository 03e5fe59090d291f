"""Python host binding of libbpg.so (ctypes over include/bpg.h).

Mirrors the reference's entry points for tests and the benchmark:
  prove(name, instance, witness, gadgets) -> (proof bytes, .coms text)
      src/prove.rs:37 `prove` through the iOS C-ABI c_prove
      (interfaces/ios/src/lib.rs:20-42)
  verify(name, instance, proof, commitments, gadgets) -> bool
      src/verify.rs:36 `verify` through c_verify (lib.rs:44-52)
Errors raise BpgError (the reference panics); the library itself never
falls back to a CPU path: without a HIP device every proving/verifying call
fails with "no HIP device available".
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# BPG_LIB_PATH: an in-tree variant build for A/B runs (scripts/ab.sh)
LIB_PATH = os.environ.get("BPG_LIB_PATH") or os.path.join(HERE, "libbpg.so")
MAX_PROOF = 417 + 64 * 31

# every symbol include/bpg.h declares
EXPORTS = [
    "c_prove", "c_verify", "free_proof", "bpg_last_error", "bpg_last_num_constraints", "bpg_set_seed",
    "bpg_clear_seed", "bpg_set_device", "bpg_ctx_create", "bpg_ctx_destroy", "bpg_gens_ensure",
    "bpg_pedersen_commit", "bpg_r1cs_prove", "bpg_r1cs_verify", "bpg_prepare", "bpg_prepared_free",
    "bpg_prove_batch", "bpg_last_timings", "bpg_msm", "bpg_synthesize", "bpg_synthesize_verifier",
    "bpg_synth_view", "bpg_synth_commitments", "bpg_synth_V", "bpg_synth_free", "bpg_mimc_hash",
    "bpg_mimc_sponge", "bpg_profile_enable", "bpg_kernel_stats", "bpg_kernel_stats_reset", "bpg_rng_selftest",
    "bpg_rng_rate", "bpg_r1cs_verify_shard", "bpg_point_sum", "bpg_kernel_femul",
    "bpg_verify_batch", "bpg_prepare_verifier", "bpg_gens_cache_dir", "bpg_ctx_set_fold_tables",
    "bpg_ctx_set_fold_pairs", "bpg_ctx_set_ipp_tail", "bpg_ctx_setup_stats", "bpg_r1cs_prove_sharded", "bpg_cs_create", "bpg_cs_free",
    "bpg_cs_commit", "bpg_cs_commit_point", "bpg_cs_multiply", "bpg_cs_allocate_multiplier", "bpg_cs_constrain",
    "bpg_cs_merkle_tree", "bpg_cs_range_proof", "bpg_cs_view", "bpg_cs_V", "bpg_prepare_shard",
    "bpg_prove_prepared", "bpg_verify_prepared", "bpg_ctx_trim", "bpg_prove_statements",
    "bpg_ctx_set_pipeline", "bpg_last_batch_stats", "bpg_last_statements_stats", "bpg_ctx_set_msm_tables",
    "bpg_set_statements_layout",
]

# bpg_allgather_fn (include/bpg.h)
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p)


class BpgError(RuntimeError):
    pass


class ProofArtifacts(ctypes.Structure):
    _fields_ = [("commitments", ctypes.c_char_p), ("proof", ctypes.POINTER(ctypes.c_uint8)),
                ("proof_len", ctypes.c_size_t), ("proof_cap", ctypes.c_size_t)]


class Lc(ctypes.Structure):
    _fields_ = [("nterms", ctypes.c_uint32), ("vars", ctypes.c_void_p), ("coeffs", ctypes.c_void_p)]


class R1csView(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_uint32), ("m", ctypes.c_uint32), ("q", ctypes.c_uint32), ("nnz", ctypes.c_uint32),
        ("a_L", ctypes.c_void_p), ("a_R", ctypes.c_void_p), ("a_O", ctypes.c_void_p),
        ("v", ctypes.c_void_p), ("v_blinding", ctypes.c_void_p),
        ("row_ptr", ctypes.c_void_p), ("term_var", ctypes.c_void_p), ("term_coeff", ctypes.c_void_p),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise BpgError("libbpg.so is not built (run __graft_entry__.build())")
        L = ctypes.CDLL(LIB_PATH)
        vp, sz, u32, u64, cp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p
        L.c_prove.restype = ctypes.POINTER(ProofArtifacts)
        L.c_prove.argtypes = [cp, cp, cp, cp]
        L.c_verify.restype = ctypes.c_bool
        L.c_verify.argtypes = [cp, cp, cp, cp, vp, sz]
        L.free_proof.argtypes = [ctypes.POINTER(ProofArtifacts)]
        L.bpg_last_error.restype = cp
        L.bpg_last_num_constraints.restype = u64
        L.bpg_set_seed.argtypes = [u64]
        L.bpg_set_device.argtypes = [ctypes.c_int]
        L.bpg_ctx_create.restype = vp
        L.bpg_ctx_create.argtypes = [ctypes.c_int]
        L.bpg_ctx_destroy.argtypes = [vp]
        L.bpg_gens_ensure.argtypes = [vp, u32]
        L.bpg_pedersen_commit.argtypes = [vp, vp, vp, u32, vp]
        L.bpg_r1cs_prove.argtypes = [vp, vp, sz, vp, vp, vp, sz, ctypes.POINTER(sz), vp]
        L.bpg_r1cs_verify.argtypes = [vp, vp, sz, vp, vp, vp, sz, vp]
        L.bpg_r1cs_verify_shard.argtypes = [vp, vp, sz, vp, vp, vp, sz, vp, u32, u32, vp]
        L.bpg_point_sum.argtypes = [vp, u32, vp]
        L.bpg_gens_cache_dir.argtypes = [cp]
        L.bpg_ctx_set_fold_tables.argtypes = [vp, ctypes.c_int]
        L.bpg_ctx_set_fold_pairs.argtypes = [vp, ctypes.c_int]
        L.bpg_ctx_set_ipp_tail.argtypes = [vp, ctypes.c_int]
        L.bpg_ctx_setup_stats.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.bpg_ctx_set_pipeline.argtypes = [vp, u32, u32, u32]
        L.bpg_ctx_set_msm_tables.argtypes = [vp, ctypes.c_int]
        L.bpg_last_batch_stats.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.bpg_last_statements_stats.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.bpg_set_statements_layout.argtypes = [u32, u32]
        L.bpg_r1cs_prove_sharded.argtypes = [vp, vp, sz, vp, vp, u32, u32, ALLGATHER_FN, vp, vp, sz,
                                             ctypes.POINTER(sz), vp]
        L.bpg_prepare.restype = vp
        L.bpg_prepare.argtypes = [vp, vp]
        L.bpg_prepared_free.argtypes = [vp]
        L.bpg_prepare_verifier.restype = vp
        L.bpg_prepare_verifier.argtypes = [vp, vp]
        L.bpg_prove_batch.argtypes = [vp, vp, sz, vp, u32, u32, vp, sz, ctypes.POINTER(sz)]
        L.bpg_verify_batch.argtypes = [vp, vp, sz, vp, vp, sz, ctypes.POINTER(sz), u32, u32, vp,
                                       ctypes.POINTER(ctypes.c_int)]
        L.bpg_last_timings.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.bpg_msm.argtypes = [vp, vp, vp, u32, vp]
        L.bpg_synthesize.restype = vp
        L.bpg_synthesize.argtypes = [cp, cp, cp]
        L.bpg_synthesize_verifier.restype = vp
        L.bpg_synthesize_verifier.argtypes = [cp, cp, cp]
        L.bpg_synth_view.restype = ctypes.POINTER(R1csView)
        L.bpg_synth_view.argtypes = [vp]
        L.bpg_synth_commitments.restype = cp
        L.bpg_synth_commitments.argtypes = [vp]
        L.bpg_synth_V.restype = vp
        L.bpg_synth_V.argtypes = [vp]
        L.bpg_synth_free.argtypes = [vp]
        L.bpg_prepare_shard.restype = vp
        L.bpg_prepare_shard.argtypes = [vp, vp, u32, u32]
        L.bpg_prove_prepared.argtypes = [vp, vp, sz, vp, ALLGATHER_FN, vp, vp, sz, ctypes.POINTER(sz)]
        L.bpg_verify_prepared.argtypes = [vp, vp, sz, vp, vp, sz, vp, u32, u32, vp]
        L.bpg_prove_statements.argtypes = [cp, vp, vp, vp, vp, u32, u32, vp]
        L.bpg_ctx_trim.restype = ctypes.c_int64
        L.bpg_ctx_trim.argtypes = [vp]
        L.bpg_cs_create.restype = vp
        L.bpg_cs_create.argtypes = [ctypes.c_int]
        L.bpg_cs_free.argtypes = [vp]
        L.bpg_cs_commit.restype = ctypes.c_int64
        L.bpg_cs_commit.argtypes = [vp, vp, vp]
        L.bpg_cs_commit_point.restype = ctypes.c_int64
        L.bpg_cs_commit_point.argtypes = [vp, vp]
        pl = ctypes.POINTER(Lc)
        L.bpg_cs_multiply.argtypes = [vp, pl, pl, ctypes.POINTER(u32)]
        L.bpg_cs_allocate_multiplier.argtypes = [vp, vp, vp, ctypes.POINTER(u32)]
        L.bpg_cs_constrain.argtypes = [vp, pl]
        L.bpg_cs_merkle_tree.argtypes = [vp, pl, pl, u32, pl, u32, cp]
        L.bpg_cs_range_proof.argtypes = [vp, pl, u32, vp]
        L.bpg_cs_view.restype = ctypes.POINTER(R1csView)
        L.bpg_cs_view.argtypes = [vp]
        L.bpg_cs_V.restype = vp
        L.bpg_cs_V.argtypes = [vp]
        L.bpg_rng_rate.restype = ctypes.c_double
        L.bpg_rng_rate.argtypes = [u32, ctypes.c_int]
        _lib = L
    return _lib


def last_error():
    return lib().bpg_last_error().decode(errors="replace")


def set_seed(seed):
    lib().bpg_set_seed(seed)


def clear_seed():
    lib().bpg_clear_seed()


def _b(s):
    return s.encode() if isinstance(s, str) else s


def prove(name, instance, witness, gadgets):
    """prove.rs:37 -> (proof bytes, commitments text)."""
    a = lib().c_prove(_b(name), _b(instance), _b(witness), _b(gadgets))
    if not a:
        raise BpgError(last_error())
    try:
        proof = bytes(a.contents.proof[:a.contents.proof_len])
        coms = a.contents.commitments.decode()
    finally:
        lib().free_proof(a)
    return proof, coms


def set_statements_layout(consumers=0, lockstep=0):
    """bpg_set_statements_layout: device threads of later prove_statements
    calls (0: min(5, threads / 2), capped by HBM) and statements each proves
    at once (0: 4)."""
    if lib().bpg_set_statements_layout(consumers, lockstep) != 0:
        raise BpgError("statements layout out of range")


def prove_statements(name, statements, threads, seeds=None):
    """bpg_prove_statements: prove.rs:37 for many distinct statements
    ((instance, witness, gadgets) texts) at once; statement k behaves as
    set_seed(seeds[k]); prove(name, *statements[k]). Returns a list of
    (proof, coms) or None per statement."""
    n = len(statements)
    arr = lambda xs: (ctypes.c_char_p * max(n, 1))(*[_b(x) for x in xs])
    ins, wit, gad = (arr([st[i] for st in statements]) for i in range(3))
    sd = (ctypes.c_uint64 * max(n, 1))(*seeds) if seeds is not None else None
    out = (ctypes.POINTER(ProofArtifacts) * max(n, 1))()
    rc = lib().bpg_prove_statements(_b(name), ins, wit, gad, sd, n, threads, out)
    if rc < 0:
        raise BpgError(last_error())
    res = []
    for k in range(n):
        a = out[k]
        if not a:
            res.append(None)
            continue
        try:
            res.append((bytes(a.contents.proof[:a.contents.proof_len]), a.contents.commitments.decode()))
        finally:
            lib().free_proof(a)
    return res


def verify(name, instance, proof, commitments, gadgets):
    """verify.rs:36 -> bool (False also on malformed input; see last_error())."""
    return bool(lib().c_verify(_b(name), _b(instance), _b(gadgets), _b(commitments), proof, len(proof)))


def num_constraints():
    return lib().bpg_last_num_constraints()


class Synth:
    """Statement synthesis without device work (flattened system export)."""

    def __init__(self, instance, witness=None, gadgets="", commitments=None):
        if commitments is None:
            h = lib().bpg_synthesize(_b(instance), _b(witness), _b(gadgets))
        else:
            h = lib().bpg_synthesize_verifier(_b(instance), _b(commitments), _b(gadgets))
        if not h:
            raise BpgError(last_error())
        self.h = h
        self.prover = commitments is None
        v = lib().bpg_synth_view(h).contents
        self.n, self.m, self.q, self.nnz = v.n, v.m, v.q, v.nnz
        self.view = v

    def names(self):
        return [l for l in lib().bpg_synth_commitments(self.h).decode().splitlines() if l]

    def vec(self, field, count):
        p = getattr(self.view, field)
        raw = ctypes.string_at(p, 32 * count) if count else b""
        return [raw[32 * i:32 * i + 32] for i in range(count)]

    def rows(self):
        v = self.view
        rp = (ctypes.c_uint32 * (self.q + 1)).from_address(v.row_ptr)
        tv = (ctypes.c_uint32 * max(self.nnz, 1)).from_address(v.term_var)
        tc = ctypes.string_at(v.term_coeff, 32 * self.nnz) if self.nnz else b""
        out = []
        for r in range(self.q):
            out.append([(tv[k], tc[32 * k:32 * k + 32]) for k in range(rp[r], rp[r + 1])])
        return out

    def V(self):
        return ctypes.string_at(lib().bpg_synth_V(self.h), 32 * self.m) if self.m else b""

    def __del__(self):
        try:
            lib().bpg_synth_free(self.h)
        except Exception:
            pass


ONE = 0          # Variable::One() (BPG_VAR(BPG_VAR_ONE, 0))
ELL = 2**252 + 27742317777372353535851937790883648493


def _coeff(c):
    """A LinearCombination coefficient: kept as given (dalek Scalars from
    be_to_scalar may be unreduced); negative ints are taken mod l."""
    if isinstance(c, int):
        return (c % ELL if c < 0 else c).to_bytes(32, "little")
    return bytes(c)


class GadgetCS:
    """Gadget-API constraint system (bpg_cs_*): the r1cs::ConstraintSystem
    calls a Gadget (src/gadget.rs:7-60) makes, recorded like ProverBuffer /
    VerifierBuffer (src/cs_buffer.rs) and flattened for the inner ABI.
    A linear combination is a list of (variable, coefficient) pairs, the
    coefficient an int (< 2^256; negative ints mod l) or 32 LE bytes."""

    def __init__(self, prover=True):
        self.h = lib().bpg_cs_create(1 if prover else 0)
        if not self.h:
            raise BpgError(last_error())
        self.prover = prover
        self._m = 0

    @staticmethod
    def _lc(terms):
        terms = list(terms)
        vars_ = (ctypes.c_uint32 * max(len(terms), 1))(*[v for v, _ in terms])
        co = ctypes.create_string_buffer(b"".join(_coeff(c) for _, c in terms) or b"\0" * 32)
        lc = Lc(len(terms), ctypes.cast(vars_, ctypes.c_void_p), ctypes.cast(co, ctypes.c_void_p))
        lc._keep = (vars_, co)
        return lc

    def commit(self, value, blinding=None):
        """Prover::commit(v, v_blinding) / Verifier::commit(V) -> Variable."""
        if self.prover:
            # v is kept as given (Scalar::from_bits: bit 255 cleared, no reduction)
            raw = (value & ((1 << 255) - 1)).to_bytes(32, "little") if isinstance(value, int) else bytes(value)
            r = lib().bpg_cs_commit(self.h, raw, _coeff(blinding))
        else:
            r = lib().bpg_cs_commit_point(self.h, value)
        if r < 0:
            raise BpgError(last_error())
        self._m += 1
        return r

    def multiply(self, left, right):
        out = (ctypes.c_uint32 * 3)()
        if lib().bpg_cs_multiply(self.h, ctypes.byref(self._lc(left)), ctypes.byref(self._lc(right)), out) != 0:
            raise BpgError(last_error())
        return out[0], out[1], out[2]

    def allocate_multiplier(self, assignment=None):
        out = (ctypes.c_uint32 * 3)()
        l, r = (None, None) if assignment is None else (_coeff(assignment[0]), _coeff(assignment[1]))
        if lib().bpg_cs_allocate_multiplier(self.h, l, r, out) != 0:
            raise BpgError(last_error())
        return out[0], out[1], out[2]

    def constrain(self, lc):
        if lib().bpg_cs_constrain(self.h, ctypes.byref(self._lc(lc))) != 0:
            raise BpgError(last_error())

    def merkle_tree(self, root, instances, witnesses, pattern):
        """MerkleTree256::new(root, instance_vars, witness_vars, pattern)
        .assemble (merkle_tree_gadget.rs:44-56); LCs as above, pattern in the
        reference's Display form ("H(W W)")."""
        keep = [self._lc(x) for x in instances], [self._lc(x) for x in witnesses]
        ia = (Lc * max(len(keep[0]), 1))(*keep[0])
        wa = (Lc * max(len(keep[1]), 1))(*keep[1])
        if lib().bpg_cs_merkle_tree(self.h, ctypes.byref(self._lc(root)), ia, len(keep[0]), wa, len(keep[1]),
                                    _b(pattern)) != 0:
            raise BpgError(last_error())

    def range_proof(self, x, bits, assignment=None):
        """utils.rs:5 range_proof(cs, x, n, x_assignment)."""
        a = None if assignment is None else _coeff(assignment)
        if lib().bpg_cs_range_proof(self.h, ctypes.byref(self._lc(x)), bits, a) != 0:
            raise BpgError(last_error())

    @property
    def view(self):
        """The flattened system (bpg_r1cs_view; valid until the next call)."""
        return lib().bpg_cs_view(self.h).contents

    def __del__(self):
        try:
            lib().bpg_cs_free(self.h)
        except Exception:
            pass


def pattern_str(p):
    """('H', l, r) / ('W',) / ('I',) tuples -> the reference's Display form."""
    return p[0] if p[0] != "H" else "H(%s %s)" % (pattern_str(p[1]), pattern_str(p[2]))


class Context:
    """Device context (generator cache in HBM) for the inner ABI."""

    def __init__(self, device=0):
        self.h = lib().bpg_ctx_create(device)
        if not self.h:
            raise BpgError(last_error())

    def set_strategy(self, fold_tables=-1, fold_pairs=-1, ipp_tail=-1, msm_tables=-1):
        """IPP fold strategy of this context's calls (bpg_ctx_set_fold_*,
        bpg_ctx_set_ipp_tail); fold_pairs 2 folds rounds in triples;
        msm_tables: fixed-base generator tables (bpg_ctx_set_msm_tables)."""
        if lib().bpg_ctx_set_fold_tables(self.h, fold_tables) != 0 or \
                lib().bpg_ctx_set_fold_pairs(self.h, fold_pairs) != 0 or \
                lib().bpg_ctx_set_ipp_tail(self.h, ipp_tail) != 0 or \
                lib().bpg_ctx_set_msm_tables(self.h, msm_tables) != 0:
            raise BpgError("bad strategy")

    def set_pipeline(self, producers=0, lockstep=0, max_inflight=0):
        """bpg_ctx_set_pipeline: layout of prove_batch on circuits prepared
        through this context afterwards (0 = automatic)."""
        if lib().bpg_ctx_set_pipeline(self.h, producers, lockstep, max_inflight) != 0:
            raise BpgError("bad pipeline layout")

    def setup_stats(self):
        arr = (ctypes.c_double * 10)()
        lib().bpg_ctx_setup_stats(self.h, arr, 10)
        return {"gens_ms": arr[0], "comb_ms": arr[1], "gens_from_cache": bool(arr[2]), "comb_alloc_ms": arr[3],
                "comb_bytes": arr[4], "msm_table_bytes": arr[5], "workspaces_parked": int(arr[6]),
                "workspace_parks": int(arr[7]), "stages_parked": int(arr[8]), "stage_parks": int(arr[9])}

    def trim(self):
        """bpg_ctx_trim: drop cached comb tables / generator slices no proof
        holds; returns the table bytes released."""
        r = lib().bpg_ctx_trim(self.h)
        if r < 0:
            raise BpgError(last_error())
        return r

    def msm(self, scalars, points):
        out = ctypes.create_string_buffer(32)
        rc = lib().bpg_msm(self.h, b"".join(scalars), b"".join(points), len(scalars), out)
        if rc != 0:
            raise BpgError("bpg_msm failed (%d): %s" % (rc, last_error()))
        return out.raw

    def pedersen(self, v, vb):
        out = ctypes.create_string_buffer(32 * max(len(v), 1))
        if lib().bpg_pedersen_commit(self.h, b"".join(v), b"".join(vb), len(v), out) != 0:
            raise BpgError(last_error())
        return [out.raw[32 * i:32 * i + 32] for i in range(len(v))]

    # `view` may be any ctypes mirror of bpg_r1cs_view (ours or the oracle's)
    def r1cs_prove(self, label, view, entropy):
        out = ctypes.create_string_buffer(MAX_PROOF)
        plen = ctypes.c_size_t(0)
        V = ctypes.create_string_buffer(32 * max(view.m, 1))
        rc = lib().bpg_r1cs_prove(self.h, label, len(label), ctypes.addressof(view), entropy, out, MAX_PROOF,
                                  ctypes.byref(plen), V)
        if rc != 0:
            raise BpgError(last_error())
        return out.raw[:plen.value], [V.raw[32 * i:32 * i + 32] for i in range(view.m)]

    def r1cs_prove_sharded(self, label, view, entropy, rank, world, allgather):
        """One proof sharded over `world` ranks (bpg_r1cs_prove_sharded).
        allgather(payload bytes) -> list of every rank's payload, rank order."""
        fn, err = _allgather_cb(allgather, world)
        out = ctypes.create_string_buffer(MAX_PROOF)
        plen = ctypes.c_size_t(0)
        V = ctypes.create_string_buffer(32 * max(view.m, 1))
        rc = lib().bpg_r1cs_prove_sharded(self.h, label, len(label), ctypes.addressof(view), entropy, rank, world,
                                          fn, None, out, MAX_PROOF, ctypes.byref(plen), V)
        if rc != 0:
            raise BpgError(last_error() + ("" if not err else " (%r)" % err[0]))
        return out.raw[:plen.value], [V.raw[32 * i:32 * i + 32] for i in range(view.m)]

    def r1cs_verify(self, label, view, V, proof, entropy=b"\x05" * 32):
        Vb = b"".join(V) or b"\0" * 32
        rc = lib().bpg_r1cs_verify(self.h, label, len(label), ctypes.addressof(view), Vb, proof, len(proof), entropy)
        if rc < 0:
            raise BpgError(last_error())
        return rc == 1

    def r1cs_verify_shard(self, label, view, V, proof, shard, nshards, entropy=b"\x05" * 32):
        """-> (ok, partial): one shard of the verifier's mega-MSM (bpg.h)."""
        Vb = b"".join(V) or b"\0" * 32
        part = ctypes.create_string_buffer(32)
        rc = lib().bpg_r1cs_verify_shard(self.h, label, len(label), ctypes.addressof(view), Vb, proof, len(proof),
                                         entropy, shard, nshards, part)
        if rc < 0:
            raise BpgError(last_error())
        return rc == 1, part.raw

    def prepare_shard(self, view, rank, world):
        """bpg_prepare_shard: this rank's slice resident in HBM, for
        Prepared.prove_one (world == 1: the whole circuit)."""
        p = lib().bpg_prepare_shard(self.h, ctypes.addressof(view), rank, world)
        if not p:
            raise BpgError(last_error())
        return Prepared(p, world)

    def prepare(self, view, verifier=False):
        """HBM-resident circuit: for prove_batch, or with verifier=True for
        verify_batch (bpg_prepare_verifier)."""
        f = lib().bpg_prepare_verifier if verifier else lib().bpg_prepare
        p = f(self.h, ctypes.addressof(view))
        if not p:
            raise BpgError(last_error())
        return Prepared(p)

    def __del__(self):
        try:
            lib().bpg_ctx_destroy(self.h)
        except Exception:
            pass


def _allgather_cb(allgather, world):
    """bpg_allgather_fn over a Python allgather(bytes) -> [bytes per rank]."""
    err = []

    def cb(_user, send, nbytes, recv):
        try:
            parts = list(allgather(ctypes.string_at(send, nbytes)))
            if len(parts) != world or any(len(p) != nbytes for p in parts):
                raise BpgError("all-gather returned %d parts of %s bytes, want %d x %d"
                               % (len(parts), sorted({len(p) for p in parts}), world, nbytes))
            ctypes.memmove(recv, b"".join(parts), nbytes * world)
            return 0
        except Exception as e:  # the library turns a failed exchange into an error status
            err.append(e)
            return -1
    return ALLGATHER_FN(cb), err


class Prepared:
    def __init__(self, h, world=1):
        self.h = h
        self.world = world

    def prove_one(self, label, entropy, allgather=None):
        """bpg_prove_prepared: one proof on the calling thread (sharded when
        prepared with world > 1: every rank calls it, allgather exchanges)."""
        fn, err = _allgather_cb(allgather or (lambda p: [p]), self.world)
        out = ctypes.create_string_buffer(MAX_PROOF)
        plen = ctypes.c_size_t(0)
        rc = lib().bpg_prove_prepared(self.h, label, len(label), entropy, fn, None, out, MAX_PROOF, ctypes.byref(plen))
        if rc != 0:
            raise BpgError(last_error() + ("" if not err else " (%r)" % err[0]))
        return out.raw[:plen.value]

    def prove_batch(self, label, entropies, threads):
        count = len(entropies)
        stride = MAX_PROOF
        out = ctypes.create_string_buffer(stride * max(count, 1))
        lens = (ctypes.c_size_t * max(count, 1))()
        rc = lib().bpg_prove_batch(self.h, label, len(label), b"".join(entropies), count, threads, out, stride, lens)
        if rc != 0:
            raise BpgError(last_error())
        return [out.raw[stride * k:stride * k + lens[k]] for k in range(count)]

    def verify_batch(self, label, V, proofs, threads, entropy=b"\x05" * 32):
        """Verifier::verify over every proof of `proofs` (bytes each) against
        the compressed commitments V (list of 32-byte points, or their
        concatenation); list of bools."""
        if isinstance(V, (list, tuple)):
            V = b"".join(V)
        count = len(proofs)
        stride = max([len(p) for p in proofs] + [1])
        buf = b"".join(p.ljust(stride, b"\0") for p in proofs)
        lens = (ctypes.c_size_t * max(count, 1))(*[len(p) for p in proofs])
        res = (ctypes.c_int * max(count, 1))()
        rc = lib().bpg_verify_batch(self.h, label, len(label), V, buf, stride, lens, count, threads, entropy, res)
        if rc != 0:
            raise BpgError(last_error())
        return [res[k] == 1 for k in range(count)]

    def verify_one(self, label, V, proof, entropy=b"\x05" * 32, shard=0, nshards=1):
        """bpg_verify_prepared on a verifier-prepared circuit: nshards == 1
        -> bool verdict; else -> (ok, 32-byte partial) of shard `shard`."""
        if isinstance(V, (list, tuple)):
            V = b"".join(V)
        part = ctypes.create_string_buffer(32)
        rc = lib().bpg_verify_prepared(self.h, label, len(label), V or b"\0" * 32, proof, len(proof), entropy,
                                       shard, nshards, part)
        if rc < 0:
            raise BpgError(last_error())
        return rc == 1 if nshards == 1 else (rc == 1, part.raw)

    def __del__(self):
        try:
            lib().bpg_prepared_free(self.h)
        except Exception:
            pass


def point_sum(points):
    """Sum of compressed Ristretto points (host code, no device needed)."""
    buf = b"".join(points)
    out = ctypes.create_string_buffer(32)
    if lib().bpg_point_sum(buf, len(points), out) != 0:
        raise BpgError(last_error() or "invalid point encoding")
    return out.raw


def last_timings():
    arr = (ctypes.c_double * 5)()
    lib().bpg_last_timings(arr, 5)
    return {"rng_ms": arr[0], "commit_ms": arr[1], "vec_ms": arr[2], "ipp_ms": arr[3], "total_ms": arr[4]}


BATCH_STATS = ("producers", "consumers", "lockstep", "inflight", "wall_ms", "fill_ms", "consumer_starved_ms",
               "producer_slot_wait_ms", "producer_draw_ms", "consumer_prove_ms", "host_bound", "hbm_free_gb",
               "est_gb_per_consumer", "consumers_by_threads", "consumers_by_hbm", "process_cpus", "hw_queues",
               "ws_gb_max")


def last_batch_stats():
    """bpg_last_batch_stats: the last prove_batch's layout and pipeline counters."""
    arr = (ctypes.c_double * len(BATCH_STATS))()
    lib().bpg_last_batch_stats(arr, len(BATCH_STATS))
    d = dict(zip(BATCH_STATS, arr))
    d["host_bound"] = bool(d["host_bound"])
    for k in ("producers", "consumers", "lockstep", "inflight", "consumers_by_threads", "consumers_by_hbm",
              "process_cpus", "hw_queues"):
        d[k] = int(d[k])
    return d


STATEMENTS_STATS = ("workers", "consumers", "limit", "wall_ms", "synth_ms", "prepare_ms", "rng_ms", "prove_ms",
                    "worker_idle_ms", "consumer_idle_ms", "bound_stage", "hbm_limit", "est_gb_per_statement",
                    "lockstep", "hbm_free_gb", "oom_retired", "est_gb_per_device_thread", "ws_gb_max")


def last_statements_stats():
    """bpg_last_statements_stats: per-stage busy / idle time of the last
    prove_statements call and the stage that bounded it."""
    arr = (ctypes.c_double * len(STATEMENTS_STATS))()
    lib().bpg_last_statements_stats(arr, len(STATEMENTS_STATS))
    d = dict(zip(STATEMENTS_STATS, arr))
    d["bound_stage"] = {0: "none", 1: "cpu workers (synthesis + prepare + rng)", 2: "device consumers"}.get(
        int(d["bound_stage"]), "?")
    for k in ("workers", "consumers", "limit", "hbm_limit", "lockstep", "oom_retired"):
        d[k] = int(d[k])
    wall = max(d["wall_ms"], 1e-9)
    d["worker_busy_frac"] = round(1 - d["worker_idle_ms"] / (wall * max(d["workers"], 1)), 3)
    d["consumer_busy_frac"] = round(1 - d["consumer_idle_ms"] / (wall * max(d["consumers"], 1)), 3)
    return d
