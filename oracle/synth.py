"""Pure-Python restatement of the reference's statement layer: the mini-language
(.inst/.wtns/.gadgets/.coms), the gadgets, the OR transform and the recording
constraint system, ending in a flattened R1CS (oracle.FlatCS) that the C
oracle proves/verifies.

TEST INFRASTRUCTURE ONLY (tests/, bench.py cpu_baseline). Mirrors:
  src/prove.rs, src/verify.rs          statement drivers
  src/lalrpop/*                        grammar + Assignments naming
  src/cs_buffer.rs, src/or/            recording CS + OR cartesian product
  src/{bounds_check,mimc_hash,merkle_tree,set_membership,less_than,
       inequality,equality}/, src/utils.rs, src/conversions.rs
  bulletproofs@2.1.0 r1cs::{Prover,Verifier}::{multiply, allocate_multiplier,
       constrain, commit}; LinearCombination ops (term concatenation).
Scalars are Python ints holding the raw 256-bit value (from_bits values may be
>= l); every arithmetic result is reduced mod l, as curve25519-dalek 3.2.0's
Scalar Add/Sub/Mul/Neg do; equality/ordering use raw bytes.
"""
import re

try:
    from . import oracle as O
except ImportError:  # loaded as a top-level module
    import oracle as O

L = 2**252 + 27742317777372353535851937790883648493
ONE, VL, VR, VO, VV = 0, 1, 2, 3, 4


def var(kind, idx):
    return (kind << 28) | idx


V_ONE = var(ONE, 0)


def b32(x):
    return x.to_bytes(32, "little")


def from_bits(b):
    """Scalar::from_bits: clear bit 255, no reduction."""
    return int.from_bytes(b, "little") & ((1 << 255) - 1)


def le_to_scalars(data):
    data = bytes(data)
    if len(data) % 32:
        data += b"\0" * (32 - len(data) % 32)
    return [from_bits(data[i:i + 32]) for i in range(0, len(data), 32)]


def be_to_scalars(data):
    return le_to_scalars(bytes(data)[::-1])


def le_to_scalar(data):
    assert len(data) <= 32
    return from_bits(bytes(data) + b"\0" * (32 - len(data)))


def be_to_scalar(data):
    return le_to_scalar(bytes(data)[::-1])


def scalar_to_be(s):
    return b32(s)[::-1]


def inv(x):
    return pow(x % L, L - 2, L)


# --------------------------------------------------------------------------
# Linear combinations: lists of (var_code, raw_scalar); ops concatenate terms
# --------------------------------------------------------------------------
def lc_const(s):
    return [(V_ONE, s)]


def lc_var(v):
    return [(v, 1)]


def lc_add(a, b):
    return a + b


def lc_sub(a, b):
    return a + [(v, (-c) % L) for v, c in b]


def lc_scale(a, s):
    return [(v, c * s % L) for v, c in a]


# --------------------------------------------------------------------------
# MiMC (src/mimc_hash/mimc.rs) with constants from tests/golden
# --------------------------------------------------------------------------
_MIMC = None


def mimc_constants():
    global _MIMC
    if _MIMC is None:
        import os
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden",
                            "mimc_round_constants.hex")
        with open(path) as f:
            _MIMC = [from_bits(bytes.fromhex(l.strip())) for l in f if l.strip()]
        assert len(_MIMC) == 486
    return _MIMC


def pkcs7(data, block):
    k = block - (len(data) % block)
    return bytes(data) + bytes([k]) * k


def strip_trailing_zeros(b):
    b = bytes(b)
    while b and b[-1] == 0:
        b = b[:-1]
    return b


def mimc_pad(blocks):
    last_le = strip_trailing_zeros(b32(blocks[-1]))
    if len(last_le) < 32:
        blocks = blocks[:-1] + [le_to_scalar(pkcs7(last_le, 32))]
    else:
        blocks = blocks + [le_to_scalar(bytes([32]) * 32)]
    return blocks


def mimc_hash(preimage):
    """mimc.rs:61-75 (sponge_1, 486 rounds, key 0)."""
    cs = mimc_constants()
    state = 0
    for blk in mimc_pad(be_to_scalars(preimage)):
        state = (state + blk) % L
        for c in cs:
            t = (state + c) % L
            state = t * t % L * t % L
        state = state % L
    return state


# --------------------------------------------------------------------------
# Recording constraint systems (bulletproofs r1cs Prover / Verifier)
# --------------------------------------------------------------------------
class Cs:
    """Single-pass recorder equivalent to ProverBuffer/VerifierBuffer + the
    final replay into the main Prover/Verifier (prove.rs:72, cs_buffer.rs).
    Operations are recorded into `self.ops` (a stack of op lists for OR
    blocks); values are evaluated eagerly (prover side)."""

    def __init__(self, prover):
        self.prover = prover
        self.aL, self.aR, self.aO = [], [], []
        self.nvars = 0
        self.v, self.vb, self.V = [], [], []
        self.ops = [[]]

    # -- Prover::commit / Verifier::commit
    def commit(self, value=None, blinding=None, V=None):
        i = len(self.v) if self.prover else len(self.V)
        if self.prover:
            self.v.append(value)
            self.vb.append(blinding)
        else:
            self.V.append(V)
        return var(VV, i)

    def eval(self, lc):
        tot = 0
        for v, c in lc:
            k, i = v >> 28, v & 0x0FFFFFFF
            val = 1 if k == ONE else [None, self.aL, self.aR, self.aO, self.v][k][i]
            tot += c * val
        return tot % L

    def _alloc(self, l=None, r=None):
        i = self.nvars
        self.nvars += 1
        if self.prover:
            self.aL.append(l % L if l is not None else 0)
            self.aR.append(r % L if r is not None else 0)
            self.aO.append(l * r % L)
        return var(VL, i), var(VR, i), var(VO, i)

    def multiply(self, left, right):
        l = r = None
        if self.prover:
            l, r = self.eval(left), self.eval(right)
        lv, rv, ov = self._alloc(l, r)
        self.ops[-1].append(("mul", list(left), list(right), lv, rv))
        return lv, rv, ov

    def allocate_multiplier(self, assignment):
        if self.prover:
            l, r = assignment
            return self._alloc(l, r)
        return self._alloc()

    def constrain(self, lc):
        self.ops[-1].append(("con", list(lc)))

    def flat_rows(self):
        rows = []
        for op in self.ops[0]:
            if op[0] == "mul":
                _, left, right, lv, rv = op
                rows.append(left + [(lv, L - 1)])
                rows.append(right + [(rv, L - 1)])
            else:
                rows.append(op[1])
        return rows

    def to_flat(self):
        rows = [[(v, b32(c % (1 << 256))) for v, c in r] for r in self.flat_rows()]
        n = self.nvars
        if self.prover:
            return O.FlatCS(n, len(self.v), [b32(x) for x in self.aL], [b32(x) for x in self.aR],
                            [b32(x) for x in self.aO], [b32(x) for x in self.v], [b32(x) for x in self.vb], rows)
        return O.FlatCS(n, len(self.V), [], [], [], [], [], rows)


def or_block(main, cache):
    """src/or/or_conjunction.rs:4-38 — replay branch multiplies, multiply out
    the cartesian product of branch constraints."""
    constraint_lists = []
    for ops in cache:
        cons = []
        for op in ops:
            if op[0] == "mul":
                main.ops[-1].append(op)
            else:
                cons.append(op[1])
        constraint_lists.append(cons)
    combos = []
    if constraint_lists:
        combos = [[c] for c in constraint_lists[0]]
        for lst in constraint_lists[1:]:
            combos = [xs + [y] for xs in combos for y in lst]
    for cons in combos:
        prod = cons[0]
        for c in cons[1:]:
            _, _, o = main.multiply(prod, c)
            prod = lc_var(o)
        main.constrain(prod)


# --------------------------------------------------------------------------
# Gadgets
# --------------------------------------------------------------------------
def range_proof(cs, x, n, x_assignment):
    """src/utils.rs:5-35"""
    exp2 = 1
    xb = b32(x_assignment) if x_assignment is not None else None
    x = list(x)
    for i in range(n):
        if xb is not None:
            bit = (xb[i // 8] >> (i % 8)) & 1
            a, b, o = cs.allocate_multiplier(((1 - bit), bit))
        else:
            a, b, o = cs.allocate_multiplier(None)
        cs.constrain(lc_var(o))
        cs.constrain(lc_add(lc_var(a), lc_sub(lc_var(b), lc_const(1))))
        x = lc_sub(x, lc_scale(lc_var(b), exp2))
        exp2 = (exp2 + exp2) % L
    cs.constrain(x)


def setup(cs, derived, rng):
    """gadget.rs:23-42: commit each derived scalar with a fresh blinding."""
    out = []
    for s in derived:
        vb = rng.scalar()
        out.append((s, cs.commit(s, vb)))
    return out


class BoundsCheck:
    def __init__(self, mn, mx):
        self.n = (len(mx) * 8) % 256
        self.min, self.max = be_to_scalar(mn), be_to_scalar(mx)

    def preprocess(self, w):
        return [(w[0] - self.min) % L, (self.max - w[0]) % L]

    def assemble(self, cs, _w, d):
        (aa, a), (ba, b) = d[0], d[1]
        cs.constrain(lc_sub(lc_add(lc_var(a), lc_var(b)), lc_const((self.max - self.min) % L)))
        range_proof(cs, lc_var(a), self.n, aa)
        range_proof(cs, lc_var(b), self.n, ba)


class MimcHash:
    def __init__(self, image):
        self.image = image

    def preprocess(self, w):
        last = w[-1]
        le = strip_trailing_zeros(b32(last))
        if len(le) < 32:
            padded = le_to_scalar(pkcs7(le, 32))
            return [padded, (padded - last) % L]
        return [le_to_scalar(bytes([32]) * 32)]

    def assemble(self, cs, w, d):
        coms = list(w)
        padded = d[0][1]
        if len(d) == 2:
            padding = d[1][1]
            last = lc_var(coms.pop())
            cs.constrain(lc_sub(lc_add(last, lc_var(padding)), lc_var(padded)))
        coms.append(padded)
        h = mimc_sponge(cs, [lc_var(v) for v in coms])
        cs.constrain(lc_sub(h, self.image))


def mimc_sponge(cs, pre):
    """mimc_hash_gadget.rs:108-150"""
    key = lc_const(0)
    state = lc_const(0)
    consts = mimc_constants()
    for v in pre:
        state = lc_add(state, v)
        p = state
        for c in consts:
            pk = lc_add(lc_add(p, key), lc_const(c))
            x, _, sqr = cs.multiply(pk, pk)
            _, _, cube = cs.multiply(lc_var(sqr), lc_var(x))
            p = lc_var(cube)
        state = lc_add(p, key)
    return state


class Merkle:
    """merkle_tree_gadget.rs:44-115. Patterns: ('W',) ('I',) ('H', l, r)."""

    def __init__(self, root, inst, wit, pattern):
        self.root, self.inst, self.wit, self.pattern = root, list(inst), list(wit), pattern

    def assemble(self, cs, _w, _d):
        w, i = list(self.wit), list(self.inst)
        h = self.parse(cs, w, i, self.pattern)
        cs.constrain(lc_sub(h, self.root))

    def parse(self, cs, w, i, p):
        def take(vals):
            assert vals, "too few variables provided to satisfy the given pattern"
            return vals.pop(0)
        if p[0] == "W":
            pre = [take(w)]
        elif p[0] == "I":
            pre = [take(i)]
        else:
            l, r = p[1], p[2]
            left = self.parse(cs, w, i, l) if l[0] == "H" else take(w if l[0] == "W" else i)
            right = self.parse(cs, w, i, r) if r[0] == "H" else take(w if r[0] == "W" else i)
            pre = [left, right]
        return mimc_sponge(cs, pre)


class SetMembership:
    def __init__(self, value, value_a, inst, inst_a):
        self.value, self.value_a, self.inst, self.inst_a = value, value_a, inst, inst_a

    def preprocess(self, w):
        return [1 if b32(e) == b32(self.value_a) else 0 for e in list(w) + list(self.inst_a)]

    def assemble(self, cs, w, d):
        bits = []
        for _, bit in d:
            bl = lc_var(bit)
            _, _, z = cs.multiply(lc_sub(lc_const(1), bl), bl)
            cs.constrain(lc_var(z))
            bits.append(bl)
        s = lc_const(0)
        for b in bits:
            s = lc_add(s, b)
        cs.constrain(lc_sub(lc_const(1), s))
        st = [lc_var(x) for x in w] + list(self.inst)
        if len(bits) != len(st):
            cs.constrain(lc_const(1))
            return
        act = lc_const(0)
        for a, b in zip(bits, st):
            _, _, pr = cs.multiply(a, b)
            act = lc_add(act, lc_var(pr))
        cs.constrain(lc_sub(self.value, act))


class LessThan:
    def __init__(self, left, la, right, ra):
        self.left, self.la, self.right, self.ra = left, la, right, ra

    def preprocess(self, _w):
        delta = (self.ra - self.la) % L
        return [delta, 0 if delta == 0 else inv(delta)]

    def assemble(self, cs, _w, d):
        (da, dv), (_, dinv) = d[0], d[1]
        range_proof(cs, self.left, 126, self.la)
        range_proof(cs, self.right, 126, self.ra)
        range_proof(cs, lc_var(dv), 126, da)
        _, _, one = cs.multiply(lc_var(dv), lc_var(dinv))
        cs.constrain(lc_sub(lc_const(1), lc_var(one)))
        cs.constrain(lc_sub(lc_sub(self.right, self.left), lc_var(dv)))


def compare_bytes(a, b):
    """inequality_gadget.rs:103-113: byte-wise from the top, >= is true."""
    x, y = b32(a), b32(b)
    for i in range(31, -1, -1):
        if x[i] > y[i]:
            return True
        if x[i] < y[i]:
            return False
    return True


class Inequality:
    def __init__(self, right, ra):
        self.right, self.ra = right, ra

    def preprocess(self, left):
        out, tot = [], 0
        for i, lft in enumerate(left):
            r = self.ra[i] if i < len(self.ra) else 0
            delta = (lft - r) % L if compare_bytes(lft, r) else (r - lft) % L
            out.append(delta)
            if delta == 0:
                out.append(0)
            else:
                di = inv(delta)
                out.append(di)
                tot = (tot + delta * di) % L
        out.append(inv(tot) if tot else 0)
        return out

    def assemble(self, cs, left, d):
        if len(self.right) != len(left):
            cs.constrain(lc_const(0))
            return
        s = lc_const(0)
        for i in range(len(left)):
            r, l_ = self.right[i], lc_var(left[i])
            delta, dinv = d[2 * i][1], d[2 * i + 1][1]
            lmr, rml = lc_sub(l_, r), lc_sub(r, l_)
            _, _, z = cs.multiply(lc_sub(lmr, lc_var(delta)), lc_sub(rml, lc_var(delta)))
            cs.constrain(lc_var(z))
            _, _, zo = cs.multiply(lc_var(delta), lc_var(dinv))
            s = lc_add(s, lc_var(zo))
        _, _, one = cs.multiply(s, lc_var(d[-1][1]))
        cs.constrain(lc_sub(lc_const(1), lc_var(one)))


class Equality:
    def __init__(self, right):
        self.right = right

    def assemble(self, cs, left, _d):
        if len(self.right) != len(left):
            cs.constrain(lc_const(1))
            return
        for r, l_ in zip(self.right, left):
            cs.constrain(lc_sub(r, lc_var(l_)))


# --------------------------------------------------------------------------
# Mini-language (src/lalrpop/*.lalrpop)
# --------------------------------------------------------------------------
_VAR_RE = re.compile(r"^\s*([CD]\d+-\d+(?:-\d+)?|I\d+|W\d+)\s*=\s*0[xX]([0-9a-fA-F]*)\s*$")


def parse_var_line(line):
    m = _VAR_RE.match(line)
    if not m:
        raise ValueError("unable to parse line: %r" % line)
    h = m.group(2)
    if len(h) % 2:
        raise ValueError("odd-length hex in %r" % line)
    return m.group(1), bytes.fromhex(h)


def tokens(line):
    return re.findall(r"\(|\)|[A-Z_]+\d*|\[|\]|\{|\}", line)


def parse_tree(toks, pos):
    """Tree rule of gadget_grammar.lalrpop:46-72 -> (inst, wit, pattern, pos)."""
    assert toks[pos] == "("
    pos += 1
    items = []
    for _ in range(2):
        t = toks[pos]
        if t == "(":
            i, w, p, pos = parse_tree(toks, pos)
            items.append((i, w, p))
        elif t[0] == "W":
            items.append(([], [t], ("W",)))
            pos += 1
        elif t[0] == "I":
            items.append(([t], [], ("I",)))
            pos += 1
        else:
            raise ValueError("bad tree token %r" % t)
    assert toks[pos] == ")"
    (i1, w1, p1), (i2, w2, p2) = items
    return i1 + i2, w1 + w2, ("H", p1, p2), pos + 1


class Rng:
    """Deterministic stand-in for thread_rng(): ChaCha20 stream (oracle)."""

    def __init__(self, seed):
        self.seed, self.off = seed, 0

    def bytes(self, n):
        b = O.seed_stream(self.seed, self.off, n)
        self.off += n
        return b

    def scalar(self):
        return int.from_bytes(self.bytes(64), "little") % L


class Statement:
    """prove.rs / verify.rs drivers over the single-pass recorder."""

    def __init__(self, prover, instance, gadgets, seed=0, witness="", coms=""):
        self.prover = prover
        self.cs = Cs(prover)
        self.rng = Rng(seed)
        self.inst = {}
        for line in instance.splitlines():
            k, v = parse_var_line(line)
            self.inst[k] = v
        self.wit = {}
        self.commits = {}       # name -> Variable
        self.com_order = []     # (name, commit index) in commit order
        if prover:
            for line in witness.splitlines():
                name, data = parse_var_line(line)
                scalars = be_to_scalars(data)
                vars_ = []
                for k, s in enumerate(scalars):
                    vb = self.rng.scalar()
                    v = self.cs.commit(s, vb)
                    vars_.append(v)
                    self.com_order.append("C%s-%d" % (name[1:], k))
                self.wit[name] = (scalars, vars_, data)
        else:
            for line in coms.splitlines():
                name, data = parse_var_line(line)
                self.commits[name] = self.cs.commit(V=data)
        lines = gadgets.splitlines()
        self.lines = list(enumerate(lines))
        self.pos = 0
        while self.pos < len(self.lines):
            idx, line = self.lines[self.pos]
            self.pos += 1
            self.conjunction(line)
            self.gadget(line, idx)

    # -- variable access (assignment_parser.rs)
    def instance(self, name, assert32=False):
        v = self.inst[name]
        if assert32:
            assert len(v) <= 32, "instance var %s is longer than 32 bytes" % name
        return v

    def witness(self, name, assert32=False):
        w = self.wit[name]
        if assert32:
            assert len(w[0]) == 1, "witness var %s is longer than 32 bytes" % name
        return w

    def com(self, name, k=0):
        return self.commits["C%s-%d" % (name[1:], k)]

    def all_coms(self, name):
        out, k = [], 0
        while "C%s-%d" % (name[1:], k) in self.commits:
            out.append(self.commits["C%s-%d" % (name[1:], k)])
            k += 1
        return out

    def derived(self, gadget, index, sub):
        return self.commits["D%d-%d-%d" % (gadget, sub, index)]

    def inquire_derived(self, gadget, index, sub):
        return self.commits.get("D%d-%d-%d" % (gadget, sub, index))

    def name_derived(self, n, gadget, sub):
        for k in range(n):
            self.com_order.append("D%d-%d-%d" % (gadget, sub, k))

    def setup(self, derived_scalars):
        return setup(self.cs, derived_scalars, self.rng)

    # -- drivers
    def conjunction(self, line):
        if line.split()[:1] == ["OR"]:
            self.or_conjunction()

    def or_conjunction(self):
        if self.pos >= len(self.lines):
            raise ValueError("unexpected end of input")
        self.cs.ops.append([])
        cache = []
        while self.pos < len(self.lines):
            idx, line = self.lines[self.pos]
            self.pos += 1
            op = (line.split() or [""])[0]
            if op == "]":
                break
            if op == "}":
                cache.append(self.cs.ops[-1])
                self.cs.ops[-1] = []
            else:
                self.conjunction(line)
                self.gadget(line, idx)
        self.cs.ops.pop()
        or_block(self.cs, cache)

    def gadget(self, line, index):
        toks = tokens(line)
        op = (line.split() or [""])[0]
        known = {"OR", "HASH", "]", "BOUND", "[", "MERKLE", "}", "EQUALS", "{", "UNEQUAL", "LESS_THAN", "SET_MEMBER"}
        if op not in known:
            raise ValueError("unknown gadget: %s" % op)
        if op == "BOUND":
            self.g_bound(toks, index)
        elif op == "HASH":
            self.g_hash(toks, index)
        elif op == "MERKLE":
            self.g_merkle(toks, index)
        elif op == "EQUALS":
            self.g_equals(toks)
        elif op == "LESS_THAN":
            self.g_less_than(toks, index)
        elif op == "UNEQUAL":
            self.g_unequal(toks, index)
        elif op == "SET_MEMBER":
            self.g_set_member(toks, index)

    def g_bound(self, t, index):
        v, mn, mx = t[1], t[2], t[3]
        assert v[0] == "W" and mn[0] == "I" and mx[0] == "I"
        g = BoundsCheck(self.instance(mn, True), self.instance(mx, True))
        if self.prover:
            s, vars_, _ = self.witness(v, True)
            d = self.setup(g.preprocess(s))
            g.assemble(self.cs, vars_, d)
            self.name_derived(len(d), index, 0)
        else:
            d = [(None, self.derived(index, 0, 0)), (None, self.derived(index, 1, 0))]
            g.assemble(self.cs, [self.com(v)], d)

    def _image_lc(self, name):
        if name[0] == "W":
            if self.prover:
                return lc_var(self.witness(name, True)[1][0])
            return lc_var(self.com(name))
        return lc_const(be_to_scalar(self.instance(name, True)))

    def g_hash(self, t, index):
        image, pre = t[1], t[2]
        assert pre[0] == "W"
        g = MimcHash(self._image_lc(image))
        if self.prover:
            s, vars_, _ = self.witness(pre)
            d = self.setup(g.preprocess(s))
            g.assemble(self.cs, vars_, d)
            self.name_derived(len(d), index, 0)
        else:
            d1 = self.derived(index, 0, 0)
            d2 = self.inquire_derived(index, 1, 0)
            d = [(None, d1)] + ([(None, d2)] if d2 is not None else [])
            g.assemble(self.cs, self.all_coms(pre), d)

    def hash_witness(self, name, index, sub):
        """prove.rs:142-172 / verify.rs:397-415"""
        if self.prover:
            s, vars_, data = self.witness(name)
            image = mimc_hash(data)
            iv = self.cs.commit(image, self.rng.scalar())
            g = MimcHash(lc_var(iv))
            d = self.setup(g.preprocess(s))
            g.assemble(self.cs, vars_, d)
            self.name_derived(1 + len(d), index, sub)
            return image, iv
        pre = self.all_coms(name)
        iv = self.derived(index, 0, sub)
        d1 = self.derived(index, 1, sub)
        d2 = self.inquire_derived(index, 2, sub)
        d = [(None, d1)] + ([(None, d2)] if d2 is not None else [])
        MimcHash(lc_var(iv)).assemble(self.cs, pre, d)
        return None, iv

    def g_merkle(self, t, index):
        root = t[1]
        inst, wit, pattern, _ = parse_tree(t, 2)
        root_lc = self._image_lc(root)
        inst_lcs = [lc_const(mimc_hash(self.instance(i))) for i in inst]
        wl = []
        for k, w in enumerate(wit):
            _, iv = self.hash_witness(w, index, k)
            wl.append(lc_var(iv))
        Merkle(root_lc, inst_lcs, wl, pattern).assemble(self.cs, [], [])

    def _var_lcs(self, name):
        """(scalars, lcs) for a witness or instance variable."""
        if name[0] == "W":
            if self.prover:
                s, vars_, _ = self.witness(name)
                return s, [lc_var(v) for v in vars_]
            return None, [lc_var(v) for v in self.all_coms(name)]
        s = be_to_scalars(self.instance(name))
        return s, [lc_const(x) for x in s]

    def g_equals(self, t):
        a, b = t[1], t[2]
        if a[0] == "I":
            a, b = b, a
        left = self.witness(a)[1] if self.prover else self.all_coms(a)
        Equality(self._var_lcs(b)[1]).assemble(self.cs, left, [])

    def g_less_than(self, t, index):
        a, b = t[1], t[2]
        if self.prover:
            ls, lv, _ = self.witness(a, True)
            rs, rv, _ = self.witness(b, True)
            g = LessThan(lc_var(lv[0]), ls[0], lc_var(rv[0]), rs[0])
            d = self.setup(g.preprocess([]))
            g.assemble(self.cs, [], d)
            self.name_derived(len(d), index, 0)
        else:
            g = LessThan(lc_var(self.com(a)), None, lc_var(self.com(b)), None)
            g.assemble(self.cs, [], [(None, self.derived(index, 0, 0)), (None, self.derived(index, 1, 0))])

    def g_unequal(self, t, index):
        a, b = t[1], t[2]
        if a[0] == "I":
            a, b = b, a
        rs, rl = self._var_lcs(b)
        if self.prover:
            ls, lv, _ = self.witness(a)
            g = Inequality(rl, rs)
            d = self.setup(g.preprocess(ls))
            g.assemble(self.cs, lv, d)
            self.name_derived(len(d), index, 0)
        else:
            left = self.all_coms(a)
            d = [(None, self.derived(index, k, 0)) for k in range(2 * len(left) + 1)]
            Inequality(rl, None).assemble(self.cs, left, d)

    def g_set_member(self, t, index):
        member, st = t[1], t[2:]
        ms, ml = self._var_lcs(member)
        if self.prover:
            mscal, mlc = ms[0], ml[0]
            hashing = len(ms) > 1
        else:
            mlc = ml[0]
            hashing = False
        wsv, wss, isl, iss = [], [], [], []
        if not hashing:
            for e in st:
                if e[0] == "W":
                    if self.prover:
                        s, v, _ = self.witness(e)
                        if len(v) == 1:
                            wss.append(s[0]); wsv.append(v[0])
                        else:
                            hashing = True
                    else:
                        c = self.all_coms(e)
                        if len(c) == 1:
                            wsv.append(c[0])
                        else:
                            hashing = True
                else:
                    s = be_to_scalars(self.instance(e))
                    if len(s) == 1:
                        iss.append(s[0]); isl.append(lc_const(s[0]))
                    else:
                        hashing = True
        if not self.prover:
            if len(ml) > 1:
                hashing = True
            d = [(None, self.derived(index, k, 0)) for k in range(len(st))]
        if hashing:
            hn = 1
            if member[0] == "W":
                img, iv = self.hash_witness(member, index, hn)
                hn += 1
                mscal, mlc = img, lc_var(iv)
            else:
                mscal = mimc_hash(self.instance(member))
                mlc = lc_const(mscal)
            wsv, wss, isl, iss = [], [], [], []
            for e in st:
                if e[0] == "W":
                    img, iv = self.hash_witness(e, index, hn)
                    hn += 1
                    wsv.append(iv); wss.append(img)
                else:
                    h = mimc_hash(self.instance(e))
                    isl.append(lc_const(h)); iss.append(h)
        if self.prover:
            g = SetMembership(mlc, mscal, isl, iss)
            d = self.setup(g.preprocess(wss))
            g.assemble(self.cs, wsv, d)
            self.name_derived(len(d), index, 0)
        else:
            SetMembership(mlc, None, isl, None).assemble(self.cs, wsv, d)


def synthesize_prover(instance, witness, gadgets, seed):
    st = Statement(True, instance, gadgets, seed=seed, witness=witness)
    return st


def entropy_for(st):
    """32 bytes of finalize entropy drawn after synthesis (program order)."""
    return st.rng.bytes(32)


def prove_statement(label, instance, witness, gadgets, seed):
    """prove.rs:37-82 under deterministic mode -> (proof, coms_text, flat)."""
    st = synthesize_prover(instance, witness, gadgets, seed)
    flat = st.cs.to_flat()
    proof, V = O.r1cs_prove(label, flat, entropy_for(st))
    coms = "".join("%s = 0x%s\n" % (name, V[i].hex()) for i, name in enumerate(st.com_order))
    return proof, coms, flat


def verify_statement(label, instance, proof, coms, gadgets, seed=1):
    """verify.rs:36-73"""
    st = Statement(False, instance, gadgets, coms=coms)
    flat = st.cs.to_flat()
    ent = Rng(seed).bytes(32)
    return O.r1cs_verify(label, flat, st.cs.V, proof, ent) == 1
