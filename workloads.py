"""Synthetic statements for the BASELINE.json configs.

Every statement is plain mini-language text (.inst/.wtns/.gadgets), generated
deterministically from a seed, with instance values (MiMC images, Merkle
roots) computed by the product's native MiMC (libbpg bpg_mimc_hash /
bpg_mimc_sponge, i.e. src/mimc_hash/mimc.rs semantics) so every statement is
satisfiable and its proofs verify.

  config 1: the reference's example.gadgets (CPU plumbing)
  config 2: 8 x BOUND, 64-bit range                  -> n = 1,024     N = 2^10
  config 3: HASH of a 2143-byte preimage             -> n = 65,124    N = 2^16
  config 4: 4 x depth-32 MERKLE paths                -> n = 252,720   N = 2^18
  config 5: 256-leaf MERKLE + SET_MEMBER(16) + BOUND -> n = 744,712   N = 2^20
"""
import ctypes
import os
import random

ROOT = os.path.dirname(os.path.abspath(__file__))


def _bpg():
    import importlib.util
    import sys
    if "bpg" in sys.modules:
        return sys.modules["bpg"]
    spec = importlib.util.spec_from_file_location("bpg", os.path.join(ROOT, "bulletproof-gadgets_amd", "bpg.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    sys.modules["bpg"] = mod
    return mod


def mimc_hash(data):
    """-> 32-byte little-endian scalar."""
    L = _bpg().lib()
    L.bpg_mimc_hash.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
    out = ctypes.create_string_buffer(32)
    if L.bpg_mimc_hash(bytes(data), len(data), out) != 0:
        raise RuntimeError("mimc_hash failed")
    return out.raw


def mimc_node(left_le, right_le):
    L = _bpg().lib()
    L.bpg_mimc_sponge.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p]
    out = ctypes.create_string_buffer(32)
    if L.bpg_mimc_sponge(left_le + right_le, 2, out) != 0:
        raise RuntimeError("mimc_sponge failed")
    return out.raw


def be_hex(le32):
    """A 32-byte LE scalar as the big-endian hex an instance line carries."""
    return le32[::-1].hex()


class Builder:
    def __init__(self, seed):
        self.rnd = random.Random(seed)
        self.inst, self.wit, self.gad = [], [], []
        self.ni = self.nw = 0

    def I(self, data):
        name = "I%d" % self.ni
        self.ni += 1
        self.inst.append("%s = 0x%s" % (name, bytes(data).hex()))
        return name

    def W(self, data):
        name = "W%d" % self.nw
        self.nw += 1
        self.wit.append("%s = 0x%s" % (name, bytes(data).hex()))
        return name

    def rbytes(self, k):
        return bytes(self.rnd.getrandbits(8) for _ in range(k))

    def text(self):
        return "\n".join(self.inst) + "\n", "\n".join(self.wit) + "\n", "\n".join(self.gad) + "\n"


def _bound(b, v_name, v):
    lo = b.I((1).to_bytes(8, "big"))
    hi = b.I(((1 << 64) - 1).to_bytes(8, "big"))
    b.gad.append("BOUND %s %s %s" % (v_name, lo, hi))


def config2(seed=1002):
    b = Builder(seed)
    for _ in range(8):
        v = b.rnd.randrange(1, (1 << 64) - 1)
        _bound(b, b.W(v.to_bytes(8, "big")), v)
    return b.text()


def config3(seed=1003):
    b = Builder(seed)
    pre = b.rbytes(2143)
    img = mimc_hash(pre)
    i0 = b.I(bytes.fromhex(be_hex(img)))
    w0 = b.W(pre)
    b.gad.append("HASH %s %s" % (i0, w0))
    return b.text()


def _path(b, depth):
    """MERKLE Ir (((W I1) I2) ... Id): witness leaf, instance siblings."""
    leaf = b.rbytes(31)
    node = mimc_hash(leaf)
    sib_names, expr = [], None
    wname = None
    pending = []
    for d in range(depth):
        sib = b.rbytes(32)
        pending.append(sib)
        node = mimc_node(node, mimc_hash(sib))
    root = b.I(bytes.fromhex(be_hex(node)))
    wname = b.W(leaf)
    expr = wname
    for sib in pending:
        expr = "(%s %s)" % (expr, b.I(sib))
    b.gad.append("MERKLE %s %s" % (root, expr))


def config4(seed=1004, paths=4, depth=32):
    b = Builder(seed)
    for _ in range(paths):
        _path(b, depth)
    return b.text()


def merkle_set_bound(seed, leaves):
    """config 5 family: a full `leaves`-leaf witness Merkle tree, a 16-element
    SET_MEMBER and a 64-bit BOUND on one committed value."""
    b = Builder(seed)
    root_name = b.I(b"\0")       # placeholder, patched below
    level, names = [], []
    for _ in range(leaves):
        leaf = b.rbytes(31)
        names.append(b.W(leaf))
        level.append(mimc_hash(leaf))
    exprs = list(names)
    while len(level) > 1:
        level = [mimc_node(level[i], level[i + 1]) for i in range(0, len(level), 2)]
        exprs = ["(%s %s)" % (exprs[i], exprs[i + 1]) for i in range(0, len(exprs), 2)]
    b.inst[0] = "%s = 0x%s" % (root_name, be_hex(level[0]))
    b.gad.append("MERKLE %s %s" % (root_name, exprs[0]))
    v = b.rnd.randrange(1, (1 << 64) - 1)
    vw = b.W(v.to_bytes(8, "big"))
    pos = b.rnd.randrange(16)
    members = [b.I((v if k == pos else b.rnd.randrange(1, 1 << 64)).to_bytes(8, "big")) for k in range(16)]
    b.gad.append("SET_MEMBER %s %s" % (vw, " ".join(members)))
    _bound(b, vw, v)
    return b.text()


def config5(seed=1005):
    return merkle_set_bound(seed, 256)


def config1():
    res = os.path.join(ROOT, "tests", "golden", "resources")
    return tuple(open(os.path.join(res, "example." + e)).read() for e in ("inst", "wtns", "gadgets"))


CONFIGS = {1: config1, 2: config2, 3: config3, 4: config4, 5: config5}
NAMES = {
    1: "example.gadgets (reference CPU plumbing case)",
    2: "8x BOUND 64-bit (~2^10)",
    3: "mimc_hash 2143-byte preimage (2^16)",
    4: "4x depth-32 merkle_tree paths over MiMC (2^18)",
    5: "merkle_tree(256 leaves)+mimc_hash+set_membership(16)+bounds_check, 2^20",
}
