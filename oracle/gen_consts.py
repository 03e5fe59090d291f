"""Derive the curve25519 / Ristretto255 field constants used by the oracle and the
device library from their definitions (RFC 9496 section 4.1; curve25519-dalek 3.2.0
`constants.rs` names), and print them as C initialisers.

Test/infra tooling: run by hand; its output is pasted into oracle/bpg_oracle.c
(5 x 51-bit limbs) and the device field header (8 x 32-bit limbs).
"""
p = 2**255 - 19


def inv(a):
    return pow(a, p - 2, p)


def sqrt(a):
    r = pow(a, (p + 3) // 8, p)
    if r * r % p != a % p:
        r = r * SQRT_M1 % p
    assert r * r % p == a % p
    return r


D = (-121665 * inv(121666)) % p
SQRT_M1 = pow(2, (p - 1) // 4, p)
# The root choice is a convention: RFC 9496 section 4.1 (= dalek constants.rs)
# fixes these representatives; check they satisfy their definitions.
SQRT_AD_MINUS_ONE = 25063068953384623474111414158702152701244531502492656460079210482610430750235
INVSQRT_A_MINUS_D = 54469307008909316920995813868745141605393597292927456921205312896311721017578
assert SQRT_AD_MINUS_ONE ** 2 % p == (-D - 1) % p
assert INVSQRT_A_MINUS_D ** 2 * ((-1 - D) % p) % p == 1
CONSTS = {
    "EDWARDS_D": D,
    "EDWARDS_D2": 2 * D % p,
    "SQRT_M1": SQRT_M1,
    "SQRT_AD_MINUS_ONE": SQRT_AD_MINUS_ONE,
    "INVSQRT_A_MINUS_D": INVSQRT_A_MINUS_D,
    "ONE_MINUS_D_SQ": (1 - D * D) % p,
    "D_MINUS_ONE_SQ": (D - 1) ** 2 % p,
}


def limbs(x, bits, n):
    return [(x >> (bits * i)) & ((1 << bits) - 1) for i in range(n)]


if __name__ == "__main__":
    for k, v in CONSTS.items():
        l51 = ", ".join("0x%013xULL" % t for t in limbs(v, 51, 5))
        l32 = ", ".join("0x%08xu" % t for t in limbs(v, 32, 8))
        print("/* %s */ {%s}" % (k, l51))
        print("/* %s */ {%s}" % (k, l32))
