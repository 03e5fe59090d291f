// Host build of the device arithmetic (csrc/device/dev_field.h) exposed over
// a C ABI so tests/test_devsim.py can check it against Python integers and
// the CPU oracle without a GPU. Test infrastructure only.
#define BPG_HOST_SIM 1
#include "../../bulletproof-gadgets_amd/csrc/device/dev_field.h"
#include <string.h>

extern "C" {
// raw limb interface (10 x u32 in, 10 x u32 out): exercises the bound rules
void sim_fe_mul_limbs(const uint32_t *a, const uint32_t *b, uint32_t *r) { fe x, y, z; memcpy(x.v, a, 40); memcpy(y.v, b, 40); fe_mul(z, x, y); memcpy(r, z.v, 40); }
void sim_fe_sq_limbs(const uint32_t *a, uint32_t *r) { fe x, z; memcpy(x.v, a, 40); fe_sq(z, x); memcpy(r, z.v, 40); }
void sim_fe_carry_limbs(const uint32_t *a, uint32_t *r) { fe x, z; memcpy(x.v, a, 40); fe_carry(z, x); memcpy(r, z.v, 40); }
void sim_fe_canon_limbs(const uint32_t *a, uint32_t *r) { fe x, z; memcpy(x.v, a, 40); fe_canon(z, x); memcpy(r, z.v, 40); }
void sim_fe_tow_limbs(const uint32_t *a, uint32_t *w) { fe x; memcpy(x.v, a, 40); fe_tow(w, x); }
// word interface (8 x u32 canonical in/out)
void sim_fe_mul(const uint32_t *a, const uint32_t *b, uint32_t *r) { fe x, y, z; fe_fromw(x, a); fe_fromw(y, b); fe_mul(z, x, y); fe_tow(r, z); }
void sim_fe_sq(const uint32_t *a, uint32_t *r) { fe x, z; fe_fromw(x, a); fe_sq(z, x); fe_tow(r, z); }
void sim_fe_add(const uint32_t *a, const uint32_t *b, uint32_t *r) { fe x, y, z; fe_fromw(x, a); fe_fromw(y, b); fe_add(z, x, y); fe_tow(r, z); }
void sim_fe_sub(const uint32_t *a, const uint32_t *b, uint32_t *r) { fe x, y, z; fe_fromw(x, a); fe_fromw(y, b); fe_sub(z, x, y); fe_tow(r, z); }
void sim_fe_invert(const uint32_t *a, uint32_t *r) { fe x, z; fe_fromw(x, a); fe_invert(z, x); fe_tow(r, z); }
void sim_sc_montmul(const uint32_t *a, const uint32_t *b, uint32_t *r) { sc x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); sc_montmul(z, x, y); memcpy(r, z.v, 32); }
void sim_sc_add(const uint32_t *a, const uint32_t *b, uint32_t *r) { sc x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); sc_add(z, x, y); memcpy(r, z.v, 32); }
void sim_sc_sub(const uint32_t *a, const uint32_t *b, uint32_t *r) { sc x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); sc_sub(z, x, y); memcpy(r, z.v, 32); }
void sim_sc_reduce(const uint32_t *a, uint32_t *r) { sc x, z; memcpy(x.v, a, 32); sc_reduce(z, x); memcpy(r, z.v, 32); }
// points: compressed in/out. op: 0 add, 1 sub, 2 add_cached, 3 sub_cached,
// 4 dbl, 5 dbl without T then add (exercises the T-less doubling),
// 9-12 identity-free run starts (Niels / cached -> extended, then + p),
// 13/14 (p +/- q without T) doubled, then + q (the folds' T-less additions)
int sim_pt_op(int op, const uint32_t *a, const uint32_t *b, uint32_t *r) {
    ge p, q, s;
    if (!ristretto_decode(p, a) || !ristretto_decode(q, b)) return -1;
    gec qc; ge_to_cached(qc, q);
    switch (op) {
        case 0: ge_add(s, p, q); break;
        case 1: ge_sub(s, p, q); break;
        case 2: ge_add_c(s, p, qc); break;
        case 3: ge_sub_c(s, p, qc); break;
        case 4: ge_dbl(s, p); break;
        case 5: { ge t; ge_dbl_t<false>(t, p); ge_dbl(t, t); ge_add_c(s, t, qc); break; }
        case 6: case 7: {   // affine Niels madd / msub, operand through the packed 96-B table form
            gen qn; ge_to_niels(qn, q);
            uint4 pk[6]; genp_store(pk, qn);
            gen qu; genp_unpack(qu, pk);
            gen_cneg(qu, op == 7);
            ge_madd(s, p, qu); break;
        }
        case 9: case 10: {  // run start of MSM pass 1 / comb fold: Niels -> extended (1M), then + p
            gen qn; ge_to_niels(qn, q); gen_cneg(qn, op == 10);
            ge t; ge_from_niels(t, qn); ge_add(s, t, p); break;
        }
        case 11: case 12: { // the same from a cached point (uses its 2dT)
            gec c2 = qc; gec_cneg(c2, op == 12);
            ge t; ge_from_cached_t(t, c2); ge_add(s, t, p); break;
        }
        case 13: { ge t; ge_add_c_t<false>(t, p, qc); ge_dbl(t, t); ge_add_c(s, t, qc); break; }   // T-less add, then dbl
        case 14: { ge t; ge_sub_c_t<false>(t, p, qc); ge_dbl(t, t); ge_add_c(s, t, qc); break; }
        default: {          // Niels -> cached (2Z = 2) path of the fold kernel
            gen qn; ge_to_niels(qn, q); gec c2; gen_to_cached(c2, qn); ge_add_c(s, p, c2); break;
        }
    }
    ristretto_encode(r, s);
    return 0;
}
int sim_from_uniform(const uint32_t *w, uint32_t *r) {
    fe r1, r2; ge p1, p2, p; fe_fromw(r1, w); fe_fromw(r2, w + 8);
    ristretto_elligator(p1, r1); ristretto_elligator(p2, r2); ge_add(p, p1, p2); ristretto_encode(r, p); return 0;
}
}
