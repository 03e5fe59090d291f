// Host build of the device arithmetic (csrc/device/dev_field.h) exposed over
// a C ABI so tests/test_devsim.py can check it against Python integers on the
// CPU. Test infrastructure only.
#define BPG_HOST_SIM 1
#include "../../bulletproof-gadgets_amd/csrc/device/dev_field.h"
#include <string.h>

extern "C" {
void sim_fe_mul(const uint32_t *a, const uint32_t *b, uint32_t *r) { fe x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); fe_mul(z, x, y); memcpy(r, z.v, 32); }
void sim_fe_sq(const uint32_t *a, uint32_t *r) { fe x, z; memcpy(x.v, a, 32); fe_sq(z, x); memcpy(r, z.v, 32); }
void sim_fe_add(const uint32_t *a, const uint32_t *b, uint32_t *r) { fe x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); fe_add(z, x, y); memcpy(r, z.v, 32); }
void sim_fe_sub(const uint32_t *a, const uint32_t *b, uint32_t *r) { fe x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); fe_sub(z, x, y); memcpy(r, z.v, 32); }
void sim_fe_canon(const uint32_t *a, uint32_t *r) { fe x, z; memcpy(x.v, a, 32); fe_canon(z, x); memcpy(r, z.v, 32); }
void sim_fe_invert(const uint32_t *a, uint32_t *r) { fe x, z; memcpy(x.v, a, 32); fe_invert(z, x); memcpy(r, z.v, 32); }
void sim_sc_montmul(const uint32_t *a, const uint32_t *b, uint32_t *r) { sc x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); sc_montmul(z, x, y); memcpy(r, z.v, 32); }
void sim_sc_add(const uint32_t *a, const uint32_t *b, uint32_t *r) { sc x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); sc_add(z, x, y); memcpy(r, z.v, 32); }
void sim_sc_sub(const uint32_t *a, const uint32_t *b, uint32_t *r) { sc x, y, z; memcpy(x.v, a, 32); memcpy(y.v, b, 32); sc_sub(z, x, y); memcpy(r, z.v, 32); }
void sim_sc_reduce(const uint32_t *a, uint32_t *r) { sc x, z; memcpy(x.v, a, 32); sc_reduce(z, x); memcpy(r, z.v, 32); }
// points: compressed in/out
int sim_pt_add(const uint32_t *a, const uint32_t *b, uint32_t *r) {
    ge p, q, s; if (!ristretto_decode(p, a) || !ristretto_decode(q, b)) return -1;
    ge_add(s, p, q); ristretto_encode(r, s); return 0;
}
int sim_pt_dbl(const uint32_t *a, uint32_t *r) { ge p, s; if (!ristretto_decode(p, a)) return -1; ge_dbl(s, p); ristretto_encode(r, s); return 0; }
int sim_from_uniform(const uint32_t *w, uint32_t *r) {
    fe r1, r2; ge p1, p2, p; fe_fromw(r1, w); fe_fromw(r2, w + 8);
    ristretto_elligator(p1, r1); ristretto_elligator(p2, r2); ge_add(p, p1, p2); ristretto_encode(r, p); return 0;
}
}
