// Host-code sanitizer driver: the statement
// layer (statement.cpp), the host crypto (hcrypto.cpp), the lockstep RNG
// (rng8.cpp) and the device arithmetic compiled for the host (dev_field.h)
// built with -fsanitize=address,undefined and driven over the reference's
// fixtures, malformed statements, the Gadget-API entry points and random
// field / scalar operands. Exit status 0 and no sanitizer report = pass.
// Test infrastructure only (tests/test_sanitize.py builds and runs it).
#define BPG_HOST_SIM 1
#include "../../bulletproof-gadgets_amd/csrc/device/dev_field.h"
#include "../../bulletproof-gadgets_amd/csrc/host/rng8.h"
#include "../../bulletproof-gadgets_amd/csrc/host/statement.h"

#include <stdio.h>

#include <fstream>
#include <random>
#include <sstream>

using namespace bpg;

static std::string slurp(const std::string &p) {
    std::ifstream f(p, std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    return ss.str();
}

static int fixtures(int argc, char **argv) {
    int n = 0;
    for (int i = 1; i < argc; i++) {
        const std::string b = argv[i];
        std::string inst = slurp(b + ".inst"), wtns = slurp(b + ".wtns"), gad = slurp(b + ".gadgets");
        thread_entropy().seeded = true;
        thread_entropy().cs.seed(7);
        Synthesis s = synthesize_prover(inst, wtns, gad);
        bpg_r1cs_view v = s.cs->view(true);
        // verifier side over made-up commitments of the right count
        std::string coms;
        for (size_t k = 0; k < s.com_names.size(); k++) coms += s.com_names[k] + " = 0x" + std::string(64, '0') + "\n";
        Synthesis t = synthesize_verifier(inst, coms, gad);
        bpg_r1cs_view w = t.cs->view(false);
        if (v.n != w.n || v.q != w.q || v.nnz != w.nnz) { fprintf(stderr, "%s: sides differ\n", b.c_str()); return -1; }
        n++;
        // malformed variants must throw, never crash
        const std::string bad[] = {gad + "\nBOUND W0", gad + "\nMERKLE I0 ((W0 I1)", "HASH", "SET_MEMBER W9999 I0",
                                   gad + "\nOR\n{\n", std::string("\xff\xfe", 2)};
        for (const std::string &g : bad) {
            try { synthesize_prover(inst, wtns, g); } catch (const std::exception &) {}
        }
        try { synthesize_prover(inst.substr(0, inst.size() / 2), wtns, gad); } catch (const std::exception &) {}
        try { synthesize_prover(inst, wtns.substr(0, wtns.size() / 3), gad); } catch (const std::exception &) {}
        try { synthesize_verifier(inst, "C0-0 = 0x12", gad); } catch (const std::exception &) {}
    }
    return n;
}

static bool gadget_api() {
    ConstraintSystem cs(true);
    std::vector<LC> wit;
    for (int k = 0; k < 8; k++) wit.push_back(LC::of(cs.commit_value(Scalar::from_u64(k + 1), Scalar::from_u64(99))));
    merkle_tree_assemble(cs, LC::cnst(Scalar::from_u64(5)), {}, wit, "H(H(H(W W) H(W W)) H(H(W W) H(W W)))");
    Scalar x = Scalar::from_u64(0x1234);
    range_proof_assemble(cs, LC::cnst(x), 16, &x);
    bool threw = false;
    try { merkle_tree_assemble(cs, LC(), {}, {}, "H(W"); } catch (const std::exception &) { threw = true; }
    return threw && cs.view(true).n > 0;
}

static bool rng_lockstep() {
    Transcript T((const uint8_t *)"san", 3);
    T.append_u64("m", 2);
    TranscriptRng base(T);
    for (int lanes = 1; lanes <= 8; lanes++) {
        uint8_t ent[8][32];
        const uint8_t *ep[8];
        for (int k = 0; k < 8; k++) { for (int i = 0; i < 32; i++) ent[k][i] = (uint8_t)(k * 13 + i + lanes); ep[k] = ent[k]; }
        Strobe8 S; S.from(base.s, lanes);
        S.meta_ad((const uint8_t *)"rng", 3);
        S.key_each(ep, 32);
        std::vector<TranscriptRng> ref;
        for (int k = 0; k < lanes; k++) { ref.push_back(base); ref.back().finalize(ent[k]); }
        uint8_t out[8][64], want[64];
        uint8_t *op[8];
        for (int k = 0; k < 8; k++) op[k] = out[k];
        for (int d = 0; d < 50; d++) {
            S.draw64(op);
            for (int k = 0; k < lanes; k++) { ref[k].fill_bytes(want, 64); if (memcmp(want, out[k], 64)) return false; }
        }
    }
    return true;
}

static bool arith() {
    std::mt19937_64 r(5);
    for (int it = 0; it < 2000; it++) {
        uint32_t a[8], b[8];
        for (int k = 0; k < 8; k++) { a[k] = (uint32_t)r(); b[k] = (uint32_t)r(); }
        a[7] &= 0x7fffffff; b[7] &= 0x7fffffff;
        fe x, y, z, w;
        fe_fromw(x, a); fe_fromw(y, b);
        fe_mul(z, x, y); fe_sq(w, z); fe_add(z, z, w); fe_sub(w, w, x);
        uint32_t o[8]; fe_tow(o, w); fe_tow(o, z);
        sc s, t, u;
        for (int k = 0; k < 8; k++) { s.v[k] = a[k]; t.v[k] = b[k]; }
        s.v[7] &= 0x0fffffff; t.v[7] &= 0x0fffffff;
        sc_montmul(u, s, t); sc_add(u, u, s); sc_sub(u, u, t); sc_reduce(u, u);
        Scalar p = Scalar::reduce(reinterpret_cast<const uint8_t *>(a)), q = Scalar::reduce(reinterpret_cast<const uint8_t *>(b));
        Scalar m = p * q + p - q;
        (void)sc_invert(m);
    }
    return true;
}

int main(int argc, char **argv) {
    int n = fixtures(argc, argv);
    if (n != argc - 1) return 1;
    if (!gadget_api()) { fprintf(stderr, "gadget api\n"); return 2; }
    if (!rng_lockstep()) { fprintf(stderr, "rng lockstep\n"); return 3; }
    if (!arith()) return 4;
    printf("sanitize ok: %d fixtures\n", n);
    return 0;
}
