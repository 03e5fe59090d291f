// statement.h — the circuit layer kept for drop-in compatibility with
// FairAds/bulletproof-gadgets: the .inst/.wtns/.gadgets/.coms mini-language
// (src/lalrpop/*), the Gadget trait (src/gadget.rs:7-60) and the gadgets
// (bounds_check, mimc_hash, merkle_tree, set_membership, less_than,
// inequality, equality, OR), producing the flattened constraint system the
// hot path consumes (include/bpg.h bpg_r1cs_view).
//
// The reference records every operation twice (a ProverBuffer on a scratch
// "BufferTranscript" prover, then a replay into the main prover,
// src/cs_buffer.rs + src/prove.rs:72). Here one recorder builds the final
// system in a single pass: top-level operations go straight into the CSR
// arrays, only OR branches (src/or/or_conjunction.rs) are buffered until the
// cartesian product is multiplied out.
#pragma once
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../../include/bpg.h"
#include "hcrypto.h"

namespace bpg {

typedef uint32_t Var;   // BPG_VAR(kind, index)
inline Var var_one() { return BPG_VAR(BPG_VAR_ONE, 0); }

// bulletproofs r1cs::LinearCombination: a list of terms; + and - concatenate.
struct LC {
    std::vector<std::pair<Var, Scalar>> t;
    LC() {}
    static LC cnst(const Scalar &s) { LC l; l.t.push_back({var_one(), s}); return l; }
    static LC of(Var v) { LC l; l.t.push_back({v, Scalar::one()}); return l; }
};
LC operator+(const LC &a, const LC &b);
LC operator-(const LC &a, const LC &b);
LC lc_scale(const LC &a, const Scalar &s);

struct StatementError : std::runtime_error {
    explicit StatementError(const std::string &m) : std::runtime_error(m) {}
};

// One recorder for both sides: `prover` evaluates assignments eagerly
// (r1cs::Prover semantics), the verifier side only counts variables
// (r1cs::Verifier).
class ConstraintSystem {
  public:
    explicit ConstraintSystem(bool prover);
    ~ConstraintSystem();
    bool prover() const { return prover_; }
    Var commit_value(const Scalar &v, const Scalar &blinding);   // Prover::commit
    Var commit_point(const uint8_t V[32]);                        // Verifier::commit
    struct Triple { Var l, r, o; };
    Triple multiply(const LC &left, const LC &right);
    Triple allocate_multiplier(const Scalar *l, const Scalar *r); // NULL on the verifier
    void constrain(const LC &lc);
    // OR support (src/or/or_conjunction.rs, prove.rs:184-220): operations of
    // an OR block are buffered per branch `{ ... }` and replayed by or_block.
    struct Op { bool mul; LC a, b; Var lv, rv; };
    void push_buffer();                              // `OR` / `[`
    void rewind();                                   // `}` closes a branch
    std::vector<std::vector<Op>> pop_buffer();       // `]`: closed branches
    void replay_mul(const Op &op);                   // branch multiply -> parent
    // results
    uint32_t n() const { return nvars_; }
    uint32_t q() const { return (uint32_t)row_ptr_.size() - 1; }
    const std::vector<Scalar> &v() const { return v_; }
    const std::vector<Scalar> &vb() const { return vb_; }
    const std::vector<uint8_t> &V() const { return V_; }
    uint32_t m() const { return prover_ ? (uint32_t)v_.size() : (uint32_t)(V_.size() / 32); }
    // Flattened view (pointers into this object).
    bpg_r1cs_view view(bool with_secrets);
  private:
    Scalar eval(const LC &lc) const;
    void emit(const LC &lc);
    void emit_minus(const LC &lc, Var v);   // emit lc - v (a multiplier's input constraint)
    bool prover_;
    uint32_t nvars_ = 0;
    std::vector<Scalar> aL_, aR_, aO_, v_, vb_;
    std::vector<uint8_t> V_;
    std::vector<uint32_t> row_ptr_{0}, term_var_;
    std::vector<uint8_t> term_coeff_;
    std::vector<uint8_t> aLb_, aRb_, aOb_, vbytes_, vbb_;
    std::vector<std::vector<Op>> stack_;        // open OR buffers
    std::vector<std::vector<std::vector<Op>>> cache_;  // closed blocks per open OR
};

// MiMC-256 (src/mimc_hash/mimc.rs:61-75), native.
Scalar mimc_hash(const std::vector<uint8_t> &preimage);
// Unpadded sponge over field elements (the Merkle node hash of
// merkle_tree_gadget.rs:106 evaluated natively).
Scalar mimc_sponge_native(const std::vector<Scalar> &blocks);

// Gadget-API building blocks over a recorder (the Gadget trait callers of
// src/gadget.rs:7-60 that build circuits in code, not in the mini-language):
// MerkleTree256::assemble (merkle_tree_gadget.rs:44-56; `pattern` in the
// reference's Display form, e.g. "H(H(W W) I)") and utils.rs:5 range_proof.
void merkle_tree_assemble(ConstraintSystem &cs, const LC &root, std::vector<LC> inst, std::vector<LC> wit,
                          const std::string &pattern);
void range_proof_assemble(ConstraintSystem &cs, const LC &x, unsigned n, const Scalar *x_assign);

// Statement drivers (src/prove.rs:37-75, src/verify.rs:36-69).
struct Synthesis {
    std::unique_ptr<ConstraintSystem> cs;
    std::vector<std::string> com_names;   // prover: `.coms` names in commit order
};
Synthesis synthesize_prover(const std::string &instance, const std::string &witness, const std::string &gadgets);
Synthesis synthesize_verifier(const std::string &instance, const std::string &commitments, const std::string &gadgets);

}  // namespace bpg
