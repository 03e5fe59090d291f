// statement.cpp — see statement.h. Gadget semantics cite the reference
// (/root/reference/src/...) per function.
#include "statement.h"

#include <algorithm>
#include <string.h>

namespace bpg {

#include "mimc_constants.inc"

// ------------------------------------------------------------ LC operators
LC operator+(const LC &a, const LC &b) {
    LC r = a;
    r.t.insert(r.t.end(), b.t.begin(), b.t.end());
    return r;
}
LC operator-(const LC &a, const LC &b) {
    LC r = a;
    r.t.reserve(a.t.size() + b.t.size());
    for (auto &x : b.t) r.t.push_back({x.first, -x.second});
    return r;
}
LC lc_scale(const LC &a, const Scalar &s) {
    LC r = a;
    for (auto &x : r.t) x.second = x.second * s;
    return r;
}

// -------------------------------------------------------- ConstraintSystem
// The flattened arrays of a 2^20 statement are ~200 MB; grown from empty for
// every statement, their reallocation copies and first-touch page faults cost
// about as much as the synthesis itself (and serialise threads on the
// process's page tables). A thread keeps the buffers of its last recorder
// (cleared, capacity intact) for the next one.
namespace {
struct CsBuffers {
    std::vector<Scalar> aL, aR, aO;
    std::vector<uint32_t> row_ptr, term_var;
    std::vector<uint8_t> term_coeff, aLb, aRb, aOb;
    bool valid = false;
};
CsBuffers &cs_pool() { static thread_local CsBuffers b; return b; }
// memset the optimiser may not drop (the buffer is reused, not freed, but the
// intent is a wipe)
void secure_wipe(void *p, size_t n) {
    if (!p || !n) return;
    memset(p, 0, n);
    __asm__ __volatile__("" : : "r"(p) : "memory");
}
}  // namespace
ConstraintSystem::ConstraintSystem(bool prover) : prover_(prover) {
    CsBuffers &b = cs_pool();
    if (b.valid) {
        b.valid = false;
        aL_.swap(b.aL); aR_.swap(b.aR); aO_.swap(b.aO);
        row_ptr_.swap(b.row_ptr); term_var_.swap(b.term_var); term_coeff_.swap(b.term_coeff);
        aLb_.swap(b.aLb); aRb_.swap(b.aRb); aOb_.swap(b.aOb);
        aL_.clear(); aR_.clear(); aO_.clear(); term_var_.clear(); term_coeff_.clear();
        row_ptr_.assign(1, 0);
    }
}
ConstraintSystem::~ConstraintSystem() {
    // the witness (a_L, a_R, a_O and their byte forms) is wiped before its
    // buffers go back to the thread's pool: the next recorder on this thread
    // (a verifier's, say) must not inherit another statement's secrets
    if (prover_) {
        secure_wipe(aL_.data(), aL_.size() * sizeof(Scalar));
        secure_wipe(aR_.data(), aR_.size() * sizeof(Scalar));
        secure_wipe(aO_.data(), aO_.size() * sizeof(Scalar));
        secure_wipe(aLb_.data(), aLb_.size());
        secure_wipe(aRb_.data(), aRb_.size());
        secure_wipe(aOb_.data(), aOb_.size());
    }
    CsBuffers &b = cs_pool();
    // retained capacity is bounded (a 2^22-gate statement's worth of terms)
    if (term_coeff_.capacity() > ((size_t)32 << 22) * 3) return;
    if (b.valid && b.term_coeff.capacity() >= term_coeff_.capacity()) return;   // keep the larger set
    aL_.swap(b.aL); aR_.swap(b.aR); aO_.swap(b.aO);
    row_ptr_.swap(b.row_ptr); term_var_.swap(b.term_var); term_coeff_.swap(b.term_coeff);
    aLb_.swap(b.aLb); aRb_.swap(b.aRb); aOb_.swap(b.aOb);
    b.valid = true;
}

Var ConstraintSystem::commit_value(const Scalar &v, const Scalar &blinding) {
    uint32_t i = (uint32_t)v_.size();
    v_.push_back(v);
    vb_.push_back(blinding);
    return BPG_VAR(BPG_VAR_V, i);
}
Var ConstraintSystem::commit_point(const uint8_t V[32]) {
    uint32_t i = (uint32_t)(V_.size() / 32);
    V_.insert(V_.end(), V, V + 32);
    return BPG_VAR(BPG_VAR_V, i);
}
// Prover::eval: sum coeff * value (dalek Mul/Add: canonical results). The
// statement layer's terms are mostly unit coefficients and constants (the
// MiMC rounds' (One, c)): c * 1 = c mod l and 1 * v = v mod l, and Add
// reduces its operands, so those terms are added without a multiplication;
// a zero coefficient adds 0 to an already canonical sum.
static inline bool sc_is_one(const Scalar &s) { return s.v[0] == 1 && !(s.v[1] | s.v[2] | s.v[3]); }
Scalar ConstraintSystem::eval(const LC &lc) const {
    Scalar acc = Scalar::zero();
    for (auto &x : lc.t) {
        const uint32_t k = BPG_VAR_KIND(x.first), i = BPG_VAR_INDEX(x.first);
        if (x.second.is_zero_raw()) continue;
        if (k == BPG_VAR_ONE) { acc = acc + x.second; continue; }
        const Scalar &val = k == BPG_VAR_L ? aL_[i] : k == BPG_VAR_R ? aR_[i] : k == BPG_VAR_O ? aO_[i] : v_[i];
        acc = acc + (sc_is_one(x.second) ? val : x.second * val);
    }
    return acc;
}
void ConstraintSystem::emit(const LC &lc) {
    const size_t k0 = term_var_.size();
    term_coeff_.resize(32 * (k0 + lc.t.size()));
    uint8_t *c = term_coeff_.data() + 32 * k0;
    for (auto &x : lc.t) {
        term_var_.push_back(x.first);
        x.second.to_bytes(c);
        c += 32;
    }
    row_ptr_.push_back((uint32_t)term_var_.size());
}
void ConstraintSystem::emit_minus(const LC &lc, Var v) {
    static const Scalar minus_one = -Scalar::one();
    const size_t k0 = term_var_.size();
    term_coeff_.resize(32 * (k0 + lc.t.size() + 1));
    uint8_t *c = term_coeff_.data() + 32 * k0;
    for (auto &x : lc.t) {
        term_var_.push_back(x.first);
        x.second.to_bytes(c);
        c += 32;
    }
    term_var_.push_back(v);
    minus_one.to_bytes(c);
    row_ptr_.push_back((uint32_t)term_var_.size());
}
// r1cs Prover::multiply / Verifier::multiply: allocate (l, r, o), constrain
// left - l = 0 and right - r = 0.
ConstraintSystem::Triple ConstraintSystem::multiply(const LC &left, const LC &right) {
    uint32_t i = nvars_++;
    Triple t{BPG_VAR(BPG_VAR_L, i), BPG_VAR(BPG_VAR_R, i), BPG_VAR(BPG_VAR_O, i)};
    if (prover_) {
        Scalar l = eval(left), r = &left == &right ? l : eval(right);
        aL_.push_back(l); aR_.push_back(r); aO_.push_back(l * r);
    }
    if (stack_.empty()) {   // left - l = 0 and right - r = 0, without copying the combinations
        emit_minus(left, t.l);
        emit_minus(right, t.r);
    } else {
        stack_.back().push_back(Op{true, left, right, t.l, t.r});
    }
    return t;
}
ConstraintSystem::Triple ConstraintSystem::allocate_multiplier(const Scalar *l, const Scalar *r) {
    uint32_t i = nvars_++;
    if (prover_) {
        if (!l || !r) throw StatementError("missing assignment");
        aL_.push_back(l->reduced()); aR_.push_back(r->reduced()); aO_.push_back(*l * *r);
    }
    return Triple{BPG_VAR(BPG_VAR_L, i), BPG_VAR(BPG_VAR_R, i), BPG_VAR(BPG_VAR_O, i)};
}
void ConstraintSystem::constrain(const LC &lc) {
    if (stack_.empty()) emit(lc);
    else stack_.back().push_back(Op{false, lc, LC(), 0, 0});
}
void ConstraintSystem::replay_mul(const Op &op) {
    if (!stack_.empty()) { stack_.back().push_back(op); return; }
    emit_minus(op.a, op.lv);
    emit_minus(op.b, op.rv);
}
void ConstraintSystem::push_buffer() { stack_.emplace_back(); cache_.emplace_back(); }
void ConstraintSystem::rewind() {
    cache_.back().push_back(std::move(stack_.back()));
    stack_.back().clear();
}
std::vector<std::vector<ConstraintSystem::Op>> ConstraintSystem::pop_buffer() {
    auto c = std::move(cache_.back());
    cache_.pop_back();
    stack_.pop_back();   // operations after the last `}` are dropped, as in or_conjunction
    return c;
}
bpg_r1cs_view ConstraintSystem::view(bool with_secrets) {
    bpg_r1cs_view v{};
    v.n = nvars_;
    v.m = m();
    v.q = q();
    v.nnz = (uint32_t)term_var_.size();
    v.row_ptr = row_ptr_.data();
    v.term_var = term_var_.data();
    v.term_coeff = term_coeff_.data();
    if (with_secrets && prover_) {
        auto pack = [](std::vector<uint8_t> &dst, const std::vector<Scalar> &src) {
            dst.resize(src.size() * 32 + 32);
            for (size_t i = 0; i < src.size(); i++) src[i].to_bytes(dst.data() + 32 * i);
        };
        pack(aLb_, aL_); pack(aRb_, aR_); pack(aOb_, aO_); pack(vbytes_, v_); pack(vbb_, vb_);
        v.a_L = aLb_.data(); v.a_R = aRb_.data(); v.a_O = aOb_.data();
        v.v = vbytes_.data(); v.v_blinding = vbb_.data();
    }
    return v;
}

// ------------------------------------------------------------------- bytes
typedef std::vector<uint8_t> Bytes;
static Scalar from_bits_vec(const uint8_t *b, size_t n) {   // n <= 32, LE, zero-padded
    uint8_t buf[32] = {0};
    memcpy(buf, b, n);
    return Scalar::from_bits(buf);
}
// conversions.rs:6-23 le_to_scalars / 26-30 be_to_scalars
static std::vector<Scalar> be_to_scalars(const Bytes &be) {
    Bytes le(be.rbegin(), be.rend());
    std::vector<Scalar> out;
    for (size_t i = 0; i < le.size(); i += 32) out.push_back(from_bits_vec(le.data() + i, std::min<size_t>(32, le.size() - i)));
    return out;
}
// conversions.rs:48-53
static Scalar be_to_scalar(const Bytes &be) {
    if (be.size() > 32) throw StatementError("the given vector is longer than 32 bytes");
    Bytes le(be.rbegin(), be.rend());
    return from_bits_vec(le.data(), le.size());
}
static Scalar le_to_scalar(const Bytes &le) {
    if (le.size() > 32) throw StatementError("the given vector is longer than 32 bytes");
    return from_bits_vec(le.data(), le.size());
}
static Bytes scalar_le(const Scalar &s) { uint8_t b[32]; s.to_bytes(b); return Bytes(b, b + 32); }
static Bytes strip_trailing_zeros(Bytes b) { while (!b.empty() && b.back() == 0) b.pop_back(); return b; }
static Bytes pkcs7(Bytes b, size_t block) {
    size_t k = block - (b.size() % block);
    b.insert(b.end(), k, (uint8_t)k);
    return b;
}

// ------------------------------------------------------------------- MiMC
static const std::vector<Scalar> &mimc_consts() {
    static std::vector<Scalar> cs = [] {
        std::vector<Scalar> v;
        const char *h = MIMC_ROUND_CONSTANTS_HEX;
        auto nib = [](char c) -> int { return c <= '9' ? c - '0' : (c | 32) - 'a' + 10; };
        for (int i = 0; i < 486; i++) {
            uint8_t b[32];
            for (int j = 0; j < 32; j++) b[j] = (uint8_t)(nib(h[64 * i + 2 * j]) << 4 | nib(h[64 * i + 2 * j + 1]));
            v.push_back(Scalar::from_bits(b));
        }
        return v;
    }();
    return cs;
}
// mimc.rs:77-97 pad (PKCS#7 on the trailing-zero-stripped LE bytes of the last block)
static std::vector<Scalar> mimc_pad(std::vector<Scalar> blocks) {
    Bytes last = strip_trailing_zeros(scalar_le(blocks.back()));
    if (last.size() < 32) {
        blocks.pop_back();
        blocks.push_back(le_to_scalar(pkcs7(last, 32)));
    } else {
        blocks.push_back(le_to_scalar(Bytes(32, 32)));
    }
    return blocks;
}
Scalar mimc_hash(const std::vector<uint8_t> &preimage) {
    const auto &cs = mimc_consts();
    Scalar state = Scalar::zero();
    for (const Scalar &blk : mimc_pad(be_to_scalars(preimage))) {
        state = state + blk;
        for (const Scalar &c : cs) {   // mimc_encryption, key = 0
            Scalar t = state + c;
            state = t * t * t;
        }
        state = state + Scalar::zero();
    }
    return state;
}

Scalar mimc_sponge_native(const std::vector<Scalar> &blocks) {
    const auto &cs = mimc_consts();
    Scalar state = Scalar::zero();
    for (const Scalar &blk : blocks) {
        state = state + blk;
        for (const Scalar &c : cs) { Scalar t = state + c; state = t * t * t; }
    }
    return state;
}

// mimc_hash_gadget.rs:108-150
static LC mimc_sponge(ConstraintSystem &cs, const std::vector<LC> &pre) {
    const auto &consts = mimc_consts();
    const Var one = var_one();
    LC key = LC::cnst(Scalar::zero());
    LC state = LC::cnst(Scalar::zero());
    // the round's LCs are rebuilt in place (same terms, same order as
    // p + key + LC::cnst(c), LC::of(sq.o), LC::of(sq.l)): no allocation per round
    LC pk, so, sl;
    so.t.resize(1);
    sl.t.resize(1);
    for (const LC &v : pre) {
        state = state + v;
        LC p = state;
        pk.t.reserve(p.t.size() + 2);
        for (const Scalar &c : consts) {
            pk.t.assign(p.t.begin(), p.t.end());
            pk.t.push_back({one, Scalar::zero()});   // + key
            pk.t.push_back({one, c});
            auto sq = cs.multiply(pk, pk);
            so.t[0] = {sq.o, Scalar::one()};
            sl.t[0] = {sq.l, Scalar::one()};
            auto cube = cs.multiply(so, sl);
            p.t.assign(1, {cube.o, Scalar::one()});
        }
        state = p + key;
    }
    return state;
}

// ---------------------------------------------------------------- gadgets
typedef std::vector<std::pair<Scalar, Var>> Derived;   // (assignment, variable)

// utils.rs:5-35
static void range_proof(ConstraintSystem &cs, LC x, unsigned n, const Scalar *x_assign) {
    Scalar exp2 = Scalar::one();
    uint8_t xb[32];
    if (x_assign) x_assign->to_bytes(xb);
    for (unsigned i = 0; i < n; i++) {
        ConstraintSystem::Triple t;
        if (x_assign) {
            unsigned bit = (xb[i / 8] >> (i % 8)) & 1;
            Scalar l = Scalar::from_u64(1 - bit), r = Scalar::from_u64(bit);
            t = cs.allocate_multiplier(&l, &r);
        } else {
            t = cs.allocate_multiplier(nullptr, nullptr);
        }
        cs.constrain(LC::of(t.o));
        cs.constrain(LC::of(t.l) + (LC::of(t.r) - LC::cnst(Scalar::one())));
        x = x - lc_scale(LC::of(t.r), exp2);
        exp2 = exp2 + exp2;
    }
    cs.constrain(x);
}

// gadget.rs:23-42 setup: commit each derived scalar with a fresh blinding
static Derived gadget_setup(ConstraintSystem &cs, const std::vector<Scalar> &derived) {
    Derived out;
    for (const Scalar &s : derived) {
        Scalar blinding = thread_entropy().random_scalar();
        out.push_back({s, cs.commit_value(s, blinding)});
    }
    return out;
}

// bounds_check_gadget.rs:14-63
struct BoundsCheck {
    Scalar min, max;
    unsigned n;
    BoundsCheck(const Bytes &mn, const Bytes &mx) {
        n = (unsigned)((mx.size() * 8) & 0xff);   // `as u8`
        min = be_to_scalar(mn);
        max = be_to_scalar(mx);
    }
    std::vector<Scalar> preprocess(const std::vector<Scalar> &w) const { return {w[0] - min, max - w[0]}; }
    void assemble(ConstraintSystem &cs, const Derived &d, bool with_assign) const {
        Var a = d[0].second, b = d[1].second;
        cs.constrain((LC::of(a) + LC::of(b)) - LC::cnst(max - min));
        range_proof(cs, LC::of(a), n, with_assign ? &d[0].first : nullptr);
        range_proof(cs, LC::of(b), n, with_assign ? &d[1].first : nullptr);
    }
};

// mimc_hash_gadget.rs:15-75
struct MimcGadget {
    LC image;
    std::vector<Scalar> preprocess(const std::vector<Scalar> &w) const {
        Scalar last = w.back();
        Bytes le = strip_trailing_zeros(scalar_le(last));
        if (le.size() < 32) {
            Scalar padded = le_to_scalar(pkcs7(le, 32));
            return {padded, padded - last};
        }
        return {le_to_scalar(Bytes(32, 32))};
    }
    void assemble(ConstraintSystem &cs, std::vector<Var> coms, const Derived &d) const {
        Var padded = d[0].second;
        if (d.size() == 2) {
            Var padding = d[1].second;
            LC last = LC::of(coms.back());
            coms.pop_back();
            cs.constrain((last + LC::of(padding)) - LC::of(padded));
        }
        coms.push_back(padded);
        std::vector<LC> pre;
        for (Var v : coms) pre.push_back(LC::of(v));
        LC h = mimc_sponge(cs, pre);
        cs.constrain(h - image);
    }
};

// merkle_tree_gadget.rs:15-115
struct Pattern {
    char kind;   // 'W', 'I', 'H'
    std::unique_ptr<Pattern> l, r;
};
static LC merkle_parse(ConstraintSystem &cs, std::vector<LC> &w, std::vector<LC> &i, const Pattern &p) {
    auto take = [](std::vector<LC> &vals) {
        if (vals.empty()) throw StatementError("too few variables provided to satisfy the given pattern");
        LC v = vals.front();
        vals.erase(vals.begin());
        return v;
    };
    std::vector<LC> pre;
    if (p.kind == 'W') pre.push_back(take(w));
    else if (p.kind == 'I') pre.push_back(take(i));
    else {
        LC left = p.l->kind == 'H' ? merkle_parse(cs, w, i, *p.l) : take(p.l->kind == 'W' ? w : i);
        LC right = p.r->kind == 'H' ? merkle_parse(cs, w, i, *p.r) : take(p.r->kind == 'W' ? w : i);
        pre.push_back(left);
        pre.push_back(right);
    }
    return mimc_sponge(cs, pre);
}

// set_membership_gadget.rs:13-131
struct SetMembership {
    LC value;
    Scalar value_a;
    std::vector<LC> inst;
    std::vector<Scalar> inst_a;
    std::vector<Scalar> preprocess(const std::vector<Scalar> &w) const {
        std::vector<Scalar> out;
        auto bit = [&](const Scalar &e) { out.push_back(e == value_a ? Scalar::one() : Scalar::zero()); };
        for (auto &e : w) bit(e);
        for (auto &e : inst_a) bit(e);
        return out;
    }
    void assemble(ConstraintSystem &cs, const std::vector<Var> &w, const Derived &d) const {
        std::vector<LC> bits;
        for (auto &x : d) {
            LC bl = LC::of(x.second);
            auto z = cs.multiply(LC::cnst(Scalar::one()) - bl, bl);
            cs.constrain(LC::of(z.o));
            bits.push_back(bl);
        }
        LC sum = LC::cnst(Scalar::zero());
        for (auto &b : bits) sum = sum + b;
        cs.constrain(LC::cnst(Scalar::one()) - sum);
        std::vector<LC> set;
        for (Var v : w) set.push_back(LC::of(v));
        for (auto &e : inst) set.push_back(e);
        if (bits.size() != set.size()) { cs.constrain(LC::cnst(Scalar::one())); return; }
        LC act = LC::cnst(Scalar::zero());
        for (size_t k = 0; k < bits.size(); k++) {
            auto pr = cs.multiply(bits[k], set[k]);
            act = act + LC::of(pr.o);
        }
        cs.constrain(value - act);
    }
};

// less_than_gadget.rs:16-66
struct LessThan {
    LC left, right;
    const Scalar *la, *ra;
    std::vector<Scalar> preprocess() const {
        Scalar delta = *ra - *la;
        return {delta, delta == Scalar::zero() ? Scalar::zero() : sc_invert(delta)};
    }
    void assemble(ConstraintSystem &cs, const Derived &d) const {
        Var delta = d[0].second, dinv = d[1].second;
        range_proof(cs, left, 126, la);
        range_proof(cs, right, 126, ra);
        range_proof(cs, LC::of(delta), 126, la ? &d[0].first : nullptr);
        auto one = cs.multiply(LC::of(delta), LC::of(dinv));
        cs.constrain(LC::cnst(Scalar::one()) - LC::of(one.o));
        cs.constrain((right - left) - LC::of(delta));
    }
};

// inequality_gadget.rs:12-113
static bool compare_bytes(const Scalar &a, const Scalar &b) {
    uint8_t x[32], y[32];
    a.to_bytes(x); b.to_bytes(y);
    for (int i = 31; i >= 0; i--) {
        if (x[i] > y[i]) return true;
        if (x[i] < y[i]) return false;
    }
    return true;
}
struct Inequality {
    std::vector<LC> right;
    std::vector<Scalar> ra;
    std::vector<Scalar> preprocess(const std::vector<Scalar> &left) const {
        std::vector<Scalar> out;
        Scalar sum = Scalar::zero();
        for (size_t i = 0; i < left.size(); i++) {
            Scalar l = left[i], r = i < ra.size() ? ra[i] : Scalar::zero();
            Scalar delta = compare_bytes(l, r) ? l - r : r - l;
            out.push_back(delta);
            if (delta == Scalar::zero()) out.push_back(Scalar::zero());
            else {
                Scalar di = sc_invert(delta);
                out.push_back(di);
                sum = sum + delta * di;
            }
        }
        out.push_back(sc_invert(sum));
        return out;
    }
    void assemble(ConstraintSystem &cs, const std::vector<Var> &left, const Derived &d) const {
        if (right.size() != left.size()) { cs.constrain(LC::cnst(Scalar::zero())); return; }
        LC sum = LC::cnst(Scalar::zero());
        for (size_t i = 0; i < left.size(); i++) {
            LC r = right[i], l = LC::of(left[i]);
            Var delta = d[2 * i].second, dinv = d[2 * i + 1].second;
            LC lmr = l - r, rml = r - l;
            auto z = cs.multiply(lmr - LC::of(delta), rml - LC::of(delta));
            cs.constrain(LC::of(z.o));
            auto zo = cs.multiply(LC::of(delta), LC::of(dinv));
            sum = sum + LC::of(zo.o);
        }
        auto one = cs.multiply(sum, LC::of(d.back().second));
        cs.constrain(LC::cnst(Scalar::one()) - LC::of(one.o));
    }
};

// equality_gadget.rs:10-32
static void equality_assemble(ConstraintSystem &cs, const std::vector<LC> &right, const std::vector<Var> &left) {
    if (right.size() != left.size()) { cs.constrain(LC::cnst(Scalar::one())); return; }
    for (size_t i = 0; i < left.size(); i++) cs.constrain(right[i] - LC::of(left[i]));
}

// --------------------------------------------------------- mini-language
// Rust str::lines(): split on \n, strip one trailing \r, no final empty line
static std::vector<std::string> rust_lines(const std::string &s) {
    std::vector<std::string> out;
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find('\n', i);
        if (j == std::string::npos) j = s.size();
        std::string l = s.substr(i, j - i);
        if (!l.empty() && l.back() == '\r') l.pop_back();
        out.push_back(l);
        i = j + 1;
    }
    return out;
}
static std::string trim(const std::string &s) {
    size_t a = s.find_first_not_of(" \t\r\n"), b = s.find_last_not_of(" \t\r\n");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}
static bool all_digits(const std::string &s, size_t from, size_t to) {
    if (from >= to) return false;
    for (size_t i = from; i < to; i++) if (s[i] < '0' || s[i] > '9') return false;
    return true;
}
// var_grammar.lalrpop: NAME "=" 0[xX][0-9a-fA-F]+
static std::pair<std::string, Bytes> parse_var_line(const std::string &line, char kind) {
    size_t eq = line.find('=');
    if (eq == std::string::npos) throw StatementError("unable to parse line: " + line);
    std::string name = trim(line.substr(0, eq)), val = trim(line.substr(eq + 1));
    bool ok = false;
    if (kind == 'C') {
        // [C|D]{1}\d+-\d+(-\d+)?
        if (!name.empty() && (name[0] == 'C' || name[0] == 'D' || name[0] == '|')) {
            size_t d1 = name.find('-', 1);
            if (d1 != std::string::npos && all_digits(name, 1, d1)) {
                size_t d2 = name.find('-', d1 + 1);
                if (d2 == std::string::npos) ok = all_digits(name, d1 + 1, name.size());
                else ok = all_digits(name, d1 + 1, d2) && all_digits(name, d2 + 1, name.size());
            }
        }
    } else {
        ok = name.size() >= 2 && name[0] == kind && all_digits(name, 1, name.size());
    }
    if (!ok) throw StatementError("unable to parse line: " + line);
    if (val.size() < 3 || val[0] != '0' || (val[1] != 'x' && val[1] != 'X'))
        throw StatementError("unable to parse hex in line: " + line);
    std::string h = val.substr(2);
    if (h.size() % 2) throw StatementError("odd-length hex in line: " + line);
    Bytes out;
    for (size_t i = 0; i < h.size(); i += 2) {
        auto nib = [&](char c) -> int {
            if (c >= '0' && c <= '9') return c - '0';
            if (c >= 'a' && c <= 'f') return c - 'a' + 10;
            if (c >= 'A' && c <= 'F') return c - 'A' + 10;
            throw StatementError("invalid hex in line: " + line);
        };
        out.push_back((uint8_t)(nib(h[i]) << 4 | nib(h[i + 1])));
    }
    return {name, out};
}
static std::vector<std::string> tokens(const std::string &line) {
    std::vector<std::string> out;
    size_t i = 0;
    while (i < line.size()) {
        char c = line[i];
        if (c == '(' || c == ')' || c == '[' || c == ']' || c == '{' || c == '}') { out.push_back(std::string(1, c)); i++; }
        else if (isalnum((unsigned char)c) || c == '_') {
            size_t j = i;
            while (j < line.size() && (isalnum((unsigned char)line[j]) || line[j] == '_')) j++;
            out.push_back(line.substr(i, j - i));
            i = j;
        } else if (isspace((unsigned char)c)) i++;
        else throw StatementError("unexpected character in line: " + line);
    }
    return out;
}
static bool is_witness(const std::string &t) { return t.size() >= 2 && t[0] == 'W' && all_digits(t, 1, t.size()); }
static bool is_instance(const std::string &t) { return t.size() >= 2 && t[0] == 'I' && all_digits(t, 1, t.size()); }

// gadget_grammar.lalrpop:46-72 (Tree)
struct Tree { std::vector<std::string> inst, wit; std::unique_ptr<Pattern> p; };
// Nesting bound of the recursive pattern parsers (a deeper text would only
// overflow the stack; the crate's own circuits nest at most 32 deep).
static const int MAX_PATTERN_DEPTH = 512;
static Tree parse_tree(const std::vector<std::string> &t, size_t &pos, int depth = 0) {
    if (depth > MAX_PATTERN_DEPTH) throw StatementError("MERKLE tree nested too deeply");
    if (pos >= t.size() || t[pos] != "(") throw StatementError("malformed MERKLE tree");
    pos++;
    Tree out;
    out.p.reset(new Pattern{'H', nullptr, nullptr});
    for (int side = 0; side < 2; side++) {
        if (pos >= t.size()) throw StatementError("malformed MERKLE tree");
        std::unique_ptr<Pattern> sub;
        if (t[pos] == "(") {
            Tree s = parse_tree(t, pos, depth + 1);
            out.inst.insert(out.inst.end(), s.inst.begin(), s.inst.end());
            out.wit.insert(out.wit.end(), s.wit.begin(), s.wit.end());
            sub = std::move(s.p);
        } else if (is_witness(t[pos])) {
            out.wit.push_back(t[pos++]);
            sub.reset(new Pattern{'W', nullptr, nullptr});
        } else if (is_instance(t[pos])) {
            out.inst.push_back(t[pos++]);
            sub.reset(new Pattern{'I', nullptr, nullptr});
        } else throw StatementError("malformed MERKLE tree");
        (side ? out.p->r : out.p->l) = std::move(sub);
    }
    if (pos >= t.size() || t[pos] != ")") throw StatementError("malformed MERKLE tree");
    pos++;
    return out;
}

// ------------------------------------------- Gadget-API entry points
// Pattern in the reference's Display form (merkle_tree_gadget.rs:21-29):
// "W", "I" or "H(<left> <right>)".
static std::unique_ptr<Pattern> parse_display_pattern(const std::string &s, size_t &pos, int depth = 0) {
    if (depth > MAX_PATTERN_DEPTH) throw StatementError("pattern nested too deeply");
    while (pos < s.size() && s[pos] == ' ') pos++;
    if (pos >= s.size()) throw StatementError("malformed pattern");
    const char c = s[pos++];
    if (c == 'W' || c == 'I') return std::unique_ptr<Pattern>(new Pattern{c, nullptr, nullptr});
    if (c != 'H' || pos >= s.size() || s[pos] != '(') throw StatementError("malformed pattern");
    pos++;
    std::unique_ptr<Pattern> p(new Pattern{'H', nullptr, nullptr});
    p->l = parse_display_pattern(s, pos, depth + 1);
    p->r = parse_display_pattern(s, pos, depth + 1);
    while (pos < s.size() && s[pos] == ' ') pos++;
    if (pos >= s.size() || s[pos] != ')') throw StatementError("malformed pattern");
    pos++;
    return p;
}
void merkle_tree_assemble(ConstraintSystem &cs, const LC &root, std::vector<LC> inst, std::vector<LC> wit,
                          const std::string &pattern) {
    size_t pos = 0;
    std::unique_ptr<Pattern> p = parse_display_pattern(pattern, pos);
    while (pos < pattern.size() && pattern[pos] == ' ') pos++;
    if (pos != pattern.size()) throw StatementError("malformed pattern");
    // merkle_parse emits constraints as it goes: refuse a pattern with more
    // leaves than variables before it starts, so a failing call leaves the
    // recorder unchanged
    size_t nw = 0, ni = 0;
    std::vector<const Pattern *> stack{p.get()};
    while (!stack.empty()) {
        const Pattern *q = stack.back();
        stack.pop_back();
        if (q->kind == 'W') nw++;
        else if (q->kind == 'I') ni++;
        else { stack.push_back(q->l.get()); stack.push_back(q->r.get()); }
    }
    if (nw > wit.size() || ni > inst.size())
        throw StatementError("too few variables provided to satisfy the given pattern");
    LC h = merkle_parse(cs, wit, inst, *p);
    cs.constrain(h - root);
}
void range_proof_assemble(ConstraintSystem &cs, const LC &x, unsigned n, const Scalar *x_assign) {
    range_proof(cs, x, n, x_assign);
}

// ------------------------------------------------------- statement driver
class Statement {
  public:
    Statement(bool prover) : cs_(new ConstraintSystem(prover)), prover_(prover) {}
    std::unique_ptr<ConstraintSystem> cs_;
    std::vector<std::string> com_names;

    void parse_instance(const std::string &inst) {
        for (auto &l : rust_lines(inst)) { auto kv = parse_var_line(l, 'I'); inst_[kv.first] = kv.second; }
    }
    // assignment_parser.rs:144-155 + commitments.rs:35-44
    void parse_witness(const std::string &wit) {
        for (auto &l : rust_lines(wit)) {
            auto kv = parse_var_line(l, 'W');
            Wit w;
            w.bytes = kv.second;
            w.scalars = be_to_scalars(kv.second);
            for (size_t k = 0; k < w.scalars.size(); k++) {
                Scalar blinding = thread_entropy().random_scalar();
                w.vars.push_back(cs_->commit_value(w.scalars[k], blinding));
                com_names.push_back("C" + kv.first.substr(1) + "-" + std::to_string(k));
            }
            wit_[kv.first] = w;
        }
    }
    // assignment_parser.rs:133-141
    void parse_commitments(const std::string &coms) {
        for (auto &l : rust_lines(coms)) {
            auto kv = parse_var_line(l, 'C');
            if (kv.second.size() != 32) throw StatementError("commitment must be 32 bytes: " + l);
            coms_[kv.first] = cs_->commit_point(kv.second.data());
        }
    }
    void run(const std::string &gadgets) {
        lines_ = rust_lines(gadgets);
        pos_ = 0;
        while (pos_ < lines_.size()) {
            size_t idx = pos_;
            const std::string line = lines_[pos_++];
            conjunction(line);
            gadget(line, idx);
        }
    }

  private:
    struct Wit { std::vector<Scalar> scalars; std::vector<Var> vars; Bytes bytes; };
    ConstraintSystem &cs() { return *cs_; }
    bool prover_;
    std::map<std::string, Bytes> inst_;
    std::map<std::string, Wit> wit_;
    std::map<std::string, Var> coms_;
    std::vector<std::string> lines_;
    size_t pos_ = 0;

    static std::string first_word(const std::string &line) {
        size_t a = line.find_first_not_of(" \t\r");
        if (a == std::string::npos) return "";
        size_t b = line.find_first_of(" \t\r", a);
        return line.substr(a, b == std::string::npos ? std::string::npos : b - a);
    }
    const Bytes &instance(const std::string &name, bool assert32) {
        auto it = inst_.find(name);
        if (it == inst_.end()) throw StatementError("missing instance var " + name);
        if (assert32 && it->second.size() > 32) throw StatementError("instance var " + name + " is longer than 32 bytes");
        return it->second;
    }
    const Wit &witness(const std::string &name, bool assert32) {
        auto it = wit_.find(name);
        if (it == wit_.end()) throw StatementError("missing witness var " + name);
        if (assert32 && it->second.scalars.size() != 1) throw StatementError("witness var " + name + " is longer than 32 bytes");
        return it->second;
    }
    Var commitment(const std::string &name, size_t k) {
        auto it = coms_.find("C" + name.substr(1) + "-" + std::to_string(k));
        if (it == coms_.end()) throw StatementError("missing commitment C" + name.substr(1) + "-" + std::to_string(k));
        return it->second;
    }
    std::vector<Var> all_commitments(const std::string &name) {
        std::vector<Var> out;
        for (size_t k = 0;; k++) {
            auto it = coms_.find("C" + name.substr(1) + "-" + std::to_string(k));
            if (it == coms_.end()) break;
            out.push_back(it->second);
        }
        return out;
    }
    Var derived(size_t gadget, size_t index, size_t sub) {
        std::string key = "D" + std::to_string(gadget) + "-" + std::to_string(sub) + "-" + std::to_string(index);
        auto it = coms_.find(key);
        if (it == coms_.end()) throw StatementError("missing commitment " + key);
        return it->second;
    }
    bool inquire_derived(size_t gadget, size_t index, size_t sub, Var &out) {
        auto it = coms_.find("D" + std::to_string(gadget) + "-" + std::to_string(sub) + "-" + std::to_string(index));
        if (it == coms_.end()) return false;
        out = it->second;
        return true;
    }
    void name_derived(size_t count, size_t gadget, size_t sub) {
        for (size_t k = 0; k < count; k++)
            com_names.push_back("D" + std::to_string(gadget) + "-" + std::to_string(sub) + "-" + std::to_string(k));
    }

    // prove.rs:122-130 parse_conjunction / 184-220 or_conjunction
    void conjunction(const std::string &line) {
        if (first_word(line) == "OR") or_conjunction();
    }
    void or_conjunction() {
        if (pos_ >= lines_.size()) throw StatementError("unexpected end of input");
        cs().push_buffer();
        while (pos_ < lines_.size()) {
            size_t idx = pos_;
            const std::string line = lines_[pos_++];
            std::string op = first_word(line);
            if (op == "]") break;
            if (op == "}") cs().rewind();
            else { conjunction(line); gadget(line, idx); }
        }
        auto blocks = cs().pop_buffer();
        // src/or/or_conjunction.rs:4-38
        std::vector<std::vector<LC>> lists;
        for (auto &ops : blocks) {
            std::vector<LC> cons;
            for (auto &op : ops) {
                if (op.mul) cs().replay_mul(op);
                else cons.push_back(op.a);
            }
            lists.push_back(std::move(cons));
        }
        if (lists.empty()) return;
        std::vector<std::vector<size_t>> combos;
        for (size_t i = 0; i < lists[0].size(); i++) combos.push_back({i});
        for (size_t l = 1; l < lists.size(); l++) {
            std::vector<std::vector<size_t>> next;
            for (auto &c : combos)
                for (size_t j = 0; j < lists[l].size(); j++) { auto d = c; d.push_back(j); next.push_back(d); }
            combos.swap(next);
        }
        for (auto &c : combos) {
            LC prod = lists[0][c[0]];
            for (size_t l = 1; l < c.size(); l++) {
                auto t = cs().multiply(prod, lists[l][c[l]]);
                prod = LC::of(t.o);
            }
            cs().constrain(prod);
        }
    }
    // prove.rs:101-119 parse_gadget (get_gadget_op panics on unknown words)
    void gadget(const std::string &line, size_t index) {
        std::string op = first_word(line);
        static const char *known[] = {"OR", "HASH", "]", "BOUND", "[", "MERKLE", "}", "EQUALS", "{", "UNEQUAL",
                                      "LESS_THAN", "SET_MEMBER"};
        bool ok = false;
        for (const char *k : known) ok = ok || op == k;
        if (!ok) throw StatementError("unknown gadget: " + op);
        auto t = tokens(line);
        if (op == "BOUND") g_bound(t, index);
        else if (op == "HASH") g_hash(t, index);
        else if (op == "MERKLE") g_merkle(t, index);
        else if (op == "EQUALS") g_equals(t);
        else if (op == "LESS_THAN") g_less_than(t, index);
        else if (op == "UNEQUAL") g_unequal(t, index);
        else if (op == "SET_MEMBER") g_set_member(t, index);
    }
    static void need(const std::vector<std::string> &t, size_t n, const char *what) {
        if (t.size() != n) throw StatementError(std::string("unable to parse ") + what + " gadget");
    }

    // prove.rs:235-258 / verify.rs:163-181
    void g_bound(const std::vector<std::string> &t, size_t index) {
        need(t, 4, "BOUND");
        if (!is_witness(t[1]) || !is_instance(t[2]) || !is_instance(t[3])) throw StatementError("unable to parse BOUND gadget");
        BoundsCheck g(instance(t[2], true), instance(t[3], true));
        if (prover_) {
            const Wit &w = witness(t[1], true);
            Derived d = gadget_setup(cs(), g.preprocess(w.scalars));
            g.assemble(cs(), d, true);
            name_derived(d.size(), index, 0);
        } else {
            commitment(t[1], 0);
            Derived d{{Scalar::zero(), derived(index, 0, 0)}, {Scalar::zero(), derived(index, 1, 0)}};
            g.assemble(cs(), d, false);
        }
    }
    LC image_lc(const std::string &name) {
        if (is_witness(name)) {
            if (prover_) return LC::of(witness(name, true).vars[0]);
            return LC::of(commitment(name, 0));
        }
        return LC::cnst(be_to_scalar(instance(name, true)));
    }
    // prove.rs:260-285 / verify.rs:183-206
    void g_hash(const std::vector<std::string> &t, size_t index) {
        need(t, 3, "HASH");
        if (!is_witness(t[2]) || !(is_witness(t[1]) || is_instance(t[1]))) throw StatementError("unable to parse HASH gadget");
        MimcGadget g{image_lc(t[1])};
        if (prover_) {
            const Wit &w = witness(t[2], false);
            Derived d = gadget_setup(cs(), g.preprocess(w.scalars));
            g.assemble(cs(), w.vars, d);
            name_derived(d.size(), index, 0);
        } else {
            Derived d{{Scalar::zero(), derived(index, 0, 0)}};
            Var d2;
            if (inquire_derived(index, 1, 0, d2)) d.push_back({Scalar::zero(), d2});
            g.assemble(cs(), all_commitments(t[2]), d);
        }
    }
    // prove.rs:142-172 / verify.rs:397-415
    std::pair<Scalar, Var> hash_witness(const std::string &name, size_t index, size_t sub) {
        if (prover_) {
            const Wit &w = witness(name, false);
            Scalar image = mimc_hash(w.bytes);
            Scalar blinding = thread_entropy().random_scalar();
            Var iv = cs().commit_value(image, blinding);
            MimcGadget g{LC::of(iv)};
            Derived d = gadget_setup(cs(), g.preprocess(w.scalars));
            g.assemble(cs(), w.vars, d);
            name_derived(1 + d.size(), index, sub);
            return {image, iv};
        }
        Var iv = derived(index, 0, sub);
        Derived d{{Scalar::zero(), derived(index, 1, sub)}};
        Var d2;
        if (inquire_derived(index, 2, sub, d2)) d.push_back({Scalar::zero(), d2});
        MimcGadget{LC::of(iv)}.assemble(cs(), all_commitments(name), d);
        return {Scalar::zero(), iv};
    }
    // prove.rs:287-318 / verify.rs:208-236
    void g_merkle(const std::vector<std::string> &t, size_t index) {
        if (t.size() < 3 || !(is_witness(t[1]) || is_instance(t[1]))) throw StatementError("unable to parse MERKLE gadget");
        size_t pos = 2;
        Tree tree = parse_tree(t, pos);
        if (pos != t.size()) throw StatementError("unable to parse MERKLE gadget");
        LC root = image_lc(t[1]);
        std::vector<LC> inst, wit;
        for (auto &i : tree.inst) inst.push_back(LC::cnst(mimc_hash(instance(i, false))));
        for (size_t k = 0; k < tree.wit.size(); k++) wit.push_back(LC::of(hash_witness(tree.wit[k], index, k).second));
        LC h = merkle_parse(cs(), wit, inst, *tree.p);
        cs().constrain(h - root);
    }
    // (scalars, lcs) of a witness or instance variable
    void var_lcs(const std::string &name, std::vector<Scalar> *s, std::vector<LC> &lcs) {
        if (is_witness(name)) {
            if (prover_) {
                const Wit &w = witness(name, false);
                if (s) *s = w.scalars;
                for (Var v : w.vars) lcs.push_back(LC::of(v));
            } else {
                for (Var v : all_commitments(name)) lcs.push_back(LC::of(v));
            }
            return;
        }
        std::vector<Scalar> sc = be_to_scalars(instance(name, false));
        if (s) *s = sc;
        for (auto &x : sc) lcs.push_back(LC::cnst(x));
    }
    // prove.rs:320-342 / verify.rs:238-256
    void g_equals(const std::vector<std::string> &t) {
        need(t, 3, "EQUALS");
        std::string a = t[1], b = t[2];
        if (is_instance(a) && is_witness(b)) std::swap(a, b);
        if (!is_witness(a) || !(is_witness(b) || is_instance(b))) throw StatementError("unable to parse EQUALS gadget");
        std::vector<Var> left = prover_ ? witness(a, false).vars : all_commitments(a);
        std::vector<LC> right;
        var_lcs(b, nullptr, right);
        equality_assemble(cs(), right, left);
    }
    // prove.rs:344-366 / verify.rs:258-276
    void g_less_than(const std::vector<std::string> &t, size_t index) {
        need(t, 3, "LESS_THAN");
        if (!is_witness(t[1]) || !is_witness(t[2])) throw StatementError("unable to parse LESS_THAN gadget");
        if (prover_) {
            const Wit &l = witness(t[1], true), &r = witness(t[2], true);
            LessThan g{LC::of(l.vars[0]), LC::of(r.vars[0]), &l.scalars[0], &r.scalars[0]};
            Derived d = gadget_setup(cs(), g.preprocess());
            g.assemble(cs(), d);
            name_derived(d.size(), index, 0);
        } else {
            LessThan g{LC::of(commitment(t[1], 0)), LC::of(commitment(t[2], 0)), nullptr, nullptr};
            Derived d{{Scalar::zero(), derived(index, 0, 0)}, {Scalar::zero(), derived(index, 1, 0)}};
            g.assemble(cs(), d);
        }
    }
    // prove.rs:368-402 / verify.rs:278-307
    void g_unequal(const std::vector<std::string> &t, size_t index) {
        need(t, 3, "UNEQUAL");
        std::string a = t[1], b = t[2];
        if (is_instance(a) && is_witness(b)) std::swap(a, b);
        if (!is_witness(a) || !(is_witness(b) || is_instance(b))) throw StatementError("unable to parse UNEQUAL gadget");
        std::vector<Scalar> rs;
        std::vector<LC> rl;
        var_lcs(b, prover_ ? &rs : nullptr, rl);
        if (prover_) {
            const Wit &l = witness(a, false);
            Inequality g{rl, rs};
            Derived d = gadget_setup(cs(), g.preprocess(l.scalars));
            g.assemble(cs(), l.vars, d);
            name_derived(d.size(), index, 0);
        } else {
            std::vector<Var> left = all_commitments(a);
            Derived d;
            for (size_t k = 0; k < 2 * left.size() + 1; k++) d.push_back({Scalar::zero(), derived(index, k, 0)});
            Inequality{rl, {}}.assemble(cs(), left, d);
        }
    }
    // prove.rs:404-514 / verify.rs:309-395
    void g_set_member(const std::vector<std::string> &t, size_t index) {
        if (t.size() < 3) throw StatementError("unable to parse SET_MEMBER gadget");
        const std::string member = t[1];
        std::vector<std::string> set(t.begin() + 2, t.end());
        for (auto &e : set)
            if (!is_witness(e) && !is_instance(e)) throw StatementError("unable to parse SET_MEMBER gadget");
        if (!is_witness(member) && !is_instance(member)) throw StatementError("unable to parse SET_MEMBER gadget");
        std::vector<Scalar> ms;
        std::vector<LC> ml;
        var_lcs(member, prover_ ? &ms : nullptr, ml);
        if (ml.empty()) throw StatementError("empty SET_MEMBER value");
        Scalar mscal = prover_ ? ms[0] : Scalar::zero();
        LC mlc = ml[0];
        bool hashing = prover_ ? ms.size() > 1 : false;
        std::vector<Var> wsv;
        std::vector<Scalar> wss, iss;
        std::vector<LC> isl;
        if (!hashing) {
            for (auto &e : set) {
                if (is_witness(e)) {
                    if (prover_) {
                        const Wit &w = witness(e, false);
                        if (w.vars.size() == 1) { wss.push_back(w.scalars[0]); wsv.push_back(w.vars[0]); }
                        else hashing = true;
                    } else {
                        auto c = all_commitments(e);
                        if (c.size() == 1) wsv.push_back(c[0]);
                        else hashing = true;
                    }
                } else {
                    auto s = be_to_scalars(instance(e, false));
                    if (s.size() == 1) { iss.push_back(s[0]); isl.push_back(LC::cnst(s[0])); }
                    else hashing = true;
                }
            }
        }
        Derived dver;
        if (!prover_) {
            if (ml.size() > 1) hashing = true;
            for (size_t k = 0; k < set.size(); k++) dver.push_back({Scalar::zero(), derived(index, k, 0)});
        }
        if (hashing) {
            size_t hn = 1;
            if (is_witness(member)) {
                auto r = hash_witness(member, index, hn++);
                mscal = r.first;
                mlc = LC::of(r.second);
            } else {
                mscal = mimc_hash(instance(member, false));
                mlc = LC::cnst(mscal);
            }
            wsv.clear(); wss.clear(); isl.clear(); iss.clear();
            for (auto &e : set) {
                if (is_witness(e)) {
                    auto r = hash_witness(e, index, hn++);
                    wsv.push_back(r.second);
                    wss.push_back(r.first);
                } else {
                    Scalar h = mimc_hash(instance(e, false));
                    isl.push_back(LC::cnst(h));
                    iss.push_back(h);
                }
            }
        }
        SetMembership g{mlc, mscal, isl, iss};
        if (prover_) {
            Derived d = gadget_setup(cs(), g.preprocess(wss));
            g.assemble(cs(), wsv, d);
            name_derived(d.size(), index, 0);
        } else {
            g.assemble(cs(), wsv, dver);
        }
    }
};

Synthesis synthesize_prover(const std::string &instance, const std::string &witness, const std::string &gadgets) {
    Statement st(true);
    st.parse_instance(instance);
    st.parse_witness(witness);
    st.run(gadgets);
    Synthesis s;
    s.cs = std::move(st.cs_);
    s.com_names = std::move(st.com_names);
    return s;
}
Synthesis synthesize_verifier(const std::string &instance, const std::string &commitments, const std::string &gadgets) {
    Statement st(false);
    st.parse_instance(instance);
    st.parse_commitments(commitments);
    st.run(gadgets);
    Synthesis s;
    s.cs = std::move(st.cs_);
    return s;
}

}  // namespace bpg
