// State-merging evaluator of has_match (beyond the reference).
//
// The reference enumerates every branch (engine.rs:45-214): one AND chain per
// path through the AST, ORed at the end.  Config 5 of BASELINE.json
// (/^a{2,8}(bc|de)+[^xyz]$/ on 512 chars) has ~2^252 of them.  The same
// boolean is a reachability problem over content positions: push a vector
// R[p] ("some path reaches position p", an encrypted boolean) through the AST,
// merging paths that meet at the same (node, position).  The circuit is then
// polynomial in L and its depth logarithmic for fixed-width loops.
//
// Exactness against the reference enumerator follows its rules node by node:
//  * SOF / EOF pass position 0 / L only; every other node visited at p >= L
//    yields nothing (engine.rs:69-71), so nullable nodes cannot skip at the end;
//  * Repeated counts: {0 if lo = 0} U [max(1,lo), max(1,lo) + at_most - at_least]
//    with at_most = hi or L - p (the lo = 0 case allows hi + 1 repetitions);
//  * Not negates each branch condition of its operand (single-char operands);
//  * Between tests char > from (the ct_ge -> smart_gt quirk) and char <= to;
//  * a structurally present branch stays present with a FALSE value (so a
//    node behind it is still visited, e.g. for the empty-Seq panic).
// Branch counts and the reference's ct_ops / cache_hits are not reproduced
// (the reference cannot finish on the inputs this targets); ct_ops reports the
// number of DAG operations created.  Verified against the enumerator on the
// golden vectors and on fuzzed patterns (tests/test_host.py).
#include <algorithm>

#include "regex.h"

namespace fr {

namespace {

constexpr int ABSENT = -1;

class Merged {
  public:
    Merged(ValueDag& dag, size_t L) : dag_(dag), L_(L) {
        VNode t{VNode::CONST};
        t.c = 1;
        T_ = dag_.add(t);
        VNode f{VNode::CONST};
        f.c = 0;
        F_ = dag_.add(f);
    }
    using Reach = std::vector<int>;  // size L+1: ABSENT or a value id

    int T() const { return T_; }
    uint64_t ops() const { return ops_; }

    int AND(int a, int b) {
        if (a == F_ || b == F_) return F_;
        if (a == T_) return b;
        if (b == T_ || a == b) return a;
        VNode n{VNode::AND};
        n.a = std::min(a, b);
        n.b = std::max(a, b);
        return add(n);
    }
    int OR(int a, int b) {
        if (a == T_ || b == T_) return T_;
        if (a == F_) return b;
        if (b == F_ || a == b) return a;
        VNode n{VNode::OR};
        n.a = std::min(a, b);
        n.b = std::max(a, b);
        return add(n);
    }
    int NOT(int a) {
        if (a == T_) return F_;
        if (a == F_) return T_;
        VNode n{VNode::NOT};
        n.a = a;
        return add(n);
    }
    int CMP(VNode::Op op, size_t p, uint8_t c) {
        VNode n{op};
        n.pos = (int)p;
        n.c = c;
        return add(n);
    }

    // merge b into a (presence: either; value: OR)
    void merge(Reach& a, const Reach& b) {
        for (size_t q = 0; q <= L_; ++q) {
            if (b[q] == ABSENT) continue;
            a[q] = a[q] == ABSENT ? b[q] : OR(a[q], b[q]);
        }
    }
    Reach below_L(const Reach& in) const {
        Reach r = in;
        r[L_] = ABSENT;
        return r;
    }
    bool empty(const Reach& r) const {
        for (int v : r)
            if (v != ABSENT) return false;
        return true;
    }

    // the single-character condition of a width-1, single-branch node at p
    // (Char, AnyChar, Between, Range, Not of those); -2 if not of that shape
    int char_cond(const Re& re, size_t p) {
        switch (re.kind) {
            case Re::CHAR: return CMP(VNode::EQ, p, re.c);
            case Re::ANY: return T_;
            case Re::BETWEEN: return AND(CMP(VNode::GT, p, re.from), CMP(VNode::LE, p, re.to));
            case Re::RANGE: {
                int r = CMP(VNode::EQ, p, re.cs[0]);
                for (size_t i = 1; i < re.cs.size(); ++i) r = OR(r, CMP(VNode::EQ, p, re.cs[i]));
                return r;
            }
            case Re::CLASS: {
                int r = -1;
                for (size_t i = 0; i + 1 < re.cs.size(); i += 2) {
                    const uint8_t lo = re.cs[i], hi = re.cs[i + 1];
                    int item;
                    if (lo == hi) {
                        item = CMP(VNode::EQ, p, lo);
                    } else {
                        const int ge = lo == 0 ? T_ : CMP(VNode::GT, p, (uint8_t)(lo - 1));
                        const int le = hi == 255 ? T_ : CMP(VNode::LE, p, hi);
                        item = AND(ge, le);
                    }
                    r = r < 0 ? item : OR(r, item);
                }
                return r;
            }
            case Re::NOT: {
                int c = char_cond(*re.a, p);
                return c == -2 ? -2 : NOT(c);
            }
            default: return -2;
        }
    }

    // minimum and (if fixed) exact width of the strings a node consumes
    static bool fixed_width(const Re& re, size_t& w) {
        switch (re.kind) {
            case Re::CHAR:
            case Re::ANY:
            case Re::BETWEEN:
            case Re::RANGE:
            case Re::CLASS:
            case Re::NOT: w = 1; return true;
            case Re::SEQ: {
                size_t s = 0;
                for (auto& x : re.xs) {
                    size_t wx;
                    if (!fixed_width(*x, wx)) return false;
                    s += wx;
                }
                w = s;
                return !re.xs.empty();
            }
            case Re::EITHER: {
                size_t wa, wb;
                if (!fixed_width(*re.a, wa) || !fixed_width(*re.b, wb) || wa != wb) return false;
                w = wa;
                return true;
            }
            case Re::REPEATED: {
                size_t wx;
                if (!re.has_lo || !re.has_hi || re.lo != re.hi || re.lo == 0 || !fixed_width(*re.a, wx)) return false;
                w = wx * re.lo;
                return true;
            }
            default: return false;
        }
    }
    static bool has_anchor(const Re& re) {
        switch (re.kind) {
            case Re::SOF:
            case Re::EOF_: return true;
            case Re::SEQ:
                for (auto& x : re.xs)
                    if (has_anchor(*x)) return true;
                return false;
            case Re::EITHER: return has_anchor(*re.a) || has_anchor(*re.b);
            case Re::OPTIONAL:
            case Re::REPEATED:
            case Re::NOT: return re.a && has_anchor(*re.a);
            default: return false;
        }
    }
    static bool nullable_or_anchor(const Re& re) {
        switch (re.kind) {
            case Re::SOF:
            case Re::EOF_:
            case Re::OPTIONAL: return true;
            case Re::REPEATED: return !re.has_lo || re.lo == 0 || nullable_or_anchor(*re.a);
            case Re::SEQ:
                for (auto& x : re.xs)
                    if (!nullable_or_anchor(*x)) return false;
                return true;
            case Re::EITHER: return nullable_or_anchor(*re.a) || nullable_or_anchor(*re.b);
            default: return false;
        }
    }

    Reach apply(const Re& re, const Reach& in) {
        Reach out(L_ + 1, ABSENT);
        switch (re.kind) {
            case Re::SOF:  // engine.rs:52-58
                out[0] = in[0];
                return out;
            case Re::EOF_:  // :59-65
                out[L_] = in[L_];
                return out;
            default: break;
        }
        const Reach r = below_L(in);  // :69-71
        switch (re.kind) {
            case Re::CHAR:
            case Re::ANY:
            case Re::BETWEEN:
            case Re::RANGE:
            case Re::CLASS:
            case Re::NOT: {
                for (size_t p = 0; p < L_; ++p) {
                    if (r[p] == ABSENT) continue;
                    int c = char_cond(re, p);
                    if (c == -2) throw Error(FR_ERR_INVALID, "merged engine: Not over a multi-branch operand");
                    out[p + 1] = AND(r[p], c);
                }
                return out;
            }
            case Re::EITHER: {  // :94-98
                out = apply(*re.a, r);
                merge(out, apply(*re.b, r));
                return out;
            }
            case Re::OPTIONAL: {  // :184-188
                out = apply(*re.a, r);
                merge(out, r);
                return out;
            }
            case Re::SEQ: {  // :189-211
                if (re.xs.empty()) {
                    if (!empty(r)) throw Error(FR_ERR_REF_PANIC, "Seq{[]}: index out of bounds (reference panics, engine.rs:189-190)");
                    return out;
                }
                Reach cur = r;
                for (auto& x : re.xs) {
                    cur = apply(*x, cur);
                    if (empty(cur)) return cur;
                }
                return cur;
            }
            case Re::REPEATED: return repeated(re, r);
            default: throw Error(FR_ERR_REF_PANIC, "unmatched regex variant");
        }
    }

  private:
    Reach repeated(const Re& re, const Reach& r) {  // :127-183
        Reach out(L_ + 1, ABSENT);
        if (empty(r)) return out;
        const uint64_t lo = re.has_lo ? re.lo : 0;
        if (re.has_hi) {
            const uint64_t hi = re.hi;
            if (lo > hi) return out;
            // counts: {0 if lo == 0} U [max(1,lo), max(1,lo) + hi - lo]
            const uint64_t first = std::max<uint64_t>(1, lo), last = first + (hi - lo);
            if (lo == 0) merge(out, r);
            Reach lev = r;
            for (uint64_t k = 1; k <= last; ++k) {
                lev = apply(*re.a, lev);
                if (empty(lev)) break;
                if (k >= first) merge(out, lev);
            }
            return out;
        }
        // unbounded: at_most = L - p.  Exact as an unbounded closure when the
        // operand consumes at least one char per repetition (no path can then
        // reach more than L - p repetitions).  A nullable operand without anchors
        // (round 3) can also repeat empty, at every position below L and with no
        // condition: a position q reached by k <= q - p non-empty repetitions is
        // reached within the reference's counts [max(1,lo), L - p] (lo = 0: up to
        // L - p + 1) by padding with empty ones, as long as the count range of the
        // entry position p is not empty: lo <= L - p.  So the closure stays exact
        // once entries with L - p < lo are dropped (engine.rs:127-183 enumerates
        // nothing there).  An operand holding an anchor matches empty only at 0 or
        // L and stays refused.
        Reach rin = r;
        if (nullable_or_anchor(*re.a)) {
            if (has_anchor(*re.a))
                throw Error(FR_ERR_INVALID,
                            "merged engine: unbounded repetition of a nullable operand holding an anchor");
            for (size_t p = 0; p <= L_; ++p)
                if (L_ - p < lo) rin[p] = ABSENT;
        }
        if (lo == 0) merge(out, rin);
        Reach lev = rin;
        const uint64_t first = std::max<uint64_t>(1, lo);
        for (uint64_t k = 1; k <= first; ++k) {
            lev = apply(*re.a, lev);
            if (empty(lev)) return out;
        }
        merge(out, closure(*re.a, lev));
        return out;
    }

    // S* = S U apply(x, S*) for a non-nullable x, merged per position
    Reach closure(const Re& x, const Reach& s) {
        size_t w;
        if (fixed_width(x, w) && w > 0) return closure_fixed(x, s, w);
        // general: increasing positions (every repetition moves right)
        Reach acc = s;
        for (size_t p = 0; p < L_; ++p) {
            if (acc[p] == ABSENT) continue;
            Reach unit(L_ + 1, ABSENT);
            unit[p] = acc[p];
            Reach step = apply(x, unit);
            for (size_t q = p + 1; q <= L_; ++q)
                if (step[q] != ABSENT) acc[q] = acc[q] == ABSENT ? step[q] : OR(acc[q], step[q]);
        }
        return acc;
    }

    // fixed width w: x_q = s_q OR (b_q AND x_{q-w}) with b_q = [x matches at q-w],
    // a boolean linear recurrence per residue class mod w, evaluated as a
    // Kogge-Stone prefix scan of the maps f(x) = a OR (b AND x):
    //   f2 o f1 = (a2 OR (b2 AND a1), b2 AND b1)        -> depth log2(L / w)
    Reach closure_fixed(const Re& x, const Reach& s, size_t w) {
        Reach out = s;
        for (size_t r0 = 0; r0 < w && r0 <= L_; ++r0) {
            std::vector<size_t> qs;
            for (size_t q = r0; q <= L_; q += w) qs.push_back(q);
            const size_t n = qs.size();
            // presence: a position is present if s is, or its predecessor is and x fits
            std::vector<int> A(n, ABSENT), B(n, ABSENT);
            std::vector<char> present(n, 0);
            for (size_t t = 0; t < n; ++t) {
                present[t] = s[qs[t]] != ABSENT;
                if (t > 0 && present[t - 1] && qs[t - 1] + w <= L_ && qs[t - 1] < L_) {
                    // x from qs[t-1]: its single-start condition
                    Reach unit(L_ + 1, ABSENT);
                    unit[qs[t - 1]] = T_;
                    const int c = apply(x, unit)[qs[t]];
                    if (c != ABSENT) {
                        present[t] = 1;
                        B[t] = c;
                    }
                }
                A[t] = s[qs[t]] == ABSENT ? F_ : s[qs[t]];
                if (B[t] == ABSENT) B[t] = F_;
            }
            // scan over maximal runs (a position absent from s and unreachable
            // breaks the chain: B = FALSE there already)
            std::vector<int> a = A, b = B;
            for (size_t d = 1; d < n; d <<= 1) {
                std::vector<int> na = a, nb = b;
                for (size_t t = d; t < n; ++t) {
                    na[t] = OR(a[t], AND(b[t], a[t - d]));
                    nb[t] = AND(b[t], b[t - d]);
                }
                a.swap(na);
                b.swap(nb);
            }
            for (size_t t = 0; t < n; ++t)
                if (present[t]) out[qs[t]] = a[t];
        }
        return out;
    }

    int add(const VNode& n) {
        ++ops_;
        return dag_.add(n);
    }

    ValueDag& dag_;
    size_t L_;
    int T_ = -1, F_ = -1;
    uint64_t ops_ = 0;
};

}  // namespace

Recorded record_has_match_merged(ValueDag& dag, size_t L, const std::string& pattern, size_t lo, size_t hi) {
    ReP re = parse(pattern);  // engine.rs:13
    if (hi > L) hi = L;
    Merged m(dag, L);
    Merged::Reach in(L + 1, ABSENT);
    for (size_t p = lo; p < hi; ++p) in[p] = m.T();  // start offsets, engine.rs:15-18
    Merged::Reach out = m.apply(*re, in);
    int res = -1;
    uint64_t present = 0;
    for (int v : out) {
        if (v == ABSENT) continue;
        ++present;
        res = res < 0 ? v : m.OR(res, v);
    }
    Recorded r;
    if (res < 0) {  // no branch at all: ct_false (engine.rs:22-26)
        VNode f{VNode::CONST};
        f.c = 0;
        res = dag.add(f);
    }
    r.root = res;
    r.ct_ops = m.ops();
    r.cache_hits = 0;
    r.n_branches = present;  // end positions reached (merged branches)
    return r;
}

}  // namespace fr
