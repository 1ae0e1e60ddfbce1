// Value DAG -> PBS gate program.  See lower.h.
#include "lower.h"

#include <algorithm>
#include <bitset>
#include <map>
#include <queue>
#include <tuple>
#include <cstring>
#include <iterator>
#include <unordered_map>

namespace fr {

void lut_eq(uint8_t* lut, int v) {
    for (int x = 0; x < 16; ++x) lut[x] = (uint8_t)(x == v);
}
void lut_sign(uint8_t* lut, int v) {
    for (int x = 0; x < 16; ++x) lut[x] = (uint8_t)(x < v ? 0 : (x == v ? 1 : 2));
}
void lut_gt3(uint8_t* lut, bool le) {
    for (int x = 0; x < 16; ++x) {
        int sh = x / 3, sl = x % 3;
        bool gt = (sh == 2) || (sh == 1 && sl == 2);
        lut[x] = (uint8_t)(le ? !gt : gt);
    }
}
void lut_at_least(uint8_t* lut, int m) {
    for (int x = 0; x < 16; ++x) lut[x] = (uint8_t)(x >= m);
}

namespace {

struct Lit {
    int gate;
    bool neg;
    bool operator<(const Lit& o) const { return gate != o.gate ? gate < o.gate : neg < o.neg; }
    bool operator==(const Lit& o) const { return gate == o.gate && neg == o.neg; }
};
struct Form {
    enum K { CONST, LIT, AND, OR, SET } k = CONST;
    int c = 0;
    Lit lit{-1, false};
    std::vector<Lit> lits;
    int pos = -1;           // SET: content position
    std::bitset<256> set;   // SET: the characters for which the form is 1
};

inline int cblock(int pos, int blk) { return -(1 + pos * 4 + blk); }

struct KeyHash {  // FNV-1a over the words of a gate key
    size_t operator()(const std::vector<int64_t>& k) const {
        uint64_t h = 1469598103934665603ULL;
        for (int64_t w : k) h = (h ^ (uint64_t)w) * 1099511628211ULL;
        return (size_t)h;
    }
};
struct SetKey {
    int pos;
    std::bitset<256> set;
    bool operator==(const SetKey& o) const { return pos == o.pos && set == o.set; }
};
struct SetKeyHash {
    size_t operator()(const SetKey& k) const { return std::hash<std::bitset<256>>()(k.set) * 1000003u + (size_t)k.pos; }
};

struct Lowerer {
    const ValueDag& dag;
    int mode;
    Program prog;
    std::unordered_map<std::vector<int64_t>, int, KeyHash> gate_index;  // hash-consing of gates
    // expand_set results by (position, set): lowering a set creates its gates once
    // (later calls only hit gate_index), so the memo returns identical forms
    std::unordered_map<SetKey, Form, SetKeyHash> set_memo;
    std::vector<Form> memo;
    std::vector<char> done;

    Lowerer(const ValueDag& d, int m) : dag(d), mode(m), memo(d.nodes.size()), done(d.nodes.size(), 0) {
        const size_t hint = std::min<size_t>(2 * d.nodes.size(), (size_t)1 << 18);  // bounded for huge DAGs
        gate_index.reserve(hint);
        set_memo.reserve(hint / 2);
        prog.gates.reserve(hint);
    }

    int add_gate(std::vector<int64_t>&& key, PGate&& g) {
        auto it = gate_index.find(key);
        if (it != gate_index.end()) return it->second;
        prog.gates.push_back(std::move(g));
        int id = (int)prog.gates.size() - 1;
        gate_index.emplace(std::move(key), id);
        return id;
    }
    // [x_{2h} + 4 x_{2h+1} ? v] over the packed nibble of char `pos`
    int nibble_gate(int kind, int pos, int half, int v, int tag) {
        PGate g;
        g.ins = {{cblock(pos, 2 * half), 1}, {cblock(pos, 2 * half + 1), 4}};
        if (kind == 0) lut_eq(g.lut, v);
        else lut_sign(g.lut, v);
        return add_gate({1, kind, pos, half, v, tag}, std::move(g));
    }
    // arbitrary 16-entry LUT over the packed nibble (x_{2h} + 4 x_{2h+1}) of char `pos`
    // (its own index, keyed without a heap-allocated key: the lowering's most frequent lookup)
    struct NibKey {
        int32_t pos, half;
        uint64_t lut_lo, lut_hi;  // the 16 LUT bytes
        bool operator==(const NibKey& o) const {
            return pos == o.pos && half == o.half && lut_lo == o.lut_lo && lut_hi == o.lut_hi;
        }
    };
    struct NibKeyHash {
        size_t operator()(const NibKey& k) const {
            uint64_t h = (uint64_t)(uint32_t)k.pos * 0x9E3779B97F4A7C15ULL ^ (uint64_t)k.half;
            h = (h ^ k.lut_lo) * 0xBF58476D1CE4E5B9ULL;
            h = (h ^ k.lut_hi) * 0x94D049BB133111EBULL;
            return (size_t)(h ^ (h >> 31));
        }
    };
    std::unordered_map<NibKey, int, NibKeyHash> nib_index;
    int nibble_lut_gate(int pos, int half, const uint8_t* lut) {
        NibKey key{pos, half, 0, 0};
        std::memcpy(&key.lut_lo, lut, 8);
        std::memcpy(&key.lut_hi, lut + 8, 8);
        auto it = nib_index.find(key);
        if (it != nib_index.end()) return it->second;
        PGate g;
        g.ins = {{cblock(pos, 2 * half), 1}, {cblock(pos, 2 * half + 1), 4}};
        std::memcpy(g.lut, lut, 16);
        prog.gates.push_back(std::move(g));
        const int id = (int)prog.gates.size() - 1;
        nib_index.emplace(key, id);
        return id;
    }
    // Lower "char at pos is in S" (S != {} and S != all).  Characters split into
    // nibbles (hi, lo); rows = hi values grouped by their lo-set, columns = lo
    // values grouped by their hi-set.
    //  * product set (one non-empty row class): AND{[hi in H], [lo in L]} — two
    //    nibble PBS, mergeable into a parent AND;
    //  * rows x cols <= 16: two class LUTs + one PBS on (cols*row + col);
    //  * otherwise OR over row classes of AND{[hi in class], [lo in L_class]}.
    Form lower_set(int pos, const std::bitset<256>& S) {
        // row h = bits 16h..16h+15 of S, read a 64-bit word at a time
        std::bitset<16> rowset[16];
        {
            const std::bitset<256> m64(~0ull);
            for (int w = 0; w < 4; ++w) {
                const unsigned long long word = ((S >> (64 * w)) & m64).to_ullong();
                for (int q = 0; q < 4; ++q) rowset[4 * w + q] = std::bitset<16>((word >> (16 * q)) & 0xFFFFu);
            }
        }
        // row classes: distinct non-empty lo-sets (class 0 = empty)
        std::vector<std::bitset<16>> rc;
        int rowcls[16];
        for (int h = 0; h < 16; ++h) {
            rowcls[h] = 0;
            if (rowset[h].none()) continue;
            int c = -1;
            for (size_t i = 0; i < rc.size(); ++i)
                if (rc[i] == rowset[h]) c = (int)i;
            if (c < 0) { rc.push_back(rowset[h]); c = (int)rc.size() - 1; }
            rowcls[h] = c + 1;
        }
        if (rc.size() == 1) {  // product set
            uint8_t lh[16], ll[16];
            bool allh = true, alll = true;
            for (int v = 0; v < 16; ++v) {
                lh[v] = (uint8_t)(rowcls[v] != 0);
                ll[v] = (uint8_t)rc[0][v];
                allh &= lh[v] != 0;
                alll &= ll[v] != 0;
            }
            Form f;
            f.k = Form::AND;
            if (!allh) f.lits.push_back(Lit{nibble_lut_gate(pos, 1, lh), false});
            if (!alll) f.lits.push_back(Lit{nibble_lut_gate(pos, 0, ll), false});
            std::sort(f.lits.begin(), f.lits.end());
            if (f.lits.size() == 1) return lit_form(f.lits[0]);
            return f;
        }
        // column classes: distinct hi-sets of each lo value
        std::vector<std::bitset<16>> cc;
        int colcls[16];
        for (int l = 0; l < 16; ++l) {
            std::bitset<16> sig;
            for (int h = 0; h < 16; ++h) sig[h] = rowset[h][l];
            int c = -1;
            for (size_t i = 0; i < cc.size(); ++i)
                if (cc[i] == sig) c = (int)i;
            if (c < 0) { cc.push_back(sig); c = (int)cc.size() - 1; }
            colcls[l] = c;
        }
        const int R = (int)rc.size() + 1, Cn = (int)cc.size();
        if (R * Cn <= 16) {
            uint8_t lh[16], ll[16];
            for (int v = 0; v < 16; ++v) {
                lh[v] = (uint8_t)rowcls[v];
                ll[v] = (uint8_t)colcls[v];
            }
            int gh = nibble_lut_gate(pos, 1, lh), gl = nibble_lut_gate(pos, 0, ll);
            PGate g;
            g.ins = {{gh, Cn}, {gl, 1}};
            for (int v = 0; v < 16; ++v) {
                int r = v / Cn, c = v % Cn;
                // representative hi for row class r, lo for column class c
                int member = 0;
                if (r >= 1 && r < R)
                    for (int l = 0; l < 16; ++l)
                        if (colcls[l] == c) { member = rc[r - 1][l]; break; }
                g.lut[v] = (uint8_t)member;
            }
            std::vector<int64_t> key{7, gh, gl, Cn};
            for (int v = 0; v < 16; ++v) key.push_back(g.lut[v]);
            return lit_form(Lit{add_gate(std::move(key), std::move(g)), false});
        }
        Form f;
        f.k = Form::OR;
        for (size_t r = 0; r < rc.size(); ++r) {
            uint8_t lh[16], ll[16];
            for (int v = 0; v < 16; ++v) {
                lh[v] = (uint8_t)(rowcls[v] == (int)r + 1);
                ll[v] = (uint8_t)rc[r][v];
            }
            std::vector<Lit> a{Lit{nibble_lut_gate(pos, 1, lh), false}, Lit{nibble_lut_gate(pos, 0, ll), false}};
            f.lits.push_back(Lit{threshold_gate(true, a), false});
        }
        std::sort(f.lits.begin(), f.lits.end());
        return f;
    }
    // SET -> general form (cheaper of S and its complement)
    Form expand_set(const Form& f) {
        if (f.set.none()) return const_form(0);
        if (f.set.all()) return const_form(1);
        const SetKey key{f.pos, f.set};
        auto it = set_memo.find(key);
        if (it != set_memo.end()) return it->second;
        Form r = expand_set_uncached(f);
        set_memo.emplace(key, r);
        return r;
    }
    Form expand_set_uncached(const Form& f) {
        Form a = lower_set(f.pos, f.set);
        if (a.k == Form::AND || a.k == Form::LIT) return a;
        Form b = negate(lower_set(f.pos, ~f.set));
        if (b.k == Form::AND || b.k == Form::LIT) return b;
        return a;
    }
    // AND / OR of m <= 16 literals as one SIGN gate:
    //   AND: s = sum - m + 1/2 > 0 ;  OR: s = sum - 1/2 > 0   (s in (-16, 16))
    int threshold_gate(bool is_and, std::vector<Lit> lits) {
        std::sort(lits.begin(), lits.end());
        PGate g;
        g.kind = GATE_SIGN;
        int negs = 0;
        std::vector<int64_t> key{2, is_and ? 1 : 0};
        for (auto& l : lits) {
            g.ins.push_back({l.gate, l.neg ? -1 : 1});
            negs += l.neg;
            key.push_back(l.gate * 2 + l.neg);
        }
        const int m = (int)lits.size();
        g.offset = 2 * negs + (is_and ? 1 - 2 * m : -1);
        return add_gate(std::move(key), std::move(g));
    }
    Lit materialize(const Form& f0) {
        if (f0.k == Form::SET) return materialize(expand_set(f0));
        const Form& f = f0;
        if (f.k == Form::LIT) return f.lit;
        if (f.k == Form::CONST) throw Error(FR_ERR_INVALID, "lowering: cannot materialize a constant");
        bool is_and = f.k == Form::AND;
        std::vector<Lit> lits = reduce(is_and, f.lits, MAX_FANIN);
        if (lits.size() == 1) return lits[0];
        return Lit{threshold_gate(is_and, lits), false};
    }
    // levels of threshold gates (fan-in <= 16, balanced chunks) until <= keep literals remain
    std::vector<Lit> reduce(bool is_and, std::vector<Lit> lits, size_t keep) {
        while (lits.size() > keep) {
            size_t m = lits.size();
            size_t chunks = (m + MAX_FANIN - 1) / MAX_FANIN;
            std::vector<Lit> next;
            size_t start = 0;
            for (size_t c = 0; c < chunks; ++c) {
                size_t len = m / chunks + (c < m % chunks ? 1 : 0);
                std::vector<Lit> part(lits.begin() + start, lits.begin() + start + len);
                start += len;
                next.push_back(part.size() == 1 ? part[0] : Lit{threshold_gate(is_and, part), false});
            }
            lits = std::move(next);
        }
        return lits;
    }
    // the parts of a root: an OR form's literals reduced to <= max_parts, else one literal
    std::vector<Lit> parts(const Form& f0, size_t max_parts) {
        if (f0.k == Form::SET) return parts(expand_set(f0), max_parts);
        if (f0.k == Form::OR && max_parts > 1) return reduce(false, f0.lits, max_parts);
        return {materialize(f0)};
    }
    static Form lit_form(Lit l) {
        Form f;
        f.k = Form::LIT;
        f.lit = l;
        return f;
    }
    static Form const_form(int c) {
        Form f;
        f.k = Form::CONST;
        f.c = c;
        return f;
    }
    // literals of f as members of an AND (is_and) or OR list
    // (f is consumed: a same-kind form hands over its literal list)
    std::vector<Lit> members(Form&& f, bool is_and) {
        if (f.k == Form::SET) return members(expand_set(f), is_and);
        if (f.k == Form::CONST) throw Error(FR_ERR_INVALID, "lowering: constant member");
        if (f.k == Form::LIT) return {f.lit};
        if ((f.k == Form::AND) == is_and) return std::move(f.lits);
        return {materialize(f)};
    }
    // operands by value: lower_t moves a node's form in at its last use, so the long
    // AND/OR chains of has_match grow their literal lists without copies
    Form combine(bool is_and, Form a0, Form b0) {
        // same-position character sets combine exactly
        if (a0.k == Form::SET && b0.k == Form::SET && a0.pos == b0.pos) {
            Form f = std::move(a0);
            f.set = is_and ? (f.set & b0.set) : (f.set | b0.set);
            if (f.set.none()) return const_form(0);
            if (f.set.all()) return const_form(1);
            return f;
        }
        Form a = a0.k == Form::SET ? expand_set(a0) : std::move(a0);
        Form b = b0.k == Form::SET ? expand_set(b0) : std::move(b0);
        // constant folding (booleans)
        if (a.k == Form::CONST) return is_and ? (a.c ? std::move(b) : const_form(0)) : (a.c ? const_form(1) : std::move(b));
        if (b.k == Form::CONST) return is_and ? (b.c ? std::move(a) : const_form(0)) : (b.c ? const_form(1) : std::move(a));
        // member lists are sorted (forms keep their literals sorted): merge, O(|a|+|b|)
        std::vector<Lit> l0 = members(std::move(a), is_and), r = members(std::move(b), is_and);
        if (l0.size() < r.size()) std::swap(l0, r);
        if (r.size() == 1) {
            // the long folds (has_match's OR over its branches, engine.rs:22-35) add one
            // literal at a time, usually past the end: insert in place instead of copying
            // the whole list per operand (quadratic in the branch count)
            // (a form's own list is sorted, unique and free of x / !x pairs: only x's
            // neighbours can complement it)
            const Lit x = r[0];
            auto it = std::lower_bound(l0.begin(), l0.end(), x);
            if (it == l0.end() || !(*it == x)) {
                if ((it != l0.end() && it->gate == x.gate) || (it != l0.begin() && (it - 1)->gate == x.gate))
                    return const_form(is_and ? 0 : 1);  // x & !x, x | !x
                l0.insert(it, x);
            }
            if (l0.size() == 1) return lit_form(l0[0]);
            Form f;
            f.k = is_and ? Form::AND : Form::OR;
            f.lits = std::move(l0);
            return f;
        }
        std::vector<Lit> l;
        l.reserve(l0.size() + r.size());
        std::merge(l0.begin(), l0.end(), r.begin(), r.end(), std::back_inserter(l));
        l.erase(std::unique(l.begin(), l.end()), l.end());
        for (size_t i = 0; i + 1 < l.size(); ++i)
            if (l[i].gate == l[i + 1].gate) return const_form(is_and ? 0 : 1);  // x & !x, x | !x
        if (l.size() == 1) return lit_form(l[0]);
        Form f;
        f.k = is_and ? Form::AND : Form::OR;
        f.lits = std::move(l);
        return f;
    }
    Form negate(const Form& f) {
        Form g = f;
        switch (f.k) {
            case Form::SET: g.set = ~f.set; break;
            case Form::CONST: g.c = f.c ^ 1; break;
            case Form::LIT: g.lit.neg = !f.lit.neg; break;
            case Form::AND:
            case Form::OR:
                g.k = f.k == Form::AND ? Form::OR : Form::AND;
                for (auto& l : g.lits) l.neg = !l.neg;
                break;
        }
        return g;
    }

    // ---------------------------------------------------------- threshold
    std::vector<int32_t> uses;  // remaining AND/OR/NOT operand uses of each node (lower_t)
    Form take(int id) {
        if (--uses[id] <= 0) return std::move(memo[id]);
        return memo[id];
    }
    Form lower_t(int id) {
        if (done[id]) return memo[id];
        uses.assign(dag.nodes.size(), 0);
        for (const VNode& n : dag.nodes)
            if (n.op == VNode::AND || n.op == VNode::OR) {
                ++uses[n.a];
                ++uses[n.b];
            } else if (n.op == VNode::NOT) {
                ++uses[n.a];
            }
        ++uses[id];  // the root's form is returned
        // iterative post-order over AND/OR/NOT chains to avoid deep recursion
        std::vector<int> st{id};
        while (!st.empty()) {
            int x = st.back();
            if (done[x]) { st.pop_back(); continue; }
            const VNode& n = dag.nodes[x];
            bool ready = true;
            if ((n.op == VNode::AND || n.op == VNode::OR || n.op == VNode::NOT)) {
                if (!done[n.a]) { st.push_back(n.a); ready = false; }
                if (n.b >= 0 && !done[n.b]) { st.push_back(n.b); ready = false; }
            }
            if (!ready) continue;
            st.pop_back();
            Form f;
            switch (n.op) {
                case VNode::POS: throw Error(FR_ERR_INVALID, "lowering: content char used as a boolean");
                case VNode::CONST: f = const_form(n.c); break;
                case VNode::EQ:
                case VNode::GT:
                case VNode::LE: {
                    f.k = Form::SET;
                    f.pos = n.pos;
                    // {c}, {ch > c} or {ch <= c}, built word-wise
                    const std::bitset<256> all = std::bitset<256>().set();
                    if (n.op == VNode::EQ) f.set.reset().set(n.c);
                    else if (n.op == VNode::GT) f.set = all << (n.c + 1);
                    else f.set = all >> (255 - n.c);
                    break;
                }
                case VNode::AND: {
                    Form fa = take(n.a);
                    f = combine(true, std::move(fa), take(n.b));
                    break;
                }
                case VNode::OR: {
                    Form fa = take(n.a);
                    f = combine(false, std::move(fa), take(n.b));
                    break;
                }
                case VNode::NOT: f = negate(take(n.a)); break;
            }
            memo[x] = std::move(f);
            done[x] = 1;
        }
        return memo[id];
    }
    int cmp_gate(const VNode& n, int tag) {
        int hi = nibble_gate(1, n.pos, 1, n.c >> 4, tag);
        int lo = nibble_gate(1, n.pos, 0, n.c & 15, tag);
        PGate g;
        g.ins = {{hi, 3}, {lo, 1}};
        lut_gt3(g.lut, n.op == VNode::LE);
        return add_gate({3, n.op, n.pos, n.c, tag}, std::move(g));
    }

    // ---------------------------------------------------------- faithful
    // one gate group per distinct reference op
    Form lower_f(int id) {
        std::vector<int> st{id};
        while (!st.empty()) {
            int x = st.back();
            if (done[x]) { st.pop_back(); continue; }
            const VNode& n = dag.nodes[x];
            bool ready = true;
            if ((n.op == VNode::AND || n.op == VNode::OR || n.op == VNode::NOT)) {
                if (!done[n.a]) { st.push_back(n.a); ready = false; }
                if (n.b >= 0 && !done[n.b]) { st.push_back(n.b); ready = false; }
            }
            if (!ready) continue;
            st.pop_back();
            Form f;
            switch (n.op) {
                case VNode::POS: throw Error(FR_ERR_INVALID, "lowering: content char used as a boolean");
                case VNode::CONST: f = const_form(n.c); break;
                case VNode::EQ: {
                    // smart_eq: both nibble tests, then [lo + hi == 2]  (3 PBS)
                    int lo = nibble_gate(0, n.pos, 0, n.c & 15, n.c);
                    int hi = nibble_gate(0, n.pos, 1, n.c >> 4, n.c);
                    PGate g;
                    g.ins = {{lo, 1}, {hi, 1}};
                    lut_eq(g.lut, 2);
                    f = lit_form(Lit{add_gate({4, n.pos, n.c}, std::move(g)), false});
                    break;
                }
                case VNode::GT:
                case VNode::LE: f = lit_form(Lit{cmp_gate(n, n.c), false}); break;
                case VNode::AND:
                case VNode::OR: {
                    bool is_and = n.op == VNode::AND;
                    const Form& a = memo[n.a];
                    const Form& b = memo[n.b];
                    PGate g;
                    int offset = 0;
                    std::vector<int64_t> key{5, is_and, x};
                    for (const Form* o : {&a, &b}) {
                        if (o->k == Form::CONST) {
                            offset += o->c;  // trivial operand (e.g. or(false, x), execution.rs:154-164)
                        } else {
                            Lit l = materialize(*o);
                            g.ins.push_back({l.gate, l.neg ? -1 : 1});
                            offset += l.neg;
                        }
                    }
                    g.offset = 2 * offset;
                    if (is_and) lut_eq(g.lut, 2);
                    else lut_at_least(g.lut, 1);
                    f = lit_form(Lit{add_gate(std::move(key), std::move(g)), false});
                    break;
                }
                case VNode::NOT: f = negate(memo[n.a]); break;  // smart_bitxor(a, 1) on a boolean: linear
            }
            memo[x] = std::move(f);
            done[x] = 1;
        }
        return memo[id];
    }

    // ---------------------------------------------------------- faithful tree
    // The faithful gates with the reference's AND/OR chains rebalanced.
    // A chain is a maximal run of AND (or OR) nodes in which every inner node is used
    // once, by the next node of the same op: the left fold of has_match
    // (engine.rs:22-35) and the Seq / Repeated AND chains (engine.rs:127-211).  A chain
    // over m operands keeps exactly m - 1 two-input gates, as lower_f makes one per node
    // (the reference's PBS count), but they form a tree of least depth: the two
    // shallowest operands are joined first (ties in operand order).  A constant operand
    // (or(false, x) is not short-circuited, execution.rs:154-164) is joined to the
    // shallowest other operand as the same trivial-offset gate lower_f makes.
    std::vector<int32_t> glv;  // level of each gate (1 + its deepest gate input)
    int gate_level(int g) {
        for (int i = (int)glv.size(); i <= g; ++i) {
            int l = 0;
            for (const PIn& in : prog.gates[i].ins)
                if (in.src >= 0) l = std::max(l, glv[in.src]);
            glv.push_back(l + 1);
        }
        return glv[g];
    }
    struct Item {
        bool is_const;
        int c;
        Lit lit;
    };
    int pair_gate(bool is_and, const Item& p, const Item& q, int chain, int k) {
        PGate g;
        int offset = 0;
        for (const Item* o : {&p, &q}) {
            if (o->is_const) {
                offset += o->c;
            } else {
                g.ins.push_back({o->lit.gate, o->lit.neg ? -1 : 1});
                offset += o->lit.neg;
            }
        }
        g.offset = 2 * offset;
        if (is_and) lut_eq(g.lut, 2);
        else lut_at_least(g.lut, 1);
        return add_gate({9, is_and, chain, k}, std::move(g));
    }
    Form lower_ft(int id) {
        const size_t nn = dag.nodes.size();
        std::vector<int32_t> nuse(nn, 0), user(nn, -1);
        for (size_t x = 0; x < nn; ++x) {
            const VNode& n = dag.nodes[x];
            if (n.op == VNode::AND || n.op == VNode::OR) {
                ++nuse[n.a], user[n.a] = (int)x;
                ++nuse[n.b], user[n.b] = (int)x;
            } else if (n.op == VNode::NOT) {
                ++nuse[n.a], user[n.a] = (int)x;
            }
        }
        ++nuse[id];  // the root is used by the result
        auto absorbed = [&](int x) {
            const VNode& n = dag.nodes[x];
            return (n.op == VNode::AND || n.op == VNode::OR) && nuse[x] == 1 && user[x] >= 0 &&
                   dag.nodes[user[x]].op == n.op;
        };
        std::vector<int> st{id};
        while (!st.empty()) {
            int x = st.back();
            if (done[x]) { st.pop_back(); continue; }
            const VNode& n = dag.nodes[x];
            bool ready = true;
            if ((n.op == VNode::AND || n.op == VNode::OR || n.op == VNode::NOT)) {
                if (!done[n.a]) { st.push_back(n.a); ready = false; }
                if (n.b >= 0 && !done[n.b]) { st.push_back(n.b); ready = false; }
            }
            if (!ready) continue;
            st.pop_back();
            Form f;
            switch (n.op) {
                case VNode::POS: throw Error(FR_ERR_INVALID, "lowering: content char used as a boolean");
                case VNode::CONST: f = const_form(n.c); break;
                case VNode::EQ:
                case VNode::GT:
                case VNode::LE:
                    lower_f(x);  // the comparison gates are lower_f's (it fills memo[x], done[x])
                    continue;
                case VNode::NOT: f = negate(memo[n.a]); break;
                case VNode::AND:
                case VNode::OR: {
                    if (absorbed(x)) break;  // an inner link: its chain root gathers its operands
                    const bool is_and = n.op == VNode::AND;
                    // the chain's operands, left to right
                    std::vector<Item> leaves;
                    std::vector<int> ds{n.b, n.a};
                    while (!ds.empty()) {
                        int y = ds.back();
                        ds.pop_back();
                        if (absorbed(y) && user[y] >= 0) {
                            ds.push_back(dag.nodes[y].b);
                            ds.push_back(dag.nodes[y].a);
                            continue;
                        }
                        const Form& o = memo[y];
                        if (o.k == Form::CONST) leaves.push_back(Item{true, o.c, Lit{-1, false}});
                        else leaves.push_back(Item{false, 0, materialize(o)});
                    }
                    // least-depth binary tree: join the two shallowest operands first
                    using QE = std::tuple<int, int, int>;  // (level, order, item index)
                    std::priority_queue<QE, std::vector<QE>, std::greater<QE>> q;
                    std::vector<Item> items;
                    std::vector<Item> consts;
                    int order = 0;
                    for (const Item& it : leaves) {
                        if (it.is_const) { consts.push_back(it); continue; }
                        items.push_back(it);
                        q.emplace(gate_level(it.lit.gate), order++, (int)items.size() - 1);
                    }
                    int k = 0;
                    auto join = [&](const Item& p, const Item& r) {
                        int g = pair_gate(is_and, p, r, x, k++);
                        items.push_back(Item{false, 0, Lit{g, false}});
                        q.emplace(gate_level(g), order++, (int)items.size() - 1);
                    };
                    size_t c0 = 0;
                    if (q.empty()) {
                        // every operand's value is a constant (a short-circuit returns its
                        // operand under a new key, execution.rs:121-164, so the op above it is
                        // real): lower_f's input-free gate, as the first join
                        if (consts.size() < 2) throw Error(FR_ERR_INVALID, "lowering: one-operand chain");
                        join(consts[0], consts[1]);
                        c0 = 2;
                    }
                    for (size_t ci = c0; ci < consts.size(); ++ci) {
                        const Item& c = consts[ci];
                        auto [lv, od, ix] = q.top();
                        q.pop();
                        (void)lv, (void)od;
                        join(items[ix], c);
                    }
                    while (q.size() > 1) {
                        auto [l1, o1, i1] = q.top();
                        q.pop();
                        auto [l2, o2, i2] = q.top();
                        q.pop();
                        (void)l1, (void)l2;
                        // operand order as in the chain (the earlier one first)
                        if (o1 < o2) join(items[i1], items[i2]);
                        else join(items[i2], items[i1]);
                    }
                    f = lit_form(items[std::get<2>(q.top())].lit);
                    break;
                }
            }
            memo[x] = std::move(f);
            done[x] = 1;
        }
        return memo[id];
    }
};

}  // namespace

void compute_levels(Program& prog) {
    int maxl = 0;
    std::vector<size_t> width;
    for (auto& g : prog.gates) {
        int l = 0;
        for (auto& in : g.ins)
            if (in.src >= 0) l = std::max(l, prog.gates[in.src].level);
        g.level = l + 1;
        maxl = std::max(maxl, g.level);
        if ((size_t)g.level >= width.size()) width.resize(g.level + 1, 0);
        width[g.level]++;
    }
    prog.levels = maxl;
    prog.max_width = 0;
    for (auto w : width) prog.max_width = std::max(prog.max_width, w);
}

Program lower(const ValueDag& dag, int root, int mode, int max_parts) {
    if (max_parts < 1 || max_parts > MAX_FANIN) throw Error(FR_ERR_INVALID, "lowering: parts must be in [1, 16]");
    Lowerer lw(dag, mode);
    Form f = mode == FR_LOWER_FAITHFUL ? lw.lower_f(root)
             : mode == FR_LOWER_FAITHFUL_TREE ? lw.lower_ft(root) : lw.lower_t(root);
    Program& p = lw.prog;
    if (f.k == Form::SET) f = lw.expand_set(f);  // (an empty or full set is a constant)
    if (f.k == Form::CONST) {
        p.outs.push_back(ProgOut{-1, 0, f.c});
    } else {
        for (const Lit& l : lw.parts(f, (size_t)max_parts))
            p.outs.push_back(ProgOut{l.gate, l.neg ? -1 : 1, l.neg ? 1 : 0});
    }
    // drop gates not reachable from the outputs (e.g. materialized then merged)
    std::vector<char> live(p.gates.size(), 0);
    for (const ProgOut& o : p.outs) {
        if (o.gate < 0) continue;
        std::vector<int> st{o.gate};
        while (!st.empty()) {
            int g = st.back();
            st.pop_back();
            if (live[g]) continue;
            live[g] = 1;
            for (auto& in : p.gates[g].ins)
                if (in.src >= 0 && !live[in.src]) st.push_back(in.src);
        }
    }
    std::vector<int> remap(p.gates.size(), -1);
    Program out;
    for (size_t g = 0; g < p.gates.size(); ++g) {
        if (!live[g]) continue;
        PGate ng = std::move(p.gates[g]);
        for (auto& in : ng.ins)
            if (in.src >= 0) in.src = remap[in.src];
        remap[g] = (int)out.gates.size();
        out.gates.push_back(std::move(ng));
    }
    for (ProgOut o : p.outs) {
        if (o.gate >= 0) o.gate = remap[o.gate];
        out.outs.push_back(o);
    }
    out.out_gate = out.outs[0].gate;
    out.out_w = out.outs[0].w;
    out.out_const = out.outs[0].cst;
    compute_levels(out);
    return out;
}

int eval_program(const Program& prog, const uint8_t* content, size_t L) {
    std::vector<int> parts;
    return eval_program_parts(prog, content, L, parts);
}

int eval_program_parts(const Program& prog, const uint8_t* content, size_t L, std::vector<int>& parts) {
    std::vector<int> val(prog.gates.size(), 0);
    for (size_t g = 0; g < prog.gates.size(); ++g) {
        const PGate& G = prog.gates[g];
        int s = G.offset;  // half units
        for (auto& in : G.ins) {
            int v;
            if (in.src >= 0) {
                v = val[in.src];
            } else {
                int cb = -in.src - 1;
                size_t pos = (size_t)(cb / 4);
                if (pos >= L) throw Error(FR_ERR_INVALID, "program references content past its end");
                v = (content[pos] >> (2 * (cb % 4))) & 3;
            }
            s += 2 * in.w * v;
        }
        if (G.kind == GATE_SIGN) {
            if ((s & 1) == 0 || s <= -32 || s >= 32) throw Error(FR_ERR_INVALID, "sign gate input out of (-16, 16) or integral");
            val[g] = s > 0 ? 1 : 0;
        } else {
            if ((s & 1) || s < 0 || s >= 32) throw Error(FR_ERR_INVALID, "program lincomb out of the 16-value message space");
            val[g] = G.lut[s / 2];
        }
    }
    parts.clear();
    if (prog.outs.size() > 1) {
        int any = 0;
        for (const ProgOut& o : prog.outs) {
            parts.push_back(o.gate < 0 ? o.cst : o.cst + o.w * val[o.gate]);
            any |= parts.back();
        }
        return any;
    }
    parts.push_back(prog.out_gate < 0 ? prog.out_const : prog.out_const + prog.out_w * val[prog.out_gate]);
    return parts[0];
}

}  // namespace fr
