// Host C++ restatement of the reference regex layer.
//   parser:      src/regex/parser.rs:146-351 (combine 4.6.6 commit semantics)
//   enumerator:  src/regex/engine.rs:45-214
//   driver:      src/regex/engine.rs:8-42
//   Execution:   src/regex/execution.rs:64-222
#include "regex.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <sstream>
#include <vector>

namespace fr {

// =================================================================== AST
// appends into one string (a small frame per level: the syntax tree may be
// MAX_AST_DEPTH deep, e.g. a long alternation's right-nested Either chain)
static void to_string_into(const Re& r, std::string& o) {
    auto num = [&](uint64_t v) { o += std::to_string(v); };
    switch (r.kind) {
        case Re::SOF: o += "SOF"; break;
        case Re::EOF_: o += "EOF"; break;
        case Re::ANY: o += "Any"; break;
        case Re::CHAR: o += "Char("; num(r.c); o += ")"; break;
        case Re::BETWEEN: o += "Between("; num(r.from); o += ","; num(r.to); o += ")"; break;
        case Re::RANGE:
            o += "Range(";
            for (size_t i = 0; i < r.cs.size(); ++i) { if (i) o += ","; num(r.cs[i]); }
            o += ")";
            break;
        case Re::NOT: o += "Not("; to_string_into(*r.a, o); o += ")"; break;
        case Re::EITHER: o += "Either("; to_string_into(*r.a, o); o += ","; to_string_into(*r.b, o); o += ")"; break;
        case Re::OPTIONAL: o += "Optional("; to_string_into(*r.a, o); o += ")"; break;
        case Re::REPEATED:
            o += "Repeated(";
            to_string_into(*r.a, o);
            o += ",";
            if (r.has_lo) num(r.lo); else o += "_";
            o += ",";
            if (r.has_hi) num(r.hi); else o += "_";
            o += ")";
            break;
        case Re::SEQ:
            o += "Seq(";
            for (size_t i = 0; i < r.xs.size(); ++i) { if (i) o += ","; to_string_into(*r.xs[i], o); }
            o += ")";
            break;
        case Re::CLASS:
            o += "Class(";
            for (size_t i = 0; i + 1 < r.cs.size(); i += 2) { if (i) o += ","; num(r.cs[i]); o += "-"; num(r.cs[i + 1]); }
            o += ")";
            break;
    }
}
std::string to_string(const Re& r) {
    std::string o;
    to_string_into(r, o);
    return o;
}

// Depth of a syntax tree, without recursion (explicit stack).
static size_t ast_depth(const Re& root) {
    size_t best = 0;
    std::vector<std::pair<const Re*, size_t>> st{{&root, 1}};
    while (!st.empty()) {
        auto [r, d] = st.back();
        st.pop_back();
        best = std::max(best, d);
        if (r->a) st.push_back({r->a.get(), d + 1});
        if (r->b) st.push_back({r->b.get(), d + 1});
        for (auto& x : r->xs) st.push_back({x.get(), d + 1});
    }
    return best;
}

static ReP mk(Re::Kind k) {
    auto r = std::make_shared<Re>();
    r->kind = k;
    return r;
}
static ReP mk_char(uint8_t c) {
    auto r = std::make_shared<Re>();
    r->kind = Re::CHAR;
    r->c = c;
    return r;
}

// case_insensitive, parser.rs:44-81: only Char is folded.
static ReP fold_case(const ReP& n) {
    auto r = std::make_shared<Re>(*n);
    switch (n->kind) {
        case Re::CHAR: {
            r->kind = Re::RANGE;
            uint8_t c = n->c;
            r->cs = {c};
            if (c >= 'a' && c <= 'z') r->cs.push_back((uint8_t)(c - 32));
            else if (c >= 'A' && c <= 'Z') r->cs.push_back((uint8_t)(c + 32));
            break;
        }
        case Re::NOT:
        case Re::OPTIONAL:
        case Re::REPEATED: r->a = fold_case(n->a); break;
        case Re::EITHER: r->a = fold_case(n->a); r->b = fold_case(n->b); break;
        case Re::SEQ:
            for (auto& x : r->xs) x = fold_case(x);
            break;
        default: break;
    }
    return r;
}

// =============================================================== parser
// Every rule returns {ok, committed, pos, node}: combine's "consumed" status.
// choice/many/optional propagate committed errors; attempt() clears them.
namespace {
struct PR {
    bool ok = false;
    bool committed = false;
    size_t pos = 0;
    ReP node;
};
inline PR ok(ReP n, size_t p) { PR r; r.ok = true; r.pos = p; r.node = std::move(n); return r; }
inline PR fail(bool committed) { PR r; r.committed = committed; return r; }

// Nesting limit of the parser (groups, bracket negations; an alternation's '|' chain is a
// loop and does not count): the recursive descent below,
// like the reference's combine parser, takes stack per level, so a hostile pattern could
// exhaust the caller's stack; past this depth the pattern is refused (FR_ERR_INVALID, a
// limit of this build: the reference would overflow its stack instead).
constexpr int MAX_NEST = 512;
// Depth limit of the syntax tree itself (every consumer -- enumerator, recorder, merged
// engine, printer -- walks it recursively): an alternation of n terms is an Either chain of
// depth n, so flat alternations up to ~4,000 terms are taken (the group limit above does
// not count them); deeper trees are refused with FR_ERR_INVALID, a limit of this build.
constexpr size_t MAX_AST_DEPTH = 4096;

struct Parser {
    const std::string& s;
    const bool ext;  // FR_GRAMMAR_EXT
    // Packrat memo: regex/term/factor/atom are pure functions of the position, but the
    // reference's grammar tries atom up to four times per factor (attempt(atom '?'),
    // three attempts of repeated, atom) and term twice per regex, so a plain recursive
    // descent takes ~5^depth calls on nested groups ("((((((((((a))))))))))" ~10^7, as
    // the reference does); memoised, every (rule, position) is parsed once.
    std::vector<PR> m_regex, m_term, m_factor, m_atom;
    std::vector<char> h_regex, h_term, h_factor, h_atom;
    int depth = 0;
    Parser(const std::string& str, bool e)
        : s(str), ext(e), m_regex(str.size() + 1), m_term(str.size() + 1), m_factor(str.size() + 1),
          m_atom(str.size() + 1), h_regex(str.size() + 1, 0), h_term(str.size() + 1, 0),
          h_factor(str.size() + 1, 0), h_atom(str.size() + 1, 0) {}
    struct Nest {  // one nesting level (restored on every exit)
        int& d;
        explicit Nest(int& dd) : d(dd) {
            if (++d > MAX_NEST)
                throw Error(FR_ERR_INVALID, "pattern nests deeper than " + std::to_string(MAX_NEST) + " levels");
        }
        ~Nest() { --d; }
    };
    template <class Fn>
    PR memo(std::vector<PR>& m, std::vector<char>& h, size_t i, Fn&& fn) {
        if (i < h.size() && h[i]) return m[i];
        PR r = fn();
        if (i < h.size()) {
            m[i] = r;
            h[i] = 1;
        }
        return r;
    }
    bool at(size_t i, char ch) const { return i < s.size() && s[i] == ch; }
    static bool letter(unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'); }
    static bool nonesc(unsigned char c) {  // parser.rs:252-254
        static const char* syms = "&;:,`~-_!@#%'\"";
        for (const char* p = syms; *p; ++p)
            if ((unsigned char)*p == c) return true;
        return false;
    }
    bool is_letter(size_t i) const { return i < s.size() && letter((unsigned char)s[i]); }
    bool is_digit(size_t i) const { return i < s.size() && s[i] >= '0' && s[i] <= '9'; }

    static uint64_t parse_digits(const std::string& d) {  // parser.rs:349-351
        if (d.empty()) throw Error(FR_ERR_REF_PANIC, "parse_digits: empty digit string (reference panics)");
        unsigned __int128 v = 0;
        for (char ch : d) {
            v = v * 10 + (unsigned)(ch - '0');
            if (v >> 64) throw Error(FR_ERR_REF_PANIC, "parse_digits: usize overflow (reference panics)");
        }
        return (uint64_t)v;
    }

    // regex := attempt(term '|' regex) | term           (parser.rs:208-222)
    PR regex(size_t i) {
        return memo(m_regex, h_regex, i, [&] { return regex_(i); });
    }
    // The right recursion runs as a loop, so an alternation of any length takes no stack
    // per alternative (only groups and bracket negations count as nesting):
    // t_k = term(p_k), p_(k+1) = t_k.pos + 1 while t_k is followed by '|'; then from the
    // last alternative back, regex(p_k) = Either(t_k, regex(p_(k+1))) if that succeeded,
    // else t_k (attempt() restores the position: the '|' is left unconsumed).
    PR regex_(size_t i) {
        std::vector<size_t> ps{i};
        std::vector<PR> ts;
        for (;;) {
            const size_t p = ps.back();
            if (ps.size() > 1 && p < h_regex.size() && h_regex[p]) break;  // regex(p) already known
            ts.push_back(term(p));
            const PR& t = ts.back();
            if (!(t.ok && at(t.pos, '|'))) break;
            ps.push_back(t.pos + 1);
        }
        // r = regex(ps[K]) for the last position reached
        size_t K = ps.size() - 1;
        PR r = ts.size() == ps.size() ? ts.back() : m_regex[ps[K]];
        if (ts.size() == ps.size()) {
            if (ps[K] < h_regex.size()) m_regex[ps[K]] = r, h_regex[ps[K]] = 1;
        }
        for (size_t k = K; k-- > 0;) {
            const PR& t = ts[k];
            if (r.ok) {
                auto e = mk(Re::EITHER);
                auto m = std::const_pointer_cast<Re>(e);
                m->a = t.node;
                m->b = r.node;
                r = ok(e, r.pos);
            } else {
                r = t;
            }
            if (k > 0 && ps[k] < h_regex.size()) m_regex[ps[k]] = r, h_regex[ps[k]] = 1;
        }
        return r;
    }
    // term := many(factor); one factor is returned unwrapped (parser.rs:224-236)
    PR term(size_t i) {
        return memo(m_term, h_term, i, [&] { return term_(i); });
    }
    PR term_(size_t i) {
        std::vector<ReP> xs;
        size_t j = i;
        for (;;) {
            PR f = factor(j);
            if (!f.ok) {
                if (f.committed) return fail(true);
                break;
            }
            xs.push_back(f.node);
            j = f.pos;
        }
        if (xs.size() == 1) return ok(xs[0], j);
        auto q = std::make_shared<Re>();
        q->kind = Re::SEQ;
        q->xs = std::move(xs);
        return ok(q, j);
    }
    // factor := attempt(atom '?') | attempt(repeated) | atom   (parser.rs:238-250)
    PR factor(size_t i) {
        return memo(m_factor, h_factor, i, [&] { return factor_(i); });
    }
    PR factor_(size_t i) {
        {
            PR a = atom(i);
            if (a.ok && at(a.pos, '?')) {
                auto q = std::make_shared<Re>();
                q->kind = Re::OPTIONAL;
                q->a = a.node;
                return ok(q, a.pos + 1);
            }
        }
        {
            PR r = repeated(i);
            if (r.ok) return r;
        }
        return atom(i);
    }
    // atom (parser.rs:256-269)
    PR atom(size_t i) {
        return memo(m_atom, h_atom, i, [&] { return atom_(i); });
    }
    PR atom_(size_t i) {
        if (at(i, '.')) return ok(mk(Re::ANY), i + 1);
        if (at(i, '\\') && i + 1 < s.size()) return ok(mk_char((uint8_t)s[i + 1]), i + 2);
        if (i < s.size() && (letter((unsigned char)s[i]) || nonesc((unsigned char)s[i])))
            return ok(mk_char((uint8_t)s[i]), i + 1);
        if (ext && is_digit(i)) return ok(mk_char((uint8_t)s[i]), i + 1);  // extension: bare digits
        if (at(i, '[')) {
            PR r = range(i + 1);
            if (r.ok && at(r.pos, ']')) return ok(r.node, r.pos + 1);
            if (!ext) return fail(true);
            // extension: attempt(reference class) failed -> general class
            PR x = ext_class(i + 1);
            if (!x.ok || !at(x.pos, ']')) return fail(true);
            return ok(x.node, x.pos + 1);
        }
        if (at(i, '(')) {
            Nest nest(depth);
            PR r = regex(i + 1);
            if (!r.ok) return fail(true);
            if (!at(r.pos, ')')) return fail(true);
            return ok(r.node, r.pos + 1);
        }
        return fail(false);
    }
    // range (parser.rs:279-294)
    PR range(size_t i) {
        if (at(i, '^')) {
            Nest nest(depth);
            PR r = range(i + 1);
            if (!r.ok) return fail(true);
            auto q = std::make_shared<Re>();
            q->kind = Re::NOT;
            q->a = r.node;
            return ok(q, r.pos);
        }
        if (is_letter(i) && at(i + 1, '-') && is_letter(i + 2)) {
            auto q = std::make_shared<Re>();
            q->kind = Re::BETWEEN;
            q->from = (uint8_t)s[i];
            q->to = (uint8_t)s[i + 2];
            return ok(q, i + 3);
        }
        if (is_letter(i)) {
            auto q = std::make_shared<Re>();
            q->kind = Re::RANGE;
            size_t j = i;
            while (is_letter(j)) q->cs.push_back((uint8_t)s[j++]);
            return ok(q, j);
        }
        return fail(false);
    }
    // grammar extension: class := '^' class | item+ ; item := cc '-' cc | cc ;
    // cc := letter | digit | '\\' byte | one of the 14 symbols except '-'
    bool class_char(size_t i, uint8_t& c, size_t& next) const {
        if (at(i, '\\') && i + 1 < s.size()) { c = (uint8_t)s[i + 1]; next = i + 2; return true; }
        if (i < s.size() && (letter((unsigned char)s[i]) || is_digit(i) || (nonesc((unsigned char)s[i]) && s[i] != '-'))) {
            c = (uint8_t)s[i];
            next = i + 1;
            return true;
        }
        return false;
    }
    PR ext_class(size_t i) {
        if (at(i, '^')) {
            Nest nest(depth);
            PR r = ext_class(i + 1);
            if (!r.ok) return fail(true);
            auto q = std::make_shared<Re>();
            q->kind = Re::NOT;
            q->a = r.node;
            return ok(q, r.pos);
        }
        auto q = std::make_shared<Re>();
        q->kind = Re::CLASS;
        size_t j = i;
        uint8_t lo, hi;
        size_t n1, n2;
        while (class_char(j, lo, n1)) {
            if (at(n1, '-') && class_char(n1 + 1, hi, n2)) {
                if (hi < lo) throw Error(FR_ERR_PARSE, "character class range out of order");
                j = n2;
            } else {
                hi = lo;
                j = n1;
            }
            q->cs.push_back(lo);
            q->cs.push_back(hi);
        }
        if (q->cs.empty()) return fail(j != i);
        return ok(q, j);
    }
    // repeated (parser.rs:296-347); always called under attempt() by factor,
    // so only success or panic is observable.
    PR repeated(size_t i) {
        {  // attempt(atom ('*'|'+'))
            PR a = atom(i);
            if (a.ok && (at(a.pos, '*') || at(a.pos, '+'))) {
                auto q = std::make_shared<Re>();
                q->kind = Re::REPEATED;
                q->a = a.node;
                if (s[a.pos] == '+') { q->has_lo = true; q->lo = 1; }
                return ok(q, a.pos + 1);
            }
        }
        {  // attempt(atom '{' digits '}')
            PR a = atom(i);
            if (a.ok && at(a.pos, '{')) {
                size_t j = a.pos + 1;
                std::string d;
                while (is_digit(j)) d.push_back(s[j++]);
                if (at(j, '}')) {
                    uint64_t n = parse_digits(d);
                    auto q = std::make_shared<Re>();
                    q->kind = Re::REPEATED;
                    q->a = a.node;
                    q->has_lo = q->has_hi = true;
                    q->lo = q->hi = n;
                    return ok(q, j + 1);
                }
            }
        }
        {  // atom '{' digits? ',' digits? '}'
            PR a = atom(i);
            if (!a.ok) return fail(a.committed);
            if (!at(a.pos, '{')) return fail(true);
            size_t j = a.pos + 1;
            std::string lo, hi;
            while (is_digit(j)) lo.push_back(s[j++]);
            if (!at(j, ',')) return fail(true);
            ++j;
            while (is_digit(j)) hi.push_back(s[j++]);
            if (!at(j, '}')) return fail(true);
            auto q = std::make_shared<Re>();
            q->kind = Re::REPEATED;
            q->a = a.node;
            if (!lo.empty()) { q->has_lo = true; q->lo = parse_digits(lo); }
            if (!hi.empty()) { q->has_hi = true; q->hi = parse_digits(hi); }
            return ok(q, j + 1);
        }
    }
};
}  // namespace

static thread_local int g_grammar = FR_GRAMMAR_REFERENCE;
int current_grammar() { return g_grammar; }
GrammarScope::GrammarScope(int grammar) : prev_(g_grammar) { g_grammar = grammar; }
GrammarScope::~GrammarScope() { g_grammar = prev_; }

ReP parse(const std::string& pattern) { return parse(pattern, g_grammar); }

ReP parse(const std::string& pattern, int grammar) {
    if (grammar != FR_GRAMMAR_REFERENCE && grammar != FR_GRAMMAR_EXT) throw Error(FR_ERR_INVALID, "unknown grammar");
    Parser ps(pattern, grammar == FR_GRAMMAR_EXT);
    const std::string& s = pattern;
    size_t i = 0;
    if (!ps.at(0, '/')) throw Error(FR_ERR_PARSE, "failed to parse regular expression");
    i = 1;
    bool sof = false, eof = false;
    if (ps.at(i, '^')) { sof = true; ++i; }
    PR r = ps.regex(i);
    if (!r.ok) throw Error(FR_ERR_PARSE, "failed to parse regular expression");
    i = r.pos;
    if (ps.at(i, '$')) { eof = true; ++i; }
    if (!ps.at(i, '/')) throw Error(FR_ERR_PARSE, "failed to parse regular expression");
    ++i;
    bool ci = false;
    if (ps.at(i, 'i')) { ci = true; ++i; }
    ReP re = r.node;
    if (ast_depth(*re) > MAX_AST_DEPTH)
        throw Error(FR_ERR_INVALID, "pattern's syntax tree is deeper than " + std::to_string(MAX_AST_DEPTH) +
                                        " levels (each alternative of an alternation is one level)");
    if (sof || eof) {
        auto q = std::make_shared<Re>();
        q->kind = Re::SEQ;
        if (sof) q->xs.push_back(mk(Re::SOF));
        q->xs.push_back(re);
        if (eof) q->xs.push_back(mk(Re::EOF_));
        re = q;
    }
    if (ci) re = fold_case(re);
    if (i != s.size())
        throw Error(FR_ERR_PARSE, "failed to parse regular expression, unexpected token at start of: " + s.substr(i));
    return re;
}

// ============================================================ value DAG
static inline uint64_t mix(uint64_t h, uint64_t v) {
    h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
    return h;
}

int ValueDag::add(const VNode& n) {
    const uint64_t h =
        mix(mix(mix(mix(mix(0, n.op), (uint64_t)(int64_t)n.a), (uint64_t)(int64_t)n.b), (uint64_t)n.pos), n.c);
    return index_.find_or_add(
        h,
        [&](int id) {
            const VNode& m = nodes[id];
            return m.op == n.op && m.a == n.a && m.b == n.b && m.pos == n.pos && m.c == n.c;
        },
        [&] {
            nodes.push_back(n);
            return (int)nodes.size() - 1;
        });
}

int ValueDag::eval(int id, const uint8_t* content, std::vector<int16_t>& memo) const {
    if (memo.size() < nodes.size()) memo.resize(nodes.size(), -1);
    // iterative post-order to avoid deep recursion on long OR chains
    std::vector<int> st{id};
    while (!st.empty()) {
        int x = st.back();
        if (memo[x] >= 0) { st.pop_back(); continue; }
        const VNode& n = nodes[x];
        bool ready = true;
        if (n.a >= 0 && memo[n.a] < 0) { st.push_back(n.a); ready = false; }
        if (n.b >= 0 && memo[n.b] < 0) { st.push_back(n.b); ready = false; }
        if (!ready) continue;
        int v = 0;
        switch (n.op) {
            case VNode::POS: v = content[n.pos]; break;
            case VNode::CONST: v = n.c; break;
            case VNode::EQ: v = content[n.pos] == n.c; break;
            case VNode::GT: v = content[n.pos] > n.c; break;
            case VNode::LE: v = content[n.pos] <= n.c; break;
            case VNode::AND: v = memo[n.a] & memo[n.b]; break;
            case VNode::OR: v = memo[n.a] | memo[n.b]; break;
            case VNode::NOT: v = memo[n.a] ^ 1; break;
        }
        memo[x] = (int16_t)v;
        st.pop_back();
    }
    return memo[id];
}

// ============================================================ Execution
int Execution::key(Tag t, int64_t a, int64_t b) {
    const uint64_t h = mix(mix(mix(0, t), (uint64_t)a), (uint64_t)b);
    return key_index_.find_or_add(
        h,
        [&](int id) {
            const KeyRec& k = keys_[id];
            return k.t == t && k.a == a && k.b == b;
        },
        [&] {
            keys_.push_back({t, a, b});
            return (int)keys_.size() - 1;
        });
}
int Execution::const_of(int k) const { return keys_[k].t == K_CONST ? (int)keys_[k].a : -1; }

template <class F>
Val Execution::with_cache(int k, F&& f) {  // execution.rs:212-222
    if ((size_t)k < cache_.size() && cache_[k] >= 0) {
        ++cache_hits_;
        return {cache_[k], k};
    }
    ++ct_ops_;
    int v = f();
    if ((size_t)k >= cache_.size()) cache_.resize(std::max<size_t>(2 * cache_.size(), (size_t)k + 1), -1);
    cache_[k] = v;
    return {v, k};
}

Val Execution::ct_constant(uint8_t c) {  // execution.rs:197-210
    VNode n{VNode::CONST};
    n.c = c;
    return {dag_.add(n), key(K_CONST, c)};
}
Val Execution::ct_pos(int at) {
    VNode n{VNode::POS};
    n.pos = at;
    return {dag_.add(n), key(K_POS, at)};
}

static VNode cmp_node(VNode::Op op, const ValueDag& d, const Val& a, const Val& b) {
    const VNode& x = d.nodes[a.value];
    const VNode& y = d.nodes[b.value];
    if (x.op != VNode::POS || y.op != VNode::CONST)
        throw Error(FR_ERR_INVALID, "comparison operands must be (content char, constant)");
    VNode n{op};
    n.pos = x.pos;
    n.c = y.c;
    return n;
}

Val Execution::ct_eq(const Val& a, const Val& b) {  // execution.rs:64-79
    int k = key(K_EQ, a.key, b.key);
    return with_cache(k, [&] { return dag_.add(cmp_node(VNode::EQ, dag_, a, b)); });
}
Val Execution::ct_ge(const Val& a, const Val& b) {  // execution.rs:81-96 (smart_gt)
    int k = key(K_GE, a.key, b.key);
    return with_cache(k, [&] { return dag_.add(cmp_node(VNode::GT, dag_, a, b)); });
}
Val Execution::ct_le(const Val& a, const Val& b) {  // execution.rs:98-113
    int k = key(K_LE, a.key, b.key);
    return with_cache(k, [&] { return dag_.add(cmp_node(VNode::LE, dag_, a, b)); });
}
Val Execution::ct_and(const Val& a, const Val& b) {  // execution.rs:115-146
    int k = key(K_AND, a.key, b.key);
    int ca = const_of(a.key), cb = const_of(b.key);
    if (ca == 1) return {b.value, k};
    if (ca == 0) return {a.value, k};
    if (cb == 1) return {a.value, k};
    if (cb == 0) return {b.value, k};
    return with_cache(k, [&] {
        VNode n{VNode::AND};
        n.a = a.value;
        n.b = b.value;
        return dag_.add(n);
    });
}
Val Execution::ct_or(const Val& a, const Val& b) {  // execution.rs:148-176
    int k = key(K_OR, a.key, b.key);
    int ca = const_of(a.key), cb = const_of(b.key);
    if (ca == 1) return {a.value, k};
    if (cb == 1) return {b.value, k};
    if (ca == 0 && cb == 0) return {a.value, k};
    return with_cache(k, [&] {
        VNode n{VNode::OR};
        n.a = a.value;
        n.b = b.value;
        return dag_.add(n);
    });
}
Val Execution::ct_not(const Val& a) {  // execution.rs:178-195
    int k = key(K_NOT, a.key);
    return with_cache(k, [&] {
        VNode n{VNode::NOT};
        n.a = a.value;
        return dag_.add(n);
    });
}

// ============================================================ enumerator
static Lazy lazy(std::function<Val(Execution&)> f) {
    return std::make_shared<const std::function<Val(Execution&)>>(std::move(f));
}
static Lazy seq_and(const Lazy& prev, const Lazy& x) {  // engine.rs:197-205
    return lazy([prev, x](Execution& ex) {
        Val rp = (*prev)(ex);
        Val rx = (*x)(ex);
        return ex.ct_and(rp, rx);
    });
}

// variants still allowed in this enumeration (record_has_match's budget)
static thread_local size_t g_budget = SIZE_MAX;
static void spend(size_t n) {
    if (n > g_budget) throw Error(FR_ERR_OOM, "variant enumeration budget exceeded");
    g_budget -= n;
}

std::vector<Branch> build_branches(size_t L, const ReP& re, size_t p) {
    switch (re->kind) {  // engine.rs:51-67
        case Re::SOF:
            if (p == 0) return {{lazy([](Execution& ex) { return ex.ct_true(); }), p}};
            return {};
        case Re::EOF_:
            if (p == L) return {{lazy([](Execution& ex) { return ex.ct_true(); }), p}};
            return {};
        default: break;
    }
    if (p >= L) return {};  // engine.rs:69-71
    switch (re->kind) {
        case Re::CHAR: {  // :74-80
            uint8_t c = re->c;
            int at = (int)p;
            return {{lazy([c, at](Execution& ex) { return ex.ct_eq(ex.ct_pos(at), ex.ct_constant(c)); }), p + 1}};
        }
        case Re::ANY:  // :81
            return {{lazy([](Execution& ex) { return ex.ct_true(); }), p + 1}};
        case Re::NOT: {  // :82-93
            std::vector<Branch> out;
            for (auto& br : build_branches(L, re->a, p)) {
                Lazy f = br.f;
                out.push_back({lazy([f](Execution& ex) { return ex.ct_not((*f)(ex)); }), br.end});
            }
            return out;
        }
        case Re::EITHER: {  // :94-98
            auto l = build_branches(L, re->a, p);
            auto r = build_branches(L, re->b, p);
            l.insert(l.end(), r.begin(), r.end());
            return l;
        }
        case Re::BETWEEN: {  // :99-111
            uint8_t f = re->from, t = re->to;
            int at = (int)p;
            return {{lazy([f, t, at](Execution& ex) {
                         Val cf = ex.ct_constant(f);
                         Val ctt = ex.ct_constant(t);
                         Val ge = ex.ct_ge(ex.ct_pos(at), cf);
                         Val le = ex.ct_le(ex.ct_pos(at), ctt);
                         return ex.ct_and(ge, le);
                     }),
                     p + 1}};
        }
        case Re::RANGE: {  // :112-126
            std::vector<uint8_t> cs = re->cs;
            int at = (int)p;
            return {{lazy([cs, at](Execution& ex) {
                         Val res = ex.ct_eq(ex.ct_pos(at), ex.ct_constant(cs[0]));
                         for (size_t i = 1; i < cs.size(); ++i) {
                             Val e = ex.ct_eq(ex.ct_pos(at), ex.ct_constant(cs[i]));
                             res = ex.ct_or(res, e);
                         }
                         return res;
                     }),
                     p + 1}};
        }
        case Re::CLASS: {  // grammar extension: OR over items of [lo <= c <= hi]
            std::vector<uint8_t> cs = re->cs;
            int at = (int)p;
            return {{lazy([cs, at](Execution& ex) {
                         Val res{};
                         for (size_t i = 0; i + 1 < cs.size(); i += 2) {
                             const uint8_t lo = cs[i], hi = cs[i + 1];
                             Val item;
                             if (lo == hi) {
                                 item = ex.ct_eq(ex.ct_pos(at), ex.ct_constant(lo));
                             } else {
                                 // c >= lo as ct_ge(c, lo - 1): ct_ge is strict (execution.rs:93)
                                 Val ge = lo == 0 ? ex.ct_true() : ex.ct_ge(ex.ct_pos(at), ex.ct_constant((uint8_t)(lo - 1)));
                                 Val le = hi == 255 ? ex.ct_true() : ex.ct_le(ex.ct_pos(at), ex.ct_constant(hi));
                                 item = ex.ct_and(ge, le);
                             }
                             res = i == 0 ? item : ex.ct_or(res, item);
                         }
                         return res;
                     }),
                     p + 1}};
        }
        case Re::REPEATED: {  // :127-183
            uint64_t at_least = re->has_lo ? re->lo : 0;
            uint64_t at_most = re->has_hi ? re->hi : (uint64_t)(L - p);
            if (at_least > at_most) return {};
            std::vector<std::vector<Branch>> res;
            if (at_least == 0) res.push_back({{lazy([](Execution& ex) { return ex.ct_true(); }), p}});
            else res.push_back({});
            {
                auto q = std::make_shared<Re>();
                q->kind = Re::SEQ;
                uint64_t reps = at_least > 1 ? at_least : 1;
                if (reps > (1u << 24)) throw Error(FR_ERR_REF_PANIC, "repetition count too large (reference exhausts memory)");
                for (uint64_t r = 0; r < reps; ++r) q->xs.push_back(re->a);
                res.push_back(build_branches(L, q, p));
            }
            // (at_least+1 ..= at_most): each step extends the previous list;
            // once a step yields nothing all later ones do too.
            for (uint64_t it = at_least + 1; it <= at_most; ++it) {
                std::vector<Branch> nxt;
                for (auto& bp : res.back())
                    for (auto& bx : build_branches(L, re->a, bp.end)) nxt.push_back({seq_and(bp.f, bx.f), bx.end});
                spend(nxt.size());
                bool empty = nxt.empty();
                res.push_back(std::move(nxt));
                if (empty) break;
            }
            std::vector<Branch> out;
            for (auto& v : res) out.insert(out.end(), v.begin(), v.end());
            return out;
        }
        case Re::OPTIONAL: {  // :184-188
            auto out = build_branches(L, re->a, p);
            out.push_back({lazy([](Execution& ex) { return ex.ct_true(); }), p});
            return out;
        }
        case Re::SEQ: {  // :189-211
            if (re->xs.empty()) throw Error(FR_ERR_REF_PANIC, "Seq{[]}: index out of bounds (reference panics, engine.rs:189-190)");
            auto conts = build_branches(L, re->xs[0], p);
            for (size_t i = 1; i < re->xs.size(); ++i) {
                std::vector<Branch> nxt;
                for (auto& bp : conts)
                    for (auto& bx : build_branches(L, re->xs[i], bp.end)) nxt.push_back({seq_and(bp.f, bx.f), bx.end});
                spend(nxt.size());
                conts = std::move(nxt);
            }
            return conts;
        }
        default: break;
    }
    throw Error(FR_ERR_REF_PANIC, "unmatched regex variant");
}

Recorded record_has_match(ValueDag& dag, size_t L, const std::string& pattern, size_t lo, size_t hi,
                          size_t branch_budget) {
    ReP re = parse(pattern);  // engine.rs:13
    if (hi > L) hi = L;
    std::vector<Lazy> branches;
    struct Budget {  // restored on every exit
        explicit Budget(size_t b) : saved(g_budget) { g_budget = b; }
        ~Budget() { g_budget = saved; }
        size_t saved;
    } budget(branch_budget);
    for (size_t i = lo; i < hi; ++i) {  // engine.rs:15-18
        auto bs = build_branches(L, re, i);
        spend(bs.size());
        for (auto& b : bs) branches.push_back(b.f);
    }
    Execution ex(dag);
    Val res;
    if (branches.size() <= 1) {  // engine.rs:22-26
        res = branches.empty() ? ex.ct_false() : (*branches[0])(ex);
    } else {  // engine.rs:27-34
        res = (*branches[0])(ex);
        for (size_t i = 1; i < branches.size(); ++i) {
            Val r = (*branches[i])(ex);
            res = ex.ct_or(res, r);
        }
    }
    Recorded out;
    out.root = res.value;
    out.ct_ops = ex.ct_operations_count();
    out.cache_hits = ex.cache_hits();
    out.n_branches = branches.size();
    return out;
}

// ------------------------------------------------------------ enumeration cost
namespace {
struct DryPanic {};   // the enumeration would panic here: no count
struct DryMemory {};  // the counter's memo reached its byte bound: no count
struct DryRes {
    std::vector<std::pair<size_t, uint64_t>> ends;  // (end position, multiplicity), ascending
    uint64_t spent = 0;                             // spend() total of one call
    uint64_t size = 0;                              // branches one call returns
};
// build_branches without the branches: every case mirrors its line above; sums and
// products saturate at cap
struct Dry {
    size_t L;
    uint64_t cap;
    uint64_t mem_cap;  // bound on the memo's bytes (entries + their stored end positions)
    std::map<std::pair<const Re*, size_t>, DryRes> memo;  // node references stay valid
    uint64_t bytes = 0;
    // a memo entry: the map node (key, DryRes, links) plus 16 B per (end, multiplicity)
    static constexpr uint64_t ENTRY_BYTES = 96, END_BYTES = 16;

    uint64_t add(uint64_t a, uint64_t b) const { return a >= cap || b >= cap || a + b >= cap ? cap : a + b; }
    uint64_t mul(uint64_t a, uint64_t b) const {
        if (!a || !b) return 0;
        return a >= cap || b >= cap || a > cap / b ? cap : std::min(cap, a * b);
    }
    void put(std::map<size_t, uint64_t>& m, size_t e, uint64_t c) const {
        uint64_t& v = m[e];
        v = add(v, c);
    }
    uint64_t total(const std::map<size_t, uint64_t>& m) const {
        uint64_t t = 0;
        for (auto& [e, c] : m) t = add(t, c);
        return t;
    }
    // the branches of bb(x, end) over every (end, multiplicity) of conts; spends into *spent
    std::map<size_t, uint64_t> extend(const std::map<size_t, uint64_t>& conts, const Re* x, uint64_t* spent) {
        std::map<size_t, uint64_t> nxt;
        for (auto& [e, c] : conts) {
            const DryRes& r = bb(x, e);
            *spent = add(*spent, mul(c, r.spent));
            for (auto& [e2, c2] : r.ends) put(nxt, e2, mul(c, c2));
        }
        return nxt;
    }
    static std::map<size_t, uint64_t> as_map(const DryRes& r) { return {r.ends.begin(), r.ends.end()}; }
    DryRes done(const std::map<size_t, uint64_t>& m, uint64_t spent) const {
        DryRes r;
        r.ends.assign(m.begin(), m.end());
        r.spent = spent;
        r.size = total(m);
        return r;
    }
    const DryRes& bb(const Re* re, size_t p) {
        const auto key = std::make_pair(re, p);
        auto it = memo.find(key);
        if (it != memo.end()) return it->second;
        DryRes r = compute(re, p);
        // a huge AST x content: no count (the caller enumerates under its own budget, as
        // without the counter) rather than a memo of unbounded size.  Every entry holds up
        // to L - p + 1 end positions, so the bound is on bytes, not entries.
        bytes += ENTRY_BYTES + END_BYTES * r.ends.size();
        if (bytes > mem_cap) throw DryMemory{};
        return memo.emplace(key, std::move(r)).first->second;
    }
    DryRes compute(const Re* re, size_t p) {
        std::map<size_t, uint64_t> out;
        switch (re->kind) {
            case Re::SOF:
                if (p == 0) put(out, p, 1);
                return done(out, 0);
            case Re::EOF_:
                if (p == L) put(out, p, 1);
                return done(out, 0);
            default: break;
        }
        if (p >= L) return done(out, 0);
        switch (re->kind) {
            case Re::CHAR:
            case Re::ANY:
            case Re::BETWEEN:
            case Re::RANGE:
            case Re::CLASS: put(out, p + 1, 1); return done(out, 0);
            case Re::NOT: return bb(re->a.get(), p);
            case Re::EITHER: {
                const DryRes& l = bb(re->a.get(), p);
                uint64_t spent = l.spent;
                out = as_map(l);
                const DryRes& r = bb(re->b.get(), p);
                spent = add(spent, r.spent);
                for (auto& [e, c] : r.ends) put(out, e, c);
                return done(out, spent);
            }
            case Re::OPTIONAL: {
                const DryRes& r = bb(re->a.get(), p);
                out = as_map(r);
                put(out, p, 1);
                return done(out, r.spent);
            }
            case Re::SEQ: {
                if (re->xs.empty()) throw DryPanic{};
                const DryRes& r0 = bb(re->xs[0].get(), p);
                uint64_t spent = r0.spent;
                std::map<size_t, uint64_t> conts = as_map(r0);
                // once saturated the count is past cap whatever follows (as Repeated below)
                for (size_t i = 1; i < re->xs.size() && spent < cap; ++i) {
                    conts = extend(conts, re->xs[i].get(), &spent);
                    spent = add(spent, total(conts));
                }
                return done(conts, spent);
            }
            case Re::REPEATED: {
                const uint64_t at_least = re->has_lo ? re->lo : 0;
                const uint64_t at_most = re->has_hi ? re->hi : (uint64_t)(L - p);
                if (at_least > at_most) return done(out, 0);
                if (at_least == 0) put(out, p, 1);
                const uint64_t reps = at_least > 1 ? at_least : 1;
                if (reps > (1u << 24)) throw DryPanic{};
                // the Seq of reps copies
                const Re* a = re->a.get();
                const DryRes& r0 = bb(a, p);
                uint64_t spent = r0.spent;
                std::map<size_t, uint64_t> conts = as_map(r0);
                for (uint64_t r = 1; r < reps && !conts.empty() && spent < cap; ++r) {
                    conts = extend(conts, a, &spent);
                    spent = add(spent, total(conts));
                }
                for (auto& [e, c] : conts) put(out, e, c);
                // at_least + 1 ..= at_most, stopping after the first empty step (or once
                // saturated: the count is then past cap whatever follows)
                for (uint64_t it = at_least + 1; it <= at_most && spent < cap; ++it) {
                    std::map<size_t, uint64_t> nxt = extend(conts, a, &spent);
                    spent = add(spent, total(nxt));
                    if (nxt.empty()) break;
                    for (auto& [e, c] : nxt) put(out, e, c);
                    conts = std::move(nxt);
                }
                return done(out, spent);
            }
            default: break;
        }
        throw DryPanic{};  // unmatched variant: the enumeration reports it
    }
};
}  // namespace

uint64_t enumeration_spent(size_t L, const ReP& re, size_t lo, size_t hi, uint64_t cap) {
    if (hi > L) hi = L;
    const size_t saved = g_budget;
    g_budget = cap;
    uint64_t spent;
    try {
        for (size_t i = lo; i < hi; ++i) spend(build_branches(L, re, i).size());  // record_has_match's loop
        spent = cap - g_budget;
    } catch (const Error& e) {
        g_budget = saved;
        if (e.code != FR_ERR_OOM) throw;
        return cap + 1;
    }
    g_budget = saved;
    return spent;
}

CostOutcome enumeration_cost(size_t L, const ReP& re, size_t lo, size_t hi, uint64_t cap, uint64_t* cost,
                             uint64_t mem_bytes) {
    if (hi > L) hi = L;
    Dry d{L, cap == UINT64_MAX ? cap : cap + 1, mem_bytes ? mem_bytes : ENUM_COST_MEM_BYTES, {}};
    uint64_t t = 0;
    try {
        for (size_t i = lo; i < hi && t < d.cap; ++i) {  // record_has_match: spend(bs.size()) per start
            const DryRes& r = d.bb(re.get(), i);
            t = d.add(t, d.add(r.spent, r.size));
        }
    } catch (const DryPanic&) {
        return COST_PANIC;
    } catch (const DryMemory&) {
        return COST_MEMORY;
    }
    *cost = t;
    return COST_COUNTED;
}

Recorded record_has_match_engine(ValueDag& dag, size_t L, const std::string& pattern, size_t lo, size_t hi,
                                 int engine) {
    if (engine == FR_ENGINE_MERGED) return record_has_match_merged(dag, L, pattern, lo, hi);
    if (engine == FR_ENGINE_ENUMERATE) return record_has_match(dag, L, pattern, lo, hi);
    // AUTO: the reference's enumeration (exact counters) while it stays within
    // a few million variants, else the state-merging evaluator.  The enumeration's cost
    // is counted first (enumeration_cost, exact), so a pattern past the budget goes
    // straight to the merged evaluator instead of building 2^22 branches and dropping
    // them (config 5 at 512 chars: ~1 s of host time per cold call).  Small enumerations
    // (/abc/ x 256: 763 variants) are tried directly: counting costs about as much as them.
    constexpr size_t budget = (size_t)1 << 22, small = (size_t)1 << 12;
    try {  // (the budget runs out while enumerating, before the dag is touched)
        return record_has_match(dag, L, pattern, lo, hi, small);
    } catch (const Error& e) {
        if (e.code != FR_ERR_OOM) throw;
    }
    {
        // no count (a panic, or the counter's memo bound: FR_ENUM_COST_BYTES overrides it,
        // tests only) -> the enumeration below decides under its budget, as without the counter
        uint64_t cost = 0, mem = 0;
        if (const char* ev = std::getenv("FR_ENUM_COST_BYTES")) mem = std::strtoull(ev, nullptr, 10);
        if (enumeration_cost(L, parse(pattern), lo, hi, budget, &cost, mem) == COST_COUNTED && cost > budget)
            return record_has_match_merged(dag, L, pattern, lo, hi);
    }
    try {
        return record_has_match(dag, L, pattern, lo, hi, budget);
    } catch (const Error& e) {
        if (e.code != FR_ERR_OOM) throw;
    }
    return record_has_match_merged(dag, L, pattern, lo, hi);
}

}  // namespace fr
