// Regex AST, parser, variant enumerator and symbolic Execution — host C++
// restatement of the reference's src/regex/{parser,engine,execution}.rs.
#pragma once
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace fr {

// ------------------------------------------------------------------ AST
// enum RegExpr, src/regex/parser.rs:8-41
struct Re;
using ReP = std::shared_ptr<const Re>;
struct Re {
    // CLASS (grammar extension, not in the reference): cs = lo0,hi0,lo1,hi1,...
    // inclusive byte ranges; one character matches if it lies in any of them
    enum Kind { SOF, EOF_, ANY, CHAR, BETWEEN, RANGE, NOT, EITHER, OPTIONAL, REPEATED, SEQ, CLASS } kind;
    uint8_t c = 0, from = 0, to = 0;
    std::vector<uint8_t> cs;
    ReP a, b;
    bool has_lo = false, has_hi = false;
    uint64_t lo = 0, hi = 0;
    std::vector<ReP> xs;
};
// canonical string form (shared with oracle/regex_oracle.py)
std::string to_string(const Re& r);
// parse(pattern): parser.rs:146-185.  Throws Error(FR_ERR_PARSE) for the
// reference's Err, Error(FR_ERR_REF_PANIC) where the reference panics.
// grammar FR_GRAMMAR_EXT (beyond the reference) additionally accepts bare
// digits as characters and bracket classes mixing letters, digits, escapes and
// ranges ([a-z0-9], [^A-Z_]) — only where the reference grammar fails, so every
// pattern the reference accepts parses to the same AST.  The default is the
// calling thread's grammar (GrammarScope), initially FR_GRAMMAR_REFERENCE.
ReP parse(const std::string& pattern, int grammar);
ReP parse(const std::string& pattern);
int current_grammar();
struct GrammarScope {  // sets the thread's grammar for parse(pattern)
    explicit GrammarScope(int grammar);
    ~GrammarScope();
    GrammarScope(const GrammarScope&) = delete;
    GrammarScope& operator=(const GrammarScope&) = delete;
  private:
    int prev_;
};

// Open-addressing index of dense ids by a 64-bit hash (linear probing, load
// <= 1/2): hash-consing of DAG nodes and Executed keys without per-bucket
// allocations.  find_or_add(h, eq, add): eq(id) tests a candidate, add()
// appends the new record and returns its id.
class IdIndex {
  public:
    template <class Eq, class Add>
    int find_or_add(uint64_t h, Eq&& eq, Add&& add) {
        if (2 * (count_ + 1) > ids_.size()) grow();
        const size_t mask = ids_.size() - 1;
        for (size_t i = (size_t)h & mask;; i = (i + 1) & mask) {
            if (ids_[i] < 0) {
                const int id = add();
                ids_[i] = id;
                hs_[i] = h;
                ++count_;
                return id;
            }
            if (hs_[i] == h && eq(ids_[i])) return ids_[i];
        }
    }

  private:
    void grow() {
        std::vector<int32_t> ids(ids_.empty() ? 1024 : 2 * ids_.size(), -1);
        std::vector<uint64_t> hs(ids.size());
        const size_t mask = ids.size() - 1;
        for (size_t j = 0; j < ids_.size(); ++j)
            if (ids_[j] >= 0) {
                size_t i = (size_t)hs_[j] & mask;
                while (ids[i] >= 0) i = (i + 1) & mask;
                ids[i] = ids_[j];
                hs[i] = hs_[j];
            }
        ids_.swap(ids);
        hs_.swap(hs);
    }
    std::vector<int32_t> ids_;
    std::vector<uint64_t> hs_;
    size_t count_ = 0;
};

// ------------------------------------------------------------ value DAG
// What the reference actually computes homomorphically: one node per distinct
// computation (hash-consed); short-circuited ops return an operand's node.
struct VNode {
    enum Op : uint8_t { POS, CONST, EQ, GT, LE, AND, OR, NOT } op;
    int32_t a = -1, b = -1;  // operand value ids (AND/OR/NOT)
    int32_t pos = 0;         // POS / EQ / GT / LE: content position
    uint8_t c = 0;           // CONST value, or the comparison constant
};

struct ValueDag {
    std::vector<VNode> nodes;
    int add(const VNode& n);
    int eval(int id, const uint8_t* content, std::vector<int16_t>& memo) const;
  private:
    IdIndex index_;
};

// ------------------------------------------------------- Execution (symbolic)
// src/regex/execution.rs:8-223: Executed keys (hash-consed), op cache,
// constant short-circuits, ct_ops / cache_hits.
struct Val {
    int32_t value;  // ValueDag id
    int32_t key;    // Executed key id
};

class Execution {
  public:
    explicit Execution(ValueDag& dag) : dag_(dag) {}
    Val ct_eq(const Val& a, const Val& b);
    Val ct_ge(const Val& a, const Val& b);  // smart_gt (execution.rs:93 quirk)
    Val ct_le(const Val& a, const Val& b);
    Val ct_and(const Val& a, const Val& b);
    Val ct_or(const Val& a, const Val& b);
    Val ct_not(const Val& a);
    Val ct_constant(uint8_t c);
    Val ct_true() { return ct_constant(1); }
    Val ct_false() { return ct_constant(0); }
    Val ct_pos(int at);
    uint64_t ct_operations_count() const { return ct_ops_; }
    uint64_t cache_hits() const { return cache_hits_; }

  private:
    enum Tag : uint8_t { K_CONST, K_POS, K_AND, K_OR, K_EQ, K_GE, K_LE, K_NOT };
    int key(Tag t, int64_t a, int64_t b = -1);
    int const_of(int key) const;  // -1 if not a Constant key
    template <class F>
    Val with_cache(int key, F&& f);
    ValueDag& dag_;
    IdIndex key_index_;
    struct KeyRec { Tag t; int64_t a, b; };
    std::vector<KeyRec> keys_;
    std::vector<int32_t> cache_;  // key id -> value id, -1 if not executed
    uint64_t ct_ops_ = 0, cache_hits_ = 0;
};

using Lazy = std::shared_ptr<const std::function<Val(Execution&)>>;
struct Branch {
    Lazy f;
    size_t end;
};
// build_branches, src/regex/engine.rs:45-214 (content only enters via its length)
std::vector<Branch> build_branches(size_t L, const ReP& re, size_t pos);

struct Recorded {
    int root = -1;  // value id of the result
    uint64_t ct_ops = 0, cache_hits = 0, n_branches = 0;
};
// has_match, src/regex/engine.rs:8-42 (start offsets restricted to [lo, hi)).
// branch_budget bounds the number of enumerated variants (Error FR_ERR_OOM past
// it); the reference itself has no bound and exhausts memory instead.
Recorded record_has_match(ValueDag& dag, size_t L, const std::string& pattern, size_t lo, size_t hi,
                          size_t branch_budget = SIZE_MAX);
// What record_has_match would spend of its branch budget (the variants it enumerates),
// counted without building a branch: per (node, position) the multiset of end positions
// with multiplicities and the spends of one call, memoised, so it is polynomial in L
// where the enumeration is exponential.  Saturates just past cap.  No count where the
// enumeration would panic (COST_PANIC: empty Seq, a repetition count the reference cannot
// allocate) or once the memo would hold more than mem_bytes (COST_MEMORY; 0: the default
// ENUM_COST_MEM_BYTES; entries and their stored end positions are counted): the caller
// then enumerates, which reproduces the error or the exact decision.
enum CostOutcome { COST_COUNTED = 0, COST_PANIC = 1, COST_MEMORY = 2 };
constexpr uint64_t ENUM_COST_MEM_BYTES = (uint64_t)256 << 20;
CostOutcome enumeration_cost(size_t L, const ReP& re, size_t lo, size_t hi, uint64_t cap, uint64_t* cost,
                             uint64_t mem_bytes = 0);
// The same by enumerating (test hook): the spends, or cap + 1 once past cap.
uint64_t enumeration_spent(size_t L, const ReP& re, size_t lo, size_t hi, uint64_t cap);
// State-merging evaluator (merged.cpp, beyond the reference): the same boolean,
// polynomial in L.  Error FR_ERR_INVALID for AST shapes it does not cover.
Recorded record_has_match_merged(ValueDag& dag, size_t L, const std::string& pattern, size_t lo, size_t hi);
// engine: FR_ENGINE_AUTO (enumerate within a budget, else merge), _ENUMERATE, _MERGED
Recorded record_has_match_engine(ValueDag& dag, size_t L, const std::string& pattern, size_t lo, size_t hi,
                                 int engine);

}  // namespace fr
