// Lowering of the recorded value DAG (what the reference computes through
// tfhe-rs smart_* calls) into a program of programmable bootstraps (PBS).
//
// Every gate is one programmable bootstrap of  s = offset/2 + sum_i w_i * in_i
// (offset in units of Delta/2, Delta = 2^59).  Inputs are content blocks (2-bit
// radix digits of the encrypted characters, src/regex/ciphertext.rs:18-29) or
// earlier gates.  Two kinds:
//  * LUT  : s integral in [0, 16), out = lut[s] (16-box test polynomial, one
//           padding bit, as tfhe-rs shortint PARAM_MESSAGE_2_CARRY_2);
//  * SIGN : s half-integral in (-16, 16), out = [s > 0] (constant test
//           polynomial: the negacyclic rotation yields +-Delta/2, then +Delta/2).
//           Threshold AND/OR of up to 16 literals in one bootstrap.
//
// FR_LOWER_FAITHFUL: one gate group per reference op (eq/gt/le = 3 PBS, and/or
//   = 1 PBS, not = linear), the decomposition of SURVEY App. D.3.
// FR_LOWER_THRESHOLD (default): AND/OR trees of the recorded circuit are
//   flattened into n-ary threshold gates (AND of m literals = [sum == m],
//   OR = [sum >= 1], m <= 15), NOT is pushed into literals (De Morgan, linear),
//   equality nibble tests are shared across constants.  Same decrypted result,
//   far fewer PBS and levels.
#pragma once
#include <cstdint>
#include <vector>

#include "regex.h"

namespace fr {

struct PIn {
    int32_t src;  // >= 0: gate index; < 0: content block -(1 + pos*4 + blk)
    int32_t w;
};
enum GateKind : int32_t { GATE_LUT = 0, GATE_SIGN = 1 };
struct PGate {
    std::vector<PIn> ins;
    int32_t offset = 0;  // units of Delta/2
    int32_t kind = GATE_LUT;
    uint8_t lut[16] = {0};
    int32_t level = 0;
};
// one boolean output: cst + w * gates[gate]   (gate == -1: the constant cst)
struct ProgOut {
    int32_t gate = -1, w = 0, cst = 0;
};
struct Program {
    std::vector<PGate> gates;
    // result = out_const + out_w * gates[out_gate]   (out_gate == -1: constant)
    int32_t out_gate = -1, out_const = 0, out_w = 0;
    // the outputs: {out_*} alone, or (lower's max_parts > 1) up to max_parts booleans
    // whose OR is the result
    std::vector<ProgOut> outs;
    int32_t levels = 0;
    size_t max_width = 0;
};

constexpr int MAX_FANIN = 16;

// max_parts > 1: a root OR (the has_match fold over start offsets, engine.rs:22-35)
// stops its threshold tree at <= max_parts literals and outputs them as parts, so the
// caller's own OR of several parts lists (start shards on several GPUs) is the
// tree's last level instead of one more.  Faithful lowerings and non-OR roots: one part.
Program lower(const ValueDag& dag, int root, int mode, int max_parts = 1);
// Plaintext semantics of a program (LUT semantics, with the [0,16) range
// check); returns the result value (several parts: their OR).
int eval_program(const Program& prog, const uint8_t* content, size_t L);
// the same, and each output's value in `parts`
int eval_program_parts(const Program& prog, const uint8_t* content, size_t L, std::vector<int>& parts);
void compute_levels(Program& prog);

// LUT builders
void lut_eq(uint8_t* lut, int v);     // [x == v]
void lut_sign(uint8_t* lut, int v);   // x < v -> 0, x == v -> 1, x > v -> 2
void lut_gt3(uint8_t* lut, bool le);  // over 3*s_hi + s_lo: gt (or its negation)
void lut_at_least(uint8_t* lut, int m);

}  // namespace fr
