// extern "C" boundary (include/fheregex.h): context, keys, ciphertext handles,
// eager gate ops (the smart_* replacements), the batched has_match engine.
#include <chrono>
#include <climits>
#include <cstdlib>
#include <map>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "device.h"
#include "fheregex.h"
#include "keys.h"
#include "rns.h"
#include "lower.h"
#include "regex.h"

namespace fr {

// PARAM_MESSAGE_2_CARRY_2 (ciphertext.rs:1): 2-bit message, 2-bit carry per block
constexpr uint64_t MESSAGE_MODULUS = 4, CARRY_MODULUS = 4;

static thread_local std::string g_last_error;
void set_last_error(const std::string& m) { g_last_error = m; }

Params params_from_c(const fr_params* c) {
    Params p;
    if (c) {
        p.k = c->k;
        p.N = c->N;
        p.n = c->n;
        p.ks_base_log = c->ks_base_log;
        p.ks_level = c->ks_level;
        p.pbs_base_log = c->pbs_base_log;
        p.pbs_level = c->pbs_level;
        p.ring = c->ring;
        p.lwe_sigma = c->lwe_sigma;
        p.glwe_sigma = c->glwe_sigma;
    }
    validate_params(p);
    return p;
}
void validate_params(const Params& p) {
    if (p.k < 1 || p.k > 4 || p.N < 256 || p.N > 4096 || (p.N & (p.N - 1)) || p.n < 1 || p.n > 1024)
        throw Error(FR_ERR_INVALID, "invalid params");
    if (p.pbs_base_log != 23 || p.pbs_level != 1) throw Error(FR_ERR_INVALID, "only the 2^23 x 1 PBS gadget is supported");
    if (p.ks_base_log < 1 || p.ks_base_log * p.ks_level > 63) throw Error(FR_ERR_INVALID, "invalid keyswitch gadget");
    if (p.ring != FR_RING_RNS && p.ring != FR_RING_FFT) throw Error(FR_ERR_INVALID, "invalid ring");
    if (p.ring == FR_RING_FFT && !((p.k == 1 && p.N == 2048) || (p.k == 2 && p.N == 1024)))
        throw Error(FR_ERR_INVALID, "the FFT ring is built for (k, N) = (1, 2048) and (2, 1024)");
}

struct Block {
    int slot = -1;     // -1: trivial block
    uint8_t triv = 0;  // value of a trivial block (message, < 16)
};
struct HandleRec {
    bool live = false;
    bool is_bool = false;  // block 0 carries 0/1, blocks 1..3 trivial zero
    Block b[4];
};

static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace fr

using namespace fr;

struct fr_plan_cache;  // cached match plans (below)

struct fr_ctx {
    Params p;
    std::unique_ptr<Device> dev;
    ClientKey ck;
    bool has_ck = false;
    std::vector<uint64_t> ksk, bsk;
    bool has_sk = false;
    std::vector<HandleRec> handles;
    std::vector<uint32_t> free_handles;
    int lowering = FR_LOWER_THRESHOLD;
    int engine = FR_ENGINE_AUTO;
    int grammar = FR_GRAMMAR_REFERENCE;
    int keygen = FR_KEYGEN_AUTO;
    bool sk_on_device = false;  // server key generated on the device (export downloads it)
    bool multi_value = true;  // merge same-input small-norm LUTs into one blind rotation
    bool async_match = true;  // has_match returns once its launches are enqueued (fr_set_async)
    uint64_t next_lane = 0;   // fr_set_lanes: consecutive asynchronous matches round-robin over the lanes
    fr_plan_cache* plans = nullptr;
    // content_signature scratch: canonical id of an arena slot, valid while sig_gen[slot] == gen
    std::vector<int32_t> sig_id;
    std::vector<uint32_t> sig_gen;
    uint32_t gen = 0;

    fr_ctx();
    ~fr_ctx();
    fr_ctx(const fr_ctx&) = delete;
    fr_ctx& operator=(const fr_ctx&) = delete;
    void clear_plans();

    Device& device() {
        if (!dev) throw Error(FR_ERR_NO_DEVICE, "host-only context: no HIP device");
        return *dev;
    }
    fr_ct new_handle(const HandleRec& r) {
        uint32_t h;
        if (!free_handles.empty()) {
            h = free_handles.back();
            free_handles.pop_back();
            handles[h] = r;
        } else {
            h = (uint32_t)handles.size();
            handles.push_back(r);
        }
        handles[h].live = true;
        return h;
    }
    HandleRec& get(fr_ct h) {
        if (h >= handles.size() || !handles[h].live) throw Error(FR_ERR_INVALID, "invalid ciphertext handle");
        return handles[h];
    }
    void release(fr_ct h) {
        HandleRec& r = get(h);
        for (auto& b : r.b)
            if (b.slot >= 0 && dev) dev->free_slot(b.slot);
        r.live = false;
        free_handles.push_back(h);
    }
};

namespace fr {

// LUTs whose multi-value factor w_f has sum(d^2) <= this share rotations
constexpr int MV_MAX_NORM2 = 8;

// ---------------------------------------------------------------- executor
// A PBS program whose negative sources refer to content blocks (input q = pos q:
// src = -(1 + q*4 + blk)) becomes a Schedule: its rotation jobs by dependency level,
// small-norm LUTs on the same linear combination merged into one multi-value job.
// Job references are abstract: in_slot[q] >= 0 is the output of program gate
// in_slot[q], in_slot[q] < 0 content block -1 - in_slot[q]; out_slot[f] is a program
// gate.  Trivial content blocks are folded into the offset.  Building a schedule
// validates every gate and allocates nothing; a host-only context builds the same
// schedule (fr_schedule_match) as the device plan, which maps the references to
// arena slots (compile_plan).
struct Schedule {
    std::vector<DevGate> jobs;      // levels concatenated
    std::vector<size_t> level_off;  // level l (0-based): jobs [level_off[l], level_off[l+1])
    size_t n_gates = 0;
    uint64_t levels = 0, max_width = 0;
};

// block(cb, &key, &triv): false if content block cb is trivial (its value in triv),
// else key identifies the block's ciphertext (the multi-value merge compares keys)
template <class Block>
static Schedule build_schedule(const std::vector<PGate>& gates, size_t n_content, bool multi_value, Block&& block) {
    // 1. validation: topological order, input range, fan-in, offsets
    std::vector<int> level(gates.size(), 0);
    int maxl = 0;
    for (size_t g = 0; g < gates.size(); ++g) {
        const PGate& G = gates[g];
        int l = 0, nin = 0, off = G.offset;
        for (auto& in : G.ins) {
            if (in.src >= 0) {
                if ((size_t)in.src >= g) throw Error(FR_ERR_INVALID, "gate program is not topologically ordered");
                l = std::max(l, level[in.src]);
                ++nin;
                continue;
            }
            const int cb = -in.src - 1;
            if ((size_t)(cb / 4) >= n_content) throw Error(FR_ERR_INVALID, "gate input out of range");
            int key = 0, triv = 0;
            if (block(cb, key, triv)) ++nin;
            else off += 2 * in.w * triv;
        }
        if (nin > 16) throw Error(FR_ERR_INVALID, "gate fan-in > 16");
        if (G.kind != GATE_SIGN && (off & 1)) throw Error(FR_ERR_INVALID, "LUT gate with a half-integral offset");
        level[g] = l + 1;
        maxl = std::max(maxl, l + 1);
    }
    std::vector<std::vector<int>> by_level(maxl + 1);
    for (size_t g = 0; g < gates.size(); ++g) by_level[level[g]].push_back((int)g);
    // 2. jobs, level by level
    Schedule S;
    S.n_gates = gates.size();
    S.level_off.push_back(0);
    for (int l = 1; l <= maxl; ++l) {
        const size_t first = S.jobs.size();
        // input signature -> open job index
        std::map<std::vector<int32_t>, size_t> open_job;
        for (int g : by_level[l]) {
            const PGate& G = gates[g];
            DevGate d;
            std::memset(&d, 0, sizeof d);
            int off = G.offset, nin = 0;
            std::vector<int32_t> sig;
            for (auto& in : G.ins) {
                int ref, key;
                if (in.src >= 0) {
                    ref = in.src;
                    key = in.src;
                } else {
                    const int cb = -in.src - 1;
                    int triv = 0;
                    if (!block(cb, key, triv)) {
                        off += 2 * in.w * triv;  // offsets are in units of Delta/2
                        continue;
                    }
                    ref = -1 - cb;
                    key = -1 - key;
                }
                d.in_slot[nin] = ref;
                d.in_w[nin] = in.w;
                sig.push_back(key);
                sig.push_back(in.w);
                ++nin;
            }
            d.n_in = nin;
            d.offset = off;
            if (G.kind == GATE_SIGN) {
                d.n_out = 1;
                d.direct = JOB_SIGN;
                d.out_slot[0] = g;
                S.jobs.push_back(d);
                continue;
            }
            const bool small = lut_w_norm2(G.lut) <= MV_MAX_NORM2;
            if (small && multi_value) {
                sig.push_back(nin);
                sig.push_back(off);
                auto it = open_job.find(sig);
                if (it != open_job.end() && S.jobs[it->second].n_out < MAX_OUT) {
                    DevGate& J = S.jobs[it->second];
                    std::memcpy(J.lut[J.n_out], G.lut, 16);
                    J.out_slot[J.n_out] = g;
                    J.n_out++;
                    J.direct = JOB_MULTI;
                    continue;
                }
                open_job[sig] = S.jobs.size();
            }
            std::memcpy(d.lut[0], G.lut, 16);
            d.n_out = 1;
            d.direct = JOB_DIRECT;
            d.out_slot[0] = g;
            S.jobs.push_back(d);
        }
        S.level_off.push_back(S.jobs.size());
        S.max_width = std::max<uint64_t>(S.max_width, S.jobs.size() - first);
    }
    S.levels = (uint64_t)maxl;
    return S;
}

// A device plan: the schedule with references mapped to arena slots (one slot per
// program gate).  The slots allocated so far are returned if compilation throws.
// A template plan (n_refs > 0) keeps its content inputs as references
// (in_slot = -1 - (4 pos + block)) that a content map bound per call resolves
// (Device::bind_content), so one plan serves every content of the same shape.
struct Plan {
    std::vector<DevGate> gates;     // levels concatenated
    std::vector<size_t> level_off;  // level l (0-based): gates [level_off[l], level_off[l+1])
    std::vector<int> slot;          // output slot per program gate
    uint64_t pbs = 0, rotations = 0, levels = 0, max_width = 0;
    size_t n_refs = 0;              // template plan: content references (4 per position)
    DevGate* d_gates = nullptr;     // device-resident copy (cached plans)
};

static void free_plan_slots(Device& dev, std::vector<int>& slot) {
    for (int& s : slot)
        if (s >= 0) dev.free_slot(s), s = -1;
}

static Plan compile_plan(fr_ctx* ctx, const std::vector<PGate>& gates, const std::vector<fr_ct>& inputs,
                         bool content_refs = false) {
    Device& dev = ctx->device();
    if (!ctx->has_sk || !dev.has_keys()) throw Error(FR_ERR_NO_KEY, "server key not generated");
    auto block_slot = [&](int cb) -> const Block& { return ctx->get(inputs[(size_t)(cb / 4)]).b[cb % 4]; };
    Schedule S = build_schedule(gates, inputs.size(), ctx->multi_value, [&](int cb, int& key, int& triv) {
        const Block& b = block_slot(cb);
        if (b.slot < 0) {
            triv = (int)b.triv;
            return false;
        }
        key = b.slot;
        return true;
    });
    Plan P;
    P.slot.assign(gates.size(), -1);
    struct Guard {
        Device& dev;
        std::vector<int>& slot;
        bool armed = true;
        ~Guard() {
            if (armed) free_plan_slots(dev, slot);
        }
    } guard{dev, P.slot};
    for (size_t g = 0; g < gates.size(); ++g) P.slot[g] = dev.alloc_slot();
    P.gates = std::move(S.jobs);
    for (DevGate& d : P.gates) {
        for (int q = 0; q < d.n_in; ++q)
            d.in_slot[q] = d.in_slot[q] >= 0 ? P.slot[d.in_slot[q]]
                           : content_refs   ? d.in_slot[q]
                                            : block_slot(-1 - d.in_slot[q]).slot;
        for (int f = 0; f < d.n_out; ++f) d.out_slot[f] = P.slot[d.out_slot[f]];
    }
    P.n_refs = content_refs ? 4 * inputs.size() : 0;
    P.level_off = std::move(S.level_off);
    P.pbs = gates.size();
    P.rotations = P.gates.size();
    P.levels = S.levels;
    P.max_width = S.max_width;
    guard.armed = false;
    return P;
}

// enqueue every level of a plan (async on the device stream)
static void launch_plan(Device& dev, const Plan& P) {
    for (size_t l = 0; l + 1 < P.level_off.size(); ++l) {
        const size_t a = P.level_off[l], n = P.level_off[l + 1] - a;
        if (P.d_gates) dev.run_level_resident(P.d_gates + a, P.gates.data() + a, n, P.n_refs);
        else dev.run_level(P.gates.data() + a, n);
    }
}

static void add_plan_stats(const Plan& P, fr_match_stats* st) {
    if (!st) return;
    st->pbs += P.pbs;
    st->blind_rotations += P.rotations;
    st->levels += P.levels;
    st->max_level_width = std::max<uint64_t>(st->max_level_width, P.max_width);
}

// Runs a program and returns one slot per gate (the caller owns those slots).
static std::vector<int> execute_gates(fr_ctx* ctx, const std::vector<PGate>& gates, const std::vector<fr_ct>& inputs,
                                      fr_match_stats* st) {
    Plan P = compile_plan(ctx, gates, inputs);
    launch_plan(ctx->device(), P);
    add_plan_stats(P, st);
    return std::move(P.slot);
}

// result handle of a program: boolean out_const + out_w * gate slot (a linear
// op, no bootstrap), or trivial.  take_slot: the output gate's slot becomes the
// result's (else the result is a fresh slot and `slots` stay untouched).  Async:
// the caller synchronises the stream before handing the result out.
static fr_ct make_output(fr_ctx* ctx, int out_gate, int out_w, int out_const, std::vector<int>& slots, bool take_slot) {
    HandleRec r;
    r.is_bool = true;
    if (out_gate < 0) {
        r.b[0].triv = (uint8_t)out_const;
    } else if (take_slot && out_w == 1 && out_const == 0) {
        r.b[0].slot = slots[out_gate];
        slots[out_gate] = -1;
    } else {
        DevGate d;
        std::memset(&d, 0, sizeof d);
        d.n_in = 1;
        d.in_slot[0] = slots[out_gate];
        d.in_w[0] = out_w;
        d.offset = 2 * out_const;
        d.out_slot[0] = ctx->device().alloc_slot();
        ctx->device().run_linear(d);
        r.b[0].slot = d.out_slot[0];
    }
    return ctx->new_handle(r);
}
static fr_ct finish_output(fr_ctx* ctx, int out_gate, int out_w, int out_const, std::vector<int>& slots,
                           bool take_slot) {
    const fr_ct h = make_output(ctx, out_gate, out_w, out_const, slots, take_slot);
    if (take_slot) free_plan_slots(ctx->device(), slots);
    ctx->device().sync();
    return h;
}

static fr_ct run_program(fr_ctx* ctx, const Program& prog, const std::vector<fr_ct>& inputs, fr_match_stats* st) {
    std::vector<int> slots = execute_gates(ctx, prog.gates, inputs, st);
    return finish_output(ctx, prog.out_gate, prog.out_w, prog.out_const, slots, true);
}

static int cblk(int pos, int blk) { return -(1 + pos * 4 + blk); }

// ------------------------------------------------------------ plan cache
// The circuit of a match is data-oblivious: it depends on (pattern, grammar,
// engine, lowering, multi-value, length, start range, batch size) and on the
// content's *shape* -- which blocks are trivial and their values, and which
// positions share a ciphertext (the multi-value merge compares inputs) -- never on
// the ciphertexts themselves.  A cached plan is a template plan (Plan::n_refs):
// its content inputs are references that each call binds to the call's arena
// slots through a content map, so a fresh ciphertext of the same shape replays
// the plan (the reference re-plans every call, engine.rs:8-42).  A cached plan
// keeps its intermediate slots and a device copy of its gate batches; a repeat
// call skips parse -> record -> lower -> compile and the descriptor uploads, and
// only binds the content and enqueues the levels.  The cache is bounded by entries
// (LRU, default 8, FR_PLAN_CACHE) and by the intermediate slots it holds (default
// 2^18 = 4.3 GB at k = 1, FR_PLAN_CACHE_SLOTS); eviction runs before the new plan
// allocates, and a plan larger than the slot budget runs uncached.
struct CachedMatch {
    std::string key;           // match_key: every numeric field first, the pattern last
    size_t parts = 1;          // fr_has_match_parts' max_parts (also in the key)
    int lane = 0;              // lane whose plan copy this is (0: lane 0; also in the key)
    std::vector<int32_t> sig;  // canonical content shape (content_signature)
    Plan plan;
    size_t n_gates = 0;        // program gates of one match (copy m's gates start at m * n_gates)
    std::vector<ProgOut> outs;  // one match's outputs (its parts, fr_has_match_parts)
    uint64_t ct_ops = 0, cache_hits = 0, n_branches = 0;
    uint64_t last_use = 0;
};

}  // namespace fr

struct fr_plan_cache {
    std::vector<std::unique_ptr<fr::CachedMatch>> entries;
    size_t capacity = 8;
    size_t slot_cap = (size_t)1 << 18;  // intermediate slots held by all cached plans
    size_t slots_held = 0;
    uint64_t clock = 0, hits = 0, misses = 0;
};

namespace fr {

static void drop_cached(fr_ctx* ctx, CachedMatch& e);

// The key is a fixed number of '|'-terminated numeric fields followed by the pattern, so a
// pattern's own text (which may contain '|' and digits) cannot make two keys collide.
static std::string match_key(fr_ctx* ctx, const char* pattern, size_t n, size_t M, size_t lo, size_t hi,
                             size_t parts, int lane) {
    std::string k;
    for (size_t v : {(size_t)ctx->grammar, (size_t)ctx->engine, (size_t)ctx->lowering, (size_t)ctx->multi_value, n, M,
                     lo, hi, parts, (size_t)lane})
        k += std::to_string(v) + "|";
    k += pattern;
    return k;
}
// Canonical shape of the content: per position and block, the trivial value
// (-1 - v), the index of the block's ciphertext in order of first appearance (>= 0:
// equal indices = the same arena slot), or markers for an absent position / a
// boolean handle.  Two contents with equal signatures lower, schedule and merge
// identically.  cmap (if given) receives the content map: block r -> slot (-1: none).
static std::vector<int32_t> content_signature(fr_ctx* ctx, const fr_ct* content, size_t n, std::vector<int>* cmap) {
    constexpr int32_t ABSENT = INT32_MIN, BOOL = INT32_MIN + 1;
    std::vector<int32_t> sig;
    sig.reserve(4 * n);
    if (cmap) cmap->assign(4 * n, -1);
    if (++ctx->gen == 0) {  // generation wrapped: forget every stamp
        std::fill(ctx->sig_gen.begin(), ctx->sig_gen.end(), 0u);
        ctx->gen = 1;
    }
    int32_t next_id = 0;
    for (size_t q = 0; q < n; ++q) {
        if (content[q] == 0xFFFFFFFFu) {
            sig.insert(sig.end(), 4, ABSENT);
            continue;
        }
        const HandleRec& h = ctx->get(content[q]);
        for (int b = 0; b < 4; ++b) {
            const int s = h.b[b].slot;
            if (h.is_bool) {
                sig.push_back(BOOL);
            } else if (s < 0) {
                sig.push_back(-1 - (int32_t)h.b[b].triv);
            } else {
                if ((size_t)s >= ctx->sig_id.size()) {
                    ctx->sig_id.resize((size_t)s + 1024);
                    ctx->sig_gen.resize((size_t)s + 1024, 0u);
                }
                if (ctx->sig_gen[s] != ctx->gen) {
                    ctx->sig_gen[s] = ctx->gen;
                    ctx->sig_id[s] = next_id++;
                }
                sig.push_back(ctx->sig_id[s]);
            }
            if (cmap) (*cmap)[4 * q + b] = s;
        }
    }
    return sig;
}

}  // namespace fr

fr_ctx::fr_ctx() : plans(new fr_plan_cache) {
    if (const char* ev = std::getenv("FR_PLAN_CACHE")) plans->capacity = (size_t)std::max(0, std::atoi(ev));
    if (const char* ev = std::getenv("FR_PLAN_CACHE_SLOTS")) plans->slot_cap = (size_t)std::max(0L, std::atol(ev));
}
void fr_ctx::clear_plans() {
    if (!plans) return;
    for (auto& e : plans->entries) fr::drop_cached(this, *e);
    plans->entries.clear();
    plans->slots_held = 0;
}
fr_ctx::~fr_ctx() {
    try {
        clear_plans();
    } catch (...) {
    }
    delete plans;
}

namespace fr {

static void drop_cached(fr_ctx* ctx, CachedMatch& e) {
    ctx->plans->slots_held -= std::min(ctx->plans->slots_held, e.plan.slot.size());
    if (!ctx->dev) return;
    ctx->dev->sync();  // no level of this plan may still be in flight (every match ends synchronised)
    free_plan_slots(*ctx->dev, e.plan.slot);
    ctx->dev->free_gates(e.plan.d_gates);
    e.plan.d_gates = nullptr;
}
// drop least-recently-used plans until `entries` and `slots` more fit
static void evict_for(fr_ctx* ctx, size_t entries, size_t slots) {
    fr_plan_cache& pc = *ctx->plans;
    while (!pc.entries.empty() &&
           (pc.entries.size() + entries > pc.capacity || pc.slots_held + slots > pc.slot_cap)) {
        size_t v = 0;
        for (size_t i = 1; i < pc.entries.size(); ++i)
            if (pc.entries[i]->last_use < pc.entries[v]->last_use) v = i;
        drop_cached(ctx, *pc.entries[v]);
        pc.entries.erase(pc.entries.begin() + (long)v);
    }
}

// M independent matches of one pattern over M contents of n positions each
// (content[m * n + q]): one plan whose program is M copies of the match's lowered
// program, so every level of the M matches shares its launches (M = 1: has_match).
// parts > 1 (fr_has_match_parts): each match returns up to `parts` booleans whose OR is
// its result, outs[m * P + j] with P = *n_parts (the same for every m).
static void match_impl(fr_ctx* ctx, const fr_ct* content, size_t n, size_t M, const char* pattern, size_t lo,
                       size_t hi, fr_ct* outs, fr_match_stats* st, size_t parts = 1, size_t* n_parts = nullptr) {
    double t0 = now_ms();
    pattern = pattern ? pattern : "";
    Device& dev = ctx->device();
    if (!ctx->has_sk || !dev.has_keys()) throw Error(FR_ERR_NO_KEY, "server key not generated");
    if (M == 0) throw Error(FR_ERR_INVALID, "no matches");
    fr_plan_cache& pc = *ctx->plans;
    CachedMatch* hit = nullptr;
    std::string key;
    std::vector<int32_t> sig;
    std::vector<int> cmap;
    // lanes (fr_set_lanes): an asynchronous match of a cacheable plan runs on the next lane,
    // with a plan of its own (its intermediate slots), so consecutive matches overlap
    const int lane =
        (ctx->async_match && dev.match_lanes() > 0 && pc.capacity) ? 1 + (int)(ctx->next_lane++ % dev.match_lanes()) : 0;
    struct LaneScope {  // left on every exit, exceptions included
        Device& d;
        bool in = false;
        void enter(int i) {
            if (i > 0) d.enter_lane(i), in = true;
        }
        ~LaneScope() {
            if (in) d.leave_lane();
        }
    } lane_scope{dev};
    if (pc.capacity) {
        key = match_key(ctx, pattern, n, M, lo, hi, parts, lane);
        sig = content_signature(ctx, content, n * M, &cmap);
        for (auto& e : pc.entries)
            if (e->parts == parts && e->lane == lane && e->key == key && e->sig == sig) hit = e.get();
    }
    fr_match_stats local{};
    Recorded rec;
    bool cached = hit != nullptr;
    double t1;
    DeviceTimers before = dev.timers();
    if (hit) {
        ++pc.hits;
        hit->last_use = ++pc.clock;
        lane_scope.enter(lane);
        dev.bind_content(cmap.data(), cmap.size());
        t1 = now_ms();
        launch_plan(dev, hit->plan);
        add_plan_stats(hit->plan, &local);
        rec.ct_ops = hit->ct_ops;
        rec.cache_hits = hit->cache_hits;
        rec.n_branches = hit->n_branches;
        const size_t nO = hit->outs.size();
        if (nO < 1 || nO > parts)  // the caller's out buffer holds M * parts handles
            throw Error(FR_ERR_INVALID, "cached plan has more outputs than the caller's parts");
        for (size_t m = 0; m < M; ++m)
            for (size_t j = 0; j < nO; ++j) {
                const ProgOut& o = hit->outs[j];
                const int og = o.gate < 0 ? -1 : o.gate + (int)(m * hit->n_gates);
                outs[m * nO + j] = make_output(ctx, og, o.w, o.cst, hit->plan.slot, false);
            }
        if (n_parts) *n_parts = nO;
        if (!ctx->async_match) dev.sync();
    } else {
        ++pc.misses;
        ValueDag dag;
        GrammarScope grammar(ctx->grammar);
        rec = record_has_match_engine(dag, n, pattern, lo, hi, ctx->engine);
        Program prog = lower(dag, rec.root, ctx->lowering, (int)parts);
        // validate the referenced content handles of every match
        for (auto& g : prog.gates)
            for (auto& in : g.ins)
                if (in.src < 0) {
                    const size_t q = (size_t)((-in.src - 1) / 4);
                    for (size_t m = 0; m < M; ++m) {
                        const fr_ct c = q < n ? content[m * n + q] : 0xFFFFFFFFu;
                        if (c == 0xFFFFFFFFu) throw Error(FR_ERR_INVALID, "content position not provided");
                        if (ctx->get(c).is_bool) throw Error(FR_ERR_INVALID, "content handle is not a radix character");
                    }
                }
        // M copies: gate g of match m is m * G + g, content block cb of match m is 4 n m + cb
        const size_t G = prog.gates.size();
        std::vector<PGate> gates;
        gates.reserve(G * M);
        for (size_t m = 0; m < M; ++m)
            for (const PGate& g0 : prog.gates) {
                PGate g = g0;
                for (auto& in : g.ins) in.src = in.src >= 0 ? in.src + (int)(m * G) : in.src - (int)(4 * n * m);
                gates.push_back(std::move(g));
            }
        std::vector<fr_ct> inputs(content, content + n * M);
        const bool keep = pc.capacity && G && G * M <= pc.slot_cap;
        if (keep) evict_for(ctx, 1, G * M);  // before the new plan allocates its slots
        Plan P = compile_plan(ctx, gates, inputs, keep);
        add_plan_stats(P, &local);
        const size_t nO = prog.outs.size();
        if (n_parts) *n_parts = nO;
        auto out_of = [&](size_t m, size_t j) {
            return prog.outs[j].gate < 0 ? -1 : prog.outs[j].gate + (int)(m * G);
        };
        if (keep) {
            // keep the plan: its slots stay allocated, its batches go to the device once
            auto e = std::make_unique<CachedMatch>();
            e->key = std::move(key);
            e->parts = parts;
            e->lane = lane;
            e->sig = std::move(sig);
            e->n_gates = G;
            e->outs = prog.outs;
            e->ct_ops = rec.ct_ops;
            e->cache_hits = rec.cache_hits;
            e->n_branches = rec.n_branches;
            e->last_use = ++pc.clock;
            e->plan = std::move(P);
            pc.slots_held += e->plan.slot.size();
            CachedMatch& c = *e;
            pc.entries.push_back(std::move(e));
            c.plan.d_gates = dev.upload_gates(c.plan.gates.data(), c.plan.gates.size(), c.plan.n_refs);
            lane_scope.enter(lane);
            dev.bind_content(cmap.data(), cmap.size());
            t1 = now_ms();
            launch_plan(dev, c.plan);
            for (size_t m = 0; m < M; ++m)
                for (size_t j = 0; j < nO; ++j)
                    outs[m * nO + j] = make_output(ctx, out_of(m, j), prog.outs[j].w, prog.outs[j].cst, c.plan.slot, false);
        } else {
            t1 = now_ms();
            launch_plan(dev, P);
            // one output takes its gate's slot; parts get copies (two parts may read one gate)
            for (size_t m = 0; m < M; ++m)
                for (size_t j = 0; j < nO; ++j)
                    outs[m * nO + j] = make_output(ctx, out_of(m, j), prog.outs[j].w, prog.outs[j].cst, P.slot, nO == 1);
            free_plan_slots(dev, P.slot);  // later users of these slots are ordered after the launches (one stream)
        }
        if (!ctx->async_match) dev.sync();
    }
    double t2 = now_ms();
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->ct_ops = rec.ct_ops;
        st->cache_hits = rec.cache_hits;
        st->n_branches = rec.n_branches;
        st->pbs = local.pbs;
        st->blind_rotations = local.blind_rotations;
        st->levels = local.levels;
        st->max_level_width = local.max_level_width;
        st->host_ms = t1 - t0;
        st->device_ms = t2 - t1;
        st->plan_cached = cached ? 1 : 0;
        if (!ctx->async_match) {
            // blocking call: this match's timers resolved at its sync.  An asynchronous
            // call returns before its kernels ran, so its timers are left 0 here (read
            // them with fr_device_timers after a synchronising call instead)
            const DeviceTimers& after = dev.timers();
            st->br_kernel_ms = after.br_ms - before.br_ms;
            st->ks_kernel_ms = after.ks_ms - before.ks_ms;
            st->br_launches = after.br_launches - before.br_launches;
            st->br_gates = after.br_gates - before.br_gates;
        }
    }
}

// eager op programs over input handles (pos 0 = a, pos 1 = b)
static Program prog_cmp_const(int kind, uint8_t c) {
    Program p;
    PGate lo, hi;
    lo.ins = {{cblk(0, 0), 1}, {cblk(0, 1), 4}};
    hi.ins = {{cblk(0, 2), 1}, {cblk(0, 3), 4}};
    PGate fin;
    if (kind == 0) {  // eq: [lo == c_lo] + [hi == c_hi] == 2
        lut_eq(lo.lut, c & 15);
        lut_eq(hi.lut, c >> 4);
        fin.ins = {{0, 1}, {1, 1}};
        lut_eq(fin.lut, 2);
    } else {  // gt / le over the signs: 3*s_hi + s_lo
        lut_sign(lo.lut, c & 15);
        lut_sign(hi.lut, c >> 4);
        fin.ins = {{1, 3}, {0, 1}};
        lut_gt3(fin.lut, kind == 2);
    }
    p.gates = {lo, hi, fin};
    p.out_gate = 2;
    p.out_w = 1;
    compute_levels(p);
    return p;
}

}  // namespace fr

// =================================================================== C-ABI
#define FR_TRY(...)                                   \
    try {                                             \
        __VA_ARGS__;                                       \
        return FR_OK;                                 \
    } catch (const fr::Error& e) {                    \
        fr::set_last_error(e.what());                 \
        return e.code;                                \
    } catch (const std::bad_alloc&) {                 \
        fr::set_last_error("out of memory");          \
        return FR_ERR_OOM;                            \
    } catch (const std::exception& e) {               \
        fr::set_last_error(e.what());                 \
        return FR_ERR_INVALID;                        \
    } catch (...) {                                   \
        fr::set_last_error("unknown error");          \
        return FR_ERR_INVALID;                        \
    }

#define NEED(x)                                                               \
    do {                                                                      \
        if (!(x)) throw fr::Error(FR_ERR_INVALID, "invalid argument: " #x);   \
    } while (0)

extern "C" {

const char* fr_last_error(void) { return fr::g_last_error.c_str(); }

int fr_default_params(fr_params* out) {
    FR_TRY({
        NEED(out);
        Params p;
        std::memset(out, 0, sizeof *out);
        out->k = p.k;
        out->N = p.N;
        out->n = p.n;
        out->ks_base_log = p.ks_base_log;
        out->ks_level = p.ks_level;
        out->pbs_base_log = p.pbs_base_log;
        out->pbs_level = p.pbs_level;
        out->ring = p.ring;
        out->lwe_sigma = p.lwe_sigma;
        out->glwe_sigma = p.glwe_sigma;
    })
}

int fr_ctx_create(const fr_params* params, int device, fr_ctx** out) {
    FR_TRY({
        NEED(out);
        *out = nullptr;
        auto ctx = std::make_unique<fr_ctx>();
        ctx->p = params_from_c(params);
        if (device >= 0) ctx->dev = std::make_unique<Device>(ctx->p, device);
        *out = ctx.release();
    })
}

int fr_ctx_destroy(fr_ctx* ctx) {
    FR_TRY({ delete ctx; })
}

int fr_set_lowering(fr_ctx* ctx, int32_t mode) {
    FR_TRY({
        NEED(ctx && (mode == FR_LOWER_FAITHFUL || mode == FR_LOWER_THRESHOLD || mode == FR_LOWER_FAITHFUL_TREE));
        ctx->lowering = mode;
    })
}

int fr_set_engine(fr_ctx* ctx, int32_t engine) {
    FR_TRY({
        NEED(ctx && engine >= FR_ENGINE_AUTO && engine <= FR_ENGINE_MERGED);
        ctx->engine = engine;
    })
}

int fr_set_keygen(fr_ctx* ctx, int32_t where) {
    FR_TRY({
        NEED(ctx && where >= FR_KEYGEN_AUTO && where <= FR_KEYGEN_DEVICE);
        ctx->keygen = where;
    })
}

int fr_set_grammar(fr_ctx* ctx, int32_t grammar) {
    FR_TRY({
        NEED(ctx && (grammar == FR_GRAMMAR_REFERENCE || grammar == FR_GRAMMAR_EXT));
        ctx->grammar = grammar;
    })
}

int fr_set_multi_value(fr_ctx* ctx, int32_t on) {
    FR_TRY({
        NEED(ctx);
        ctx->multi_value = on != 0;
    })
}

int fr_dev_blind_rotate_multi(fr_ctx* ctx, const uint64_t* in, const uint8_t* luts, int32_t n_out, int32_t direct,
                              uint64_t* out) {
    FR_TRY({
        NEED(ctx && in && luts && out);
        ctx->device().blind_rotate_multi_host(in, luts, n_out, direct, out);
    })
}

int fr_set_profiling(fr_ctx* ctx, int32_t on) {
    FR_TRY({
        NEED(ctx && on >= 0 && on <= 2);  // 0 off, 1 blind-rotation timers, 2 the keyswitch timers too
        ctx->device().set_profiling(on);
    })
}

int fr_device_info(fr_ctx* ctx, char* buf, size_t len) {
    FR_TRY({
        NEED(ctx && buf && len);
        std::string s = ctx->dev ? ctx->dev->info() : std::string("host-only");
        std::snprintf(buf, len, "%s", s.c_str());
    })
}

int fr_load_client_key(fr_ctx* ctx, const uint8_t* data, size_t len) {
    FR_TRY({
        NEED(ctx && data);
        ClientKey ck = parse_client_key(data, len);
        if ((size_t)ctx->p.k * ctx->p.N != ck.s_big.size() || (size_t)ctx->p.n != ck.s_small.size())
            throw Error(FR_ERR_INVALID, "client key dimensions do not match the context params");
        // the radix encoding this build implements: PARAM_MESSAGE_2_CARRY_2, 4 blocks per
        // character (ciphertext.rs:1,12-13,43-44); a key of other parameters would decode wrong
        if (ck.message_modulus != MESSAGE_MODULUS || ck.carry_modulus != CARRY_MODULUS || ck.num_blocks != 4)
            throw Error(FR_ERR_INVALID, "client key: message/carry modulus or block count other than "
                                        "PARAM_MESSAGE_2_CARRY_2 with 4 blocks");
        ctx->ck = std::move(ck);
        ctx->has_ck = true;
        ctx->has_sk = false;
    })
}

int fr_gen_client_key(fr_ctx* ctx, uint64_t seed) {
    FR_TRY({
        NEED(ctx);
        ctx->ck = gen_client_key(ctx->p, seed);
        ctx->has_ck = true;
        ctx->has_sk = false;
    })
}

int fr_serialize_client_key(fr_ctx* ctx, uint8_t* buf, size_t cap, size_t* written) {
    FR_TRY({
        NEED(ctx && written);
        if (!ctx->has_ck) throw Error(FR_ERR_NO_KEY, "client key not loaded");
        const std::vector<uint8_t> b = serialize_client_key(ctx->ck);
        *written = b.size();
        if (!buf) return FR_OK;  // size query
        NEED(cap >= b.size());
        std::memcpy(buf, b.data(), b.size());
    })
}

int fr_gen_server_key(fr_ctx* ctx, uint64_t seed) {
    FR_TRY({
        NEED(ctx);
        if (!ctx->has_ck) throw Error(FR_ERR_NO_KEY, "client key not loaded");
        const bool on_dev = ctx->dev && ctx->p.ring == FR_RING_FFT && ctx->keygen != FR_KEYGEN_HOST;
        if (ctx->keygen == FR_KEYGEN_DEVICE && !on_dev)
            throw Error(ctx->dev ? FR_ERR_INVALID : FR_ERR_NO_DEVICE, "device keygen needs a device and the FFT ring");
        ctx->has_sk = false;
        if (on_dev) {
            ctx->ksk.clear();
            ctx->bsk.clear();
            ctx->dev->gen_server_key(ctx->ck, seed);
        } else {
            gen_ksk(ctx->p, ctx->ck, seed, ctx->ksk);
            gen_bsk(ctx->p, ctx->ck, seed, ctx->bsk);
            if (ctx->dev) ctx->dev->upload_keys(ctx->ksk, ctx->bsk);
        }
        ctx->sk_on_device = on_dev;
        ctx->has_sk = true;
    })
}

int fr_server_key_sizes(fr_ctx* ctx, size_t* ksk_len, size_t* bsk_len) {
    FR_TRY({
        NEED(ctx);
        const Params& p = ctx->p;
        if (ksk_len) *ksk_len = (size_t)p.big() * p.ks_level * (p.n + 1);
        if (bsk_len) *bsk_len = p.bsk_len();
    })
}

int fr_export_server_key(fr_ctx* ctx, uint64_t* ksk, size_t ksk_len, uint64_t* bsk, size_t bsk_len) {
    FR_TRY({
        NEED(ctx);
        if (!ctx->has_sk) throw Error(FR_ERR_NO_KEY, "server key not generated");
        if (ctx->sk_on_device) {
            ctx->device().download_server_key(ksk, ksk_len, bsk, bsk_len);
            return FR_OK;
        }
        if (ksk) {
            NEED(ksk_len == ctx->ksk.size());
            std::memcpy(ksk, ctx->ksk.data(), 8 * ksk_len);
        }
        if (bsk) {
            NEED(bsk_len == ctx->bsk.size());
            std::memcpy(bsk, ctx->bsk.data(), 8 * bsk_len);
        }
    })
}

int fr_load_server_key(fr_ctx* ctx, const uint64_t* ksk, size_t ksk_len, const uint64_t* bsk, size_t bsk_len) {
    FR_TRY({
        NEED(ctx && ksk && bsk);
        const Params& p = ctx->p;
        if (ksk_len != (size_t)p.big() * p.ks_level * (p.n + 1) || bsk_len != p.bsk_len())
            throw Error(FR_ERR_INVALID, "server key lengths do not match the context params (fr_server_key_sizes)");
        ctx->has_sk = false;
        std::vector<uint64_t> k(ksk, ksk + ksk_len), b(bsk, bsk + bsk_len);
        if (ctx->dev) ctx->dev->upload_keys(k, b);
        ctx->ksk = std::move(k);
        ctx->bsk = std::move(b);
        ctx->sk_on_device = false;
        ctx->has_sk = true;
    })
}

int fr_encrypt_blocks(fr_ctx* ctx, const uint8_t* msgs, size_t count, uint64_t seed, uint64_t first_block,
                      uint64_t* out) {
    FR_TRY({
        NEED(ctx && (msgs || !count) && (out || !count));
        if (!ctx->has_ck) throw Error(FR_ERR_NO_KEY, "client key not loaded");
        for (size_t i = 0; i < count; ++i) NEED(msgs[i] < 16);
        encrypt_blocks(ctx->p, ctx->ck, msgs, count, seed, first_block, out);
    })
}

// radix messages of a string (ciphertext.rs:18-29: 4 blocks of 2 bits, least significant first)

static std::vector<uint8_t> str_blocks(const char* s, size_t len) {
    std::vector<uint8_t> msgs(4 * len);
    for (size_t i = 0; i < len; ++i) {
        const uint8_t c = (uint8_t)s[i];
        if (c > 127) throw Error(FR_ERR_NON_ASCII, "content contains non-ascii characters");
        for (int b = 0; b < 4; ++b) msgs[4 * i + b] = (c >> (2 * b)) & 3;
    }
    return msgs;
}

int fr_encrypt_str(fr_ctx* ctx, const char* s, size_t len, uint64_t seed, uint64_t* out) {
    FR_TRY({
        NEED(ctx && (s || !len) && (out || !len));
        if (!ctx->has_ck) throw Error(FR_ERR_NO_KEY, "client key not loaded");
        const std::vector<uint8_t> msgs = str_blocks(s, len);
        encrypt_blocks(ctx->p, ctx->ck, msgs.data(), msgs.size(), seed, 0, out);
    })
}

int fr_encrypt_upload_str(fr_ctx* ctx, const char* s, size_t len, uint64_t seed, fr_ct* out) {
    FR_TRY({
        NEED(ctx && (s || !len) && (out || !len));
        if (!ctx->has_ck) throw Error(FR_ERR_NO_KEY, "client key not loaded");
        Device& dev = ctx->device();
        const std::vector<uint8_t> msgs = str_blocks(s, len);
        std::vector<int> slots(msgs.size());
        for (auto& x : slots) x = dev.alloc_slot();
        try {
            dev.encrypt_to_slots(ctx->ck, msgs.data(), msgs.size(), seed, 0, slots.data());
        } catch (...) {
            for (int x : slots) dev.free_slot(x);
            throw;
        }
        for (size_t i = 0; i < len; ++i) {
            HandleRec r;
            for (int b = 0; b < 4; ++b) r.b[b].slot = slots[4 * i + b];
            out[i] = ctx->new_handle(r);
        }
    })
}

// bincode (fixint, little endian) of tfhe-rs 0.2 RadixCiphertext:
//   u64 n_blocks, then per block: u64 len, len x u64 LWE words, u64 degree,
//   u64 message_modulus, u64 carry_modulus
int fr_radix_serialize(fr_ctx* ctx, const uint64_t* blocks, size_t n_blocks, uint64_t degree, uint8_t* buf,
                       size_t cap, size_t* written) {
    FR_TRY({
        NEED(ctx && (blocks || !n_blocks) && written);
        const size_t L = (size_t)ctx->p.lwe_len();
        const size_t need = 8 + n_blocks * (8 * (L + 4));
        *written = need;
        if (!buf) return FR_OK;  // size query
        NEED(cap >= need);
        uint8_t* o = buf;
        auto put = [&](uint64_t v) {
            std::memcpy(o, &v, 8);
            o += 8;
        };
        put(n_blocks);
        for (size_t b = 0; b < n_blocks; ++b) {
            put(L);
            std::memcpy(o, blocks + b * L, 8 * L);
            o += 8 * L;
            put(degree);
            put(MESSAGE_MODULUS);
            put(CARRY_MODULUS);
        }
    })
}

int fr_radix_deserialize(fr_ctx* ctx, const uint8_t* buf, size_t len, uint64_t* blocks, size_t max_blocks,
                         size_t* n_blocks) {
    FR_TRY({
        NEED(ctx && buf && n_blocks);
        const size_t L = (size_t)ctx->p.lwe_len();
        size_t off = 0;
        auto get = [&]() -> uint64_t {
            if (off + 8 > len) throw Error(FR_ERR_INVALID, "radix ciphertext: truncated");
            uint64_t v;
            std::memcpy(&v, buf + off, 8);
            off += 8;
            return v;
        };
        const uint64_t nb = get();
        if (nb > (len - 8) / (8 * (L + 4))) throw Error(FR_ERR_INVALID, "radix ciphertext: bad block count");
        *n_blocks = (size_t)nb;
        if (!blocks) return FR_OK;  // size query
        NEED(max_blocks >= nb);
        for (uint64_t b = 0; b < nb; ++b) {
            if (get() != L) throw Error(FR_ERR_INVALID, "radix ciphertext: LWE size does not match the parameters");
            if (off + 8 * L > len) throw Error(FR_ERR_INVALID, "radix ciphertext: truncated");
            std::memcpy(blocks + b * L, buf + off, 8 * L);
            off += 8 * L;
            // the comparison LUTs read clean 2-bit blocks (x0 + 4 x1 in [0, 16)); a block
            // carrying a carry (degree > message_modulus - 1) would decode silently wrong
            if (get() > MESSAGE_MODULUS - 1)
                throw Error(FR_ERR_INVALID, "radix ciphertext: block degree exceeds message_modulus - 1 (carries not propagated)");
            if (get() != MESSAGE_MODULUS || get() != CARRY_MODULUS)
                throw Error(FR_ERR_INVALID, "radix ciphertext: message/carry modulus does not match the parameters");
        }
        if (off != len) throw Error(FR_ERR_INVALID, "radix ciphertext: trailing bytes");
    })
}

int fr_decode_block(fr_ctx* ctx, const uint64_t* lwe, uint32_t* v) {
    FR_TRY({
        NEED(ctx && lwe && v);
        if (!ctx->has_ck) throw Error(FR_ERR_NO_KEY, "client key not loaded");
        *v = decode16(lwe_phase(ctx->p, ctx->ck, lwe));
    })
}

int fr_decrypt_radix(fr_ctx* ctx, const uint64_t* blocks, uint64_t* value) {
    FR_TRY({
        NEED(ctx && blocks && value);
        if (!ctx->has_ck) throw Error(FR_ERR_NO_KEY, "client key not loaded");
        uint64_t v = 0;
        for (int b = 0; b < 4; ++b) {
            uint32_t d = decode16(lwe_phase(ctx->p, ctx->ck, blocks + (size_t)b * ctx->p.lwe_len()));
            v += (uint64_t)(d % 4) << (2 * b);
        }
        *value = v & 0xFF;
    })
}

int fr_upload_radix(fr_ctx* ctx, const uint64_t* blocks, size_t n, fr_ct* out) {
    FR_TRY({
        NEED(ctx && (blocks || !n) && (out || !n));
        Device& dev = ctx->device();
        const int L = ctx->p.lwe_len();
        std::vector<int> slots(4 * n);
        for (auto& s : slots) s = dev.alloc_slot();
        dev.write_slots(slots.data(), slots.size(), blocks);
        for (size_t i = 0; i < n; ++i) {
            HandleRec r;
            for (int b = 0; b < 4; ++b) r.b[b].slot = slots[4 * i + b];
            out[i] = ctx->new_handle(r);
        }
        (void)L;
    })
}

int fr_upload_bool(fr_ctx* ctx, const uint64_t* lwe, size_t n, fr_ct* out) {
    FR_TRY({
        NEED(ctx && (lwe || !n) && (out || !n));
        Device& dev = ctx->device();
        std::vector<int> slots(n);
        for (auto& s : slots) s = dev.alloc_slot();
        dev.write_slots(slots.data(), n, lwe);
        for (size_t i = 0; i < n; ++i) {
            HandleRec r;
            r.is_bool = true;
            r.b[0].slot = slots[i];
            out[i] = ctx->new_handle(r);
        }
    })
}

int fr_download_radix(fr_ctx* ctx, fr_ct h, uint64_t* out) {
    FR_TRY({
        NEED(ctx && out);
        HandleRec& r = ctx->get(h);
        const int L = ctx->p.lwe_len();
        for (int b = 0; b < 4; ++b) {
            uint64_t* o = out + (size_t)b * L;
            if (r.b[b].slot >= 0) {
                ctx->device().read_slot(r.b[b].slot, o);
            } else {  // trivial block (shortint create_trivial): zero mask, body m * Delta
                std::memset(o, 0, 8 * (size_t)L);
                o[L - 1] = (uint64_t)r.b[b].triv << DELTA_LOG;
            }
        }
    })
}

int fr_release(fr_ctx* ctx, fr_ct h) {
    FR_TRY({
        NEED(ctx);
        ctx->release(h);
    })
}

int fr_trivial(fr_ctx* ctx, uint8_t value, fr_ct* out) {
    FR_TRY({  // create_trivial_radix, ciphertext.rs:8-30
        NEED(ctx && out);
        HandleRec r;
        for (int b = 0; b < 4; ++b) r.b[b].triv = (value >> (2 * b)) & 3;
        *out = ctx->new_handle(r);
    })
}

static int cmp_const_op(fr_ctx* ctx, fr_ct a, uint8_t c, fr_ct* out, int kind) {
    FR_TRY({
        NEED(ctx && out);
        if (ctx->get(a).is_bool) throw Error(FR_ERR_INVALID, "comparison operand must be a radix character");
        Program p = prog_cmp_const(kind, c);
        *out = run_program(ctx, p, {a}, nullptr);
    })
}
int fr_eq_const(fr_ctx* ctx, fr_ct a, uint8_t c, fr_ct* out) { return cmp_const_op(ctx, a, c, out, 0); }
int fr_gt_const(fr_ctx* ctx, fr_ct a, uint8_t c, fr_ct* out) { return cmp_const_op(ctx, a, c, out, 1); }
int fr_le_const(fr_ctx* ctx, fr_ct a, uint8_t c, fr_ct* out) { return cmp_const_op(ctx, a, c, out, 2); }

static int bitop(fr_ctx* ctx, fr_ct a, fr_ct b, fr_ct* out, bool is_and) {
    FR_TRY({
        NEED(ctx && out);
        const HandleRec& ha = ctx->get(a);
        const HandleRec& hb = ctx->get(b);
        if (ha.is_bool && hb.is_bool) {  // booleans: one bivariate PBS on block 0
            Program p;
            PGate g;
            g.ins = {{cblk(0, 0), 1}, {cblk(1, 0), 1}};
            if (is_and) lut_eq(g.lut, 2);
            else lut_at_least(g.lut, 1);
            p.gates = {g};
            p.out_gate = 0;
            p.out_w = 1;
            compute_levels(p);
            *out = run_program(ctx, p, {a, b}, nullptr);
        } else {  // general radix: per block, LUT over 4*x + y
            std::vector<PGate> gates(4);
            for (int blk = 0; blk < 4; ++blk) {
                gates[blk].ins = {{cblk(0, blk), 4}, {cblk(1, blk), 1}};
                for (int v = 0; v < 16; ++v) gates[blk].lut[v] = (uint8_t)(is_and ? ((v >> 2) & (v & 3)) : ((v >> 2) | (v & 3)));
            }
            std::vector<int> slots = execute_gates(ctx, gates, {a, b}, nullptr);
            ctx->device().sync();
            HandleRec r;
            for (int blk = 0; blk < 4; ++blk) r.b[blk].slot = slots[blk];
            *out = ctx->new_handle(r);
        }
    })
}
int fr_and(fr_ctx* ctx, fr_ct a, fr_ct b, fr_ct* out) { return bitop(ctx, a, b, out, true); }
int fr_or(fr_ctx* ctx, fr_ct a, fr_ct b, fr_ct* out) { return bitop(ctx, a, b, out, false); }

int fr_not(fr_ctx* ctx, fr_ct a, fr_ct* out) {
    FR_TRY({  // smart_bitxor(a, trivial 1), execution.rs:178-195
        NEED(ctx && out);
        const HandleRec ha = ctx->get(a);
        if (ha.is_bool) {
            HandleRec r;
            r.is_bool = true;
            if (ha.b[0].slot < 0) {
                r.b[0].triv = ha.b[0].triv ^ 1;
            } else {
                DevGate d;
                std::memset(&d, 0, sizeof d);
                d.n_in = 1;
                d.in_slot[0] = ha.b[0].slot;
                d.in_w[0] = -1;
                d.offset = 2;
                d.out_slot[0] = ctx->device().alloc_slot();
                ctx->device().run_linear(d);
                ctx->device().sync();
                r.b[0].slot = d.out_slot[0];
            }
            *out = ctx->new_handle(r);
        } else {  // general radix: block 0 through a LUT, blocks 1..3 copied
            HandleRec r;
            std::vector<PGate> gates(1);
            gates[0].ins = {{cblk(0, 0), 1}};
            for (int v = 0; v < 16; ++v) gates[0].lut[v] = (uint8_t)((v & 3) ^ 1);
            std::vector<int> slots = execute_gates(ctx, gates, {a}, nullptr);
            r.b[0].slot = slots[0];
            for (int blk = 1; blk < 4; ++blk) {
                if (ha.b[blk].slot < 0) {
                    r.b[blk] = ha.b[blk];
                    continue;
                }
                DevGate d;
                std::memset(&d, 0, sizeof d);
                d.n_in = 1;
                d.in_slot[0] = ha.b[blk].slot;
                d.in_w[0] = 1;
                d.out_slot[0] = ctx->device().alloc_slot();
                ctx->device().run_linear(d);
                r.b[blk].slot = d.out_slot[0];
            }
            ctx->device().sync();
            *out = ctx->new_handle(r);
        }
    })
}

int fr_or_many(fr_ctx* ctx, const fr_ct* in, size_t n, fr_ct* out) {
    FR_TRY({
        NEED(ctx && out && (in || !n));
        std::vector<fr_ct> inputs;
        int triv_or = 0;
        for (size_t i = 0; i < n; ++i) {
            const HandleRec& h = ctx->get(in[i]);
            if (!h.is_bool) throw Error(FR_ERR_INVALID, "fr_or_many: inputs must be booleans");
            if (h.b[0].slot < 0) triv_or |= h.b[0].triv & 1;
            else inputs.push_back(in[i]);
        }
        HandleRec r;
        r.is_bool = true;
        if (triv_or || inputs.empty()) {
            r.b[0].triv = (uint8_t)triv_or;
            *out = ctx->new_handle(r);
            return FR_OK;
        }
        if (inputs.size() == 1) {  // copy
            DevGate d;
            std::memset(&d, 0, sizeof d);
            d.n_in = 1;
            d.in_slot[0] = ctx->get(inputs[0]).b[0].slot;
            d.in_w[0] = 1;
            d.out_slot[0] = ctx->device().alloc_slot();
            ctx->device().run_linear(d);
            ctx->device().sync();
            r.b[0].slot = d.out_slot[0];
            *out = ctx->new_handle(r);
            return FR_OK;
        }
        // balanced tree of <= 16-input threshold ORs
        Program p;
        std::vector<int> cur;  // sources: negative = input q, else gate
        for (size_t q = 0; q < inputs.size(); ++q) cur.push_back(cblk((int)q, 0));
        while (cur.size() > 1) {
            std::vector<int> next;
            size_t m = cur.size(), chunks = (m + MAX_FANIN - 1) / MAX_FANIN, start = 0;
            for (size_t c = 0; c < chunks; ++c) {
                size_t len = m / chunks + (c < m % chunks ? 1 : 0);
                if (len == 1) {
                    next.push_back(cur[start]);
                } else {
                    PGate g;  // OR of <= 16 booleans: sign of sum - 1/2
                    for (size_t t = 0; t < len; ++t) g.ins.push_back({cur[start + t], 1});
                    g.kind = GATE_SIGN;
                    g.offset = -1;
                    p.gates.push_back(g);
                    next.push_back((int)p.gates.size() - 1);
                }
                start += len;
            }
            cur = next;
        }
        p.out_gate = cur[0];
        p.out_w = 1;
        compute_levels(p);
        *out = run_program(ctx, p, inputs, nullptr);
    })
}

int fr_run_gates(fr_ctx* ctx, fr_gate* gates, size_t n) {
    FR_TRY({
        NEED(ctx && (gates || !n));
        std::vector<fr_ct> inputs;
        std::vector<std::pair<fr_ct, int>> seen;
        auto input_index = [&](fr_ct h) -> int {
            for (size_t i = 0; i < inputs.size(); ++i)
                if (inputs[i] == h) return (int)i;
            ctx->get(h);
            inputs.push_back(h);
            return (int)inputs.size() - 1;
        };
        std::vector<PGate> pg(n);
        for (size_t j = 0; j < n; ++j) {
            const fr_gate& g = gates[j];
            NEED(g.n_in >= 0 && g.n_in <= 16 && (g.kind == GATE_LUT || g.kind == GATE_SIGN));
            pg[j].offset = g.offset;
            pg[j].kind = g.kind;
            std::memcpy(pg[j].lut, g.lut, 16);
            for (int q = 0; q < g.n_in; ++q) {
                if (g.in[q] & 0x80000000u) {
                    uint32_t src = g.in[q] & 0x7FFFFFFFu;
                    NEED(src < j);
                    pg[j].ins.push_back({(int)src, g.in_w[q]});
                } else {
                    NEED(g.in_block[q] >= 0 && g.in_block[q] < 4);
                    pg[j].ins.push_back({cblk(input_index(g.in[q]), g.in_block[q]), g.in_w[q]});
                }
            }
        }
        std::vector<int> slots = execute_gates(ctx, pg, inputs, nullptr);
        ctx->device().sync();
        for (size_t j = 0; j < n; ++j) {
            HandleRec r;
            r.is_bool = true;
            r.b[0].slot = slots[j];
            gates[j].out = ctx->new_handle(r);
        }
    })
}

int fr_has_match(fr_ctx* ctx, const fr_ct* content, size_t n, const char* pattern, fr_ct* out, fr_match_stats* st) {
    FR_TRY({
        NEED(ctx && out && pattern && (content || !n));
        match_impl(ctx, content, n, 1, pattern, 0, n, out, st);
    })
}

int fr_set_plan_cache(fr_ctx* ctx, size_t capacity) {
    FR_TRY({
        NEED(ctx);
        ctx->plans->capacity = capacity;
        evict_for(ctx, 0, 0);  // drop the least recently used beyond the new capacity
    })
}

int fr_set_lanes(fr_ctx* ctx, int32_t n) {
    FR_TRY({
        NEED(ctx && n >= 1 && n <= 8);
        Device& dev = ctx->device();
        if (n == 1 ? dev.match_lanes() == 0 : dev.match_lanes() == n) return FR_OK;
        // the lanes' plan copies go with the lanes (their slots are held by the cache)
        fr_plan_cache& pc = *ctx->plans;
        for (size_t i = pc.entries.size(); i-- > 0;)
            if (pc.entries[i]->lane != 0) {
                drop_cached(ctx, *pc.entries[i]);
                pc.entries.erase(pc.entries.begin() + (long)i);
            }
        dev.set_lanes(n);
        ctx->next_lane = 0;
    })
}

int fr_set_async(fr_ctx* ctx, int32_t on) {
    FR_TRY({
        NEED(ctx);
        ctx->async_match = on != 0;
    })
}

int fr_set_plan_cache_slots(fr_ctx* ctx, size_t max_slots) {
    FR_TRY({
        NEED(ctx);
        ctx->plans->slot_cap = max_slots;
        evict_for(ctx, 0, 0);
    })
}

int fr_plan_cache_stats(fr_ctx* ctx, uint64_t* entries, uint64_t* slots, uint64_t* hits, uint64_t* misses) {
    FR_TRY({
        NEED(ctx);
        const fr_plan_cache& pc = *ctx->plans;
        if (entries) *entries = pc.entries.size();
        if (slots) *slots = pc.slots_held;
        if (hits) *hits = pc.hits;
        if (misses) *misses = pc.misses;
    })
}

int fr_has_match_batch(fr_ctx* ctx, const fr_ct* content, size_t n_chars, size_t n_matches, const char* pattern,
                       fr_ct* out, fr_match_stats* st) {
    FR_TRY({
        NEED(ctx && out && pattern && n_matches && (content || !n_chars));
        match_impl(ctx, content, n_chars, n_matches, pattern, 0, n_chars, out, st);
    })
}

int fr_has_match_range(fr_ctx* ctx, const fr_ct* content, size_t n, const char* pattern, size_t lo, size_t hi,
                       fr_ct* out, fr_match_stats* st) {
    FR_TRY({
        NEED(ctx && out && pattern && (content || !n) && lo <= hi);
        match_impl(ctx, content, n, 1, pattern, lo, hi, out, st);
    })
}

int fr_has_match_parts(fr_ctx* ctx, const fr_ct* content, size_t n, const char* pattern, size_t lo, size_t hi,
                       size_t max_parts, fr_ct* out, size_t* n_parts, fr_match_stats* st) {
    FR_TRY({
        NEED(ctx && out && n_parts && pattern && (content || !n) && lo <= hi);
        NEED(max_parts >= 1 && max_parts <= (size_t)MAX_FANIN);
        match_impl(ctx, content, n, 1, pattern, lo, hi, out, st, max_parts, n_parts);
    })
}

int fr_debug_enumeration_cost(const char* pattern, int32_t grammar, size_t n_chars, size_t lo, size_t hi,
                              uint64_t cap, uint64_t mem_bytes, int32_t enumerate, int32_t* outcome,
                              uint64_t* counted, uint64_t* enumerated) {
    FR_TRY({
        NEED(pattern && outcome && counted && enumerated && lo <= hi && cap < UINT64_MAX);
        NEED(grammar == FR_GRAMMAR_REFERENCE || grammar == FR_GRAMMAR_EXT);
        GrammarScope scope(grammar);
        ReP re = parse(pattern);
        uint64_t c = 0;
        const CostOutcome o = enumeration_cost(n_chars, re, lo, hi, cap, &c, mem_bytes);
        *outcome = o == COST_COUNTED ? FR_COST_COUNTED : o == COST_PANIC ? FR_COST_PANIC : FR_COST_MEMORY;
        *counted = o == COST_COUNTED ? c : 0;
        *enumerated = enumerate ? enumeration_spent(n_chars, re, lo, hi, cap) : 0;
    })
}

int fr_plain_match_parts(const char* content, size_t len, const char* pattern, size_t lo, size_t hi, int32_t lowering,
                         int32_t engine, int32_t grammar, size_t max_parts, fr_plain_result* out, int32_t* parts,
                         size_t* n_parts) {
    FR_TRY({
        NEED((content || !len) && pattern && out && parts && n_parts && lo <= hi);
        NEED(max_parts >= 1 && max_parts <= (size_t)MAX_FANIN);
        NEED(lowering >= FR_LOWER_FAITHFUL && lowering <= FR_LOWER_FAITHFUL_TREE);
        NEED(engine >= FR_ENGINE_AUTO && engine <= FR_ENGINE_MERGED);
        NEED(grammar == FR_GRAMMAR_REFERENCE || grammar == FR_GRAMMAR_EXT);
        ValueDag dag;
        GrammarScope scope(grammar);
        Recorded rec = record_has_match_engine(dag, len, pattern, lo, hi, engine);
        std::vector<int16_t> memo;
        std::memset(out, 0, sizeof *out);
        out->ct_ops = rec.ct_ops;
        out->cache_hits = rec.cache_hits;
        out->n_branches = rec.n_branches;
        out->result_recorded = dag.eval(rec.root, (const uint8_t*)content, memo);
        Program prog = lower(dag, rec.root, lowering, (int)max_parts);
        out->pbs = prog.gates.size();
        out->levels = (uint64_t)prog.levels;
        out->max_level_width = prog.max_width;
        std::vector<int> vals;
        out->result_lowered = eval_program_parts(prog, (const uint8_t*)content, len, vals);
        for (size_t j = 0; j < vals.size(); ++j) parts[j] = vals[j];
        *n_parts = vals.size();
    })
}

int fr_parse(const char* pattern, char* buf, size_t len) {
    return fr_parse_ex(pattern, FR_GRAMMAR_REFERENCE, buf, len);
}

int fr_parse_ex(const char* pattern, int32_t grammar, char* buf, size_t len) {
    FR_TRY({
        NEED(pattern && buf && len);
        std::string s = to_string(*parse(pattern, grammar));
        if (s.size() + 1 > len) throw Error(FR_ERR_INVALID, "buffer too small");
        std::memcpy(buf, s.c_str(), s.size() + 1);
    })
}

int fr_plain_match_ex(const char* content, size_t len, const char* pattern, size_t lo, size_t hi, int32_t lowering,
                      int32_t engine, fr_plain_result* out) {
    return fr_plain_match_g(content, len, pattern, lo, hi, lowering, engine, FR_GRAMMAR_REFERENCE, out);
}

int fr_plain_match_g(const char* content, size_t len, const char* pattern, size_t lo, size_t hi, int32_t lowering,
                     int32_t engine, int32_t grammar, fr_plain_result* out) {
    FR_TRY({
        NEED((content || !len) && pattern && out && lo <= hi);
        NEED(engine >= FR_ENGINE_AUTO && engine <= FR_ENGINE_MERGED);
        NEED(grammar == FR_GRAMMAR_REFERENCE || grammar == FR_GRAMMAR_EXT);
        ValueDag dag;
        GrammarScope scope(grammar);
        Recorded rec = record_has_match_engine(dag, len, pattern, lo, hi, engine);
        std::vector<int16_t> memo;
        std::memset(out, 0, sizeof *out);
        out->ct_ops = rec.ct_ops;
        out->cache_hits = rec.cache_hits;
        out->n_branches = rec.n_branches;
        out->result_recorded = dag.eval(rec.root, (const uint8_t*)content, memo);
        Program prog = lower(dag, rec.root, lowering);
        out->pbs = prog.gates.size();
        out->levels = (uint64_t)prog.levels;
        out->max_level_width = prog.max_width;
        out->result_lowered = eval_program(prog, (const uint8_t*)content, len);
    })
}

int fr_plain_match(const char* content, size_t len, const char* pattern, size_t lo, size_t hi, int32_t lowering,
                   fr_plain_result* out) {
    return fr_plain_match_ex(content, len, pattern, lo, hi, lowering, FR_ENGINE_ENUMERATE, out);
}

int fr_dev_keyswitch(fr_ctx* ctx, const uint64_t* in, size_t count, uint64_t* out) {
    FR_TRY({
        NEED(ctx && in && out);
        ctx->device().keyswitch_host(in, count, out);
    })
}
int fr_dev_blind_rotate(fr_ctx* ctx, const uint64_t* in, const uint8_t* luts, size_t count, uint64_t* out) {
    FR_TRY({
        NEED(ctx && in && luts && out);
        ctx->device().blind_rotate_host(in, luts, count, out);
    })
}
int fr_dev_ring_mul(fr_ctx* ctx, const uint64_t* a, const uint64_t* b, size_t count, uint64_t* out) {
    FR_TRY({
        NEED(ctx && a && b && out);
        ctx->device().ring_mul_host(a, b, count, out);
    })
}
int fr_dev_bench_pbs(fr_ctx* ctx, const fr_ct* in, size_t count, int32_t iters, double* br_ms, double* total_ms) {
    FR_TRY({
        NEED(ctx && in && count && iters > 0 && br_ms && total_ms);
        Device& dev = ctx->device();
        if (!ctx->has_sk) throw Error(FR_ERR_NO_KEY, "server key not generated");
        std::vector<DevGate> gates(count);
        std::vector<int> outs(count);
        for (size_t i = 0; i < count; ++i) {
            const HandleRec& h = ctx->get(in[i]);
            DevGate& d = gates[i];
            std::memset(&d, 0, sizeof d);
            int nin = 0, off = 0;
            // pack x0 + 4*x1 of a radix char (or a boolean's block 0): an eq-nibble PBS
            const int w[2] = {1, 4};
            for (int b = 0; b < (h.is_bool ? 1 : 2); ++b) {
                if (h.b[b].slot < 0) {
                    off += w[b] * h.b[b].triv;
                    continue;
                }
                d.in_slot[nin] = h.b[b].slot;
                d.in_w[nin] = w[b];
                ++nin;
            }
            d.n_in = nin;
            d.offset = 2 * off;
            lut_eq(d.lut[0], 1);
            d.n_out = 1;
            d.direct = JOB_DIRECT;
            outs[i] = dev.alloc_slot();
            d.out_slot[0] = outs[i];
        }
        dev.bench_pbs(gates, iters, br_ms, total_ms);
        for (int s : outs) dev.free_slot(s);
    })
}

uint64_t fr_debug_scalar(int32_t op, uint64_t x, uint64_t y) {
    switch (op) {
        case 0: return rns::crt((uint32_t)(x % rns::P0), (uint32_t)(x % rns::P1));
        case 1: return (uint64_t)(int64_t)rns::decompose((uint32_t)(x % rns::P0), (uint32_t)(x % rns::P1));
        case 2: return rns::to_torus((uint32_t)(x % rns::P0), (uint32_t)(x % rns::P1));
        case 3: return mod_switch(x, (int)y);
        case 4: {
            int32_t d[5];
            ks_decompose<3, 5>(x, d);
            return (uint64_t)(int64_t)d[y % 5];
        }
        default: return 0;
    }
}

}  // extern "C"

// ------------------------------------------------------------ level-sharded matches
// One match split across ranks (the reference folds ct_or over the
// start offsets of engine.rs:15-35, and anchored patterns have a single start,
// engine.rs:51-57): every rank compiles the same plan over its own copy of the
// content, runs a contiguous slice of every level's rotation jobs, and all-gathers
// the level's output LWEs device to device (fr_shard_export / fr_shard_import into
// the caller's device buffers, e.g. RCCL all_gather); every rank then holds the
// level's outputs and goes on to the next.  The plan keeps its slots and a device
// copy of its batches, so repeat runs only enqueue.
struct fr_shard {
    fr::Plan plan;
    int32_t out_gate = -1, out_w = 0, out_const = 0;
    std::vector<std::vector<int>> out_slots;     // per level: output slots in job order
    std::vector<std::vector<uint32_t>> out_off;  // per level: first output of each job (+ total)
    fr_match_stats stats{};
};

namespace fr {
static const std::vector<int>& shard_level_range(const fr_shard* sh, uint32_t level, uint32_t b, uint32_t e,
                                                 uint32_t& first, uint32_t& count) {
    if (level >= sh->out_off.size()) throw Error(FR_ERR_INVALID, "shard: level out of range");
    const auto& off = sh->out_off[level];
    if (b > e || e + 1 > off.size()) throw Error(FR_ERR_INVALID, "shard: job range out of range");
    first = off[b];
    count = off[e] - off[b];
    return sh->out_slots[level];
}
}  // namespace fr

int fr_shard_plan(fr_ctx* ctx, const fr_ct* content, size_t n, const char* pattern, size_t lo, size_t hi,
                  fr_shard** out, fr_match_stats* st) {
    FR_TRY({
        NEED(ctx && out && pattern && (content || !n) && lo <= hi);
        Device& dev = ctx->device();
        if (!ctx->has_sk || !dev.has_keys()) throw Error(FR_ERR_NO_KEY, "server key not generated");
        const double t0 = now_ms();
        ValueDag dag;
        GrammarScope grammar(ctx->grammar);
        Recorded rec = record_has_match_engine(dag, n, pattern, lo, hi, ctx->engine);
        Program prog = lower(dag, rec.root, ctx->lowering);
        for (auto& g : prog.gates)
            for (auto& in : g.ins)
                if (in.src < 0) {
                    const size_t q = (size_t)((-in.src - 1) / 4);
                    if (q >= n || content[q] == 0xFFFFFFFFu) throw Error(FR_ERR_INVALID, "content position not provided");
                    if (ctx->get(content[q]).is_bool) throw Error(FR_ERR_INVALID, "content handle is not a radix character");
                }
        auto sh = std::make_unique<fr_shard>();
        sh->plan = compile_plan(ctx, prog.gates, std::vector<fr_ct>(content, content + n));
        struct Guard {
            fr_ctx* ctx;
            fr_shard* sh;
            ~Guard() {
                if (sh) free_plan_slots(ctx->device(), sh->plan.slot);
            }
        } guard{ctx, sh.get()};
        Plan& P = sh->plan;
        P.d_gates = dev.upload_gates(P.gates.data(), P.gates.size());
        sh->out_gate = prog.out_gate;
        sh->out_w = prog.out_w;
        sh->out_const = prog.out_const;
        for (size_t l = 0; l + 1 < P.level_off.size(); ++l) {
            std::vector<int> slots;
            std::vector<uint32_t> off{0};
            for (size_t j = P.level_off[l]; j < P.level_off[l + 1]; ++j) {
                for (int f = 0; f < P.gates[j].n_out; ++f) slots.push_back(P.gates[j].out_slot[f]);
                off.push_back((uint32_t)slots.size());
            }
            sh->out_slots.push_back(std::move(slots));
            sh->out_off.push_back(std::move(off));
        }
        fr_match_stats& s = sh->stats;
        s.ct_ops = rec.ct_ops;
        s.cache_hits = rec.cache_hits;
        s.n_branches = rec.n_branches;
        s.pbs = P.pbs;
        s.blind_rotations = P.rotations;
        s.levels = P.levels;
        s.max_level_width = P.max_width;
        s.host_ms = now_ms() - t0;
        if (st) *st = s;
        guard.sh = nullptr;
        *out = sh.release();
    })
}
int fr_shard_levels(const fr_shard* sh, uint32_t* levels) {
    FR_TRY({
        NEED(sh && levels);
        *levels = (uint32_t)sh->out_off.size();
    })
}
int fr_shard_jobs(const fr_shard* sh, uint32_t level, uint32_t* jobs) {
    FR_TRY({
        NEED(sh && jobs && level < sh->out_off.size());
        *jobs = (uint32_t)sh->out_off[level].size() - 1;
    })
}
int fr_shard_outputs(const fr_shard* sh, uint32_t level, uint32_t begin, uint32_t end, uint32_t* n_lwe) {
    FR_TRY({
        NEED(sh && n_lwe);
        uint32_t first, count;
        shard_level_range(sh, level, begin, end, first, count);
        *n_lwe = count;
    })
}
int fr_shard_run(fr_ctx* ctx, fr_shard* sh, uint32_t level, uint32_t begin, uint32_t end) {
    FR_TRY({
        NEED(ctx && sh);
        uint32_t first, count;
        shard_level_range(sh, level, begin, end, first, count);
        const Plan& P = sh->plan;
        const size_t a = P.level_off[level] + begin;
        ctx->device().run_level_resident(P.d_gates + a, P.gates.data() + a, end - begin);
    })
}
int fr_shard_export(fr_ctx* ctx, fr_shard* sh, uint32_t level, uint32_t begin, uint32_t end, uint64_t* dev_dst) {
    FR_TRY({
        NEED(ctx && sh);
        uint32_t first, count;
        const std::vector<int>& slots = shard_level_range(sh, level, begin, end, first, count);
        NEED(dev_dst || !count);
        ctx->device().slots_to_device(slots.data() + first, count, dev_dst);
    })
}
int fr_shard_import(fr_ctx* ctx, fr_shard* sh, uint32_t level, uint32_t begin, uint32_t end, const uint64_t* dev_src) {
    FR_TRY({
        NEED(ctx && sh);
        uint32_t first, count;
        const std::vector<int>& slots = shard_level_range(sh, level, begin, end, first, count);
        NEED(dev_src || !count);
        ctx->device().device_to_slots(slots.data() + first, count, dev_src);
    })
}
int fr_shard_finish(fr_ctx* ctx, fr_shard* sh, fr_ct* out, fr_match_stats* st) {
    FR_TRY({
        NEED(ctx && sh && out);
        *out = finish_output(ctx, sh->out_gate, sh->out_w, sh->out_const, sh->plan.slot, false);
        if (st) *st = sh->stats;
    })
}
int fr_shard_free(fr_ctx* ctx, fr_shard* sh) {
    FR_TRY({
        NEED(ctx);
        if (!sh) return FR_OK;
        std::unique_ptr<fr_shard> own(sh);
        if (ctx->dev) {
            ctx->dev->sync();
            free_plan_slots(*ctx->dev, sh->plan.slot);
            ctx->dev->free_gates(sh->plan.d_gates);
            sh->plan.d_gates = nullptr;
        }
    })
}

// The same schedule without a device (CPU evaluators, tests): every content
// position of [0, n_chars) is taken as an encrypted radix character.
int fr_schedule_match(size_t n_chars, const char* pattern, size_t lo, size_t hi, int32_t lowering, int32_t engine,
                      int32_t grammar, int32_t multi_value, fr_job* jobs, size_t jobs_cap, size_t* n_jobs,
                      uint32_t* level_off, size_t level_cap, size_t* n_levels, int32_t* out3) {
    size_t n_parts = 0;
    return fr_schedule_match_parts(n_chars, pattern, lo, hi, lowering, engine, grammar, multi_value, 1, jobs, jobs_cap,
                                   n_jobs, level_off, level_cap, n_levels, out3, &n_parts);
}

int fr_schedule_match_parts(size_t n_chars, const char* pattern, size_t lo, size_t hi, int32_t lowering,
                            int32_t engine, int32_t grammar, int32_t multi_value, size_t max_parts, fr_job* jobs,
                            size_t jobs_cap, size_t* n_jobs, uint32_t* level_off, size_t level_cap, size_t* n_levels,
                            int32_t* outs3, size_t* n_parts) {
    FR_TRY({
        NEED(pattern && n_jobs && n_levels && outs3 && n_parts && lo <= hi);
        NEED(max_parts >= 1 && max_parts <= (size_t)MAX_FANIN);
        ValueDag dag;
        GrammarScope gs(grammar);
        Recorded rec = record_has_match_engine(dag, n_chars, pattern, lo, hi, engine);
        Program prog = lower(dag, rec.root, lowering, (int)max_parts);
        Schedule S = build_schedule(prog.gates, n_chars, multi_value != 0, [](int cb, int& key, int&) {
            key = cb;
            return true;
        });
        *n_jobs = S.jobs.size();
        *n_levels = S.level_off.size() - 1;
        *n_parts = prog.outs.size();
        for (size_t j = 0; j < prog.outs.size(); ++j) {
            outs3[3 * j] = prog.outs[j].gate;
            outs3[3 * j + 1] = prog.outs[j].w;
            outs3[3 * j + 2] = prog.outs[j].cst;
        }
        if (jobs) {
            NEED(jobs_cap >= S.jobs.size());
            static_assert(sizeof(fr_job) == sizeof(DevGate), "fr_job mirrors DevGate");
            // (an empty schedule's vector has no storage: memcpy's source must not be null,
            // UBSan finding of tests/test_fuzz_inputs.py)
            if (!S.jobs.empty()) std::memcpy(jobs, S.jobs.data(), sizeof(DevGate) * S.jobs.size());
        }
        if (level_off) {
            NEED(level_cap >= S.level_off.size());
            for (size_t l = 0; l < S.level_off.size(); ++l) level_off[l] = (uint32_t)S.level_off[l];
        }
    })
}

// device-to-device booleans (block 0 of a handle), e.g. per-rank partial results
// gathered over RCCL: no host round trip of the LWE
int fr_export_bool_device(fr_ctx* ctx, const fr_ct* h, size_t n, uint64_t* dev_dst) {
    FR_TRY({
        NEED(ctx && (h || !n) && (dev_dst || !n));
        Device& dev = ctx->device();
        std::vector<int> slots(n), tmp;
        struct Guard {
            Device& dev;
            std::vector<int>& tmp;
            ~Guard() {
                for (int s : tmp) dev.free_slot(s);
            }
        } guard{dev, tmp};
        for (size_t i = 0; i < n; ++i) {
            const HandleRec& r = ctx->get(h[i]);
            if (r.b[0].slot >= 0) {
                slots[i] = r.b[0].slot;
                continue;
            }
            // a trivial block 0 (e.g. a start range that cannot match): its trivial LWE
            std::vector<uint64_t> lwe((size_t)ctx->p.lwe_len(), 0);
            lwe.back() = (uint64_t)r.b[0].triv << DELTA_LOG;
            tmp.push_back(dev.alloc_slot());
            dev.write_slots(&tmp.back(), 1, lwe.data());
            slots[i] = tmp.back();
        }
        dev.slots_to_device(slots.data(), n, dev_dst);
    })
}
int fr_export_bool_device_async(fr_ctx* ctx, const fr_ct* h, size_t n, uint64_t* dev_dst) {
    FR_TRY({
        NEED(ctx && (h || !n) && (dev_dst || !n));
        if (n > 16) throw Error(FR_ERR_INVALID, "fr_export_bool_device_async: at most 16 handles");
        std::vector<int> slots(n);
        for (size_t i = 0; i < n; ++i) {
            const HandleRec& r = ctx->get(h[i]);
            if (r.b[0].slot < 0) return fr_export_bool_device(ctx, h, n, dev_dst);  // trivial: synchronising path
            slots[i] = r.b[0].slot;
        }
        ctx->device().slots_to_device_async(slots.data(), n, dev_dst);
    })
}
int fr_stream(fr_ctx* ctx, void** stream) {
    FR_TRY({
        NEED(ctx && stream);
        *stream = ctx->device().stream();
    })
}
int fr_import_bool_device(fr_ctx* ctx, const uint64_t* dev_src, size_t n, fr_ct* out) {
    FR_TRY({
        NEED(ctx && out && (dev_src || !n));
        Device& dev = ctx->device();
        std::vector<int> slots;
        try {
            for (size_t i = 0; i < n; ++i) slots.push_back(dev.alloc_slot());
            dev.device_to_slots(slots.data(), n, dev_src);
        } catch (...) {
            for (int s : slots) dev.free_slot(s);
            throw;
        }
        for (size_t i = 0; i < n; ++i) {
            HandleRec r;
            r.is_bool = true;
            r.b[0].slot = slots[i];
            out[i] = ctx->new_handle(r);
        }
    })
}
int fr_device_timers_latency(fr_ctx* ctx, double* br_ms, uint64_t* br_launches, uint64_t* br_gates) {
    FR_TRY({
        NEED(ctx);
        Device& dev = ctx->device();
        dev.sync();
        const DeviceTimers& t = dev.timers();
        if (br_ms) *br_ms = t.lat_br_ms;
        if (br_launches) *br_launches = t.lat_launches;
        if (br_gates) *br_gates = t.lat_gates;
    })
}
int fr_device_timers_pair(fr_ctx* ctx, double* br_ms, uint64_t* br_launches, uint64_t* br_gates) {
    FR_TRY({
        NEED(ctx);
        Device& dev = ctx->device();
        dev.sync();
        const DeviceTimers& t = dev.timers();
        if (br_ms) *br_ms = t.pair_br_ms;
        if (br_launches) *br_launches = t.pair_launches;
        if (br_gates) *br_gates = t.pair_gates;
    })
}
int fr_device_timers(fr_ctx* ctx, double* br_ms, double* ks_ms, uint64_t* br_launches, uint64_t* br_gates) {
    FR_TRY({
        NEED(ctx);
        Device& dev = ctx->device();
        dev.sync();
        const DeviceTimers& t = dev.timers();
        if (br_ms) *br_ms = t.br_ms;
        if (ks_ms) *ks_ms = t.ks_ms;
        if (br_launches) *br_launches = t.br_launches;
        if (br_gates) *br_gates = t.br_gates;
    })
}
