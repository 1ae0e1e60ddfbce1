/*
 * fheregex.h — C-ABI of the MI355X-native gate-bootstrap executor under the
 * homomorphic regex engine of RKlompUU/fhe-regex.
 *
 * The boundary sits exactly where the reference's Execution layer calls into
 * tfhe-rs (the `tfhe::integer::ServerKey` it owns):
 *
 *   reference call site (src/regex/...)              replaced by
 *   ------------------------------------------------ ---------------------------
 *   execution.rs:76   sk.smart_eq(ct_char, ct_const)  fr_eq_const
 *   execution.rs:93   sk.smart_gt(ct_char, ct_const)  fr_gt_const   (ct_ge quirk)
 *   execution.rs:110  sk.smart_le(ct_char, ct_const)  fr_le_const
 *   execution.rs:143  sk.smart_bitand(a, b)           fr_and
 *   execution.rs:173  sk.smart_bitor(a, b)            fr_or
 *   execution.rs:190  sk.smart_bitxor(a, trivial 1)   fr_not
 *   ciphertext.rs:8-30 create_trivial_radix(sk, m)    fr_trivial
 *   ciphertext.rs:42-45 gen_keys_radix(PARAM_MESSAGE_2_CARRY_2, 4)
 *                                                     fr_gen_client_key + fr_gen_server_key
 *   engine.rs:248-254 read_test_keys: bincode::deserialize + ServerKey::new
 *                                                     fr_load_client_key + fr_gen_server_key
 *   engine.rs:238-246 generate_test_keys: bincode::serialize(client key)
 *                                                     fr_serialize_client_key
 *   engine.rs:8 has_match(sk, ...): a server holding only sk
 *                                                     fr_export_server_key -> fr_load_server_key
 *   ciphertext.rs:32-40 encrypt_str / RadixClientKey::encrypt
 *                                                     fr_encrypt_str (client side, test/bench)
 *   mod.rs:17 / engine.rs:289 RadixClientKey::decrypt fr_decrypt_radix (client side)
 *   engine.rs:8-42    has_match(sk, content, pattern) fr_has_match (whole engine, batched)
 *
 * Conventions: every function returns FR_OK (0) or a negative FR_ERR_* code;
 * the message of the last error on this thread is fr_last_error().  No C++
 * exception crosses the ABI.  Ciphertexts are opaque handles (fr_ct) into a
 * device arena owned by the context; inputs are never mutated and every op
 * writes a fresh handle (the reference always passes clones,
 * execution.rs:74-76).  One fr_ctx per GPU, driven by one host thread.
 * Host buffers are caller-owned and copied in or out.
 *
 * LWE layout on the wire: (k*N + 1) little-endian u64 per block, mask then
 * body, torus 2^64, under the reference's flattened GLWE ("big") key; a radix
 * ciphertext is 4 such blocks, least significant 2-bit digit first
 * (ciphertext.rs:18-29).
 */
#ifndef FHEREGEX_H
#define FHEREGEX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
    FR_OK = 0,
    FR_ERR_INVALID = -1,      /* bad argument / handle */
    FR_ERR_PARSE = -2,        /* pattern does not parse: reference returns Err (engine.rs:13) */
    FR_ERR_REF_PANIC = -3,    /* the reference would panic (parser.rs:349-351, engine.rs:189-190) */
    FR_ERR_NO_DEVICE = -4,    /* GPU op on a host-only context, or the HIP device is unusable */
    FR_ERR_HIP = -5,          /* HIP runtime error */
    FR_ERR_NO_KEY = -6,       /* client or server key missing */
    FR_ERR_OOM = -7,          /* arena / allocation exhausted */
    FR_ERR_NON_ASCII = -8,    /* encrypt_str on non-ASCII content (ciphertext.rs:33-35) */
};

/* Ring of the blind rotation.  FR_RING_FFT: GLWE/GGSW on the
 * 2^64 torus with an f64 negacyclic FFT (tfhe-rs's own representation);
 * FR_RING_RNS: Z_Q[X]/(X^N+1), Q = 998244353 * 1004535809, exact NTTs.  The
 * server key (fr_export_server_key) is a torus BSK for FFT, mod Q for RNS. */
enum { FR_RING_RNS = 0, FR_RING_FFT = 1 };

typedef struct fr_ctx fr_ctx;
typedef uint32_t fr_ct; /* ciphertext handle: a radix (4 blocks), boolean (block 0 + zeros) or trivial */

typedef struct {
    int32_t k;            /* GLWE dimension (reference: 1)            */
    int32_t N;            /* polynomial size (reference: 2048)        */
    int32_t n;            /* small LWE dimension (742)                */
    int32_t ks_base_log;  /* 3 */
    int32_t ks_level;     /* 5 */
    int32_t pbs_base_log; /* 23 */
    int32_t pbs_level;    /* 1 */
    int32_t ring;         /* blind-rotation ring: FR_RING_RNS (0) or FR_RING_FFT (1) */
    double lwe_sigma;
    double glwe_sigma;
} fr_params;

typedef struct {
    uint64_t ct_ops;        /* reference Execution::ct_operations_count (execution.rs:56-58) */
    uint64_t cache_hits;    /* reference Execution::cache_hits (execution.rs:60-62) */
    uint64_t n_branches;    /* variants enumerated by build_branches (engine.rs:15-18) */
    uint64_t pbs;           /* LUT evaluations (gate outputs) executed */
    uint64_t blind_rotations; /* blind rotations (several LUTs may share one: multi-value bootstrapping) */
    uint64_t levels;        /* dependent PBS levels (launch batches) */
    uint64_t max_level_width;
    double host_ms;         /* parse + enumerate + record + lower + compile (plan-cache hit: the lookup) */
    double device_ms;       /* device execution, wall (fr_set_async on: until the launches are enqueued) */
    /* This match's kernel timers (fr_set_profiling on).  Filled only by a blocking call
     * (fr_set_async(ctx, 0)); an asynchronous call returns before its kernels run and
     * leaves them 0: read fr_device_timers after a synchronising call instead. */
    double br_kernel_ms;    /* sum of blind-rotation kernel durations (HIP events) */
    double ks_kernel_ms;    /* sum of lincomb+keyswitch kernel durations (HIP events) */
    uint64_t br_launches;
    uint64_t br_gates;      /* bootstraps across all blind-rotation launches */
    uint64_t plan_cached;   /* 1: the match replayed a cached plan (fr_set_plan_cache) */
} fr_match_stats;

/* ----- context ----- */
/* device >= 0: HIP device ordinal; device == -1: host-only context (parse,
 * record, plan, keygen, plaintext evaluation; GPU ops return FR_ERR_NO_DEVICE). */
int fr_ctx_create(const fr_params* params, int device, fr_ctx** out);
int fr_ctx_destroy(fr_ctx* ctx);
const char* fr_last_error(void);
int fr_default_params(fr_params* out); /* PARAM_MESSAGE_2_CARRY_2, k=1, N=2048 */

/* ----- keys ----- */
/* bincode RadixClientKey (tfhe-rs 0.2 layout, reference test_data/client_key). */
int fr_load_client_key(fr_ctx* ctx, const uint8_t* bincode, size_t len);
/* A fresh client key (gen_keys_radix(&PARAM_MESSAGE_2_CARRY_2, 4), ciphertext.rs:44):
 * uniform binary GLWE key (k*N bits, flattened: the big LWE key) and LWE key (n bits)
 * drawn from a ChaCha20 stream of `seed` (the reference draws from the OS CSPRNG; a seed
 * makes the key reproducible), the parameter block of the context's params.  Replaces
 * any loaded client key and drops the server key. */
int fr_gen_client_key(fr_ctx* ctx, uint64_t seed);
/* bincode of the context's client key in the layout fr_load_client_key reads
 * (engine.rs:238-246 generate_test_keys): for a loaded key, the loaded bytes exactly.
 * buf == NULL: size query (*written = bytes needed). */
int fr_serialize_client_key(fr_ctx* ctx, uint8_t* buf, size_t cap, size_t* written);
/* Deterministic server key (KSK mod 2^64; BSK on the 2^64 torus for the FFT
 * ring, mod Q for the RNS ring) from the client key and a seed
 * (ServerKey::new, engine.rs:252; gen_keys_radix, ciphertext.rs:44).  With a
 * device and the FFT ring it is generated on the GPU (FR_KEYGEN_AUTO); the
 * host generator gives the same words bit for bit (fr_set_keygen). */
int fr_gen_server_key(fr_ctx* ctx, uint64_t seed);
enum { FR_KEYGEN_AUTO = 0, FR_KEYGEN_HOST = 1, FR_KEYGEN_DEVICE = 2 };
int fr_set_keygen(fr_ctx* ctx, int32_t where);
/* Export the server key: ksk = kN*ks_level*(n+1) u64 ; bsk = W*(k+1)^2*N u64
 * (coefficient domain, torus 2^64 (FFT ring) or mod Q = 998244353*1004535809
 * (RNS ring), layout [w][row][component][coef]).
 * k = 1 or the FFT ring: bootstrapping-key unrolling, W = 3*ceil(n/2) GGSWs,
 * w = 3t+g encrypts s_2t*s_2t+1, s_2t*(1-s_2t+1), (1-s_2t)*s_2t+1 for g = 0, 1, 2;
 * RNS ring with k > 1: W = n, GGSW w encrypts s_w.  Sizes from
 * fr_server_key_sizes.  Either may be NULL. */
int fr_export_server_key(fr_ctx* ctx, uint64_t* ksk, size_t ksk_len, uint64_t* bsk, size_t bsk_len);
int fr_server_key_sizes(fr_ctx* ctx, size_t* ksk_len, size_t* bsk_len);
/* Install a server key in fr_export_server_key's layout: a server context that
 * holds only `sk`, as has_match(sk, content, pattern) takes it (engine.rs:8), never
 * the client key (the reference keeps both in one process: gen_keys, ciphertext.rs:42-45;
 * ServerKey::new, engine.rs:252).  Needs no client key; any client key stays.  The
 * device transforms the BSK into its ring's domain as after fr_gen_server_key.  Lengths
 * other than fr_server_key_sizes' -> FR_ERR_INVALID.  This is the build's own layout,
 * not tfhe-rs's bincode ServerKey. */
int fr_load_server_key(fr_ctx* ctx, const uint64_t* ksk, size_t ksk_len, const uint64_t* bsk, size_t bsk_len);

/* ----- client side (tests / bench; not on the timed path) ----- */
int fr_encrypt_str(fr_ctx* ctx, const char* s, size_t len, uint64_t seed, uint64_t* out /* len*4*(kN+1) */);
int fr_encrypt_blocks(fr_ctx* ctx, const uint8_t* msgs, size_t count, uint64_t seed, uint64_t first_block,
                      uint64_t* out /* count*(kN+1) */);
int fr_decrypt_radix(fr_ctx* ctx, const uint64_t* blocks /* 4*(kN+1) */, uint64_t* value);
int fr_decode_block(fr_ctx* ctx, const uint64_t* lwe, uint32_t* msg_and_carry);

/* ----- ciphertext arena ----- */
int fr_upload_radix(fr_ctx* ctx, const uint64_t* blocks /* n*4*(kN+1) */, size_t n, fr_ct* out /* n */);
int fr_upload_bool(fr_ctx* ctx, const uint64_t* lwe /* n*(kN+1) */, size_t n, fr_ct* out);
/* encrypt_str (ciphertext.rs:32-40) on the device, straight into n_chars
 * content handles: the same ciphertext words as fr_encrypt_str (same seed),
 * without the host encryption and the 64 KB-per-char upload. */
int fr_encrypt_upload_str(fr_ctx* ctx, const char* s, size_t len, uint64_t seed, fr_ct* out /* len */);
/* Wire format of a radix ciphertext: bincode (fixint, little endian) of tfhe-rs
 * 0.2 RadixCiphertext — u64 n_blocks, then per block u64 len (= kN+1), the LWE
 * words, u64 degree, u64 message_modulus (4), u64 carry_modulus (4).  [ext]
 * unverified against tfhe-rs (absent here); follows the conventions of the
 * verified client-key layout (Vec<u64> = u64 length + words, usize = u64).
 * buf == NULL / blocks == NULL: size query only. */
int fr_radix_serialize(fr_ctx* ctx, const uint64_t* blocks, size_t n_blocks, uint64_t degree, uint8_t* buf, size_t cap,
                       size_t* written);
int fr_radix_deserialize(fr_ctx* ctx, const uint8_t* buf, size_t len, uint64_t* blocks, size_t max_blocks,
                         size_t* n_blocks);
int fr_download_radix(fr_ctx* ctx, fr_ct h, uint64_t* out /* 4*(kN+1) */);
int fr_release(fr_ctx* ctx, fr_ct h);
int fr_trivial(fr_ctx* ctx, uint8_t value, fr_ct* out);

/* ----- eager gate ops: one call per reference smart_* call ----- */
int fr_eq_const(fr_ctx* ctx, fr_ct a, uint8_t c, fr_ct* out);
int fr_gt_const(fr_ctx* ctx, fr_ct a, uint8_t c, fr_ct* out);
int fr_le_const(fr_ctx* ctx, fr_ct a, uint8_t c, fr_ct* out);
int fr_and(fr_ctx* ctx, fr_ct a, fr_ct b, fr_ct* out);
int fr_or(fr_ctx* ctx, fr_ct a, fr_ct b, fr_ct* out);
int fr_not(fr_ctx* ctx, fr_ct a, fr_ct* out);
/* OR of n boolean ciphertexts (multi-GPU partial-result reduction). */
int fr_or_many(fr_ctx* ctx, const fr_ct* in, size_t n, fr_ct* out);

/* ----- batched gate program ----- */
/* One programmable bootstrap of s = offset/2 + sum_i w_i * in_i (offset in
 * units of Delta/2; inputs are boolean/radix-block handles, block in_block[i]
 * of in[i]).  kind FR_GATE_LUT: s integral in [0,16), out = lut[s];
 * kind FR_GATE_SIGN: s half-integral in (-16,16), out = [s > 0] (threshold
 * AND/OR of up to 16 booleans). */
enum { FR_GATE_LUT = 0, FR_GATE_SIGN = 1 };
typedef struct {
    int32_t n_in;
    int32_t offset;
    int32_t kind;
    fr_ct in[16];
    int8_t in_block[16];
    int8_t in_w[16];
    uint8_t lut[16];
    fr_ct out; /* filled by fr_run_gates: a fresh boolean handle */
} fr_gate;
/* Runs n gates; a gate may consume the output of an earlier gate in the same
 * call by referencing FR_GATE_REF(j) as its input handle.  Level-scheduled
 * into batched device launches. */
#define FR_GATE_REF(j) (0x80000000u | (uint32_t)(j))
int fr_run_gates(fr_ctx* ctx, fr_gate* gates, size_t n);

/* ----- the engine (engine.rs:8-42) ----- */
/* Enumerate, record, lower and execute has_match over content handles.  The
 * result is a boolean radix handle (decrypts to 0/1).  Pattern errors return
 * FR_ERR_PARSE / FR_ERR_REF_PANIC like the reference.  By default the call returns
 * once the match's launches are enqueued on the context's stream: the result
 * handle can be used at once (every later operation of the context is ordered after
 * the match, and downloads wait for it), so consecutive matches overlap their host
 * work with the device's; fr_set_async(ctx, 0) makes the engine calls block until
 * the device has finished. */
int fr_set_async(fr_ctx* ctx, int32_t on);
/* Lanes (round 5; serving with one key): n >= 2 gives the context's device n more
 * streams ("lanes") beside its own, each with its own keyswitch scratch and content map;
 * consecutive asynchronous
 * matches of a cacheable plan go round-robin over the lanes (each lane its own copy of the
 * plan), so one match's small levels share the chip with the next match's first level.
 * Every other operation runs on lane 0 after the lanes' enqueued work (device-side event
 * waits); results are bit-identical to n = 1.  n = 1 (default): one stream.  1 <= n <= 8. */
int fr_set_lanes(fr_ctx* ctx, int32_t n);
int fr_has_match(fr_ctx* ctx, const fr_ct* content, size_t n_chars, const char* pattern, fr_ct* out,
                 fr_match_stats* stats);
/* Same, restricted to start offsets [start_lo, start_hi) — the per-GPU shard of
 * the start-offset partition (the OR over shards equals has_match). */
int fr_has_match_range(fr_ctx* ctx, const fr_ct* content, size_t n_chars, const char* pattern, size_t start_lo,
                       size_t start_hi, fr_ct* out, fr_match_stats* stats);
/* Same start range, the result as *n_parts <= max_parts booleans out[0..n_parts) whose OR
 * is fr_has_match_range's result (round 5).  The threshold lowering's OR tree over the
 * range's start offsets (engine.rs:22-35) stops once <= max_parts literals remain, so a
 * caller OR-ing the parts of W start shards (W * max_parts <= 16: one threshold OR) spends
 * the tree's last level once instead of once per shard plus once to combine.  Faithful
 * lowerings, and roots that are not an OR, give one part.  1 <= max_parts <= 16; out has
 * room for max_parts handles; each part is a boolean handle of its own. */
int fr_has_match_parts(fr_ctx* ctx, const fr_ct* content, size_t n_chars, const char* pattern, size_t start_lo,
                       size_t start_hi, size_t max_parts, fr_ct* out, size_t* n_parts, fr_match_stats* stats);
/* n_matches independent has_match calls of one pattern over n_matches contents
 * of n_chars each (content[m * n_chars + q], out[m]): the matches' circuits run
 * as one plan, so each dependency level of all matches shares its launches
 * (throughput mode; every out[m] is bit-identical to fr_has_match on content m).
 * stats: ct_ops / cache_hits / n_branches of one match; pbs, blind_rotations of
 * the batch; levels of one match (= of the batch). */
int fr_has_match_batch(fr_ctx* ctx, const fr_ct* content, size_t n_chars, size_t n_matches, const char* pattern,
                       fr_ct* out, fr_match_stats* stats);
/* Plan cache: has_match circuits are data-oblivious, so the lowered, compiled
 * plan of (pattern, grammar, engine, lowering, multi-value, n_chars, batch size,
 * start range, content shape) is kept -- its intermediate slots and its
 * device-resident gate batches -- and a repeat call binds the call's content
 * slots (a content map read by the keyswitch) and enqueues the levels.  The
 * content shape is which blocks are trivial (and their values) and which
 * positions share a ciphertext, not the ciphertexts: fresh content of the same
 * shape hits.  capacity = plans kept (LRU; default 8, env FR_PLAN_CACHE); 0
 * disables and frees every cached plan.  max_slots bounds the intermediate arena
 * slots all cached plans hold ((kN+1) u64 each; default 2^18, env
 * FR_PLAN_CACHE_SLOTS); eviction runs before a new plan allocates, and a plan
 * larger than max_slots runs uncached. */
int fr_set_plan_cache(fr_ctx* ctx, size_t capacity);
int fr_set_plan_cache_slots(fr_ctx* ctx, size_t max_slots);
int fr_plan_cache_stats(fr_ctx* ctx, uint64_t* entries, uint64_t* slots, uint64_t* hits, uint64_t* misses);

/* Booleans (block 0 of each handle) to / from a device buffer of n * (kN+1) u64
 * (the start-offset shards' partial results gathered over RCCL without a host
 * round trip; the reference's final ct_or fold, engine.rs:22-35).  Both
 * synchronise the library's stream before returning. */
int fr_export_bool_device(fr_ctx* ctx, const fr_ct* h, size_t n, uint64_t* dev_dst);
int fr_import_bool_device(fr_ctx* ctx, const uint64_t* dev_src, size_t n, fr_ct* out);
/* Stream-ordered export (n <= 16): enqueued on the library's stream (fr_stream) after
 * every earlier operation of the context, returns without synchronising; a caller
 * orders its own stream after it with an event (e.g. the RCCL all-gather of the
 * start-offset shards, which then never blocks the host between matches).  Handles
 * with a trivial block 0 take the synchronising path. */
int fr_export_bool_device_async(fr_ctx* ctx, const fr_ct* h, size_t n, uint64_t* dev_dst);
/* The context's HIP stream (hipStream_t): every device operation of the context is
 * ordered on it. */
int fr_stream(fr_ctx* ctx, void** stream);
/* Accumulated kernel timers of the profiling mode (fr_set_profiling): blind
 * rotation and (level 2) keyswitch milliseconds, launches and bootstraps. */
int fr_device_timers(fr_ctx* ctx, double* br_ms, double* ks_ms, uint64_t* br_launches, uint64_t* br_gates);
/* The part of those blind-rotation timers spent in latency-shape launches (at
 * most one bootstrap per CU: one workgroup per CU). */
int fr_device_timers_latency(fr_ctx* ctx, double* br_ms, uint64_t* br_launches, uint64_t* br_gates);
/* ... and in pair-shape launches (FFT ring, k = 1: two bootstraps per workgroup in the
 * latency geometry, for batches above the latency shape's limit). */
int fr_device_timers_pair(fr_ctx* ctx, double* br_ms, uint64_t* br_launches, uint64_t* br_gates);

/* ----- one match split across ranks ----- */
/* The reference folds ct_or over the branches of every start offset
 * (engine.rs:15-35, each branch a chain of execution.rs:76-190 calls); anchored
 * patterns have one start (engine.rs:51-57), so start offsets alone do not
 * spread their work.  A shard plan splits every dependency level of the lowered
 * circuit instead: each rank compiles the same plan over its copy of the
 * content (same pattern, content length and start range on every rank), runs a
 * contiguous slice [begin, end) of each level's rotation jobs, exports the
 * slice's output LWEs (kN+1 u64 each, job order) into a device buffer, and after
 * an all-gather imports the other ranks' slices; the last level's output then
 * exists on the ranks that hold it (fr_shard_finish).  Levels are 0-based.
 * export / import synchronise the library's stream before returning; the
 * caller orders its own stream (the all-gather) around them.  The plan reads the
 * content handles' arena slots as they were at fr_shard_plan: the content must
 * stay alive (not fr_release'd) until fr_shard_free.  fr_shard_plan merges
 * same-input gates by arena slot, so its levels equal fr_schedule_match's only
 * when every content handle is distinct and encrypted (fheregex.closure_parts
 * checks that the two agree). */
typedef struct fr_shard fr_shard;
int fr_shard_plan(fr_ctx* ctx, const fr_ct* content, size_t n_chars, const char* pattern, size_t start_lo,
                  size_t start_hi, fr_shard** out, fr_match_stats* stats);
int fr_shard_levels(const fr_shard* sh, uint32_t* levels);
int fr_shard_jobs(const fr_shard* sh, uint32_t level, uint32_t* jobs);
int fr_shard_outputs(const fr_shard* sh, uint32_t level, uint32_t begin, uint32_t end, uint32_t* n_lwe);
int fr_shard_run(fr_ctx* ctx, fr_shard* sh, uint32_t level, uint32_t begin, uint32_t end); /* async */
int fr_shard_export(fr_ctx* ctx, fr_shard* sh, uint32_t level, uint32_t begin, uint32_t end, uint64_t* dev_dst);
int fr_shard_import(fr_ctx* ctx, fr_shard* sh, uint32_t level, uint32_t begin, uint32_t end, const uint64_t* dev_src);
/* boolean result handle (valid on a rank that ran or imported the last level) */
int fr_shard_finish(fr_ctx* ctx, fr_shard* sh, fr_ct* out, fr_match_stats* stats);
int fr_shard_free(fr_ctx* ctx, fr_shard* sh);

/* The schedule of such a plan without a device (CPU evaluators, tests): rotation
 * job j of level l is jobs[level_off[l] .. level_off[l+1]); every content
 * position of [0, n_chars) counts as an encrypted radix character.  in_ref[q] >= 0
 * is the output of program gate in_ref[q], in_ref[q] < 0 content block
 * -1 - in_ref[q] (= 4 pos + block, LSB block first); job input s = offset/2 +
 * sum w_q in_q (units of Delta); kind 1: out_gate[0] = lut[0][s]; kind 0
 * (multi-value): out_gate[f] = lut[f][s], f < n_out; kind 2: [s > 0].  out3 =
 * (out_gate, out_w, out_const): result = out_const + out_w * gate (out_gate < 0:
 * the constant).  Pass jobs / level_off = NULL to query the sizes. */
typedef struct {
    int32_t n_in;
    int32_t offset;
    int32_t in_ref[16];
    int32_t in_w[16];
    int32_t n_out;
    int32_t kind;
    int32_t out_gate[8];
    uint8_t lut[8][16];
} fr_job;
int fr_schedule_match(size_t n_chars, const char* pattern, size_t start_lo, size_t start_hi, int32_t lowering,
                      int32_t engine, int32_t grammar, int32_t multi_value, fr_job* jobs, size_t jobs_cap,
                      size_t* n_jobs, uint32_t* level_off, size_t level_cap, size_t* n_levels, int32_t* out3);
/* The schedule of fr_has_match_parts' program: outs3[3j .. 3j+2] = part j's (out_gate,
 * out_w, out_const), j < *n_parts (outs3 has room for 3 * max_parts). */
int fr_schedule_match_parts(size_t n_chars, const char* pattern, size_t start_lo, size_t start_hi, int32_t lowering,
                            int32_t engine, int32_t grammar, int32_t multi_value, size_t max_parts, fr_job* jobs,
                            size_t jobs_cap, size_t* n_jobs, uint32_t* level_off, size_t level_cap, size_t* n_levels,
                            int32_t* outs3, size_t* n_parts);

/* ----- host-only introspection (tests; no device needed) ----- */
/* Canonical AST string of parse(pattern) (parser.rs:146-185). */
int fr_parse(const char* pattern, char* buf, size_t buflen);
/* Symbolic has_match over a plaintext content string: reference counters and
 * the plaintext result of the recorded circuit and of the lowered PBS program. */
typedef struct {
    uint64_t ct_ops, cache_hits, n_branches;
    uint64_t pbs, levels, max_level_width;
    int32_t result_recorded; /* value of the recorded reference op DAG */
    int32_t result_lowered;  /* value of the lowered PBS program (plaintext LUT semantics) */
} fr_plain_result;
int fr_plain_match(const char* content, size_t len, const char* pattern, size_t start_lo, size_t start_hi,
                   int32_t lowering, fr_plain_result* out);

/* Evaluation engine of the regex (fr_set_engine, fr_plain_match_ex):
 * FR_ENGINE_ENUMERATE: the reference's variant enumeration (engine.rs:45-214),
 *   exact ct_ops / cache_hits; exponential on deep variant trees (BASELINE
 *   config 5 exhausts memory, as in the reference).
 * FR_ENGINE_MERGED: state-merging evaluation (beyond the reference): the same
 *   decrypted result, a circuit polynomial in the content length and of
 *   logarithmic depth for fixed-width loops; ct_ops counts circuit operations.
 * FR_ENGINE_AUTO (default): enumerate within 2^22 variants, else merged. */
enum { FR_ENGINE_AUTO = 0, FR_ENGINE_ENUMERATE = 1, FR_ENGINE_MERGED = 2 };
/* Pattern grammar (fr_set_grammar, fr_parse_ex, fr_plain_match_g):
 * FR_GRAMMAR_REFERENCE (default): parser.rs:146-351 exactly ([a-z0-9] is Err).
 * FR_GRAMMAR_EXT (beyond the reference, opt-in): also bare digits as
 *   characters and bracket classes mixing letters, digits, escapes and
 *   inclusive ranges — [a-z0-9], [^A-Z_], [\-a] — tried only where the
 *   reference grammar fails, so every pattern the reference accepts keeps its
 *   AST (including [a-z]'s strict lower bound, engine.rs:99-111). */
enum { FR_GRAMMAR_REFERENCE = 0, FR_GRAMMAR_EXT = 1 };
int fr_set_grammar(fr_ctx* ctx, int32_t grammar);
int fr_parse_ex(const char* pattern, int32_t grammar, char* buf, size_t buflen);
int fr_plain_match_g(const char* content, size_t len, const char* pattern, size_t start_lo, size_t start_hi,
                     int32_t lowering, int32_t engine, int32_t grammar, fr_plain_result* out);
/* FR_ENGINE_AUTO's decision: the variants the reference's enumeration would build for
 * starts [start_lo, start_hi) of n_chars -- *counted from the AST without building them,
 * *enumerated by running it (enumerate != 0; else 0) -- each saturating at cap + 1.
 * *outcome says whether there is a count: FR_COST_COUNTED; FR_COST_PANIC, where the
 * enumeration would panic (engine.rs:189-190, or a repetition it cannot allocate);
 * FR_COST_MEMORY, where the counter's memo would exceed mem_bytes (0: the bound AUTO uses,
 * 256 MiB; entries and the end positions they store are counted).  Without a count *counted
 * is 0 and AUTO enumerates under its budget, as it would without the counter.  AUTO goes
 * straight to the merged engine iff the count is > 2^22. */
enum { FR_COST_COUNTED = 0, FR_COST_PANIC = 1, FR_COST_MEMORY = 2 };
int fr_debug_enumeration_cost(const char* pattern, int32_t grammar, size_t n_chars, size_t start_lo, size_t start_hi,
                              uint64_t cap, uint64_t mem_bytes, int32_t enumerate, int32_t* outcome,
                              uint64_t* counted, uint64_t* enumerated);
/* fr_plain_match_g of fr_has_match_parts' program: out->result_lowered is the OR of the
 * parts, parts[0..*n_parts) their plaintext values (room for max_parts). */
int fr_plain_match_parts(const char* content, size_t len, const char* pattern, size_t start_lo, size_t start_hi,
                         int32_t lowering, int32_t engine, int32_t grammar, size_t max_parts, fr_plain_result* out,
                         int32_t* parts, size_t* n_parts);
int fr_set_engine(fr_ctx* ctx, int32_t engine);
int fr_plain_match_ex(const char* content, size_t len, const char* pattern, size_t start_lo, size_t start_hi,
                      int32_t lowering, int32_t engine, fr_plain_result* out);

/* lowering modes for fr_plain_match / fr_set_lowering:
 * FR_LOWER_FAITHFUL: one gate group per reference op (eq/gt/le = 3 PBS, and/or = 1,
 *   not linear), in the reference's fold order (engine.rs:22-35: depth #branches).
 * FR_LOWER_THRESHOLD (default): threshold gates of fan-in <= 16, multi-value LUTs.
 * FR_LOWER_FAITHFUL_TREE: FR_LOWER_FAITHFUL's gates, the same PBS count, with every
 *   AND/OR chain whose inner links are used once rebalanced into a binary tree of
 *   least depth (/abc/ x 256: 3,047 PBS in 13 levels, not 257). */
enum { FR_LOWER_FAITHFUL = 0, FR_LOWER_THRESHOLD = 1, FR_LOWER_FAITHFUL_TREE = 2 };
int fr_set_lowering(fr_ctx* ctx, int32_t mode);
/* Multi-value bootstrapping: gates of one level that read the same linear
 * combination share one blind rotation (default on). */
int fr_set_multi_value(fr_ctx* ctx, int32_t on);
/* Device profiling: 0 off; 1 blind-rotation timers (HIP stop events stamped by the
 * launches themselves, hipExtLaunchKernel: no marker packets, no syncs; a level's blind
 * rotation runs from its keyswitch's stop event to its own, the launch gap between them
 * included; what bench.py's timed region uses; FR_TIMER_CHAIN=0 stamps a start event on
 * the blind rotation instead, 9-15 us more per launch); 2 also the keyswitch timers (start
 * and stop events on every level's keyswitch, ~30 us per /abc/ x 256 match).  Timers
 * resolve at the next synchronisation.  Any other value is FR_ERR_INVALID. */
int fr_set_profiling(fr_ctx* ctx, int32_t on);

/* ----- single-stage device entry points (parity tests of each kernel) ----- */
/* in: count*(kN+1) torus LWEs -> out: count*(n+1) keyswitched LWEs */
int fr_dev_keyswitch(fr_ctx* ctx, const uint64_t* in, size_t count, uint64_t* out);
/* in: count*(n+1) keyswitched LWEs, luts: count*16 -> out: count*(kN+1) */
int fr_dev_blind_rotate(fr_ctx* ctx, const uint64_t* in, const uint8_t* luts, size_t count, uint64_t* out);
/* one blind rotation with n_out LUTs (direct: n_out == 1, LUT polynomial
 * rotated itself; else multi-value) -> out: n_out*(kN+1) */
int fr_dev_blind_rotate_multi(fr_ctx* ctx, const uint64_t* in, const uint8_t* luts, int32_t n_out, int32_t direct,
                              uint64_t* out);
/* negacyclic product in Z_Q[X]/(X^N+1) (Q = 998244353 * 1004535809, inputs in
 * [0, Q)) through the device RNS NTT: count pairs */
int fr_dev_ring_mul(fr_ctx* ctx, const uint64_t* a, const uint64_t* b, size_t count, uint64_t* out);
/* Full timed PBS batch for roofline measurement: count gates of the given
 * lut over the uploaded boolean/radix handles; returns BR kernel ms. */
int fr_dev_bench_pbs(fr_ctx* ctx, const fr_ct* in, size_t count, int32_t iters, double* br_ms, double* total_ms);

int fr_device_info(fr_ctx* ctx, char* buf, size_t buflen);

/* Scalar maps shared by host and device code (test hook): op 0 = CRT of the
 * residues of x (identity on [0, Q)), 1 = PBS gadget digit of x mod Q (signed,
 * as u64), 2 = Z_Q -> 2^64 torus of x mod Q (from its residues),
 * 3 = modulus switch of x to 2^y, 4 = keyswitch digit y (0..4) of x (signed, as u64). */
uint64_t fr_debug_scalar(int32_t op, uint64_t x, uint64_t y);

#ifdef __cplusplus
}
#endif
#endif
