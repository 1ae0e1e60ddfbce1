// Device executor interface (HIP, gfx950).  Kernels live in device.hip.
#pragma once
#include <cstdint>
#include <vector>

#include "common.h"

namespace fr {

constexpr int MAX_OUT = 8;
// One blind-rotation job as the device sees it:
//   c = offset*2^58 + sum_q w_q * arena[in_slot_q];  KS; blind rotation of the
//   test polynomial; out_slot[f] <- LUT_f(c) for f < n_out.
// direct = 1: the test polynomial is LUT_0's own (one output).  direct = 0:
// multi-value bootstrapping, test polynomial (Delta/2)*sum_j X^j and one
// sparse small-integer product w_f per output (see k_blind_rotate).
// direct = 2: sign gate, test polynomial (Delta/2)*sum_j X^j, one output
// [c > 0] obtained as +-Delta/2 + Delta/2.
enum : int32_t { JOB_MULTI = 0, JOB_DIRECT = 1, JOB_SIGN = 2 };
struct DevGate {
    int32_t n_in;
    int32_t offset;  // units of Delta/2 = 2^58
    int32_t in_slot[16];
    int32_t in_w[16];
    int32_t n_out;
    int32_t direct;
    int32_t out_slot[MAX_OUT];
    uint8_t lut[MAX_OUT][16];
};
static_assert(sizeof(DevGate) == 304, "DevGate layout");
// sum of squared w_f coefficients of a LUT (noise growth of its factored output)
int lut_w_norm2(const uint8_t* lut);

struct DeviceTimers {
    double br_ms = 0, ks_ms = 0;
    uint64_t br_launches = 0, br_gates = 0, lut_outputs = 0;
    // the part of the above in latency-shape launches (at most one bootstrap per CU)
    double lat_br_ms = 0;
    uint64_t lat_launches = 0, lat_gates = 0;
    // the part in pair-shape launches (k = 1, two bootstraps per workgroup)
    double pair_br_ms = 0;
    uint64_t pair_launches = 0, pair_gates = 0;
};

struct ClientKey;

class Device {
  public:
    Device(const Params& p, int device);
    ~Device();
    Device(const Device&) = delete;
    Device& operator=(const Device&) = delete;

    const Params& params() const { return p_; }
    int device() const { return dev_; }

    // keys: KSK torus 2^64 [i][j][t]; BSK coefficient domain mod Q [i][r][c][coef]
    void upload_keys(const std::vector<uint64_t>& ksk, const std::vector<uint64_t>& bsk);
    bool has_keys() const { return d_ksk_ && (d_bsk_ || d_fbsk_[0]); }
    // server-key generation on the device (keygen.hip; FFT ring): the same keys
    // as gen_ksk + gen_bsk on the host, bit for bit; the torus keys stay on the
    // device for download_server_key
    void gen_server_key(const ClientKey& ck, uint64_t seed);
    void download_server_key(uint64_t* ksk, size_t ksk_len, uint64_t* bsk, size_t bsk_len);
    // fresh encryptions of block messages (encrypt_blocks, keys.h) written into
    // allocated arena slots, bit-identical to the host encryption
    void encrypt_to_slots(const ClientKey& ck, const uint8_t* msgs, size_t count, uint64_t seed, uint64_t first_block,
                          const int* slots);

    // arena of big-LWE slots
    int alloc_slot();
    void free_slot(int s);
    void write_slots(const int* slots, size_t n, const uint64_t* host /* n * lwe_len */);
    void read_slot(int slot, uint64_t* host /* lwe_len */);
    // packed device-to-device copies of slots (lwe_len u64 each) to / from a device
    // buffer owned by the caller; both synchronise the library's stream on return
    void slots_to_device(const int* slots, size_t n, uint64_t* dst);
    void device_to_slots(const int* slots, size_t n, const uint64_t* src);
    // stream-ordered slots_to_device for n <= 16 (the slot list travels as a kernel
    // argument): returns once enqueued; order other streams after it with an event on stream()
    void slots_to_device_async(const int* slots, size_t n, uint64_t* dst);
    void* stream() const { return stream_; }
    void zero_slot(int slot);

    // run one dependency level of gates (all independent), async on the stream
    void run_level(const DevGate* gates, size_t n);
    // the same for a batch already resident on the device (upload_gates); `host`
    // is its host copy (validated when uploaded; read for the profiling counters).
    // n_refs > 0: the batch reads content references (in_slot = -1 - r, r < n_refs)
    // through the content map bound last (bind_content, at least n_refs entries)
    void run_level_resident(const DevGate* d_gates, const DevGate* host, size_t n, size_t n_refs = 0);
    // validated (content references r < n_refs allowed), synchronous
    DevGate* upload_gates(const DevGate* gates, size_t n, size_t n_refs = 0);
    // content map of a template plan: reference r reads arena slot cmap[r] (-1: not
    // read by the plan).  Stream-ordered: launches enqueued after this call see it,
    // launches enqueued before it keep the previous map.
    void bind_content(const int* cmap, size_t n);
    void free_gates(DevGate* d);                            // after the stream drained
    // linear combination without bootstrap (NOT of a boolean): out = offset*2^58 + sum w*in
    void run_linear(const DevGate& g);
    void sync();

    // Lanes (serving without key copies): lane 0 is the stream above; lanes 1..n are
    // further streams of this device with their own keyswitch / digit scratch and content
    // map, sharing the keys and the arena.  Between enter_lane(i) and leave_lane() every
    // launch goes to lane i's stream, ordered after everything enqueued on lane 0 so far.
    // Work on lane 0 waits (device-side, by event) for every lane's enqueued work before it
    // runs; slots freed while a lane may still read them return to the free list only after
    // a host synchronisation of every lane (sync()).
    void set_lanes(int n);                                 // n = 1: lane 0 only; n >= 2: lanes 1..n beside it
    int match_lanes() const { return (int)lanes_.size(); }  // lanes asynchronous matches go to
    void enter_lane(int i);
    void leave_lane();
    void set_profiling(int level) { profiling_ = level; }
    DeviceTimers& timers() { return timers_; }

    // single-stage entry points for parity tests
    void keyswitch_host(const uint64_t* in, size_t count, uint64_t* out);
    void blind_rotate_host(const uint64_t* ks_in, const uint8_t* luts, size_t count, uint64_t* out);
    // one job with n_out LUTs on one keyswitched input (multi-value or direct)
    void blind_rotate_multi_host(const uint64_t* ks_in, const uint8_t* luts, int n_out, int direct, uint64_t* out);
    void ring_mul_host(const uint64_t* a, const uint64_t* b, size_t count, uint64_t* out);
    // repeated full-PBS batches on resident inputs (bench / roofline)
    void bench_pbs(const std::vector<DevGate>& gates, int iters, double* br_ms, double* total_ms);

    std::string info() const;

  private:
    struct LaneState {
        void* stream = nullptr;
        uint64_t* d_ks = nullptr;
        size_t batch_cap = 0;
        int8_t* d_dig = nullptr;
        size_t dig_cap = 0;
        int* d_cmap = nullptr;
        int* h_cmap[2] = {nullptr, nullptr};
        void* cmap_ev[2] = {nullptr, nullptr};
        size_t cmap_cap = 0, cmap_n = 0;
        int cmap_stage = 0;
        void* done_ev = nullptr;  // recorded on the lane's stream when it is left
        bool pending = false;     // work enqueued since lane 0 last waited for it
    };
    std::vector<LaneState> lanes_;  // lanes 1..n
    int lane_ = 0;                  // current lane
    bool lanes_pending_ = false;
    bool lanes_unsynced_ = false;   // lane work not yet host-synchronised (deferred frees)
    void* main_ev_ = nullptr;       // lane 0's progress, waited for by a lane on entry
    std::vector<int> deferred_free_;
    void swap_lane(LaneState& l);
    // the stream of the current lane; on lane 0 it first waits (device-side) for the lanes
    void* cur_stream();
    void join_lanes();
    void sync_all();  // host-synchronise every lane, recycle the deferred slots
    void free_lane(LaneState& l);
    void ensure_arena(size_t slots);
    void ensure_batch(size_t n);
    // pinned staging ring for gate descriptors: a buffer is rewritten only after
    // its previous H2D copy completed (no stream-wide sync between levels)
    DevGate* stage_acquire();
    void stage_copy(size_t n);
    void validate_gates(const DevGate* gates, size_t n, size_t n_refs = 0) const;
    void launch_level(const DevGate* d_gates, const DevGate* host, size_t n);
    // profiling: per-level event triples resolved at sync() (no sync per level)
    void* take_event();
    void resolve_timers();
    void ensure_digits(size_t rows);
    // ev_start / ev_stop (profiling): HIP events stamped by the kernels' own dispatch
    // (hipExtLaunchKernel) -- the first kernel's start and the last one's end -- so timing
    // adds no marker packets between dependent launches (each cost ~5 us of gap)
    void launch_ks(const DevGate* d_gates, size_t n, uint64_t* d_ks, void* ev_start = nullptr, void* ev_stop = nullptr);
    void launch_br(const DevGate* d_gates, const uint64_t* d_ks, size_t n, void* ev_start = nullptr,
                   void* ev_stop = nullptr);
    // FR_RING_FFT (fft.hip)
    void init_fft();
    void upload_fft_bsk(const std::vector<uint64_t>& bsk);
    void launch_br_fft(const DevGate* d_gates, const uint64_t* d_ks, size_t n, void* stream, void* ev_start = nullptr,
                       void* ev_stop = nullptr);
    void free_fft();
    void build_ksk_limbs();  // d_kl_ from d_ksk_
    void stage_slot_list(const int* slots, size_t n);  // -> d_slot_list_ (stream order)
    int* d_slot_list_ = nullptr;
    size_t slot_list_cap_ = 0;
    // content map (bind_content): device copy (rewritten in stream order), pinned
    // staging ring, entries bound
    int* d_cmap_ = nullptr;
    int* h_cmap_[2] = {nullptr, nullptr};
    void* cmap_ev_[2] = {nullptr, nullptr};
    size_t cmap_cap_ = 0, cmap_n_ = 0;
    int cmap_stage_ = 0;

    Params p_;
    int dev_;
    int e_ = 8;        // residues per lane in the NTT kernels (8 or 16; measured: 8 wins for k=1 and k=2)
    int e_small_ = 8;  // ... for launches of at most small_batch_ bootstraps
    size_t small_batch_ = 256;
    void* stream_ = nullptr;  // hipStream_t
    uint64_t* d_ksk_ = nullptr;
    uint64_t* d_tbsk_ = nullptr;  // torus BSK of a device-generated key (export)
    int8_t* d_kl_ = nullptr;      // KSK as balanced byte limbs [col*8 + limb][k] (MFMA keyswitch)
    int kl_cols_ = 0;
    bool ks_mfma_ = true;         // FR_KS_MFMA=0: the VALU lincomb+keyswitch kernel
    size_t ks_mr4_min_ = 96;      // FR_KS_MR4_MIN: batches from this size use 4 row tiles per wave (k_ks_glds; ab_ks_glds.log: 100 gates 44 -> 37 us, 64 gates no gain)
    int ks_mc_ = 0;               // FR_KS_MC=2: two column tiles per wave in the 4-row-tile shape (else one)
    int ks_split_ = 0;            // FR_KS_SPLIT: K slices (a divisor of kN*ks_level/256; 0: auto)
    int ks_xcd_ = 1;              // FR_KS_XCD=0: plain workgroup order of the MFMA keyswitch (k_ks_mfma)
    bool ks_dig16_ = true;        // FR_KS_DIG16=0: the digit pass with byte stores (k_ks_digits)
    bool ks_lds_ = true;          // FR_KS_LDS=0: four-row-tile keyswitch without the LDS-DMA ring (k_ks_mfma<4, 1>)
    int8_t* d_dig_ = nullptr;     // keyswitch digits [rows][kN*ks_level]
    size_t dig_cap_ = 0;
    uint32_t* d_bsk_ = nullptr;  // NTT domain [i][r][c][prime][slot], Montgomery form, scaled by 1/N
    uint32_t* d_tw_ = nullptr;   // Montgomery zeta per prime [2][N]
    // FR_RING_FFT: Fourier BSK [w][r][c][m][lane] (complex f64, scaled by 1/M), twiddles,
    // psi quadrant table, leaf exponents (fft.h)
    int fft_e_ = 4;           // complex points per lane in the throughput shape (4, 8 or 16)
    size_t fft_small_ = 256;  // launches of at most this many bootstraps use the latency shape
    // k = 1: larger launches up to this many use the pair shape (2 per workgroup; every size
    // by default: profiles/r03/ab_pair_shape.log)
    size_t fft_pair_ = SIZE_MAX;
    bool fft_dual_ = false;  // FR_FFT_DUAL=1: the dual shape instead of the pair (experiment)
    // Fourier BSK, one copy per lane geometry in use: [0] E = 4 (latency shape, always),
    // [1] E = 8, [2] E = 16 (the throughput shape's when fft_e_ is that)
    double* d_fbsk_[3] = {nullptr, nullptr, nullptr};
    static int fbsk_index(int E) { return E == 4 ? 0 : E == 8 ? 1 : 2; }
    bool fbsk_needed(int E) const { return E == 4 || E == fft_e_; }
    double* d_ftw_ = nullptr;
    double* d_fqt_ = nullptr;   // psi^k, k < 2N
    uint16_t* d_fleaf_ = nullptr;
    uint64_t* d_arena_ = nullptr;
    size_t arena_cap_ = 0;
    std::vector<int> free_slots_;
    size_t next_slot_ = 0;
    DevGate* d_gates_ = nullptr;
    DevGate* h_stage_[2] = {nullptr, nullptr};  // pinned staging ring
    void* stage_ev_[2] = {nullptr, nullptr};
    int stage_ = 0;
    struct PendingTimer {
        void* ev[4];  // KS start, KS end, BR start, BR end
        size_t gates, outs;
        bool lat, pair, ks;
        bool chain;  // BR timed from the keyswitch's end event (no start event on the BR launch)
    };
    bool latency_shape(size_t n) const;  // launch_br's shape choice for n bootstraps
    bool pair_shape(size_t n) const;     // (FFT ring, k = 1: the pair shape)
    std::vector<PendingTimer> pending_;
    std::vector<void*> event_pool_;
    uint64_t* d_ks_ = nullptr;
    size_t batch_cap_ = 0;
    int profiling_ = 0;  // fr_set_profiling level
    bool timer_chain_ = true;  // level 1: stop events only (FR_TIMER_CHAIN=0: start + stop on the BR launch)
    DeviceTimers timers_;
    void* ev_[4] = {nullptr, nullptr, nullptr, nullptr};
};

}  // namespace fr
