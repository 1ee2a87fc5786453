// sw_capi.cpp — host driver behind the C ABI (include/sw_amd.h).
//
// What the reference does per query (SWSolver.cu:266-404) and what replaces it:
//   * pad/encode the query and upload it to __constant__ (:267-299)
//       -> a 32 x qpad int8 query PROFILE (score of every residue code against
//          every query row, pre-biased by the gap for the linear kernels),
//          built on the host and copied once per query (tiny: 32 B/row);
//   * re-pack the whole database into managed memory on every query,
//     longest-first, 32 lanes per block (:301-371)
//       -> sw_db_create packs ONCE into 64-lane blocks of 16-residue groups,
//          sorted longest-first, and keeps the result resident in HBM;
//   * launch in chunks with cudaDeviceSynchronize after each (:332-354,379)
//       -> one asynchronous launch per kernel on the handle's stream;
//   * read managed scores back in packing order (:383-390)
//       -> kernels write scores[id] directly.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "sw_amd.h"
#include "sw_kernels.h"
#include "sw_plan.h"

namespace {

thread_local std::string g_err;

// fp16 represents every integer in [-kF16Span, kF16Span] exactly
constexpr int kF16Span = 2048;

// packed fp16 pair (v, v) of a small integer (|v| <= 2048: exact)
uint32_t f16_pair(int v) {
    const _Float16 x = static_cast<_Float16>(static_cast<float>(v));
    uint16_t b;
    std::memcpy(&b, &x, 2);
    return static_cast<uint32_t>(b) | (static_cast<uint32_t>(b) << 16);
}

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// record event k of the current scan's set on stream s
#define MARK(k, s)                                  \
    do {                                            \
        HIPCHECK(hipEventRecord(h->ev[k], (s)));    \
        *h->ev_rec |= 1u << (k);                    \
    } while (0)


#define HIPCHECK(expr)                                                                  \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(SW_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));   \
    } while (0)

// ---- built-in matrices (code order ARNDCQEGHILKMFPSTWYVBJZX*) ------------
// BLOSUM50 exactly as tabulated in the reference, SWSolver.cu:54-81.
const int8_t kBlosum50Ref[625] = {
    5, -2, -1, -2, -1, -1, -1, 0, -2, -1, -2, -1, -1, -3, -1, 1, 0, -3, -2, 0, -2, -2, -1, -1, 0,
    -2, 7, -1, -2, -4, 1, 0, -3, 0, -4, -3, 3, -2, -3, -3, -1, -1, -3, -1, -3, -1, -3, 0, -1, 0,
    -1, -1, 7, 2, -2, 0, 0, 0, 1, -3, -4, 0, -2, -4, -2, 1, 0, -4, -2, -3, 5, -4, 0, -1, 0,
    -2, -2, 2, 8, -4, 0, 2, -1, -1, -4, -4, -1, -4, -5, -1, 0, -1, -5, -3, -4, 6, -4, 1, -1, 0,
    -1, -4, -2, -4, 13, -3, -3, -3, -3, -2, -2, -3, -2, -2, -4, -1, -1, -5, -3, -1, -3, -2, -3, -1, 0,
    -1, 1, 0, 0, -3, 7, 2, -2, 1, -3, -2, 2, 0, -4, -1, 0, -1, -1, -1, -3, 0, -3, 4, -1, 0,
    -1, 0, 0, 2, -3, 2, 6, -3, 0, -4, -3, 1, -2, -3, -1, -1, -1, -3, -2, -3, 1, -3, 5, -1, 0,
    0, -3, 0, -1, -3, -2, -3, 8, -2, -4, -4, -2, -3, -4, -2, 0, -2, -3, -3, -4, -1, -4, -2, -1, 0,
    -2, 0, 1, -1, -3, 1, 0, -2, 10, -4, -3, 0, -1, -1, -2, -1, -2, -3, 2, -4, 0, -3, 0, -1, 0,
    -1, -4, -3, -4, -2, -3, -4, -4, -4, 5, 2, -3, 2, 0, -3, -3, -1, -3, -1, 4, -4, 4, -3, -1, 0,
    -2, -3, -4, -4, -2, -2, -3, -4, -3, 2, 5, -3, 3, 1, -4, -3, -1, -2, -1, 1, -4, 4, -3, -1, 0,
    -1, 3, 0, -1, -3, 2, 1, -2, 0, -3, -3, 6, -2, -4, -1, 0, -1, -3, -2, -3, 0, -3, 1, -1, 0,
    -1, -2, -2, -4, -2, 0, -2, -3, -1, 2, 3, -2, 7, 0, -3, -2, -1, -1, 0, 1, -3, 2, -1, -1, 0,
    -3, -3, -4, -5, -2, -4, -3, -4, -1, 0, 1, -4, 0, 8, -4, -3, -2, 1, 4, -1, -4, 1, -4, -1, 0,
    -1, -3, -2, -1, -4, -1, -1, -2, -2, -3, -4, -1, -3, -4, 10, -1, -1, -4, -3, -3, -2, -3, -1, -1, 0,
    1, -1, 1, 0, -1, 0, -1, 0, -1, -3, -3, 0, -2, -3, -1, 5, 2, -4, -2, -2, 0, -3, 0, -1, 0,
    0, -1, 0, -1, -1, -1, -1, -2, -2, -1, -1, -1, -1, -2, -1, 2, 5, -3, -2, 0, 0, -1, -1, -1, 0,
    -3, -3, -4, -5, -5, -1, -3, -3, -3, -3, -2, -3, -1, 1, -4, -4, -3, 15, 2, -3, -5, -2, -2, -1, 0,
    -2, -1, -2, -3, -3, -1, -2, -3, 2, -1, -1, -2, 0, 4, -3, -2, -2, 2, 8, -1, -3, -1, -2, -1, 0,
    0, -3, -3, -4, -1, -3, -3, -4, -4, 4, 1, -3, 1, -1, -3, -2, 0, -3, -1, 5, -3, 2, -3, -1, 0,
    -2, -1, 5, 6, -3, 0, 1, -1, 0, -4, -4, 0, -3, -4, -2, 0, 0, -5, -3, -3, 6, -4, 1, -1, 0,
    -2, -3, -4, -4, -2, -3, -3, -4, -3, 4, 4, -3, 2, 1, -3, -3, -1, -2, -1, 2, -4, 4, -3, -1, 0,
    -1, 0, 0, 1, -3, 4, 5, -2, 0, -3, -3, 1, -1, -4, -1, 0, -1, -2, -2, -3, 1, -3, 5, -1, 0,
    -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, 0,
    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
};

// NCBI BLOSUM62 with J; an option of this build (the reference has none).
const int8_t kBlosum62[625] = {
    4, -1, -2, -2, 0, -1, -1, 0, -2, -1, -1, -1, -1, -2, -1, 1, 0, -3, -2, 0, -2, -1, -1, 0, -4,
    -1, 5, 0, -2, -3, 1, 0, -2, 0, -3, -2, 2, -1, -3, -2, -1, -1, -3, -2, -3, -1, -2, 0, -1, -4,
    -2, 0, 6, 1, -3, 0, 0, 0, 1, -3, -3, 0, -2, -3, -2, 1, 0, -4, -2, -3, 3, -3, 0, -1, -4,
    -2, -2, 1, 6, -3, 0, 2, -1, -1, -3, -4, -1, -3, -3, -1, 0, -1, -4, -3, -3, 4, -3, 1, -1, -4,
    0, -3, -3, -3, 9, -3, -4, -3, -3, -1, -1, -3, -1, -2, -3, -1, -1, -2, -2, -1, -3, -1, -3, -2, -4,
    -1, 1, 0, 0, -3, 5, 2, -2, 0, -3, -2, 1, 0, -3, -1, 0, -1, -2, -1, -2, 0, -2, 3, -1, -4,
    -1, 0, 0, 2, -4, 2, 5, -2, 0, -3, -3, 1, -2, -3, -1, 0, -1, -3, -2, -2, 1, -3, 4, -1, -4,
    0, -2, 0, -1, -3, -2, -2, 6, -2, -4, -4, -2, -3, -3, -2, 0, -2, -2, -3, -3, -1, -4, -2, -1, -4,
    -2, 0, 1, -1, -3, 0, 0, -2, 8, -3, -3, -1, -2, -1, -2, -1, -2, -2, 2, -3, 0, -3, 0, -1, -4,
    -1, -3, -3, -3, -1, -3, -3, -4, -3, 4, 2, -3, 1, 0, -3, -2, -1, -3, -1, 3, -3, 3, -3, -1, -4,
    -1, -2, -3, -4, -1, -2, -3, -4, -3, 2, 4, -2, 2, 0, -3, -2, -1, -2, -1, 1, -4, 3, -3, -1, -4,
    -1, 2, 0, -1, -3, 1, 1, -2, -1, -3, -2, 5, -1, -3, -1, 0, -1, -3, -2, -2, 0, -3, 1, -1, -4,
    -1, -1, -2, -3, -1, 0, -2, -3, -2, 1, 2, -1, 5, 0, -2, -1, -1, -1, -1, 1, -3, 2, -1, -1, -4,
    -2, -3, -3, -3, -2, -3, -3, -3, -1, 0, 0, -3, 0, 6, -4, -2, -2, 1, 3, -1, -3, 0, -3, -1, -4,
    -1, -2, -2, -1, -3, -1, -1, -2, -2, -3, -3, -1, -2, -4, 7, -1, -1, -4, -3, -2, -2, -3, -1, -2, -4,
    1, -1, 1, 0, -1, 0, 0, 0, -1, -2, -2, 0, -1, -2, -1, 4, 1, -3, -2, -2, 0, -2, 0, 0, -4,
    0, -1, 0, -1, -1, -1, -1, -2, -2, -1, -1, -1, -1, -2, -1, 1, 5, -2, -2, 0, -1, -1, -1, 0, -4,
    -3, -3, -4, -4, -2, -2, -3, -2, -2, -3, -2, -3, -1, 1, -4, -3, -2, 11, 2, -3, -4, -2, -3, -2, -4,
    -2, -2, -2, -3, -2, -1, -2, -3, 2, -1, -1, -2, -1, 3, -3, -2, -2, 2, 7, -1, -3, -1, -2, -1, -4,
    0, -3, -3, -3, -1, -2, -2, -3, -3, 3, 1, -2, 1, -1, -2, -2, 0, -3, -1, 4, -3, 2, -2, -1, -4,
    -2, -1, 3, 4, -3, 0, 1, -1, 0, -3, -4, 0, -3, -3, -2, 0, -1, -4, -3, -3, 4, -3, 1, -1, -4,
    -1, -2, -3, -3, -1, -2, -3, -4, -3, 3, 3, -3, 2, 0, -3, -2, -1, -2, -1, 2, -3, 3, -3, -1, -4,
    -1, 0, 0, 1, -3, 3, 4, -2, 0, -3, -3, 1, -1, -3, -1, 0, -1, -3, -2, -2, 1, -3, 4, -1, -4,
    0, -1, -1, -1, -2, -1, -1, -1, -1, -1, -1, -1, -1, -1, -2, 0, 0, -2, -1, -1, -1, -1, -1, -1, -4,
    -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, -4, 1,
};

int8_t g_encode_lut[256];
bool g_lut_ready = false;

void init_lut() {
    if (g_lut_ready) return;
    static const char letters[] = "ARNDCQEGHILKMFPSTWYVBJZX";  // SWSolver.cu:17-40
    for (int c = 0; c < 256; ++c) g_encode_lut[c] = SW_CODE_STAR;  // SWSolver.cu:119
    for (int k = 0; k < 24; ++k) g_encode_lut[static_cast<unsigned char>(letters[k])] = static_cast<int8_t>(k);
    g_lut_ready = true;
}

int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

int default_threads() {
    unsigned n = std::thread::hardware_concurrency();
    if (n == 0) n = 4;
    return static_cast<int>(std::min(16u, n));  // GPU boxes expose many more CPUs than our share
}

// f(i) for i in [0, n) on up to default_threads() threads, `grain` indices
// per grab (at least one grab per thread).
template <class F>
void parallel_for(int64_t n, F&& f, int64_t grain = 64) {
    const int nt = static_cast<int>(std::min<int64_t>(default_threads(), std::max<int64_t>(1, n / grain)));
    if (nt <= 1) {
        for (int64_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<int64_t> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t)
        th.emplace_back([&] {
            for (;;) {
                const int64_t i0 = next.fetch_add(grain);
                if (i0 >= n) break;
                const int64_t i1 = std::min(n, i0 + grain);
                for (int64_t i = i0; i < i1; ++i) f(i);
            }
        });
    for (auto& t : th) t.join();
}

// A vector element type that resize() leaves uninitialised (the database's
// host copy is filled by parallel copies right after).
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        if constexpr (sizeof...(A) == 0) ::new (static_cast<void*>(p)) U;
        else ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};

// Subject indices sorted by length, longest first, stable (file order
// within a length): a counting sort when lengths are bounded, else
// std::stable_sort.
std::vector<int64_t> length_order(const std::vector<int64_t>& offs, int64_t n) {
    std::vector<int64_t> order(n);
    int64_t maxl = 0;
    for (int64_t k = 0; k < n; ++k) maxl = std::max(maxl, offs[k + 1] - offs[k]);
    if (maxl > (int64_t(1) << 22)) {
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) {
            return offs[x + 1] - offs[x] > offs[y + 1] - offs[y];
        });
        return order;
    }
    std::vector<int64_t> start(static_cast<size_t>(maxl) + 2, 0);
    for (int64_t k = 0; k < n; ++k) ++start[static_cast<size_t>(maxl - (offs[k + 1] - offs[k]) + 1)];
    for (size_t l = 1; l < start.size(); ++l) start[l] += start[l - 1];
    for (int64_t k = 0; k < n; ++k) order[start[static_cast<size_t>(maxl - (offs[k + 1] - offs[k]))]++] = k;
    return order;
}

}  // namespace

int swk::set_error(int code, const std::string& msg) { return fail(code, msg); }

// ---------------------------------------------------------------------------
struct ScanEvents {
    // 0 fork, 1 intra done (side), 2 inter done (main), 3 end, and around
    // each inter kernel on its own stream: 4/5 the cooperative kernel
    // (side2), 6/7 the per-wave kernel (main)
    hipEvent_t ev[8] = {};
    unsigned rec = 0;  // bit k: ev[k] was recorded by this scan (read_events
                       // falls back for the others: each record is a packet
                       // the command processor spends microseconds on)
    int launches = 0;
    bool merged = false;  // one merged launch (sw_scan_lpt): ev6..ev7 is the whole scan's fp16 pass
};

namespace {
sw_opts default_opts() {
    sw_opts o;
    std::memset(&o, 0, sizeof o);
    o.size = static_cast<int32_t>(sizeof o);
    for (int32_t* f : {&o.lpt, &o.lpt_pipe, &o.quad_width, &o.pair_width, &o.pair_group, &o.coop_width,
                       &o.coop_skew, &o.intra_x2, &o.intra_x2_rows, &o.intra_i16_first, &o.inter_i16_span,
                       &o.int16_guard, &o.rescue_stats, &o.tail_pairs, &o.lpt_persist, &o.lpt_rows,
                       &o.tri_width, &o.lpt_pipe_tail, &o.drain_spin})
        *f = -1;
    return o;
}
}  // namespace

struct sw_handle {
    int device = 0;
    int cus = 0;  // compute units of the device
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // One event set per scan since the last sw_timing_reset (grows as needed,
    // reused after a reset), so a caller can time many back-to-back scans
    // without synchronising between them.
    std::vector<ScanEvents> evpool;
    size_t nscans = 0;
    hipEvent_t* ev = nullptr;  // event set of the current scan
    unsigned* ev_rec = nullptr;
    // The intra kernel runs on a side stream, concurrently with the inter
    // kernel (fork/join through ev[0] and ev[1]).
    hipStream_t side = nullptr;
    hipStream_t side2 = nullptr;  // the cooperative wide-block kernel
    // Deferred rescue tails (the queries of a batch but the last): a scan's
    // re-scoring stages (int16 / int32 list kernels) run on `tail` after its
    // fp16 passes, while the next query's fp16 passes start on the main and
    // side streams.  Lists and boundary rows of the tail are its own
    // (parity-indexed lists, sw_db::d_rbnd_*), so nothing is shared with the
    // passes running beside it.
    hipStream_t tail = nullptr;
    hipEvent_t main_done = nullptr, side_done = nullptr;  // fp16 passes of the scan being deferred
    hipEvent_t tail_done[2] = {};                         // per list parity
    bool tail_pending[2] = {};
    int parity = 0;                                       // list set of the next scan
    hipEvent_t coop_done = nullptr;
    hipEvent_t fork2 = nullptr;  // side2 starts after the rescue counters are reset
    // per-query workspace: profiles (inter: [32][stride]; intra: lane-slotted
    // chunks) built on the device by the scan's first launch.  A ring of
    // slots: a deferred rescue tail (batches) may still read the profiles of
    // the scan before while the next scan builds its own.  Reusing a slot
    // waits until the scan that last used it has started on the device, so
    // the host runs at most kProfSlots scans ahead of the GPU: the adaptive
    // choices (the fp16 passes' flagged counts read back without waiting,
    // scan_impl) then see scans a few queries back instead of none at all
    // when many scans are enqueued at once.
    struct ProfSlot {
        int8_t* d = nullptr;
        size_t dcap = 0;
        // the end event (ev[3]) of the slot's last scan: reusing the slot
        // waits for it.  Not an event of its own: each event record is a
        // packet the command processor spends ~5 us on between two kernels
        // (rocprofv3 trace of C2's 1/8 share, scripts/step_gaps.py)
        hipEvent_t last_end = nullptr;
        bool pending = false;
        hipEvent_t tail_read = nullptr;  // a deferred rescue tail has read the slot
        bool tail_pending = false;
    };
    // pinned staging of database uploads (build_db): the host packs one
    // buffer while the other's copy runs
    uint8_t* stage[2] = {};
    size_t stage_cap = 0;
    hipEvent_t stage_ev[2] = {};
    bool stage_pending[2] = {};
    static constexpr int kProfSlots = 4;
    ProfSlot prof[kProfSlots];
    int prof_next = 0;
    int32_t* d_scores = nullptr;  // for the synchronous sw_scan
    size_t scores_cap = 0;
    int64_t* d_topk_work = nullptr;  // device top-K workspace
    std::string last_kernel = "none";  // per-wave inter kernel of the last scan
    std::string last_intra = "none";   // long-subject kernel of the last scan
    size_t topk_cap = 0;
    bool timed = false;
    bool had_intra = false;
    int launches = 0;
    // host-mapped fault word (swk::DrainArgs::fault): set by a kernel that
    // had to skip work it could not do (list_wait_take's timeout); the next
    // call on the handle fails with SW_E_DEVICE instead of returning scores
    int32_t* h_fault = nullptr;
    int32_t* d_fault = nullptr;
    int open_slot = -1;  // profile slot pending on an ev[3] this scan has not recorded yet
    sw_opts opts = default_opts();  // kernel-form overrides (sw_set_opts); all -1 = the library's choice
};

// Faults reported so far (any handle): a drain that gave up on an entry
// left claimed entries of its database's rescue lists un-reset, so every
// database re-initialises its lists at its first scan after a fault
// (sw_db::list_epoch) and later scans are exact again.
static std::atomic<uint64_t> g_fault_epoch{0};

// A kernel of this handle reported a fault since the last check (sw_kernels.h
// list_wait_take): fail loudly, once.
static int check_fault(sw_handle* h) {
    if (h && h->h_fault && __atomic_load_n(h->h_fault, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(h->h_fault, 0, __ATOMIC_RELEASE);
        g_fault_epoch.fetch_add(1);
        return fail(SW_E_DEVICE, "sw_scan_lpt: a claimed rescue-list entry never appeared; the handle's scans "
                                 "since the last successful call may hold unrescued scores");
    }
    return SW_OK;
}

struct sw_db {
    sw_handle* h = nullptr;
    int64_t n = 0;
    int64_t residues = 0;
    int32_t max_len = 0;
    int32_t max_id = -1;
    int32_t long_threshold = 0;
    // inter part
    int64_t nblocks = 0;
    int64_t packed_cells = 0;
    uint8_t* d_res = nullptr;
    size_t res_bytes = 0;
    uint64_t* d_blk_off = nullptr;
    uint32_t* d_blk_groups = nullptr;
    uint32_t* d_blk_cols = nullptr;      // block widths rounded to 8 columns (sw_inter_x2s)
    int32_t* d_lane_ids = nullptr;
    int32_t* d_ids = nullptr;            // every subject's result id (sw_scan_topk), on first use
    int rid_identity = -1;               // result ids are 0 .. n-1 in order (1), or not (0); -1 unknown
    int32_t* d_bnd_h = nullptr;
    int32_t* d_bnd_f = nullptr;
    // two rescue lists [count, block ids...] of nblocks + 1 ints each: the
    // 16-bit kernels' flagged blocks (list A), and the fp16 chain's second
    // stage's (list B)
    // (two parities of these lists: consecutive scans of a batch alternate)
    int32_t* d_rescue = nullptr;
    int32_t* d_lrescue = nullptr;        // [count, subjects...] x 2: the intra rescue chain's lists
    uint64_t list_epoch = 0;             // g_fault_epoch when the lists were last known clean
    // boundary rows of deferred rescue tails (inter H, F; intra H, F), when
    // device memory allows them (else the tails run in stream order)
    int32_t* d_rbnd_h = nullptr;
    int32_t* d_rbnd_f = nullptr;
    int32_t* d_rlbnd_h = nullptr;
    int32_t* d_rlbnd_f = nullptr;
    bool rbnd_tried = false;
    // the intra chain's order (scan_impl): the fp16 pass's flagged count read
    // back after the scan (pinned, event-gated), and per scoring the shortest
    // query seen to flag over half of the long subjects
    int32_t* h_lcount = nullptr;
    hipEvent_t lcount_ev = nullptr;
    bool lcount_pending = false;
    uint64_t lcount_qhash = 0;
    bool lcount_seen = false;  // the last observation read back (see icount_seen)
    uint64_t lseen_key = 0, lseen_qhash = 0;
    int32_t lseen_qlen = 0;
    uint64_t lcount_key = 0;
    int32_t lcount_qlen = 0;
    std::vector<std::pair<uint64_t, int32_t>> i16_first;
    // the inter scan's counterpart: the fp16 pass's flagged count and largest
    // flagged block (pinned pair, event-gated) and per (scoring, query
    // length) the span of widest blocks the int16 kernel then takes first
    int32_t* h_icount = nullptr;
    hipEvent_t icount_ev = nullptr;
    bool icount_pending = false;
    uint64_t icount_key = 0;
    int32_t icount_qlen = 0;
    int32_t icount_nr = 0;
    uint64_t icount_qhash = 0;
    // the last observation read back: a scan repeating it (same query,
    // scoring and split) does not read it back again
    bool icount_seen = false;
    uint64_t seen_key = 0, seen_qhash = 0;
    int32_t seen_qlen = 0, seen_nr = 0;
    struct SpanObs {
        uint64_t key;
        int32_t qlen;
        int32_t span;
    };
    std::vector<SpanObs> i16_span;
    int32_t last_i16_span = 0;
    uint64_t* h_trace = nullptr;         // sw_opts trace_file: host-mapped block timeline
    size_t trace_entries = 0;            // ... its entries: per block, then per merged-launch workgroup
    std::vector<uint32_t> h_blk_groups;  // block widths (16-column groups), widest first
    std::vector<int64_t> h_blk_res;      // unpadded residues per block
    int32_t last_ncoop = 0;              // blocks the last scan gave the coop kernel
    int32_t last_npair = 0;              // blocks the last scan ran by wave pairs
    bool last_lpt = false;               // the last scan was one merged launch (sw_scan_lpt)
    std::vector<int32_t> h_llen;         // long subjects' lengths, longest first
    // sw_scan_lpt work tables (longest first), per scan shape
    struct LptTable {
        int32_t qpad, rows /* per pass */, qpad_intra, ri, npair, group /* quad blocks */, tail /* tail-pair blocks */, n;
        bool affine;
        bool tri;  // the group blocks by 3-wave groups with a spare wave (InterArgs::blk_tri)
        int32_t npipe;  // the longest pairs, in the pipelined form
        int32_t pipe_opt;  // sw_opts lpt_pipe the table was built under
        int32_t pipe_tail;  // pairs [pipe_tail, ...) pipelined too (the shortest)
        int32_t tail_opt;   // sw_opts lpt_pipe_tail the table was built under
        int32_t* d_order;
        std::vector<float> cost;  // estimated duration of each entry, longest first
    };
    std::vector<LptTable> lpt_tables;
    bool last_pair_merged = false;
    bool last_drain = false;             // the last scan's merged launch drained its own rescue lists
    // device copies of the merged launch's drain arguments (swk::DrainArgs),
    // one per distinct content (profile slot x list parity x score buffer
    // x query shape): uploaded once, then reused with no copy per scan
    static constexpr int kDrainSlots = 32;
    swk::DrainArgs* d_drain = nullptr;
    swk::DrainArgs* h_drain = nullptr;   // pinned: the copies' sources
    std::vector<std::vector<uint64_t>> drain_keys;  // what each slot's content is a function of
    int drain_next = 0;
    // intra part (long subjects)
    int64_t nlong = 0;
    int32_t long_max = 0;
    uint8_t* d_lres = nullptr;
    size_t lres_bytes = 0;
    uint64_t* d_loff = nullptr;
    int32_t* d_llen = nullptr;
    int32_t* d_lid = nullptr;
    int32_t* d_lbnd_h = nullptr;
    int32_t* d_lbnd_f = nullptr;
    // host copies kept to allow re-partitioning when the threshold changes
    std::vector<uint8_t, NoInitAlloc<uint8_t>> h_residues;
    std::vector<int64_t> h_offsets;
    std::vector<int32_t> h_ids;
    std::unordered_map<int32_t, int64_t> id_index;  // result id -> subject (built on first sw_align)
    bool built = false;
    size_t device_bytes = 0;
    // synthetic database (sw_db_create_synthetic): residues are generated
    // on the device from (seed, id_base + local id); h_residues stays empty
    bool synthetic = false;
    uint64_t seed = 0;
    int64_t id_base = 0;
};

namespace {

// The planning policies' view of a database (sw_plan.h).
swplan::PlanDb plan_view(const sw_db* db) {
    swplan::PlanDb v;
    v.n = db->n;
    v.residues = db->residues;
    v.nblocks = db->nblocks;
    v.nlong = db->nlong;
    v.long_threshold = db->long_threshold;
    v.blk_groups = db->h_blk_groups.data();
    v.llen = db->h_llen.data();
    v.opts = &db->h->opts;
    v.cus = db->h->cus;
    return v;
}

// ---- adaptive routing: what earlier scans of this database observed --------
// The intra chain's order.  Linear scoring with cheap gaps makes random
// pairs' scores grow with their lengths, so on long subjects the fp16 pass
// can flag many of them and its time on those is wasted.  Once a scan with
// the same scoring (skey) has flagged over a third of the long subjects at a
// query no longer than this one, the int16 form runs first, over all of them
// (the int16 cell costs ~1.4x the fp16 one, so fp16 first + int16 over the
// flagged fraction p wins while p < ~0.3).  The last observation is read
// here once its event has completed (scan_impl_body records it).  opt =
// sw_opts intra_i16_first: 0 / 1 never / always, else the observations.
bool adapt_intra_i16_first(sw_db* db, uint64_t skey, int32_t qlen, int32_t opt) {
    if (db->lcount_pending && hipEventQuery(db->lcount_ev) == hipSuccess) {
        db->lcount_pending = false;
        db->lcount_seen = true;
        db->lseen_key = db->lcount_key;
        db->lseen_qhash = db->lcount_qhash;
        db->lseen_qlen = db->lcount_qlen;
        if (3 * static_cast<int64_t>(*db->h_lcount) > db->nlong) {
            bool seen = false;
            for (auto& e : db->i16_first)
                if (e.first == db->lcount_key) {
                    e.second = std::min(e.second, db->lcount_qlen);
                    seen = true;
                }
            if (!seen) db->i16_first.emplace_back(db->lcount_key, db->lcount_qlen);
        }
    }
    bool intra_i16_first = false;
    if (opt == 0 || opt == 1) {
        intra_i16_first = opt == 1;
    } else {
        for (const auto& e : db->i16_first)
            if (e.first == skey && e.second <= qlen) intra_i16_first = true;
    }
    return intra_i16_first;
}

// The same for the inter scan, per block: long queries under cheap linear
// gaps put the WIDEST blocks (length-sorted, ids 0, 1, ...) in the fp16
// guard band, and their re-scoring by the list kernel (one wave per block,
// every pass in turn) takes longer than the whole scan.  A scan with the
// same scoring whose fp16 pass flagged most of blocks [0, span) makes
// later queries at least as long run those blocks in int16, by wave pairs
// beside the fp16 launch.  opt = sw_opts inter_i16_span: n forces n blocks (0: off).
int32_t adapt_inter_i16_span(sw_db* db, uint64_t skey, int32_t qlen, int32_t opt) {
    if (db->icount_pending && hipEventQuery(db->icount_ev) == hipSuccess) {
        db->icount_pending = false;
        db->icount_seen = true;
        db->seen_key = db->icount_key;
        db->seen_qhash = db->icount_qhash;
        db->seen_qlen = db->icount_qlen;
        db->seen_nr = db->icount_nr;
        const int32_t cnt = db->h_icount[0], span = db->h_icount[1] + 1;
        // most of [nr, span) flagged: not a few high-scoring hits far out
        if (cnt > 0 && span > db->icount_nr && 2 * static_cast<int64_t>(cnt) >= span - db->icount_nr) {
            // keep a staircase per scoring: drop what the new observation
            // dominates (a query at least as long with a span no larger),
            // skip it if an existing one dominates it
            const uint64_t k = db->icount_key;
            const int32_t q = db->icount_qlen;
            bool dominated = false;
            for (const auto& e : db->i16_span)
                if (e.key == k && e.qlen <= q && e.span >= span) dominated = true;
            if (!dominated) {
                db->i16_span.erase(std::remove_if(db->i16_span.begin(), db->i16_span.end(),
                                                  [&](const sw_db::SpanObs& e) {
                                                      return e.key == k && e.qlen >= q && e.span <= span;
                                                  }),
                                   db->i16_span.end());
                db->i16_span.push_back({k, q, span});
            }
        }
    }
    int32_t i16_span = 0;
    if (opt >= 0) {
        i16_span = opt;
    } else {
        for (const auto& o : db->i16_span)
            if (o.key == skey && o.qlen <= qlen) i16_span = std::max(i16_span, o.span);
    }
    i16_span = static_cast<int32_t>(std::min<int64_t>(std::max(i16_span, 0), db->nblocks));
    return i16_span;
}

void free_dev(sw_db* db) {
    void* ptrs[] = {db->d_res, db->d_blk_off, db->d_blk_groups, db->d_blk_cols, db->d_lane_ids, db->d_bnd_h, db->d_bnd_f,
                    db->d_rescue, db->d_lres, db->d_loff, db->d_llen, db->d_lid, db->d_lbnd_h, db->d_lbnd_f,
                    db->d_lrescue, db->d_rbnd_h, db->d_rbnd_f, db->d_rlbnd_h, db->d_rlbnd_f, db->d_ids};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    db->d_res = nullptr; db->d_blk_off = nullptr; db->d_blk_groups = nullptr; db->d_lane_ids = nullptr;
    db->d_blk_cols = nullptr;
    db->d_bnd_h = nullptr; db->d_bnd_f = nullptr; db->d_rescue = nullptr; db->d_lres = nullptr; db->d_loff = nullptr;
    db->d_llen = nullptr; db->d_lid = nullptr; db->d_lbnd_h = nullptr; db->d_lbnd_f = nullptr;
    db->d_lrescue = nullptr;
    db->d_rbnd_h = db->d_rbnd_f = db->d_rlbnd_h = db->d_rlbnd_f = nullptr;
    db->d_ids = nullptr;
    db->rbnd_tried = false;
    for (auto& t : db->lpt_tables) (void)hipFree(t.d_order);
    db->lpt_tables.clear();
    if (db->d_drain) (void)hipFree(db->d_drain);
    if (db->h_drain) (void)hipHostFree(db->h_drain);
    db->d_drain = nullptr;
    db->h_drain = nullptr;
    db->drain_keys.clear();
    db->drain_next = 0;
    if (db->h_trace) (void)hipHostFree(db->h_trace);  // sized for this block layout
    db->h_trace = nullptr;
    db->trace_entries = 0;
    db->lcount_pending = false;
    db->lcount_seen = false;
    db->i16_first.clear();  // the long partition may change
    db->icount_pending = false;
    db->icount_seen = false;
    db->i16_span.clear();   // ... and the block layout
    db->device_bytes = 0;
    db->built = false;
}

template <class T>
int upload(T** dptr, const std::vector<T>& v, hipStream_t s, size_t* acc) {
    if (v.empty()) { *dptr = nullptr; return SW_OK; }
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(dptr), v.size() * sizeof(T)));
    HIPCHECK(hipMemcpyAsync(*dptr, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
    *acc += v.size() * sizeof(T);
    return SW_OK;
}

// ---- synthetic databases -------------------------
// Swiss-Prot composition (percent), codes 0..19 = A R N D C Q E G H I L K M F
// P S T W Y V (the same table as synth.py).
const double kSwissProtFreq[20] = {8.25, 5.53, 4.06, 5.45, 1.37, 3.93, 6.75, 7.07, 2.27, 5.96,
                                   9.66, 5.84, 2.42, 3.86, 4.70, 6.56, 5.34, 1.08, 2.92, 6.87};
constexpr uint64_t kLenSalt = 0x4C454E475448ull;  // "LENGTH"

// Acklam's rational approximation of the standard normal quantile.
double norm_quantile(double p) {
    static const double a[6] = {-3.969683028665376e+01, 2.209460984245205e+02, -2.759285104469687e+02,
                                1.383577518672690e+02, -3.066479806614716e+01, 2.506628277459239e+00};
    static const double b[5] = {-5.447609879822406e+01, 1.615858368580409e+02, -1.556989798598866e+02,
                                6.680131188771972e+01, -1.328068155288572e+01};
    static const double c[6] = {-7.784894002430293e-03, -3.223964580411365e-01, -2.400758277161838e+00,
                                -2.549732539343734e+00, 4.374664141464968e+00, 2.938163982698783e+00};
    static const double d[4] = {7.784695709041462e-03, 3.224671290700398e-01, 2.445134137142996e+00,
                                3.754408661907416e+00};
    const double pl = 0.02425;
    if (p < pl) {
        const double q = std::sqrt(-2 * std::log(p));
        return (((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
               ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
    }
    if (p > 1 - pl) {
        const double q = std::sqrt(-2 * std::log(1 - p));
        return -(((((c[0] * q + c[1]) * q + c[2]) * q + c[3]) * q + c[4]) * q + c[5]) /
               ((((d[0] * q + d[1]) * q + d[2]) * q + d[3]) * q + 1);
    }
    const double q = p - 0.5, r = q * q;
    return (((((a[0] * r + a[1]) * r + a[2]) * r + a[3]) * r + a[4]) * r + a[5]) * q /
           (((((b[0] * r + b[1]) * r + b[2]) * r + b[3]) * r + b[4]) * r + 1);
}

struct SynthTables {
    int32_t len[4096];     // log-normal length quantiles: median 290, sigma 0.657, in [5, 35213]
    uint8_t lut[65536];    // uniform u16 -> residue code
    uint8_t lut_stored[65536];  // ... as stored on the device (swk::kStored)
    SynthTables() {
        for (int k = 0; k < 4096; ++k) {
            const double z = norm_quantile((k + 0.5) / 4096.0);
            const double L = std::nearbyint(std::exp(std::log(290.0) + 0.657 * z));
            len[k] = static_cast<int32_t>(std::min(35213.0, std::max(5.0, L)));
        }
        double sum = 0, acc = 0;
        for (double f : kSwissProtFreq) sum += f;
        int64_t edges[20];
        for (int c = 0; c < 20; ++c) {
            acc += kSwissProtFreq[c] / sum;
            edges[c] = static_cast<int64_t>(std::nearbyint(acc * 65536.0));
        }
        edges[19] = 65536;
        int c = 0;
        for (int v = 0; v < 65536; ++v) {
            while (c < 19 && edges[c] <= v) ++c;
            lut[v] = static_cast<uint8_t>(c);
            lut_stored[v] = swk::kStored[c];
        }
    }
};

const SynthTables& synth_tables() {
    static const SynthTables t;
    return t;
}

int32_t synth_length(uint64_t seed, uint64_t gid) {
    return synth_tables().len[swk::synth_hash(seed, gid, kLenSalt) >> 52];
}

void synth_residues(uint64_t seed, uint64_t gid, int64_t L, uint8_t* out) {
    const uint8_t* lut = synth_tables().lut;
    for (int64_t j = 0; j < L; j += 4) {
        const uint64_t h = swk::synth_hash(seed, gid, static_cast<uint64_t>(j >> 2));
        for (int e = 0; e < 4 && j + e < L; ++e) out[j + e] = lut[(h >> (16 * e)) & 0xffffu];
    }
}

// Residues of subject k (host): stored, or regenerated for synthetic dbs.
void subject_residues(const sw_db* db, int64_t k, uint8_t* out) {
    const int64_t L = db->h_offsets[k + 1] - db->h_offsets[k];
    if (db->synthetic)
        synth_residues(db->seed, static_cast<uint64_t>(db->id_base + db->h_ids[k]), L, out);
    else
        std::memcpy(out, db->h_residues.data() + db->h_offsets[k], L);
}

// Upload bytes produced unit by unit (unit u covers [bounds[u], bounds[u+1])
// of `dev` and fill(u, dst) writes all of it, padding included) through the
// handle's two pinned staging buffers: chunks of whole units are packed on
// the host's cores into one buffer while the previous chunk's H2D copy runs
// (the reference packs byte by byte into managed memory on one thread,
// SWSolver.cu:309-359).
constexpr size_t kStageBytes = size_t(32) << 20;

template <class F>
int staged_upload(sw_handle* h, uint8_t* dev, const std::vector<uint64_t>& bounds, F&& fill) {
    const int64_t nu = static_cast<int64_t>(bounds.size()) - 1;
    if (nu <= 0 || bounds.back() == bounds.front()) return SW_OK;
    uint64_t maxu = 0;
    for (int64_t u = 0; u < nu; ++u) maxu = std::max<uint64_t>(maxu, bounds[u + 1] - bounds[u]);
    const size_t cap = std::max<size_t>(kStageBytes, maxu);
    if (cap > h->stage_cap) {
        for (int b = 0; b < 2; ++b) {
            if (h->stage_pending[b]) HIPCHECK(hipEventSynchronize(h->stage_ev[b]));
            h->stage_pending[b] = false;
            if (h->stage[b]) HIPCHECK(hipHostFree(h->stage[b]));
            h->stage[b] = nullptr;
        }
        h->stage_cap = 0;
        for (int b = 0; b < 2; ++b)
            HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&h->stage[b]), cap, hipHostMallocDefault));
        h->stage_cap = cap;
    }
    int b = 0;
    for (int64_t u0 = 0; u0 < nu;) {
        int64_t u1 = u0 + 1;
        while (u1 < nu && bounds[u1 + 1] - bounds[u0] <= h->stage_cap) ++u1;
        if (h->stage_pending[b]) HIPCHECK(hipEventSynchronize(h->stage_ev[b]));
        uint8_t* buf = h->stage[b];
        const uint64_t base = bounds[u0];
        parallel_for(u1 - u0, [&](int64_t i) { fill(u0 + i, buf + (bounds[u0 + i] - base)); }, 1);
        HIPCHECK(hipMemcpyAsync(dev + base, buf, bounds[u1] - base, hipMemcpyHostToDevice, h->stream));
        HIPCHECK(hipEventRecord(h->stage_ev[b], h->stream));
        h->stage_pending[b] = true;
        b ^= 1;
        u0 = u1;
    }
    return SW_OK;
}

// Pack: sort by length (descending, stable), route subjects longer than the
// threshold to the intra kernel, deal the rest into 64-lane blocks of
// 16-residue groups.  Lanes past a subject's end hold kPadCode.
int build_db(sw_db* db) {
    hipStream_t s = db->h->stream;
    const int64_t n = db->n;
    const std::vector<int64_t> order = length_order(db->h_offsets, n);
    auto len = [&](int64_t k) { return db->h_offsets[k + 1] - db->h_offsets[k]; };
    int64_t nlong = 0;
    while (nlong < n && len(order[nlong]) > db->long_threshold) ++nlong;

    // ---- intra (long) part: plain concatenation, 64-byte aligned starts
    std::vector<uint64_t> loff(nlong + 1);
    std::vector<int32_t> llen(nlong), lid(nlong);
    uint64_t ltotal = 0;
    for (int64_t k = 0; k < nlong; ++k) {
        const int64_t src = order[k];
        loff[k] = ltotal;
        llen[k] = static_cast<int32_t>(len(src));
        lid[k] = db->h_ids[src];
        ltotal += round_up(len(src), 64);
    }
    loff[nlong] = ltotal;

    // ---- inter part
    const int64_t nshort = n - nlong;
    const int64_t nblocks = (nshort + swk::kLanes - 1) / swk::kLanes;
    std::vector<uint64_t> blk_off(nblocks + 1);
    std::vector<uint32_t> blk_groups(nblocks), blk_cols(nblocks);
    std::vector<int32_t> lane_ids(nblocks * swk::kLanes, -1);
    std::vector<int64_t> blk_res(nblocks, 0);  // unpadded residues per block
    uint64_t total = 0;
    for (int64_t b = 0; b < nblocks; ++b) {
        const int64_t first = nlong + b * swk::kLanes;  // longest subject of the block
        const int64_t w = round_up(len(order[first]), swk::kGroupCols);
        blk_off[b] = total;
        blk_groups[b] = static_cast<uint32_t>(w / swk::kGroupCols);
        blk_cols[b] = static_cast<uint32_t>(round_up(len(order[first]), 8));
        total += static_cast<uint64_t>(blk_groups[b]) * swk::kGroupBytes;
    }
    blk_off[nblocks] = total;
    std::vector<int32_t> lane_len(db->synthetic ? nblocks * swk::kLanes : 0, 0);
    parallel_for(nblocks, [&](int64_t b) {
        for (int l = 0; l < swk::kLanes; ++l) {
            const int64_t k = nlong + b * swk::kLanes + l;
            if (k >= n) break;
            const int64_t src = order[k];
            lane_ids[b * swk::kLanes + l] = db->h_ids[src];
            blk_res[b] += len(src);
            if (db->synthetic) lane_len[b * swk::kLanes + l] = static_cast<int32_t>(len(src));
        }
    });
    // one block's bytes: [group][lane][16 codes], kPadCode past each subject;
    // codes are stored as swk::kStored (the profile rows follow it)
    auto stored = [](uint8_t* d, const uint8_t* p, int64_t m) {
        for (int64_t j = 0; j < m; ++j) d[j] = swk::kStored[p[j]];
    };
    auto fill_block = [&](int64_t b, uint8_t* dst) {
        std::memset(dst, swk::kPadCode, static_cast<size_t>(blk_groups[b]) * swk::kGroupBytes);
        for (int l = 0; l < swk::kLanes; ++l) {
            const int64_t k = nlong + b * swk::kLanes + l;
            if (k >= n) break;
            const int64_t src = order[k], L = len(src);
            const uint8_t* p = db->h_residues.data() + db->h_offsets[src];
            uint8_t* d = dst + l * swk::kGroupCols;
            int64_t j = 0;
            for (; j + swk::kGroupCols <= L; j += swk::kGroupCols, d += swk::kGroupBytes) stored(d, p + j, swk::kGroupCols);
            if (j < L) stored(d, p + j, L - j);
        }
    };
    auto fill_long = [&](int64_t k, uint8_t* dst) {
        const int64_t src = order[k];
        std::memset(dst, swk::kPadCode, loff[k + 1] - loff[k]);
        stored(dst, db->h_residues.data() + db->h_offsets[src], len(src));
    };
    blk_off.pop_back();

    size_t acc = 0;
    int rc;
    if (db->synthetic) {
        // residues generated in HBM from (seed, global id); ids in lane_ids
        // and lid are local (0..n-1), global = id_base + local
        if (total) HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_res), total));
        if (ltotal) HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_lres), ltotal));
        acc += total + ltotal;
    } else {
        // residues through pinned staging, packed in parallel chunks
        std::vector<uint64_t> bounds(blk_off);
        bounds.push_back(total);
        if (total) {
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_res), total));
            if ((rc = staged_upload(db->h, db->d_res, bounds, fill_block))) return rc;
        }
        if (ltotal) {
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_lres), ltotal));
            if ((rc = staged_upload(db->h, db->d_lres, loff, fill_long))) return rc;
        }
        acc += total + ltotal;
    }
    if ((rc = upload(&db->d_blk_off, blk_off, s, &acc))) return rc;
    if ((rc = upload(&db->d_blk_groups, blk_groups, s, &acc))) return rc;
    if ((rc = upload(&db->d_blk_cols, blk_cols, s, &acc))) return rc;
    if ((rc = upload(&db->d_lane_ids, lane_ids, s, &acc))) return rc;
    loff.pop_back();
    if ((rc = upload(&db->d_loff, loff, s, &acc))) return rc;
    if ((rc = upload(&db->d_llen, llen, s, &acc))) return rc;
    if ((rc = upload(&db->d_lid, lid, s, &acc))) return rc;
    if (db->synthetic) {
        int32_t* d_lane_len = nullptr;
        uint8_t* d_lut = nullptr;
        size_t tmp = 0;
        if ((rc = upload(&d_lane_len, lane_len, s, &tmp))) return rc;
        const SynthTables& T = synth_tables();
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&d_lut), sizeof T.lut_stored));
        HIPCHECK(hipMemcpyAsync(d_lut, T.lut_stored, sizeof T.lut_stored, hipMemcpyHostToDevice, s));
        swk::SynthFill f{};
        f.res = db->d_res;
        f.blk_off = db->d_blk_off;
        f.blk_groups = db->d_blk_groups;
        f.lane_local = db->d_lane_ids;
        f.lane_len = d_lane_len;
        f.nblocks = nblocks;
        f.lres = db->d_lres;
        f.loff = db->d_loff;
        f.llen = db->d_llen;
        f.lid = db->d_lid;
        f.nlong = static_cast<int32_t>(nlong);
        f.seed = db->seed;
        f.id_base = db->id_base;
        f.lut = d_lut;
        HIPCHECK(swk::launch_synth_fill(f, s));
        HIPCHECK(hipStreamSynchronize(s));
        if (d_lane_len) HIPCHECK(hipFree(d_lane_len));
        HIPCHECK(hipFree(d_lut));
    }
    HIPCHECK(hipStreamSynchronize(s));  // host vectors go out of scope
    db->h_blk_groups = blk_groups;
    db->h_blk_res = blk_res;
    db->h_llen = llen;
    db->res_bytes = total;
    db->lres_bytes = ltotal;
    db->nblocks = nblocks;
    db->nlong = nlong;
    db->long_max = nlong ? static_cast<int32_t>(len(order[0])) : 0;
    db->packed_cells = static_cast<int64_t>(total);  // one byte per scanned (lane, column)
    db->device_bytes = acc;
    db->built = true;
    return SW_OK;
}

// Boundary rows are only needed when the query spans more than one strip;
// allocate on first need and keep.
int ensure_bnd(sw_db* db, bool affine, bool intra_f) {
    if (db->res_bytes && !db->d_bnd_h) {
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_bnd_h), db->res_bytes * 4));
        db->device_bytes += db->res_bytes * 4;
    }
    if (affine && db->res_bytes && !db->d_bnd_f) {
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_bnd_f), db->res_bytes * 4));
        db->device_bytes += db->res_bytes * 4;
    }
    if (db->lres_bytes && !db->d_lbnd_h) {
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_lbnd_h), db->lres_bytes * 4));
        db->device_bytes += db->lres_bytes * 4;
    }
    if ((affine || intra_f) && db->lres_bytes && !db->d_lbnd_f) {
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_lbnd_f), db->lres_bytes * 4));
        db->device_bytes += db->lres_bytes * 4;
    }
    return SW_OK;
}

// The deferred tails' own boundary rows, sized as ensure_bnd's: H always, F
// only for affine scoring (inter) or when the intra form keeps F (intra_f).
// Arrays a later scan needs are allocated then.  False when device memory
// would drop below a quarter of the card's (a 50M-subject database keeps its
// tails in stream order); a refused size is not tried again for this layout.
bool ensure_rbnd(sw_db* db, bool affine, bool intra_f) {
    void** p[4] = {reinterpret_cast<void**>(&db->d_rbnd_h), reinterpret_cast<void**>(&db->d_rbnd_f),
                   reinterpret_cast<void**>(&db->d_rlbnd_h), reinterpret_cast<void**>(&db->d_rlbnd_f)};
    const size_t sz[4] = {db->res_bytes * 4, affine ? db->res_bytes * 4 : 0, db->lres_bytes * 4,
                          (affine || intra_f) ? db->lres_bytes * 4 : 0};
    size_t need = 0;
    for (int k = 0; k < 4; ++k)
        if (sz[k] && !*p[k]) need += sz[k];
    if (need == 0) return true;
    if (db->rbnd_tried) return false;
    size_t freeb = 0, totalb = 0;
    if (hipMemGetInfo(&freeb, &totalb) != hipSuccess || freeb < need + totalb / 4) {
        db->rbnd_tried = true;
        return false;
    }
    for (int k = 0; k < 4; ++k)
        if (sz[k] && !*p[k]) {
            if (hipMalloc(p[k], sz[k]) != hipSuccess) {
                *p[k] = nullptr;
                (void)hipGetLastError();
                db->rbnd_tried = true;
                return false;
            }
            db->device_bytes += sz[k];
        }
    return true;
}

int check_scoring(const sw_scoring* sc, const int8_t** mat, int* go, int* ge) {
    *mat = kBlosum50Ref;
    *go = 2;
    *ge = 2;
    if (sc) {
        if (sc->matrix) *mat = sc->matrix;
        *go = sc->gap_open;
        *ge = sc->gap_extend;
    }
    if (*go <= 0 || *ge <= 0 || *go > 1000 || *ge > 1000)
        return fail(SW_E_INVALID, "gap penalties must be in 1..1000");
    for (int k = 0; k < 625; ++k)
        if ((*mat)[k] < -100 || (*mat)[k] > 100) return fail(SW_E_INVALID, "matrix entries must be in -100..100");
    return SW_OK;
}

// Query profiles.  Inter kernel: prof[c][i] = S[q_i][c] (+ gap for the
// linear kernels) for residue codes c < 25; rows c >= 25 (the pad code) and
// columns i >= qlen score 0 (+ gap).  A zero-score pad row/column can never
// raise the maximum (every such cell is <= max(0, its diagonal, its gap
// predecessors)).  Intra kernel: the same values laid out per chunk of
// 64*ri query rows as [code][lane][RIP] so each lane's ri rows are contiguous.
struct Profiles {
    int8_t* dev = nullptr;  // device copy of this scan's profiles
    int32_t stride = 0;      // inter profiles: entries per code row
    size_t off8 = 0;         // int8 inter profile (biased for linear)
    size_t off16 = 0;        // int16 inter profile (packed kernels)
    size_t intra_off = 0;    // lane-slotted intra profile
    size_t total = 0;
    int slot = 0;            // the handle's profile slot holding them
};

// Built on the device (swk::sw_build_profile, one launch per 2,048 query
// rows; the first also zeroes the rescue lists' counters `reset`) in one of
// the handle's profile slots, on the scan's stream.
int build_profiles(sw_handle* h, const uint8_t* q, int32_t qlen, const int8_t* mat, int go, bool affine,
                   int32_t qpad_inter, bool want16, int ri, int32_t qpad_intra, int32_t* const (&reset)[10],
                   Profiles* P) {
    for (int32_t i = 0; i < qlen; ++i)
        if (q[i] >= SW_ALPHABET) return fail(SW_E_INVALID, "query residue code out of range (use sw_encode)");
    const int bias = affine ? 0 : go;
    P->stride = static_cast<int32_t>(round_up(std::max<int32_t>(qpad_inter, 16), 16));
    const size_t n = static_cast<size_t>(swk::kProfileRows) * P->stride;
    size_t at = 0;
    auto take = [&](size_t bytes) {
        const size_t o = at;
        at = round_up(static_cast<int64_t>(at + bytes), 256);
        return o;
    };
    P->off8 = take(n);
    P->off16 = want16 ? take(2 * n) : 0;
    const int rip = swk::intra_rip(ri);
    const size_t intra_bytes = ri ? static_cast<size_t>(qpad_intra / (swk::kLanes * ri)) * swk::intra_chunk_bytes(ri) : 0;
    P->intra_off = take(intra_bytes);
    P->total = at;
    P->slot = h->prof_next;
    sw_handle::ProfSlot& S = h->prof[h->prof_next];
    h->prof_next = (h->prof_next + 1) % sw_handle::kProfSlots;
    if (S.pending) HIPCHECK(hipEventSynchronize(S.last_end));
    S.pending = false;
    if (P->total > S.dcap) {
        if (S.d) {
            HIPCHECK(hipStreamSynchronize(h->stream));  // scans in flight may still read it
            if (S.tail_pending) HIPCHECK(hipEventSynchronize(S.tail_read));
            S.tail_pending = false;
            HIPCHECK(hipFree(S.d));
        }
        S.dcap = std::max<size_t>(P->total, 1 << 16);
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&S.d), S.dcap));
    }
    P->dev = S.d;
    // on the scan's stream: after the scans before it (the slot's last
    // reader among them), before this one
    if (S.tail_pending) {  // a deferred tail still reads the slot's last profiles
        HIPCHECK(hipStreamWaitEvent(h->stream, S.tail_read, 0));
        S.tail_pending = false;
    }
    swk::ProfileArgs a{};
    a.p8 = S.d + P->off8;
    a.p16 = want16 ? reinterpret_cast<int16_t*>(S.d + P->off16) : nullptr;
    a.pin = ri ? S.d + P->intra_off : nullptr;
    a.stride = P->stride;
    a.qlen = qlen;
    a.bias = bias;
    a.ri = ri;
    a.rip = rip;
    a.qpad_intra = ri ? qpad_intra : 0;
    for (int k = 0; k < 10; ++k) a.reset[k] = reset[k];
    std::memcpy(a.mat, mat, 625);
    const int32_t rows = std::max(P->stride, a.qpad_intra);
    for (int32_t r0 = 0; r0 < rows; r0 += swk::kProfQueryChunk) {
        a.row0 = r0;
        a.row1 = std::min(rows, r0 + swk::kProfQueryChunk);
        const int32_t nq = std::max(0, std::min(a.row1, qlen) - r0);
        if (nq) std::memcpy(a.q, q + r0, static_cast<size_t>(nq));
        HIPCHECK(swk::launch_build_profile(a, h->stream));
        for (auto& p : a.reset) p = nullptr;  // once
    }
    S.last_end = h->ev[3];  // recorded at the end of this scan (scan_impl)
    S.pending = true;
    h->open_slot = P->slot;  // until ev[3] is recorded (scan_impl cleans up if it fails first)
    return SW_OK;
}

// The work table of sw_scan_lpt for this scan shape (built once, cached).
int lpt_table(sw_db* db, int32_t qpad, int rows, int32_t qpad_intra, int ri, int32_t npair, int32_t nquad,
              int32_t ntail, bool affine, bool tri, const int32_t** order, int* n, int32_t* npipe_out,
              int32_t* pipe_tail_out) {
    for (const auto& t : db->lpt_tables)
        if (t.qpad == qpad && t.rows == rows && t.qpad_intra == qpad_intra && t.ri == ri && t.npair == npair && t.group == nquad &&
            t.tail == ntail && t.pipe_opt == db->h->opts.lpt_pipe && t.affine == affine && t.tri == tri &&
            t.tail_opt == db->h->opts.lpt_pipe_tail) {
            *order = t.d_order;
            *n = t.n;
            *npipe_out = t.npipe;
            *pipe_tail_out = t.pipe_tail;
            return SW_OK;
        }
    const swplan::LptPlan pl = swplan::lpt_plan(plan_view(db), qpad, rows, qpad_intra, ri, npair, nquad, ntail,
                                                affine, tri);
    const std::vector<int32_t>& ord = pl.order;
    const std::vector<float>& cost = pl.cost;
    const int64_t npipe = pl.npipe, pipe_tail = pl.pipe_tail;
    sw_db::LptTable t{qpad, rows, qpad_intra, ri, npair, nquad, ntail, static_cast<int32_t>(ord.size()), affine, tri,
                      static_cast<int32_t>(npipe), db->h->opts.lpt_pipe, static_cast<int32_t>(pipe_tail),
                      db->h->opts.lpt_pipe_tail, nullptr, cost};
    HIPCHECK(hipMalloc(reinterpret_cast<void**>(&t.d_order), ord.size() * sizeof(int32_t)));
    HIPCHECK(hipMemcpy(t.d_order, ord.data(), ord.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    db->device_bytes += ord.size() * sizeof(int32_t);
    if (db->lpt_tables.size() >= 8) {
        (void)hipFree(db->lpt_tables.front().d_order);
        db->lpt_tables.erase(db->lpt_tables.begin());
    }
    db->lpt_tables.push_back(t);
    *order = t.d_order;
    *n = t.n;
    *npipe_out = t.npipe;
    *pipe_tail_out = t.pipe_tail;
    return SW_OK;
}

// The device copy of a merged launch's drain arguments (swk::DrainArgs: read
// from the kernel arguments, the drain's values stayed in registers across
// the scan loops and spilled).  `key` lists everything the content is a
// function of (profile slot, list parity, score buffer, query length,
// scoring, split); a miss uploads the content in stream order, a hit (every
// scan of a steady loop after the first few) costs no copy.
int drain_blob(sw_db* db, hipStream_t s, const std::vector<uint64_t>& key, const swk::DrainArgs& d,
               const swk::DrainArgs** out) {
    if (!db->d_drain) {
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_drain), sw_db::kDrainSlots * sizeof(swk::DrainArgs)));
        HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&db->h_drain), sw_db::kDrainSlots * sizeof(swk::DrainArgs),
                               hipHostMallocDefault));
        db->device_bytes += sw_db::kDrainSlots * sizeof(swk::DrainArgs);
    }
    for (size_t k = 0; k < db->drain_keys.size(); ++k)
        if (db->drain_keys[k] == key) {
            *out = db->d_drain + k;
            return SW_OK;
        }
    // a slot is rewritten only after the 31 uploads since its last one, each
    // in stream order behind the scans that read it
    const int k = db->drain_next;
    db->drain_next = (k + 1) % sw_db::kDrainSlots;
    if (static_cast<int>(db->drain_keys.size()) <= k) db->drain_keys.resize(k + 1);
    db->drain_keys[k] = key;
    db->h_drain[k] = d;
    HIPCHECK(hipMemcpyAsync(db->d_drain + k, &db->h_drain[k], sizeof d, hipMemcpyHostToDevice, s));
    *out = db->d_drain + k;
    return SW_OK;
}

// The handle's stream waits for every deferred rescue tail still pending, so
// what completes on it (a non-deferred scan, the end of a batch) includes
// the rescued scores of the scans before it.
int join_tails(sw_handle* h) {
    for (int q = 0; q < 2; ++q)
        if (h->tail_pending[q]) {
            HIPCHECK(hipStreamWaitEvent(h->stream, h->tail_done[q], 0));
            h->tail_pending[q] = false;
        }
    return SW_OK;
}

// A ranking asked for with a scan (sw_scan_rank_device, sw_scan_topk): the
// k best keys of the scan's scores over the database's subjects — result id
// r, global id gid ? gid[r] : id_base + r — into out (device, k keys).
struct RankReq {
    int32_t k;
    const int32_t* gid;
    int64_t id_base;
    int64_t* out;
};

// The ranking input over a database's subjects: its scores through the
// result ids (db->d_ids, uploaded on first use), or directly when the ids
// are 0 .. n-1 in order (the default).
int rank_src(sw_db* db, const int32_t* scores, const RankReq& rq, swk::TopkSrc* src) {
    if (db->rid_identity < 0) {
        db->rid_identity = db->max_id + 1 == db->n;
        for (int64_t k = 0; db->rid_identity == 1 && k < db->n; ++k) db->rid_identity = db->h_ids[k] == k;
    }
    *src = swk::TopkSrc{};
    src->scores = scores;
    src->gid = rq.gid;
    src->id_base = rq.id_base;
    if (!db->rid_identity) {
        if (!db->d_ids) {
            HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_ids), static_cast<size_t>(db->n) * sizeof(int32_t)));
            HIPCHECK(hipMemcpy(db->d_ids, db->h_ids.data(), static_cast<size_t>(db->n) * sizeof(int32_t),
                               hipMemcpyHostToDevice));
            db->device_bytes += static_cast<size_t>(db->n) * sizeof(int32_t);
        }
        src->rid = db->d_ids;
    }
    return SW_OK;
}

// The handle's top-K workspace holds at least `need` bytes; a new one
// starts with the one-launch top-K's counter at zero (swk::launch_topk).
int ensure_topk_work(sw_handle* h, size_t need) {
    if (need > h->topk_cap) {
        if (h->d_topk_work) {
            HIPCHECK(hipStreamSynchronize(h->stream));
            HIPCHECK(hipFree(h->d_topk_work));
        }
        h->topk_cap = std::max<size_t>(need, 1 << 20);
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&h->d_topk_work), h->topk_cap));
        HIPCHECK(hipMemsetAsync(h->d_topk_work, 0, 256, h->stream));
    }
    return SW_OK;
}

int next_events(sw_handle* h) {
    if (h->nscans >= 4096) h->nscans = 0;  // bound the pool; older sums are dropped
    if (h->nscans == h->evpool.size()) {
        ScanEvents se;
        for (auto& e : se.ev) HIPCHECK(hipEventCreate(&e));
        h->evpool.push_back(se);
    }
    h->ev = h->evpool[h->nscans].ev;
    h->ev_rec = &h->evpool[h->nscans].rec;
    *h->ev_rec = 0;
    h->evpool[h->nscans].launches = 0;
    h->evpool[h->nscans].merged = false;
    ++h->nscans;
    return SW_OK;
}

// A scan's ranking: a top-K launch on the scan's stream after every stage
// that writes its scores.
int rank_after(sw_handle* h, sw_db* db, const int32_t* scores_dev, const RankReq& rq) {
    swk::TopkSrc src;
    int rc;
    if ((rc = rank_src(db, scores_dev, rq, &src))) return rc;
    if ((rc = ensure_topk_work(h, swk::topk_workspace_bytes(db->n, rq.k)))) return rc;
    HIPCHECK(swk::launch_topk(src, db->n, rq.k, rq.out, h->d_topk_work, h->stream));
    ++h->launches;
    return SW_OK;
}

// defer: another scan follows on this handle before the caller waits (the
// queries of a batch but the last): this scan's rescue tail may run on the
// tail stream beside the next scan's fp16 passes (sw_handle::tail).
// rq (nullable): rank the scan's scores too (a top-K launch after every
// stage that writes them, before the scan's end event).
int scan_impl_body(sw_handle* h, const sw_db* cdb, const uint8_t* query, int32_t qlen, const sw_scoring* sc,
              int32_t* scores_dev, bool defer = false, const RankReq* rq = nullptr) {
    sw_db* db = const_cast<sw_db*>(cdb);
    if (!h || !db || (!query && qlen > 0) || qlen < 0 || !scores_dev) return fail(SW_E_INVALID, "null argument");
    if (rq) defer = false;  // the ranking reads every rescued score
    const int8_t* mat;
    int go, ge, rc;
    if ((rc = check_fault(h))) return rc;
    if ((rc = check_scoring(sc, &mat, &go, &ge))) return rc;
    // The linear kernels keep S + gap in an int8 profile; if that does not
    // fit, score with the affine kernels (open == extend is the same DP).
    bool biased_fits = true;
    for (int k = 0; k < 625; ++k)
        if (mat[k] + go > 127) biased_fits = false;
    const bool affine = go != ge || !biased_fits;
    if (!db->built && (rc = build_db(db))) return rc;
    HIPCHECK(hipSetDevice(h->device));
    h->launches = 0;
    h->had_intra = false;
    if ((rc = next_events(h))) return rc;

    // The packed int16 kernel is exact when no H, E, F or H_diag + S can
    // leave int16: H <= qlen * max S, plus one profile entry (+ gap bias).
    int max_s = 0;
    for (int k = 0; k < 625; ++k) max_s = std::max<int>(max_s, mat[k]);
    // Beyond that bound the two-strips kernel runs guarded (saturating lanes
    // flag their block for int32 re-scoring) as long as one cell's increment
    // stays far inside the guard band (kSat16 leaves 1152).
    //   m16 = 2: int16 exact; 1: guarded int16 allowed; 0: int32 only
    // Affine 16-bit scans run the fp16 biased cell first; its values sit up
    // to 26 ge above the true ones, so absurd gap / matrix scales (far beyond
    // any published scheme) go straight to int32.
    const bool f16_fits = 2 * max_s + 27 * ge + go < 1024;
    const int x2_ok = !f16_fits                                                   ? 0
                      : (static_cast<int64_t>(qlen) + 2) * (max_s + go) < 32767 ? 2
                      : (max_s + go < 1000 && ge < 1000)                       ? 1
                                                                               : 0;
    const swk::InterShape shape = swk::inter_shape(affine, x2_ok, h->opts);
    const int R = shape.R;
    int32_t qpad_inter = static_cast<int32_t>(round_up(qlen, R));  // (the merged linear launch: see lpt_rows)
    // (the merged launch's drain takes the int32 rows per lane from ri2, below)
    int ri = db->nlong ? swk::intra_rows_for(qlen, db->long_max) : 0;
    int32_t qpad_intra = ri ? static_cast<int32_t>(round_up(qlen, static_cast<int64_t>(swk::kLanes) * ri)) : 0;
    // Long subjects: two per wave in packed fp16 (sw_intra_x2) when the guard
    // applies, with the int32 sw_intra re-scoring the subjects it flags
    // (SW_INTRA_X2=0: int32 only).
    const sw_opts& O = h->opts;
    const bool intra_x2 = db->nlong && x2_ok >= 1 && O.intra_x2 != 0;
    // (20 rows per lane only where no merged launch can take the scan: no
    // inter blocks; where the fp16 bias of row 19 fits, as f16_fits; and by
    // the cost model for affine gaps only, see intra_x2_rows_for)
    const bool ri2_wide = db->nblocks == 0 && 2 * max_s + (swk::intra_bias_rows(swk::kIntraX2MaxRI) + 1) * ge + go < 1024;
    int ri2 =
        intra_x2 ? swk::intra_x2_rows_for(qlen, db->long_max, ri2_wide ? (affine ? 2 : 1) : 0, O.intra_x2_rows) : 0;
    // Affine scans with inter blocks take the merged launch (intra rows 4, 6
    // or 8 only) even where the cost model prefers more rows per lane for the
    // long subjects alone: its tail pairs and looped grid win more (C3's long
    // queries at 8 rows: +1.3 %; under linear gaps the wider form stays,
    // -6.9 % at 8 rows: profiles/r05_ab/c3_ri8/).  Tentative: a scan that
    // does not take the merged launch after all (below) gets the cost
    // model's rows back.
    const int ri2_model = ri2;
    if (affine && ri2 > 8 && db->nblocks && O.intra_x2_rows < 0) ri2 = 8;
    // The intra chain's order from the database's earlier scans
    // (adapt_intra_i16_first), keyed by the scoring and the query:
    uint64_t skey = 1469598103934665603ull;  // FNV-1a of the scoring
    for (int k = 0; k < 625; ++k) skey = (skey ^ static_cast<uint8_t>(mat[k])) * 1099511628211ull;
    skey = ((skey ^ static_cast<uint32_t>(go)) * 1099511628211ull ^ static_cast<uint32_t>(ge)) * 1099511628211ull;
    uint64_t qhash = 1469598103934665603ull;  // FNV-1a of the query (which
    for (int32_t k = 0; k < qlen; ++k) qhash = (qhash ^ query[k]) * 1099511628211ull;  // readbacks repeat)
    const bool intra_i16_first = adapt_intra_i16_first(db, skey, qlen, O.intra_i16_first) && intra_x2;
    // ... and the inter scan's widest blocks in int16 first (adapt_inter_i16_span)
    const int32_t i16_span = adapt_inter_i16_span(db, skey, qlen, O.inter_i16_span);
    int32_t qpad_intra2 = ri2 ? static_cast<int32_t>(round_up(qlen, static_cast<int64_t>(swk::kLanes) * ri2)) : 0;
    // Empty query: every score is 0 (the reference's kernel leaves maxScore 0).
    if (qlen == 0) {
        db->last_ncoop = 0;
        db->last_npair = 0;
        h->last_kernel = "none";
        h->last_intra = "none";
        // a non-deferred scan completes on the handle's stream: so do the
        // earlier scans' deferred tails (a batch may end with an empty query)
        if (!defer && (rc = join_tails(h))) return rc;
        MARK(0, h->stream);
        if (db->max_id >= 0)
            HIPCHECK(hipMemsetAsync(scores_dev, 0, static_cast<size_t>(db->max_id + 1) * 4, h->stream));
        if (rq && (rc = rank_after(h, db, scores_dev, *rq))) return rc;
        for (int k = 1; k < 8; ++k) MARK(k, h->stream);
        h->timed = true;
        return SW_OK;
    }
    Profiles P;
    const bool x2 = shape.x2s;
    // int32 re-scoring of blocks a 16-bit kernel flags near saturation
    const bool rescue = swk::inter_needs_rescue(shape, x2_ok);
    const bool f16 = shape.f16;
    const int32_t qpad_rescue = rescue ? static_cast<int32_t>(round_up(qlen, swk::rescue_rows(affine))) : 0;
    // fp16 chain stage 2 (the int16 two-strips 32x8 kernel): 64-row passes
    // (the linear list kernel is the 48x4 shape: 96-row passes)
    const int32_t qpad_list = f16 ? static_cast<int32_t>(round_up(qlen, affine ? 64 : 96)) : 0;
    // widest blocks first, one cooperative workgroup each (int32, int8-profile paths)
    // two-strips scans: the widest blocks by wave pairs (at least two passes)
    const int32_t npair =
        (db->nblocks && swk::inter_has_pair(shape) && qpad_inter > R) ? swplan::pair_blocks(plan_view(db)) : 0;
    const int32_t ncoop =
        (!npair && db->nblocks) ? swplan::coop_blocks(plan_view(db), swk::inter_coop_divisor(shape)) : 0;
    db->last_ncoop = ncoop;
    db->last_npair = npair;
    db->last_pair_merged = npair != 0;
    // One merged launch for the fp16 scan, longest work first (sw_scan_lpt):
    // the inter groups + single waves and the long subjects' fp16 pass, when
    // the scan takes exactly that shape.  Measured (profiles/r02_strong/lpt/,
    // r02_round/): C2's 1/8 share 1.92 -> 1.45 ms, 1/4 2.57 -> 2.29.  On the
    // whole C2 database it was 2 % slower than two concurrent launches until
    // the launch drained its own rescue lists (no rescue launches or events
    // after it): now 7.19 -> 7.12 ms under affine scoring (C3 and C4's share
    // unchanged), but under linear gaps 4.57 -> 5.03 ms (profiles/r04_*/);
    // since round 5's tail pairs, looped grid and 96-row linear passes the
    // whole C2 database under linear gaps too: 16,512 -> 16,777 GCUPS
    // (profiles/r05_ab/lpt_linear_c2/).  Every scan of that shape takes it;
    // sw_opts lpt 0 / 1 forces either form.
    const bool lpt_want = O.lpt >= 0 ? O.lpt == 1 : true;
    const bool lpt = lpt_want && db->nlong && db->nblocks && intra_x2 && !intra_i16_first &&
                     f16 && rescue && npair && !ncoop && i16_span == 0 &&
                     swk::lpt_supported(ri2);
    db->last_lpt = lpt;
    if (!lpt && ri2 != ri2_model) {  // the separate intra launch: the cost model's shape
        ri2 = ri2_model;
        qpad_intra2 = static_cast<int32_t>(round_up(qlen, static_cast<int64_t>(swk::kLanes) * ri2));
    }
    // ... and that launch re-scores what it flags itself (sw_scan_lpt's drain,
    // swk::DrainArgs): no rescue launches after it, on boundary rows of its
    // own (the deferred tails', when device memory allows them), with the
    // int32 long-subject stage at the fp16 form's rows per lane
    const bool drain = lpt && ensure_rbnd(db, affine, intra_x2);
    db->last_drain = drain;
    if (drain) {
        ri = ri2;
        qpad_intra = static_cast<int32_t>(round_up(qlen, static_cast<int64_t>(swk::kLanes) * ri));
    }
    // The merged launch under linear gaps runs 96-row passes (48-row strips):
    // its widest blocks' wave groups need fewer rounds (a 375-aa query: 4
    // passes, one round of a quad, against 6 passes and two rounds of 64
    // rows), and the share's span is those blocks' latency;
    // the linear cell's registers leave room for the taller strips.  Affine
    // scans keep 64 rows (their E column would not fit).  sw_opts lpt_rows.
    const int lpt_rows = (lpt && !affine && O.lpt_rows != 64 && round_up(qlen, 96) > 96) ? 96 : 64;
    if (lpt_rows == 96) qpad_inter = static_cast<int32_t>(round_up(qlen, 96));
    const int32_t qpad_coop = ncoop ? static_cast<int32_t>(round_up(qlen, swk::inter_coop_rows())) : 0;
    // lists A and B, the largest flagged block, a spare word, the dequeue
    // heads of A and B (the merged launch's drain); every entry starts at -1
    // (sw_kernels.h: whoever takes an entry resets it)
    const int64_t rstride = 2 * (db->nblocks + 1) + 4;
    const int64_t lstride = 2 * (db->nlong + 1) + 2;  // intra lists 1 and 2, their heads
    if (rescue && db->nblocks && !db->d_rescue) {
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_rescue), 2 * rstride * sizeof(int32_t)));
        HIPCHECK(hipMemsetAsync(db->d_rescue, 0xff, 2 * rstride * sizeof(int32_t), h->stream));
        db->device_bytes += 2 * rstride * sizeof(int32_t);
    }
    const bool multi_inter = qpad_inter > R || qpad_rescue > swk::rescue_rows(affine) ||
                             qpad_coop > swk::inter_coop_rows() || qpad_list > (affine ? 64 : 96);
    const bool multi_intra = (ri && qpad_intra > swk::kLanes * ri) || (ri2 && qpad_intra2 > swk::kLanes * ri2);
    if ((multi_inter || multi_intra) && (rc = ensure_bnd(db, affine, intra_x2))) return rc;
    if (intra_x2 && !db->d_lrescue) {  // two lists: [count, subjects...] x 2
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&db->d_lrescue), 2 * lstride * sizeof(int32_t)));
        HIPCHECK(hipMemsetAsync(db->d_lrescue, 0xff, 2 * lstride * sizeof(int32_t), h->stream));
        db->device_bytes += 2 * lstride * sizeof(int32_t);
    }
    if (db->list_epoch != g_fault_epoch.load()) {  // a fault since: entries may be left claimed
        if ((rc = join_tails(h))) return rc;
        if (db->d_rescue) HIPCHECK(hipMemsetAsync(db->d_rescue, 0xff, 2 * rstride * sizeof(int32_t), h->stream));
        if (db->d_lrescue) HIPCHECK(hipMemsetAsync(db->d_lrescue, 0xff, 2 * lstride * sizeof(int32_t), h->stream));
        db->list_epoch = g_fault_epoch.load();
    }
    // this scan's list set; a deferred tail of the scan before last used it
    const int par = h->parity;
    h->parity ^= 1;
    if (h->tail_pending[par]) {
        HIPCHECK(hipStreamWaitEvent(h->stream, h->tail_done[par], 0));
        h->tail_pending[par] = false;
    }
    // The drain re-scores on the deferred tails' boundary rows (d_rbnd_*,
    // d_rlbnd_*): a non-merged scan just before this one (a longer query
    // routed int16-first, say) may still be running its tail on those rows,
    // so the merged launch starts after every pending tail.
    if (drain && (rc = join_tails(h))) return rc;
    int32_t* const listA = db->d_rescue ? db->d_rescue + par * rstride : nullptr;  // [count, ids...]
    int32_t* const listB = listA ? listA + db->nblocks + 1 : nullptr;
    int32_t* const maxA = listA ? listA + 2 * (db->nblocks + 1) : nullptr;
    int32_t* const list1 = db->d_lrescue ? db->d_lrescue + par * lstride : nullptr;  // flagged by the fp16 pass
    int32_t* const list2 = list1 ? list1 + db->nlong + 1 : nullptr;                  // ... and again by int16
    int32_t* const headA = listA ? maxA + 2 : nullptr;  // the drain's dequeue heads: A, B, 1, 2
    // the merged launch's work counter (the spare word; persistent form)
    int32_t* const lpt_next = (lpt && listA && O.lpt_persist != 0) ? maxA + 1 : nullptr;
    int32_t* const head1 = list1 ? list2 + db->nlong + 1 : nullptr;
    // the rescue tail on its own stream and boundary rows (see sw_handle::tail)
    const bool deferred = !drain && defer && (!(multi_inter || multi_intra) || ensure_rbnd(db, affine, intra_x2));
    hipStream_t const ts = deferred ? h->tail : h->stream;

    // the profiles, and the rescue lists' counters (inter A, B, largest
    // flagged block; intra 1, 2) zeroed by the same launch, before the fork
    // so the side streams see them
    {
        int32_t* const cA = (rescue && db->nblocks) ? listA : nullptr;
        int32_t* const c1 = (db->nlong && intra_x2) ? list1 : nullptr;
        int32_t* const reset[10] = {cA, (cA && f16) ? listB : nullptr, (cA && f16) ? maxA : nullptr, c1,
                                    c1 ? list2 : nullptr, drain ? headA : nullptr, drain ? headA + 1 : nullptr,
                                    drain ? head1 : nullptr, drain ? head1 + 1 : nullptr, lpt_next};
        if ((rc = build_profiles(h, query, qlen, mat, go, affine,
                                 std::max({qpad_inter, qpad_rescue, qpad_coop, qpad_list, qpad_intra2}),
                                 x2 || intra_x2, ri, qpad_intra, reset, &P)))
            return rc;
    }
    h->evpool[h->nscans - 1].merged = lpt;
    // fork: the side streams start when the main stream reaches ev[0] (the
    // merged launch has none: its scan time runs from ev[6])
    if (!lpt) MARK(0, h->stream);
    h->last_intra = "none";
    // the long subjects' stream: a side stream, concurrent with the inter
    // kernels; with the merged launch, the main stream after it (only the
    // rescue stages are left to run)
    hipStream_t is = lpt ? h->stream : h->side;
    swk::IntraArgs lpt_intra{}, lpt_i32{};  // the merged launch's fp16 pass and its drain's int32 stage
    // the long subjects' kernels: all of them, or (lpt_done) those after the
    // fp16 pass the merged launch ran
    // The long subjects' rescue stages (the int16 form over the fp16 pass's
    // list, then int32 over what is left), on stream st with boundary rows
    // bh / bf: right after the passes (stream order), or deferred to the
    // tail stream with the tail's own boundary rows.
    swk::IntraArgs tail_x{}, tail_ia{};
    bool intra_tail = false;
    auto launch_intra_tail = [&](hipStream_t st, int32_t* bh, int32_t* bf) -> int {
        if (!intra_i16_first) {
            // the int16 form re-scores the fp16 pass's list (scores near
            // 2048: high-scoring pairs, or linear scoring with cheap gaps)
            // and flags near-32767 ones
            swk::IntraArgs y = tail_x;
            y.bnd_h = bh;
            y.bnd_f = bf;
            y.list_count = list1;
            y.subj_list = list1 + 1;
            y.rescue_count = list2;
            y.rescue_list = list2 + 1;
            HIPCHECK(swk::launch_intra_x2_list16(y, ri2, st));
            ++h->launches;
        }
        // int32 re-scoring of what is left (device-side list)
        swk::IntraArgs ia = tail_ia;
        ia.bnd_h = bh;
        ia.bnd_f = bf;
        HIPCHECK(swk::launch_intra(ia, ri, affine, st));
        ++h->launches;
        return SW_OK;
    };
    // The inter scan's rescue tail: the int16 packed kernel over the blocks
    // the fp16 kernel flagged (list A: scores near 2048; it flags its own
    // near-32767 ones into list B), then int32 over list B (list A for the
    // int16 scans), on stream st with boundary rows bh / bf.
    swk::InterArgs tail_a{};
    bool inter_tail = false;
    auto launch_inter_tail = [&](hipStream_t st, int32_t* bh, int32_t* bf) -> int {
        if (f16) {
            swk::InterArgs r = tail_a;
            r.bnd_h = bh;
            r.bnd_f = bf;
            r.qpad = qpad_list;
            r.blk_list = listA + 1;
            r.blk_count = listA;
            r.rescue_list = listB + 1;
            r.rescue_count = listB;
            r.rescue_max = nullptr;
            HIPCHECK(swk::launch_inter_x2s_list(r, affine, st));
            ++h->launches;
        }
        swk::InterArgs r = tail_a;
        r.bnd_h = bh;
        r.bnd_f = bf;
        r.prof = P.dev + P.off8;
        r.qpad = qpad_rescue;
        r.blk_list = (f16 ? listB : listA) + 1;
        r.blk_count = f16 ? listB : listA;
        r.rescue_list = nullptr;
        r.rescue_count = nullptr;
        HIPCHECK(swk::launch_inter_rescue(r, affine, st));
        ++h->launches;
        return SW_OK;
    };
    // the long subjects' kernels: all of them, or (lpt_done) those after the
    // fp16 pass the merged launch ran
    auto launch_long = [&](bool lpt_done) -> int {
        if (!lpt_done && is != h->stream) HIPCHECK(hipStreamWaitEvent(is, h->ev[0], 0));
        swk::IntraArgs ia{};
        ia.residues = db->d_lres;
        ia.subj_off = db->d_loff;
        ia.subj_len = db->d_llen;
        ia.subj_id = db->d_lid;
        ia.nsubj = static_cast<int32_t>(db->nlong);
        ia.prof = P.dev + P.intra_off;
        ia.qpad = qpad_intra;
        ia.gap_open = go;
        ia.gap_extend = ge;
        ia.bnd_h = db->d_lbnd_h;
        ia.bnd_f = db->d_lbnd_f;
        ia.scores = scores_dev;
        h->last_intra = intra_x2 ? "sw_intra_x2<" + std::to_string(ri2) + (intra_i16_first ? ",int16>" : ">")
                                 : "sw_intra<" + std::to_string(ri) + (affine ? ",affine>" : ",linear>");
        h->had_intra = true;
        if (!intra_x2) {  // int32 over every long subject
            HIPCHECK(swk::launch_intra(ia, ri, affine, is));
            ++h->launches;
            return SW_OK;
        }
        swk::IntraArgs x = ia;
        x.prof = P.dev + P.off16;
        x.prof_stride = P.stride;
        x.bias = affine ? 0 : go;  // the linear profile holds S + gap
        x.qpad = qpad_intra2;
        // biased cell: stored values up to (RI + 10) ge above the true ones,
        // offset by zero = -2048 + 2 ge as the inter cell's (the lowest value
        // an addition reads is a rebased row -1 H of bias -2 ge: exact)
        const int zero = -kF16Span + 2 * ge;
        x.sat_limit = kF16Span - zero - 2 * std::max(max_s, 1) - swk::intra_bias_rows(ri2) * ge;
        for (int j = 0; j < swk::kIntraSteps; ++j) x.f16_step[j] = f16_pair(j * ge + zero);
        x.f16_zero = f16_pair(zero);
        x.f16_gog = f16_pair(go - ge);
        if (intra_i16_first) {
            // the int16 form over every long subject, flagging near-32767 ones
            x.rescue_count = list2;
            x.rescue_list = list2 + 1;
            HIPCHECK(swk::launch_intra_x2_int16(x, ri2, is));
            h->launches += 1;
        } else {
            x.rescue_count = list1;
            x.rescue_list = list1 + 1;
            if (lpt && !lpt_done) {  // the merged launch runs this pass
                lpt_intra = x;
                lpt_i32 = ia;
                return SW_OK;
            }
            if (!lpt_done) {
                HIPCHECK(swk::launch_intra_x2(x, ri2, is));
                ++h->launches;
            }
            // the fp16 pass's flagged count, read by a later scan
            if (!db->h_lcount) {
                HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&db->h_lcount), sizeof(int32_t),
                                       hipHostMallocDefault));
                HIPCHECK(hipEventCreateWithFlags(&db->lcount_ev, hipEventDisableTiming));
            }
            const bool lseen = db->lcount_seen && db->lseen_key == skey && db->lseen_qhash == qhash &&
                               db->lseen_qlen == qlen;
            if (!db->lcount_pending && !lseen) {
                HIPCHECK(hipMemcpyAsync(db->h_lcount, list1, sizeof(int32_t), hipMemcpyDeviceToHost, is));
                HIPCHECK(hipEventRecord(db->lcount_ev, is));
                db->lcount_pending = true;
                db->lcount_key = skey;
                db->lcount_qlen = qlen;
                db->lcount_qhash = qhash;
            }
            if (drain) return SW_OK;  // the merged launch re-scored its flagged subjects itself
        }
        tail_x = x;
        tail_ia = ia;
        tail_ia.list_count = list2;
        tail_ia.subj_list = list2 + 1;
        intra_tail = true;
        if (deferred) {  // after the fp16 pass; launched on the tail stream below
            HIPCHECK(hipEventRecord(h->side_done, is));
            return SW_OK;
        }
        return launch_intra_tail(is, db->d_lbnd_h, db->d_lbnd_f);
    };
    if (db->nlong && (rc = launch_long(false))) return rc;
    if (!lpt) MARK(1, db->nlong ? is : h->stream);
    if (db->nblocks) {
        swk::InterArgs a{};
        a.residues = db->d_res;
        a.blk_off = db->d_blk_off;
        a.blk_groups = db->d_blk_groups;
        a.blk_cols = db->d_blk_cols;
        a.lane_ids = db->d_lane_ids;
        a.nblocks = static_cast<int32_t>(db->nblocks);
        a.prof = P.dev + (x2 ? P.off16 : P.off8);
        a.prof_stride = P.stride;
        a.qpad = qpad_inter;
        a.gap_open = go;
        a.gap_extend = ge;
        a.bnd_h = db->d_bnd_h;
        a.bnd_f = db->d_bnd_f;
        a.scores = scores_dev;
        if (O.trace_file[0]) {
            if (!db->h_trace) {
                // one entry per block, then one per workgroup of a merged
                // launch (at most nblocks inter + nlong / 8 intra workgroups)
                db->trace_entries = static_cast<size_t>(2 * db->nblocks + db->nlong + 8);
                HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&db->h_trace), 32 * db->trace_entries,
                                       hipHostMallocMapped));
                std::memset(db->h_trace, 0, 32 * db->trace_entries);
            }
            HIPCHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.trace), db->h_trace, 0));
        }
        // the widest blocks the int16 kernel takes first (see i16_span)
        const int32_t nr = (f16 && rescue && npair && !ncoop) ? i16_span : 0;
        db->last_i16_span = nr;
        if (rescue) {
            a.rescue_count = listA;
            a.rescue_list = listA + 1;
            if (f16) a.rescue_max = maxA;  // counters reset before the fork
            // fp16 exact range: every integer in [-2048, 2048].  The cell
            // stores true + bias + zero with zero = -2048 + 2 ge, which
            // nearly doubles the range of true values: the lowest value a
            // later addition reads is a rebased H of bias -ge (>= -2048:
            // exact); values further below lose to the floor, which sits at
            // zero or above, and only need their order.  H grows by <= max S
            // per cell and the biased cell stores values up to 26 ge above
            // the true ones (bias (15 + 7 + 2) ge, + 2 ge in the profile).
            const int zero = -kF16Span + 2 * ge;
            a.sat_limit = kF16Span - zero - 2 * std::max(max_s, 1) - 26 * ge;
            for (int j = 0; j < 32; ++j) a.f16_step[j] = f16_pair(j * ge + zero);
            a.f16_gog = f16_pair(go - ge);
            a.f16_zero = f16_pair(zero);
            a.f16_diff[0] = f16_pair(4 * ge);
            a.f16_diff[1] = f16_pair(8 * ge);
            a.f16_diff[2] = f16_pair(16 * ge);
        }
        if (ncoop) {
            // on its own stream, so the per-wave kernel fills the GPU beside it
            swk::InterArgs c = a;
            c.qpad = qpad_coop;
            c.prof = P.dev + P.off8;  // the coop kernel reads the int8 profile
            HIPCHECK(hipStreamWaitEvent(h->side2, h->ev[0], 0));
            MARK(4, h->side2);
            HIPCHECK(swk::launch_inter_coop(c, ncoop, affine, h->opts.coop_skew != 0, h->side2));
            MARK(5, h->side2);
            HIPCHECK(hipEventRecord(h->coop_done, h->side2));
            ++h->launches;
            a.blk_first = ncoop;
        } else if (nr) {
            // blocks [0, nr) in int16 by wave pairs beside the fp16 launch;
            // their near-32767 ones go to list B (the int32 stage)
            swk::InterArgs c = a;
            c.nblocks = nr;
            c.blk_base = 0;
            c.rescue_list = listB + 1;
            c.rescue_count = listB;
            c.rescue_max = nullptr;
            HIPCHECK(hipEventRecord(h->fork2, h->stream));
            HIPCHECK(hipStreamWaitEvent(h->side2, h->fork2, 0));
            MARK(4, h->side2);
            HIPCHECK(swk::launch_inter_x2p(c, affine, false, false, 2, h->side2));
            MARK(5, h->side2);
            HIPCHECK(hipEventRecord(h->coop_done, h->side2));
            ++h->launches;
        }
        MARK(6, h->stream);
        int32_t ntail = 0;  // merged launch: the narrowest blocks by pairs
        int32_t ntri = 0;   // ... and the widest by 3-wave groups
        if (lpt) {
            // one launch: the inter groups + single waves and the long
            // subjects' fp16 pass, longest work first; then the long
            // subjects' rescue stages
            a.blk_base = 0;
            a.blk_first = npair;
            const int32_t* order = nullptr;
            int nwg = 0;
            ntri = affine ? swplan::lpt_tri_blocks(plan_view(db), npair, qpad_inter / lpt_rows) : 0;
            const int32_t nquad = ntri ? ntri : swplan::lpt_quad_blocks(plan_view(db), npair);
            a.blk_quad = nquad;
            a.blk_tri = ntri ? 1 : 0;
            ntail = swplan::lpt_tail_blocks(plan_view(db), npair, qpad_inter / lpt_rows);
            a.blk_tail = static_cast<int32_t>(db->nblocks) - ntail;
            int32_t npipe = 0, pipe_tail = 0;
            if ((rc = lpt_table(db, qpad_inter, lpt_rows, qpad_intra2, ri2, npair, nquad, ntail, affine, ntri != 0,
                                &order, &nwg, &npipe, &pipe_tail)))
                return rc;
            lpt_intra.pipe_pairs = npipe;
            lpt_intra.pipe_tail = pipe_tail;
            const swk::DrainArgs* dargs = nullptr;
            if (drain) {
                // the four rescue stages of launch_inter_tail / launch_intra_tail,
                // on the tails' boundary rows (sw_kernels.h DrainArgs)
                swk::DrainArgs d{};
                d.a16 = a;
                d.a16.bnd_h = db->d_rbnd_h;
                d.a16.bnd_f = db->d_rbnd_f;
                d.a16.qpad = qpad_list;
                d.a16.rescue_list = listB + 1;
                d.a16.rescue_count = listB;
                d.a16.rescue_max = nullptr;
                d.a16.trace = nullptr;
                d.a32 = a;
                d.a32.bnd_h = db->d_rbnd_h;
                d.a32.bnd_f = db->d_rbnd_f;
                d.a32.prof = P.dev + P.off8;
                d.a32.qpad = qpad_rescue;
                d.a32.rescue_list = nullptr;
                d.a32.rescue_count = nullptr;
                d.a32.rescue_max = nullptr;
                d.a32.trace = nullptr;
                d.i16 = lpt_intra;
                d.i16.bnd_h = db->d_rlbnd_h;
                d.i16.bnd_f = db->d_rlbnd_f;
                d.i16.rescue_list = list2 + 1;
                d.i16.rescue_count = list2;
                d.i32 = lpt_i32;
                d.i32.bnd_h = db->d_rlbnd_h;
                d.i32.bnd_f = db->d_rlbnd_f;
                d.lists[0] = listA;
                d.lists[1] = listB;
                d.lists[2] = list1;
                d.lists[3] = list2;
                d.heads[0] = headA;
                d.heads[1] = headA + 1;
                d.heads[2] = head1;
                d.heads[3] = head1 + 1;
                d.fault = h->d_fault;
                d.spin = O.drain_spin >= 0 ? O.drain_spin : (1 << 22);
                // (every field of d the blob's bytes depend on)
                const std::vector<uint64_t> key = {
                    reinterpret_cast<uint64_t>(P.dev), P.off8, P.off16, P.intra_off, static_cast<uint64_t>(par),
                    reinterpret_cast<uint64_t>(scores_dev), static_cast<uint64_t>(qlen), skey,
                    static_cast<uint64_t>(npair) | static_cast<uint64_t>(a.blk_tri) << 32,
                    static_cast<uint64_t>(nquad) | static_cast<uint64_t>(ntail) << 32,
                    static_cast<uint64_t>(P.stride),
                    reinterpret_cast<uint64_t>(a.trace),
                    static_cast<uint64_t>(ri2) | static_cast<uint64_t>(lpt_rows) << 16 |
                        static_cast<uint64_t>(npipe) << 32,
                    static_cast<uint64_t>(static_cast<uint32_t>(pipe_tail)),
                    static_cast<uint64_t>(static_cast<uint32_t>(d.spin))};
                if ((rc = drain_blob(db, h->stream, key, d, &dargs))) return rc;
            }
            HIPCHECK(swk::launch_scan_lpt(a, lpt_intra, order, nwg, affine, ri2, h->cus, h->stream, dargs, lpt_next,
                                          O.lpt_persist >= 2 ? O.lpt_persist : 0, lpt_rows));
            // (a draining launch ends the scan: its end event is ev[3])
            if (!drain) MARK(7, h->stream);
            if ((rc = launch_long(true))) return rc;
        } else if (npair) {
            // one launch: pairs for blocks [nr, npair), one wave per block after
            a.blk_base = nr;
            a.blk_first = std::max(npair, nr);
            HIPCHECK(swk::launch_inter_x2p(a, affine, f16, true, swplan::pair_group(plan_view(db)), h->stream));
        } else {
            HIPCHECK(swk::launch_inter(a, affine, shape, h->stream));
        }
        h->last_kernel = swk::inter_kernel_name(shape, affine);
        if (npair) h->last_kernel.replace(0, std::strlen("sw_inter_x2s"), "sw_inter_x2p");  // + wave pairs
        if (lpt && lpt_rows == 96) h->last_kernel.replace(h->last_kernel.find("<32,"), 4, "<48,");  // 48-row strips
        if (nr) h->last_kernel += "+int16[0," + std::to_string(nr) + ")";
        if (ntail) h->last_kernel += "+tail" + std::to_string(ntail);
        if (ntri) h->last_kernel += "+tri" + std::to_string(ntri);
        if (lpt) h->last_kernel += drain ? "+lpt+drain" : "+lpt";
        if (!lpt) MARK(7, h->stream);
        ++h->launches;
        if (ncoop || nr) HIPCHECK(hipStreamWaitEvent(h->stream, h->coop_done, 0));
        const bool seen = db->icount_seen && db->seen_key == skey && db->seen_qhash == qhash &&
                          db->seen_qlen == qlen && db->seen_nr == nr;
        if (f16 && rescue && !db->icount_pending && !seen) {
            // the fp16 pass's flagged count and largest flagged block, read
            // by a later scan (no synchronisation here), after every fp16
            // launch that appends to list A has joined the main stream
            if (!db->h_icount) {
                HIPCHECK(hipHostMalloc(reinterpret_cast<void**>(&db->h_icount), 2 * sizeof(int32_t),
                                       hipHostMallocDefault));
                HIPCHECK(hipEventCreateWithFlags(&db->icount_ev, hipEventDisableTiming));
            }
            HIPCHECK(hipMemcpyAsync(db->h_icount, listA, sizeof(int32_t), hipMemcpyDeviceToHost, h->stream));
            HIPCHECK(hipMemcpyAsync(db->h_icount + 1, maxA, sizeof(int32_t), hipMemcpyDeviceToHost, h->stream));
            HIPCHECK(hipEventRecord(db->icount_ev, h->stream));
            db->icount_pending = true;
            db->icount_key = skey;
            db->icount_qlen = qlen;
            db->icount_nr = nr;
            db->icount_qhash = qhash;
        }
        tail_a = a;
        inter_tail = rescue && !drain;
        if (deferred && inter_tail) HIPCHECK(hipEventRecord(h->main_done, h->stream));
        else if (inter_tail && (rc = launch_inter_tail(h->stream, db->d_bnd_h, db->d_bnd_f))) return rc;
    }
    if (deferred && (inter_tail || intra_tail)) {
        // this scan's rescue tail beside the next scan's fp16 passes
        if (inter_tail) {
            HIPCHECK(hipStreamWaitEvent(ts, h->main_done, 0));
            if ((rc = launch_inter_tail(ts, db->d_rbnd_h, db->d_rbnd_f))) return rc;
        }
        if (intra_tail) {
            HIPCHECK(hipStreamWaitEvent(ts, h->side_done, 0));
            if ((rc = launch_intra_tail(ts, db->d_rlbnd_h, db->d_rlbnd_f))) return rc;
        }
        HIPCHECK(hipEventRecord(h->tail_done[par], ts));
        h->tail_pending[par] = true;
        sw_handle::ProfSlot& S = h->prof[P.slot];
        HIPCHECK(hipEventRecord(S.tail_read, ts));
        S.tail_pending = true;
    }
    if (!db->nblocks)
        for (int k = 6; k < 8; ++k) MARK(k, h->stream);
    // (the merged launch has no separate inter end, nor a side stream to join)
    if (!lpt) MARK(2, h->stream);
    if (db->nlong && !lpt) HIPCHECK(hipStreamWaitEvent(h->stream, h->ev[1], 0));
    // the scan completes on the handle's stream: so do earlier deferred tails
    if (!deferred && (rc = join_tails(h))) return rc;
    if (rq && (rc = rank_after(h, db, scores_dev, *rq))) return rc;
    MARK(3, h->stream);
    h->open_slot = -1;
    h->evpool[h->nscans - 1].launches = h->launches;
    h->timed = true;
    if (O.rescue_stats == 1) {  // diagnostics: what the guard bands flagged (synchronises)
        HIPCHECK(hipStreamSynchronize(h->stream));
        HIPCHECK(hipStreamSynchronize(h->tail));
        int32_t cA = 0, cB = 0, l1 = 0, l2 = 0;
        std::vector<int32_t> ids;
        if (listA) {
            HIPCHECK(hipMemcpy(&cA, listA, 4, hipMemcpyDeviceToHost));
            HIPCHECK(hipMemcpy(&cB, listB, 4, hipMemcpyDeviceToHost));
            ids.resize(static_cast<size_t>(cA));
            if (cA) HIPCHECK(hipMemcpy(ids.data(), listA + 1, 4 * ids.size(), hipMemcpyDeviceToHost));
        }
        if (list1) {
            HIPCHECK(hipMemcpy(&l1, list1, 4, hipMemcpyDeviceToHost));
            HIPCHECK(hipMemcpy(&l2, list2, 4, hipMemcpyDeviceToHost));
        }
        int64_t res = 0;
        int32_t wmin = 1 << 30, wmax = 0, bmin = 1 << 30, bmax = -1;
        for (int32_t b : ids) {
            if (b < 0) continue;  // (taken entries are reset to -1: a drained list shows counts only)
            res += db->h_blk_res[b];
            wmin = std::min<int32_t>(wmin, db->h_blk_groups[b] * 16);
            wmax = std::max<int32_t>(wmax, db->h_blk_groups[b] * 16);
            bmin = std::min(bmin, b);
            bmax = std::max(bmax, b);
        }
        std::fprintf(stderr,
                     "rescue: qlen %d go %d ge %d: inter %d/%lld blocks flagged (ids %d..%d, widths %d..%d, "
                     "%lld of %lld residues), %d again; pairs %d; intra %d/%lld flagged, %d again\n",
                     qlen, go, ge, cA, static_cast<long long>(db->nblocks), bmin, bmax, wmin, wmax,
                     static_cast<long long>(res), static_cast<long long>(db->residues), cB, npair, l1,
                     static_cast<long long>(db->nlong), l2);
    }
    return SW_OK;
}

// A scan that fails after its profiles were built leaves the profile slot
// pending on an end event it never recorded: a later scan reusing the slot
// would not wait for the kernels this one queued.  Drain the handle's streams
// and release the slot instead.
int scan_impl(sw_handle* h, const sw_db* db, const uint8_t* query, int32_t qlen, const sw_scoring* sc,
              int32_t* scores_dev, bool defer = false, const RankReq* rq = nullptr) {
    const int rc = scan_impl_body(h, db, query, qlen, sc, scores_dev, defer, rq);
    if (h && h->open_slot >= 0) {
        for (hipStream_t st : {h->stream, h->side, h->side2, h->tail})
            if (st) (void)hipStreamSynchronize(st);
        h->prof[h->open_slot].pending = false;
        h->open_slot = -1;
    }
    return rc;
}

int ensure_scores(sw_handle* h, size_t n) {
    if (n > h->scores_cap) {
        if (h->d_scores) HIPCHECK(hipFree(h->d_scores));
        h->scores_cap = std::max<size_t>(n, 1024);
        HIPCHECK(hipMalloc(reinterpret_cast<void**>(&h->d_scores), h->scores_cap * 4));
    }
    return SW_OK;
}

}  // namespace

namespace {
int topk_impl(sw_handle* h, const int32_t* scores, const int64_t* keys, int64_t n, int64_t id_base,
              const int32_t* ids, int32_t k, int64_t* out) {
    if (!h || !out || n < 0 || k <= 0 || k > 4096 || (n > 0 && !scores && !keys))
        return fail(SW_E_INVALID, "bad top-k arguments (1 <= k <= 4096)");
    if (id_base < 0 || id_base + n > (int64_t(1) << 31)) return fail(SW_E_INVALID, "ids must fit in 31 bits");
    HIPCHECK(hipSetDevice(h->device));
    int rc;
    if ((rc = check_fault(h))) return rc;
    if ((rc = ensure_topk_work(h, swk::topk_workspace_bytes(n, k)))) return rc;
    swk::TopkSrc src{};
    src.scores = keys ? nullptr : scores;
    src.keys = keys;
    src.gid = ids;
    src.id_base = id_base;
    HIPCHECK(swk::launch_topk(src, n, k, out, h->d_topk_work, h->stream));
    return SW_OK;
}
}  // namespace

// ===========================================================================
extern "C" {

int32_t sw_version(void) { return 10000 * 0 + 100 * 1 + 0; }

#ifndef SW_SOURCE_ID
#define SW_SOURCE_ID "unknown"
#endif
const char* sw_build_id(void) { return SW_SOURCE_ID; }

const char* sw_last_error(void) { return g_err.c_str(); }

int sw_encode(const char* ascii, int64_t n, uint8_t* codes) {
    if ((!ascii || !codes) && n > 0) return fail(SW_E_INVALID, "null argument");
    init_lut();
    for (int64_t i = 0; i < n; ++i) codes[i] = static_cast<uint8_t>(g_encode_lut[static_cast<unsigned char>(ascii[i])]);
    return SW_OK;
}

int sw_builtin_matrix(int32_t id, int8_t* out625) {
    if (!out625) return fail(SW_E_INVALID, "null argument");
    if (id == SW_MATRIX_BLOSUM50_REF) {
        std::memcpy(out625, kBlosum50Ref, 625);
    } else if (id == SW_MATRIX_BLOSUM62) {
        std::memcpy(out625, kBlosum62, 625);
    } else if (id == SW_MATRIX_IDENTITY3) {
        for (int a = 0; a < 25; ++a)
            for (int b = 0; b < 25; ++b) out625[a * 25 + b] = static_cast<int8_t>(a == b ? 3 : -3);
    } else if (id == SW_MATRIX_BLOSUM50_CHAR) {
        // the letters score as BLOSUM50_REF; '*' (and
        // everything convertStringToChar maps to it) -5, '*' vs '*' +1
        std::memcpy(out625, kBlosum50Ref, 625);
        for (int k = 0; k < 25; ++k) out625[SW_CODE_STAR * 25 + k] = out625[k * 25 + SW_CODE_STAR] = -5;
        out625[SW_CODE_STAR * 25 + SW_CODE_STAR] = 1;
    } else {
        return fail(SW_E_INVALID, "unknown matrix id");
    }
    return SW_OK;
}

int sw_create(int32_t device, sw_handle** out) {
    if (!out) return fail(SW_E_INVALID, "null argument");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SW_E_NODEVICE, "no HIP device visible");
    if (device < 0 || device >= ndev) return fail(SW_E_INVALID, "device index out of range");
    HIPCHECK(hipSetDevice(device));
    auto* h = new (std::nothrow) sw_handle();
    if (!h) return fail(SW_E_NOMEM, "out of host memory");
    h->device = device;
    // the device's CUs, once (the merged launch's slot counts: lpt_tail_blocks,
    // the looped grid's size)
    if (hipDeviceGetAttribute(&h->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) h->cus = 0;
    hipError_t e = hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking);
    if (e != hipSuccess) { delete h; return fail(SW_E_HIP, hipGetErrorString(e)); }
    h->own_stream = true;
    // side and side2 are created with the handle, right after its own
    // stream: HIP maps normal-priority streams onto GPU_MAX_HW_QUEUES (4)
    // hardware queues, least-used first, and two streams sharing a queue run
    // in order.  Created here they take the queues beside the own stream.
    // Created on first use instead, side2 shared the caller's queue
    // and the int16 launch beside the fp16 one ran after it (C3 under the
    // reference scoring 12,840 -> 8,900 GCUPS).
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->side2, hipStreamNonBlocking);
    // The deferred rescue tails (batches) run at high priority: HIP serves
    // those streams from a separate queue pool, so a tail never shares a
    // hardware queue with the next query's scan (sharing one, the next
    // scan waited behind the tail: C3, the reference scoring's long queries
    // stalled 9-13 ms each behind their int16 list kernel).
    if (e == hipSuccess) {
        int least = 0, greatest = 0;
        e = hipDeviceGetStreamPriorityRange(&least, &greatest);
        if (e == hipSuccess) e = hipStreamCreateWithPriority(&h->tail, hipStreamNonBlocking, greatest);
    }
    for (hipEvent_t* ev : {&h->main_done, &h->side_done, &h->tail_done[0], &h->tail_done[1]})
        if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    for (auto& S : h->prof) {
        if (e == hipSuccess) e = hipEventCreateWithFlags(&S.tail_read, hipEventDisableTiming);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->coop_done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&h->fork2, hipEventDisableTiming);
    if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void**>(&h->h_fault), sizeof(int32_t), hipHostMallocMapped);
    if (e == hipSuccess) {
        *h->h_fault = 0;
        e = hipHostGetDevicePointer(reinterpret_cast<void**>(&h->d_fault), h->h_fault, 0);
    }
    for (auto& ev : h->stage_ev)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) { delete h; return fail(SW_E_HIP, hipGetErrorString(e)); }
    *out = h;
    return SW_OK;
}

int sw_destroy(sw_handle* h) {
    if (!h) return SW_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    for (auto& se : h->evpool)
        for (auto& ev : se.ev)
            if (ev) (void)hipEventDestroy(ev);
    if (h->side) (void)hipStreamSynchronize(h->side);
    if (h->side2) (void)hipStreamSynchronize(h->side2);
    if (h->tail) (void)hipStreamSynchronize(h->tail);
    for (auto& S : h->prof) {
        if (S.d) (void)hipFree(S.d);
        if (S.tail_read) (void)hipEventDestroy(S.tail_read);
    }
    if (h->d_scores) (void)hipFree(h->d_scores);
    if (h->d_topk_work) (void)hipFree(h->d_topk_work);
    for (int b = 0; b < 2; ++b) {
        if (h->stage[b]) (void)hipHostFree(h->stage[b]);
        if (h->stage_ev[b]) (void)hipEventDestroy(h->stage_ev[b]);
    }
    if (h->side) (void)hipStreamDestroy(h->side);
    if (h->side2) (void)hipStreamDestroy(h->side2);
    if (h->tail) (void)hipStreamDestroy(h->tail);
    for (hipEvent_t ev : {h->main_done, h->side_done, h->tail_done[0], h->tail_done[1]})
        if (ev) (void)hipEventDestroy(ev);
    if (h->coop_done) (void)hipEventDestroy(h->coop_done);
    if (h->fork2) (void)hipEventDestroy(h->fork2);
    if (h->h_fault) (void)hipHostFree(h->h_fault);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return SW_OK;
}

void* sw_stream(sw_handle* h) { return h ? reinterpret_cast<void*>(h->stream) : nullptr; }

int sw_opts_init(sw_opts* o) {
    if (!o) return fail(SW_E_INVALID, "null argument");
    *o = default_opts();
    return SW_OK;
}

// The one place the library reads its SW_* variables (tests and A/B scripts
// call it; the scan path reads the handle's sw_opts only).
int sw_opts_from_env(sw_opts* o) {
    int rc;
    if ((rc = sw_opts_init(o))) return rc;
    const struct {
        const char* name;
        int32_t* field;
    } ints[] = {{"SW_LPT", &o->lpt},
                {"SW_LPT_PIPE", &o->lpt_pipe},
                {"SW_QUAD_WIDTH", &o->quad_width},
                {"SW_PAIR_WIDTH", &o->pair_width},
                {"SW_PAIR_GROUP", &o->pair_group},
                {"SW_COOP_WIDTH", &o->coop_width},
                {"SW_COOP_SKEW", &o->coop_skew},
                {"SW_INTRA_X2", &o->intra_x2},
                {"SW_INTRA_X2_RI", &o->intra_x2_rows},
                {"SW_INTRA_I16_FIRST", &o->intra_i16_first},
                {"SW_INTER_I16_SPAN", &o->inter_i16_span},
                {"SW_INT16_GUARD", &o->int16_guard},
                {"SW_RESCUE_STATS", &o->rescue_stats},
                {"SW_TAIL_PAIRS", &o->tail_pairs},
                {"SW_LPT_PERSIST", &o->lpt_persist},
                {"SW_LPT_ROWS", &o->lpt_rows},
                {"SW_TRI_WIDTH", &o->tri_width},
                {"SW_LPT_PIPE_TAIL", &o->lpt_pipe_tail},
                {"SW_DRAIN_SPIN", &o->drain_spin}};
    for (const auto& k : ints)
        if (const char* e = std::getenv(k.name); e && e[0]) *k.field = std::atoi(e);
    if (const char* e = std::getenv("SW_INTER_VARIANT"))
        std::snprintf(o->inter_variant, sizeof o->inter_variant, "%s", e);
    if (const char* e = std::getenv("SW_TRACE_FILE")) std::snprintf(o->trace_file, sizeof o->trace_file, "%s", e);
    return SW_OK;
}

int sw_set_opts(sw_handle* h, const sw_opts* o) {
    if (!h || !o) return fail(SW_E_INVALID, "null argument");
    if (o->size != static_cast<int32_t>(sizeof(sw_opts)))
        return fail(SW_E_INVALID, "sw_opts.size mismatch (initialise with sw_opts_init)");
    if (o->pair_group != -1 && o->pair_group != 2 && o->pair_group != 4)
        return fail(SW_E_INVALID, "sw_opts.pair_group must be -1, 2 or 4");
    h->opts = *o;
    h->opts.inter_variant[sizeof h->opts.inter_variant - 1] = 0;
    h->opts.trace_file[sizeof h->opts.trace_file - 1] = 0;
    return SW_OK;
}

int sw_get_opts(const sw_handle* h, sw_opts* o) {
    if (!h || !o) return fail(SW_E_INVALID, "null argument");
    *o = h->opts;
    return SW_OK;
}

int sw_set_stream(sw_handle* h, void* hip_stream) {
    if (!h) return fail(SW_E_INVALID, "null handle");
    HIPCHECK(hipStreamSynchronize(h->stream));
    if (h->own_stream) HIPCHECK(hipStreamDestroy(h->stream));
    if (hip_stream) {
        h->stream = reinterpret_cast<hipStream_t>(hip_stream);
        h->own_stream = false;
    } else {
        HIPCHECK(hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking));
        h->own_stream = true;
    }
    return SW_OK;
}

int sw_db_create(sw_handle* h, const uint8_t* residues, const int64_t* offsets, int64_t n, const int32_t* ids,
                 sw_db** out) {
    if (!h || !out || n < 0 || (n > 0 && !offsets)) return fail(SW_E_INVALID, "null argument");
    *out = nullptr;
    if (n > 0 && offsets[0] != 0) return fail(SW_E_INVALID, "offsets[0] must be 0");
    for (int64_t k = 0; k < n; ++k)
        if (offsets[k + 1] < offsets[k]) return fail(SW_E_INVALID, "offsets must be non-decreasing");
    const int64_t total = n > 0 ? offsets[n] : 0;
    if (total > 0 && !residues) return fail(SW_E_INVALID, "null residues");
    for (int64_t k = 0; k < n; ++k)
        if (offsets[k + 1] - offsets[k] > (int64_t(1) << 30)) return fail(SW_E_INVALID, "subject too long");
    auto* db = new (std::nothrow) sw_db();
    if (!db) return fail(SW_E_NOMEM, "out of host memory");
    db->h = h;
    db->n = n;
    try {
        db->h_residues.resize(static_cast<size_t>(total));
        db->h_offsets.assign(offsets, offsets + n + 1);
        if (n == 0) db->h_offsets.assign(1, 0);
        db->h_ids.resize(n);
        for (int64_t k = 0; k < n; ++k) db->h_ids[k] = ids ? ids[k] : static_cast<int32_t>(k);
    } catch (...) {
        delete db;
        return fail(SW_E_NOMEM, "out of host memory");
    }
    // copy and validate in parallel 1 MiB pieces
    constexpr int64_t kPiece = int64_t(1) << 20;
    std::atomic<bool> bad{false};
    parallel_for((total + kPiece - 1) / kPiece, [&](int64_t c) {
        const int64_t lo = c * kPiece, hi = std::min(total, lo + kPiece);
        std::memcpy(db->h_residues.data() + lo, residues + lo, static_cast<size_t>(hi - lo));
        uint8_t m = 0;
        for (int64_t k = lo; k < hi; ++k) m = std::max(m, residues[k]);
        if (m >= SW_ALPHABET) bad = true;
    }, 1);
    if (bad) {
        delete db;
        return fail(SW_E_INVALID, "residue code out of range (use sw_encode)");
    }
    db->residues = total;
    for (int64_t k = 0; k < n; ++k) {
        db->max_len = std::max<int32_t>(db->max_len, static_cast<int32_t>(offsets[k + 1] - offsets[k]));
        if (db->h_ids[k] < 0) { delete db; return fail(SW_E_INVALID, "ids must be >= 0"); }
        db->max_id = std::max(db->max_id, db->h_ids[k]);
    }
    db->long_threshold = swplan::default_long_threshold(plan_view(db));
    HIPCHECK(hipSetDevice(h->device));
    int rc = build_db(db);
    if (rc) { free_dev(db); delete db; return rc; }
    *out = db;
    return SW_OK;
}

// ---- binary database file ---------------------------
namespace {
constexpr char kDbMagic[8] = {'S', 'W', 'A', 'M', 'D', 'D', 'B', '1'};
struct DbFileHeader {
    char magic[8];
    int64_t n;         // subjects
    int64_t residues;  // total residue codes
    int32_t max_len;
    int32_t version;   // 1
    uint64_t fnv;      // FNV-1a 64 over offsets, ids and residues
};

uint64_t fnv1a(uint64_t h, const void* p, size_t n) {
    const auto* b = static_cast<const uint8_t*>(p);
    for (size_t k = 0; k < n; ++k) h = (h ^ b[k]) * 1099511628211ull;
    return h;
}
}  // namespace

int sw_db_save(const sw_db* db, const char* path) {
    if (!db || !path) return fail(SW_E_INVALID, "null argument");
    // length-sorted (descending, stable), ids kept: loading gives identical scores[id]
    const int64_t n = db->n;
    const std::vector<int64_t> order = length_order(db->h_offsets, n);
    auto len = [&](int64_t k) { return db->h_offsets[k + 1] - db->h_offsets[k]; };
    std::vector<int64_t> offs(n + 1, 0);
    std::vector<int32_t> ids(n);
    std::vector<uint8_t> res(static_cast<size_t>(db->residues));
    for (int64_t k = 0; k < n; ++k) {
        const int64_t src = order[k];
        subject_residues(db, src, res.data() + offs[k]);
        offs[k + 1] = offs[k] + len(src);
        ids[k] = db->h_ids[src];
    }
    DbFileHeader hd{};
    std::memcpy(hd.magic, kDbMagic, 8);
    hd.n = n;
    hd.residues = db->residues;
    hd.max_len = db->max_len;
    hd.version = 1;
    uint64_t f = 1469598103934665603ull;
    f = fnv1a(f, offs.data(), offs.size() * sizeof(int64_t));
    f = fnv1a(f, ids.data(), ids.size() * sizeof(int32_t));
    hd.fnv = fnv1a(f, res.data(), res.size());
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return fail(SW_E_IO, std::string("cannot open ") + path);
    bool ok = std::fwrite(&hd, sizeof hd, 1, fp) == 1 &&
              std::fwrite(offs.data(), sizeof(int64_t), offs.size(), fp) == offs.size() &&
              (n == 0 || std::fwrite(ids.data(), sizeof(int32_t), ids.size(), fp) == ids.size()) &&
              (res.empty() || std::fwrite(res.data(), 1, res.size(), fp) == res.size());
    ok = (std::fclose(fp) == 0) && ok;
    if (!ok) return fail(SW_E_IO, std::string("write failed: ") + path);
    return SW_OK;
}

int sw_db_load(sw_handle* h, const char* path, sw_db** out) {
    if (!h || !path || !out) return fail(SW_E_INVALID, "null argument");
    *out = nullptr;
    FILE* fp = std::fopen(path, "rb");
    if (!fp) return fail(SW_E_IO, std::string("cannot open ") + path);
    DbFileHeader hd{};
    std::vector<int64_t> offs;
    std::vector<int32_t> ids;
    std::vector<uint8_t> res;
    int rc = SW_OK;
    if (std::fread(&hd, sizeof hd, 1, fp) != 1 || std::memcmp(hd.magic, kDbMagic, 8) != 0 || hd.version != 1 ||
        hd.n < 0 || hd.residues < 0 || hd.n > (int64_t(1) << 40) || hd.residues > (int64_t(1) << 44)) {
        rc = fail(SW_E_IO, std::string("not a database file (sw_db_save format 1): ") + path);
    } else {
        try {
            offs.resize(hd.n + 1);
            ids.resize(hd.n);
            res.resize(static_cast<size_t>(hd.residues));
        } catch (...) {
            rc = fail(SW_E_NOMEM, "out of host memory");
        }
        if (!rc && (std::fread(offs.data(), sizeof(int64_t), offs.size(), fp) != offs.size() ||
                    (hd.n && std::fread(ids.data(), sizeof(int32_t), ids.size(), fp) != ids.size()) ||
                    (hd.residues && std::fread(res.data(), 1, res.size(), fp) != res.size())))
            rc = fail(SW_E_IO, std::string("truncated database file: ") + path);
    }
    std::fclose(fp);
    if (rc) return rc;
    uint64_t f = 1469598103934665603ull;
    f = fnv1a(f, offs.data(), offs.size() * sizeof(int64_t));
    f = fnv1a(f, ids.data(), ids.size() * sizeof(int32_t));
    if (fnv1a(f, res.data(), res.size()) != hd.fnv || offs.back() != hd.residues)
        return fail(SW_E_IO, std::string("database file checksum mismatch: ") + path);
    return sw_db_create(h, res.data(), offs.data(), hd.n, ids.data(), out);
}

int sw_synth_tables(int32_t* len4096, uint8_t* lut65536) {
    const SynthTables& T = synth_tables();
    if (len4096) std::memcpy(len4096, T.len, sizeof T.len);
    if (lut65536) std::memcpy(lut65536, T.lut, sizeof T.lut);
    return SW_OK;
}

int sw_synth_lengths(uint64_t seed, int64_t id_base, int64_t n, int32_t* lengths) {
    if (n < 0 || (n > 0 && !lengths) || id_base < 0) return fail(SW_E_INVALID, "null argument");
    parallel_for(n, [&](int64_t k) { lengths[k] = synth_length(seed, static_cast<uint64_t>(id_base + k)); });
    return SW_OK;
}

int sw_db_create_synthetic(sw_handle* h, uint64_t seed, int64_t id_base, int64_t n, sw_db** out) {
    if (!h || !out || n < 0 || id_base < 0 || n > (int64_t(1) << 31) - 1) return fail(SW_E_INVALID, "bad argument");
    *out = nullptr;
    auto* db = new (std::nothrow) sw_db();
    if (!db) return fail(SW_E_NOMEM, "out of host memory");
    db->h = h;
    db->n = n;
    db->synthetic = true;
    db->seed = seed;
    db->id_base = id_base;
    try {
        std::vector<int32_t> L(n);
        sw_synth_lengths(seed, id_base, n, L.data());
        db->h_offsets.assign(n + 1, 0);
        for (int64_t k = 0; k < n; ++k) db->h_offsets[k + 1] = db->h_offsets[k] + L[k];
        db->h_ids.resize(n);
        for (int64_t k = 0; k < n; ++k) db->h_ids[k] = static_cast<int32_t>(k);
        for (int64_t k = 0; k < n; ++k) db->max_len = std::max(db->max_len, L[k]);
    } catch (...) {
        delete db;
        return fail(SW_E_NOMEM, "out of host memory");
    }
    db->residues = db->h_offsets[n];
    db->max_id = static_cast<int32_t>(n - 1);
    db->long_threshold = swplan::default_long_threshold(plan_view(db));
    HIPCHECK(hipSetDevice(h->device));
    int rc = build_db(db);
    if (rc) { free_dev(db); delete db; return rc; }
    *out = db;
    return SW_OK;
}

int sw_db_subjects(const sw_db* db, int64_t* lengths, int32_t* ids) {
    if (!db) return fail(SW_E_INVALID, "null argument");
    for (int64_t k = 0; k < db->n; ++k) {
        if (lengths) lengths[k] = db->h_offsets[k + 1] - db->h_offsets[k];
        if (ids) ids[k] = db->h_ids[k];
    }
    return SW_OK;
}

int sw_db_free(sw_db* db) {
    if (!db) return SW_OK;
    (void)hipSetDevice(db->h->device);
    (void)hipStreamSynchronize(db->h->stream);
    if (db->h->side) (void)hipStreamSynchronize(db->h->side);
    if (db->h->tail) (void)hipStreamSynchronize(db->h->tail);
    if (db->h_trace) {  // the last scan's block timeline (tail analysis builds)
        if (const char* path = db->h->opts.trace_file; path[0])
            if (FILE* f = std::fopen(path, "wb")) {
                std::fwrite(db->h_trace, 32, db->trace_entries, f);
                std::fclose(f);
            }
    }
    if (db->h_lcount) (void)hipHostFree(db->h_lcount);
    if (db->lcount_ev) (void)hipEventDestroy(db->lcount_ev);
    if (db->h_icount) (void)hipHostFree(db->h_icount);
    if (db->icount_ev) (void)hipEventDestroy(db->icount_ev);
    free_dev(db);
    delete db;
    return SW_OK;
}

int sw_db_reset_adaptive(sw_db* db) {
    if (!db) return fail(SW_E_INVALID, "null argument");
    // a readback still in flight lands in the same pinned words later, in
    // stream order before any readback a later scan issues: ignoring it is safe
    db->lcount_pending = false;
    db->lcount_seen = false;
    db->i16_first.clear();
    db->icount_pending = false;
    db->icount_seen = false;
    db->i16_span.clear();
    return SW_OK;
}

int sw_db_get_stats(const sw_db* db, sw_db_stats* out) {
    if (!db || !out) return fail(SW_E_INVALID, "null argument");
    out->n_subjects = db->n;
    out->residues = db->residues;
    out->packed_cells = db->packed_cells;
    out->n_blocks = db->nblocks;
    out->n_long = db->nlong;
    out->device_bytes = static_cast<int64_t>(db->device_bytes);
    out->max_length = db->max_len;
    out->long_threshold = db->long_threshold;
    out->coop_blocks = db->built ? db->last_ncoop : 0;
    out->coop_residues = 0;
    for (int32_t b = 0; b < out->coop_blocks; ++b) out->coop_residues += db->h_blk_res[b];
    out->pair_blocks = db->built ? db->last_npair : 0;
    out->pair_merged = db->built && db->last_pair_merged ? 1 : 0;
    out->pair_residues = 0;
    for (int32_t b = 0; b < out->pair_blocks; ++b) out->pair_residues += db->h_blk_res[b];
    out->max_id = db->max_id;
    return SW_OK;
}

int sw_db_set_long_threshold(sw_db* db, int32_t threshold) {
    if (!db) return fail(SW_E_INVALID, "null argument");
    if (threshold < 0) return fail(SW_E_INVALID, "threshold must be >= 0");
    const int32_t t = threshold == 0 ? swplan::default_long_threshold(plan_view(db)) : threshold;
    if (t == db->long_threshold && db->built) return SW_OK;
    HIPCHECK(hipSetDevice(db->h->device));
    HIPCHECK(hipStreamSynchronize(db->h->stream));
    if (db->h->side) HIPCHECK(hipStreamSynchronize(db->h->side));
    if (db->h->tail) HIPCHECK(hipStreamSynchronize(db->h->tail));
    free_dev(db);
    db->long_threshold = t;
    return build_db(db);
}

int sw_scan_device(sw_handle* h, const sw_db* db, const uint8_t* query, int32_t qlen, const sw_scoring* sc,
                   int32_t* scores_dev) {
    return scan_impl(h, db, query, qlen, sc, scores_dev);
}

int sw_scan(sw_handle* h, const sw_db* db, const uint8_t* query, int32_t qlen, const sw_scoring* sc,
            int32_t* scores_host) {
    if (!h || !db || !scores_host) return fail(SW_E_INVALID, "null argument");
    const size_t n = static_cast<size_t>(db->max_id + 1);
    if (n == 0) return SW_OK;
    int rc;
    HIPCHECK(hipSetDevice(h->device));
    if ((rc = ensure_scores(h, n))) return rc;
    // slots that no subject maps to read 0
    HIPCHECK(hipMemsetAsync(h->d_scores, 0, n * 4, h->stream));
    if ((rc = scan_impl(h, db, query, qlen, sc, h->d_scores))) return rc;
    HIPCHECK(hipMemcpyAsync(scores_host, h->d_scores, n * 4, hipMemcpyDeviceToHost, h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    return check_fault(h);
}

namespace {
int check_batch(const int64_t* qoffsets, int32_t nq) {
    if (nq > 0 && qoffsets[0] < 0) return fail(SW_E_INVALID, "bad query offsets");
    for (int32_t k = 0; k < nq; ++k) {
        const int64_t ql = qoffsets[k + 1] - qoffsets[k];
        if (ql < 0 || ql > (int64_t(1) << 24)) return fail(SW_E_INVALID, "bad query offsets");
    }
    return SW_OK;
}
}  // namespace

int sw_scan_batch_device(sw_handle* h, const sw_db* db, const uint8_t* queries, const int64_t* qoffsets, int32_t nq,
                         const sw_scoring* sc, int32_t* scores_dev) {
    if (!h || !db || nq < 0 || (nq > 0 && (!qoffsets || !queries || !scores_dev)))
        return fail(SW_E_INVALID, "null argument");
    int rc;
    if ((rc = check_batch(qoffsets, nq))) return rc;
    const size_t n = static_cast<size_t>(db->max_id + 1);
    // back to back on the handle's stream: no host synchronisation between
    // queries (profiles go through the slot ring), so the GPU never idles
    // ... and each query's rescue tail runs beside the next query's passes,
    // when a later non-empty query (a real scan, which joins the tails) follows
    int32_t last_scan = -1;
    for (int32_t k = 0; k < nq; ++k)
        if (qoffsets[k + 1] > qoffsets[k]) last_scan = k;
    for (int32_t k = 0; k < nq; ++k)
        if ((rc = scan_impl(h, db, queries + qoffsets[k], static_cast<int32_t>(qoffsets[k + 1] - qoffsets[k]), sc,
                            scores_dev + k * n, k < last_scan)))
            return rc;
    // every tail has joined the handle's stream by now; join again in case a
    // scan above fell back to stream order after deferring an earlier one
    HIPCHECK(hipSetDevice(h->device));
    return join_tails(h);
}

int sw_scan_batch(sw_handle* h, const sw_db* db, const uint8_t* queries, const int64_t* qoffsets, int32_t nq,
                  const sw_scoring* sc, int32_t* scores_host) {
    if (!h || !db || nq < 0 || (nq > 0 && (!qoffsets || !queries || !scores_host)))
        return fail(SW_E_INVALID, "null argument");
    int rc;
    if ((rc = check_batch(qoffsets, nq))) return rc;
    const size_t n = static_cast<size_t>(db->max_id + 1);
    if (n == 0 || nq == 0) return SW_OK;
    HIPCHECK(hipSetDevice(h->device));
    // chunks of queries whose score rows fit in ~1 GiB of device memory
    const int32_t chunk = static_cast<int32_t>(std::max<size_t>(1, std::min<size_t>(nq, (size_t(1) << 30) / (n * 4))));
    if ((rc = ensure_scores(h, chunk * n))) return rc;
    for (int32_t k0 = 0; k0 < nq; k0 += chunk) {
        const int32_t m = std::min(chunk, nq - k0);
        HIPCHECK(hipMemsetAsync(h->d_scores, 0, m * n * 4, h->stream));  // unmapped slots read 0
        if ((rc = sw_scan_batch_device(h, db, queries, qoffsets + k0, m, sc, h->d_scores))) return rc;
        HIPCHECK(hipMemcpyAsync(scores_host + k0 * n, h->d_scores, m * n * 4, hipMemcpyDeviceToHost, h->stream));
        HIPCHECK(hipStreamSynchronize(h->stream));
        if ((rc = check_fault(h))) return rc;
    }
    return SW_OK;
}

namespace {
int read_events(const ScanEvents& se, sw_timing* t) {
    HIPCHECK(hipEventSynchronize(se.ev[3]));
    // intra runs on the side stream from the fork (ev0) to ev1; inter on the
    // main stream from ev0 to ev2; they overlap.
    // (events a scan did not record: the intra and inter spans fall back to
    // the whole scan, the cooperative kernel's to 0; a scan without a fork,
    // the merged launch, starts at ev6)
    auto has = [&](int k) { return (se.rec >> k & 1u) != 0; };
    const hipEvent_t start = has(0) ? se.ev[0] : se.ev[6];
    float t01 = 0, t02 = 0, t03 = 0;
    HIPCHECK(hipEventElapsedTime(&t03, start, se.ev[3]));
    t01 = t02 = t03;
    if (has(1)) HIPCHECK(hipEventElapsedTime(&t01, start, se.ev[1]));
    if (has(2)) HIPCHECK(hipEventElapsedTime(&t02, start, se.ev[2]));
    float t45 = 0, t67 = 0;
    if (has(4) && has(5)) HIPCHECK(hipEventElapsedTime(&t45, se.ev[4], se.ev[5]));
    // (a merged launch that drains its own rescue lists ends the scan: ev[3])
    if (has(6)) HIPCHECK(hipEventElapsedTime(&t67, se.ev[6], has(7) ? se.ev[7] : se.ev[3]));
    if (se.merged) {  // the merged launch: no separate intra span
        t01 = 0;
        t02 = t67;
    }
    t->intra_ms += t01;
    t->inter_ms += t02;
    t->total_ms += t03;
    t->coop_ms += t45;
    t->wave_ms += t67;
    t->launches += se.launches;
    return SW_OK;
}
}  // namespace

int sw_get_timing(sw_handle* h, sw_timing* out) {
    if (!h || !out) return fail(SW_E_INVALID, "null argument");
    std::memset(out, 0, sizeof(*out));
    if (!h->timed || h->nscans == 0) return SW_OK;
    return read_events(h->evpool[h->nscans - 1], out);
}

int sw_stream_wait_scan(sw_handle* h, void* hip_stream) {
    if (!h) return fail(SW_E_INVALID, "null handle");
    int rc;
    if ((rc = check_fault(h))) return rc;  // (a completed earlier scan's fault)
    if (!h->timed || h->nscans == 0) return SW_OK;  // no scan yet: nothing to wait for
    HIPCHECK(hipSetDevice(h->device));
    HIPCHECK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(hip_stream), h->evpool[h->nscans - 1].ev[3], 0));
    return SW_OK;
}

const char* sw_last_kernel(sw_handle* h) { return h ? h->last_kernel.c_str() : "none"; }
const char* sw_last_intra_kernel(sw_handle* h) { return h ? h->last_intra.c_str() : "none"; }

int sw_timing_reset(sw_handle* h) {
    if (!h) return fail(SW_E_INVALID, "null argument");
    h->nscans = 0;
    h->timed = false;
    return SW_OK;
}

int sw_timing_total(sw_handle* h, sw_timing* out, int32_t* nscans) {
    if (!h || !out || !nscans) return fail(SW_E_INVALID, "null argument");
    std::memset(out, 0, sizeof(*out));
    *nscans = static_cast<int32_t>(h->nscans);
    for (size_t k = 0; k < h->nscans; ++k) {
        int rc = read_events(h->evpool[k], out);
        if (rc) return rc;
    }
    return SW_OK;
}

int sw_topk(const int32_t* scores, int64_t n, int32_t k, int32_t* out_ids, int32_t* out_scores) {
    if ((!scores && n > 0) || k < 0 || (k > 0 && (!out_ids || !out_scores))) return fail(SW_E_INVALID, "null argument");
    const int64_t kk = std::min<int64_t>(k, n);
    std::vector<int32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0);
    auto cmp = [&](int32_t a, int32_t b) { return scores[a] != scores[b] ? scores[a] > scores[b] : a < b; };
    std::partial_sort(idx.begin(), idx.begin() + kk, idx.end(), cmp);
    for (int64_t i = 0; i < kk; ++i) {
        out_ids[i] = idx[i];
        out_scores[i] = scores[idx[i]];
    }
    for (int64_t i = kk; i < k; ++i) {
        out_ids[i] = -1;
        out_scores[i] = 0;
    }
    return SW_OK;
}

int sw_topk_device(sw_handle* h, const int32_t* scores_dev, int64_t n, int64_t id_base, int32_t k,
                   int64_t* keys_out_dev) {
    return topk_impl(h, scores_dev, nullptr, n, id_base, nullptr, k, keys_out_dev);
}

int sw_topk_device_ids(sw_handle* h, const int32_t* scores_dev, int64_t n, const int32_t* ids_dev, int32_t k,
                       int64_t* keys_out_dev) {
    if (n > 0 && !ids_dev) return fail(SW_E_INVALID, "null id map");
    return topk_impl(h, scores_dev, nullptr, n, 0, ids_dev, k, keys_out_dev);
}

int sw_topk_keys_device(sw_handle* h, const int64_t* keys_dev, int64_t n, int32_t k, int64_t* keys_out_dev) {
    return topk_impl(h, nullptr, keys_dev, n, 0, nullptr, k, keys_out_dev);
}

int sw_scan_rank_device(sw_handle* h, const sw_db* cdb, const uint8_t* query, int32_t qlen, const sw_scoring* sc,
                        int32_t* scores_dev, int32_t k, const int32_t* gid_dev, int64_t id_base,
                        int64_t* keys_out_dev) {
    sw_db* db = const_cast<sw_db*>(cdb);
    if (!h || !db || !scores_dev || !keys_out_dev || k <= 0 || k > 4096)
        return fail(SW_E_INVALID, "bad argument (1 <= k <= 4096)");
    if (!gid_dev && (id_base < 0 || id_base + db->max_id >= (int64_t(1) << 31)))
        return fail(SW_E_INVALID, "ids must fit in 31 bits");
    const RankReq rq{k, gid_dev, gid_dev ? 0 : id_base, keys_out_dev};
    return scan_impl(h, db, query, qlen, sc, scores_dev, false, &rq);
}

int sw_scan_topk(sw_handle* h, const sw_db* cdb, const uint8_t* query, int32_t qlen, const sw_scoring* sc, int32_t k,
                 int64_t* keys_host) {
    sw_db* db = const_cast<sw_db*>(cdb);
    if (!h || !db || !keys_host || k <= 0 || k > 4096) return fail(SW_E_INVALID, "bad argument (1 <= k <= 4096)");
    if (db->n == 0) {
        for (int32_t i = 0; i < k; ++i) keys_host[i] = INT64_MIN;
        return SW_OK;
    }
    int rc;
    HIPCHECK(hipSetDevice(h->device));
    const size_t slots = static_cast<size_t>(db->max_id + 1);
    if ((rc = ensure_scores(h, slots + static_cast<size_t>(2 * k) + 2))) return rc;  // scores, then the k keys
    int64_t* keys_dev = reinterpret_cast<int64_t*>(h->d_scores + round_up(static_cast<int64_t>(slots), 2));
    // the ranking runs over the result ids of the subjects (rank_src)
    const RankReq rq{k, nullptr, 0, keys_dev};
    if ((rc = scan_impl(h, db, query, qlen, sc, h->d_scores, false, &rq))) return rc;
    HIPCHECK(hipMemcpyAsync(keys_host, keys_dev, static_cast<size_t>(k) * sizeof(int64_t), hipMemcpyDeviceToHost,
                            h->stream));
    HIPCHECK(hipStreamSynchronize(h->stream));
    return check_fault(h);
}

int sw_align(sw_handle* h, const sw_db* cdb, const uint8_t* query, int32_t qlen, const sw_scoring* sc,
             const int32_t* ids, int32_t n, sw_alignment* out, char* ops, int64_t ops_stride) {
    sw_db* db = const_cast<sw_db*>(cdb);
    if (!h || !db || n < 0 || qlen < 0 || (qlen > 0 && !query) || (n > 0 && (!ids || !out)) ||
        (ops && ops_stride <= 0))
        return fail(SW_E_INVALID, "null argument");
    const int8_t* mat;
    int go, ge, rc;
    if ((rc = check_scoring(sc, &mat, &go, &ge))) return rc;
    for (int32_t i = 0; i < qlen; ++i)
        if (query[i] >= SW_ALPHABET) return fail(SW_E_INVALID, "query residue code out of range (use sw_encode)");
    if (db->id_index.empty())
        for (int64_t k = 0; k < db->n; ++k) db->id_index.emplace(db->h_ids[k], k);
    std::vector<int64_t> sidx(n);
    for (int32_t k = 0; k < n; ++k) {
        auto it = db->id_index.find(ids[k]);
        if (it == db->id_index.end()) return fail(SW_E_INVALID, "sw_align: id not in the database");
        sidx[k] = it->second;
    }
    std::memset(out, 0, sizeof(sw_alignment) * static_cast<size_t>(n));
    if (n == 0 || qlen == 0) return SW_OK;
    HIPCHECK(hipSetDevice(h->device));
    auto slen_of = [&](int64_t k) { return db->h_offsets[k + 1] - db->h_offsets[k]; };
    // groups of hits whose direction arrays fit a 1 GiB budget
    const int64_t W1 = static_cast<int64_t>(qlen) + 1;
    int32_t k0 = 0;
    while (k0 < n) {
        int64_t bytes = 0, res = 0;
        int32_t k1 = k0;
        while (k1 < n) {
            const int64_t b = (qlen + slen_of(sidx[k1]) + 1) * W1;
            if (k1 > k0 && bytes + b > (int64_t(1) << 30)) break;
            bytes += b;
            res += slen_of(sidx[k1]);
            ++k1;
        }
        const int32_t m = k1 - k0;
        std::vector<uint8_t> hsub(static_cast<size_t>(std::max<int64_t>(res, 1)));
        std::vector<int64_t> hoff(m + 1, 0), hdoff(m, 0);
        int64_t dacc = 0;
        for (int32_t k = 0; k < m; ++k) {
            const int64_t src = sidx[k0 + k], L = slen_of(src);
            subject_residues(db, src, hsub.data() + hoff[k]);
            hoff[k + 1] = hoff[k] + L;
            hdoff[k] = dacc;
            dacc += (qlen + L + 1) * W1;
        }
        uint8_t *dq = nullptr, *dsub = nullptr, *ddir = nullptr;
        int64_t *doff = nullptr, *ddoff = nullptr;
        int8_t* dmat = nullptr;
        int32_t *dh = nullptr, *dout = nullptr;
        char* dops = nullptr;
        auto cleanup = [&]() {
            void* ptrs[] = {dq, dsub, ddir, doff, ddoff, dmat, dh, dout, dops};
            for (void* p : ptrs)
                if (p) (void)hipFree(p);
        };
        hipError_t e = hipSuccess;
        auto alloc = [&](auto** p, size_t b) {
            if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(b, 1));
        };
        alloc(&dq, qlen);
        alloc(&dsub, hsub.size());
        alloc(&doff, (m + 1) * sizeof(int64_t));
        alloc(&ddoff, m * sizeof(int64_t));
        alloc(&dmat, 625);
        alloc(&ddir, static_cast<size_t>(dacc));
        // H: three diagonals; affine also two of E and two of F
        alloc(&dh, static_cast<size_t>(m) * (go != ge ? 7 : 3) * W1 * sizeof(int32_t));
        alloc(&dout, static_cast<size_t>(m) * 6 * sizeof(int32_t));
        if (ops) alloc(&dops, static_cast<size_t>(m) * ops_stride);
        if (e == hipSuccess) e = hipMemcpyAsync(dq, query, qlen, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(dsub, hsub.data(), hsub.size(), hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(doff, hoff.data(), (m + 1) * sizeof(int64_t), hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(ddoff, hdoff.data(), m * sizeof(int64_t), hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(dmat, mat, 625, hipMemcpyHostToDevice, h->stream);
        if (e == hipSuccess) {
            swk::AlignArgs a{};
            a.query = dq;
            a.qlen = qlen;
            a.subj = dsub;
            a.subj_off = doff;
            a.n = m;
            a.mat = dmat;
            a.gap = go;
            a.gap_extend = ge;
            a.dirs = ddir;
            a.dirs_off = ddoff;
            a.hbuf = dh;
            a.out = dout;
            a.ops = dops;
            a.ops_stride = ops ? ops_stride : 0;
            e = swk::launch_align(a, h->stream);
        }
        std::vector<int32_t> hout(static_cast<size_t>(m) * 6);
        if (e == hipSuccess)
            e = hipMemcpyAsync(hout.data(), dout, hout.size() * sizeof(int32_t), hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess && ops)
            e = hipMemcpyAsync(ops + static_cast<int64_t>(k0) * ops_stride, dops, static_cast<size_t>(m) * ops_stride,
                               hipMemcpyDeviceToHost, h->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(h->stream);
        cleanup();
        if (e != hipSuccess) return fail(SW_E_HIP, hipGetErrorString(e));
        for (int32_t k = 0; k < m; ++k) {
            sw_alignment& o = out[k0 + k];
            if (slen_of(sidx[k0 + k]) == 0) continue;  // empty subject: all zero (as the oracle)
            o.score = hout[6 * k];
            o.q_begin = hout[6 * k + 1];
            o.q_end = hout[6 * k + 2];
            o.s_begin = hout[6 * k + 3];
            o.s_end = hout[6 * k + 4];
            o.ops_len = hout[6 * k + 5];
        }
        k0 = k1;
    }
    return SW_OK;
}

int sw_score_pair(sw_handle* h, const uint8_t* query, int32_t qlen, const uint8_t* subject, int32_t slen,
                  const sw_scoring* sc, int32_t* score) {
    if (!h || !score || slen < 0 || qlen < 0) return fail(SW_E_INVALID, "null argument");
    const int64_t offs[2] = {0, slen};
    const int32_t id = 0;
    sw_db* db = nullptr;
    int rc = sw_db_create(h, subject, offs, 1, &id, &db);
    if (rc) return rc;
    // a single pair takes the wavefront kernel (all subjects longer than 1)
    if ((rc = sw_db_set_long_threshold(db, 1))) { sw_db_free(db); return rc; }
    rc = sw_scan(h, db, query, qlen, sc, score);
    sw_db_free(db);
    return rc;
}

}  // extern "C"
