// sw_group.cpp — one database searched by several GPUs of one process
// (north_star: "main.cpp scan loop -> HIP-stream batch driver
// + RCCL db shard").  The reference is single-GPU: main.cpp:54-56 calls
// smith_waterman_cuda (SWSolver.cu:266-404) once, on the default device.
//
// Layered on the single-device C ABI (sw_amd.h): a group owns one sw_handle
// per device; a group database deals the subjects to the devices by LPT over
// their lengths (residue-balanced, deterministic: longest first, each to the
// lightest shard, the lowest device index on ties) and keeps one resident
// sw_db per device.  Scans run on every device at once, one host thread per
// device.  The only exchange is the top-K: each device ranks its shard
// (sw_topk_device_ids: keys carry the GLOBAL id, so ties break the same way
// on every device count), one ncclAllGather over RCCL gives every device all
// G x K keys, and device 0 merges them (sw_topk_keys_device).  Full scores
// (sw_group_scan, the reference's result vector) come back per device and are
// scattered by id on the host.
//
// RCCL is loaded at run time (dlopen of librccl.so.1: the one already in the
// process, e.g. PyTorch's, or /opt/rocm's), so the library has no link-time
// RCCL dependency, and only when the first sw_group_topk needs it: creating a
// group and sw_group_scan (the drop-in's full result vector, no collective)
// never touch RCCL.  A group that names one device twice (tests on a one-GPU
// box) cannot form an RCCL communicator, and a process where librccl cannot
// be loaded or ncclCommInitAll fails falls back the same way: the exchange
// goes through the host (same keys, same merge kernel) and sw_group_info says
// which path ran and why.  A group of one device runs the RCCL path with a
// one-rank communicator.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstring>
#include <functional>
#include <queue>
#include <string>
#include <thread>
#include <vector>

#include "sw_amd.h"
#include "sw_kernels.h"

namespace {

int gfail(int code, const std::string& msg) { return swk::set_error(code, msg); }

#define GHIP(expr)                                                                        \
    do {                                                                                  \
        hipError_t e_ = (expr);                                                           \
        if (e_ != hipSuccess) return gfail(SW_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

struct Rccl {
    void* lib = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool load(std::string* why) {
        if (lib) return true;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            lib = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (lib) break;
        }
        if (!lib) {
            *why = std::string("cannot load librccl: ") + dlerror();
            return false;
        }
        init_all = reinterpret_cast<decltype(init_all)>(dlsym(lib, "ncclCommInitAll"));
        destroy = reinterpret_cast<decltype(destroy)>(dlsym(lib, "ncclCommDestroy"));
        all_gather = reinterpret_cast<decltype(all_gather)>(dlsym(lib, "ncclAllGather"));
        group_start = reinterpret_cast<decltype(group_start)>(dlsym(lib, "ncclGroupStart"));
        group_end = reinterpret_cast<decltype(group_end)>(dlsym(lib, "ncclGroupEnd"));
        error_string = reinterpret_cast<decltype(error_string)>(dlsym(lib, "ncclGetErrorString"));
        if (!init_all || !destroy || !all_gather || !group_start || !group_end || !error_string) {
            *why = "librccl lacks an entry point";
            return false;
        }
        return true;
    }
};

Rccl& rccl() {
    static Rccl r;
    return r;
}

// Run f(d) for every device d on its own thread; the first failure's code
// and text are re-raised on the calling thread (sw_last_error is per thread).
int for_each_device(int n, const std::function<int(int)>& f) {
    std::vector<int> rc(n, SW_OK);
    std::vector<std::string> err(n);
    std::vector<std::thread> th;
    for (int d = 0; d < n; ++d)
        th.emplace_back([&, d] {
            rc[d] = f(d);
            if (rc[d] != SW_OK) err[d] = sw_last_error();
        });
    for (auto& t : th) t.join();
    for (int d = 0; d < n; ++d)
        if (rc[d] != SW_OK) return gfail(rc[d], "device " + std::to_string(d) + ": " + err[d]);
    return SW_OK;
}

}  // namespace

struct sw_group {
    std::vector<int32_t> devices;
    std::vector<sw_handle*> h;
    std::vector<ncclComm_t> comms;  // empty: host exchange
    bool distinct = false;          // every device listed once: RCCL possible
    bool comm_tried = false;        // communicators created (or failed) already
    // per device: K local keys, G x K gathered keys, capacity in keys
    std::vector<int64_t*> d_keys, d_all;
    int32_t kcap = 0;
    int64_t* d_final = nullptr;  // merged keys on device 0
    std::string exchange = "none";
};

struct sw_gdb {
    sw_group* g = nullptr;
    std::vector<sw_db*> db;
    std::vector<std::vector<int32_t>> ids;  // per shard: local k -> global result id
    std::vector<int32_t*> d_ids;            // device copies (top-K id maps)
    std::vector<int32_t*> d_scores;         // per device: local scores (device)
    int64_t n = 0;
    int32_t max_id = -1;
};

namespace {

int ensure_keys(sw_group* g, int32_t k) {
    if (k <= g->kcap) return SW_OK;
    const int n = static_cast<int>(g->devices.size());
    for (int d = 0; d < n; ++d) {
        GHIP(hipSetDevice(g->devices[d]));
        if (g->d_keys[d]) GHIP(hipFree(g->d_keys[d]));
        if (g->d_all[d]) GHIP(hipFree(g->d_all[d]));
        GHIP(hipMalloc(reinterpret_cast<void**>(&g->d_keys[d]), sizeof(int64_t) * k));
        GHIP(hipMalloc(reinterpret_cast<void**>(&g->d_all[d]), sizeof(int64_t) * k * n));
    }
    GHIP(hipSetDevice(g->devices[0]));
    if (g->d_final) GHIP(hipFree(g->d_final));
    GHIP(hipMalloc(reinterpret_cast<void**>(&g->d_final), sizeof(int64_t) * k));
    g->kcap = k;
    return SW_OK;
}

// The exchange path, decided at the first top-K: one RCCL communicator per
// device (ncclCommInitAll) when the devices are distinct and RCCL loads and
// initialises, else the host exchange.
void ensure_comms(sw_group* g) {
    if (g->comm_tried) return;
    g->comm_tried = true;
    const int ndev = static_cast<int>(g->devices.size());
    if (!g->distinct) return;
    std::string why;
    if (!rccl().load(&why)) {
        g->exchange = "host (" + why + ")";
        return;
    }
    g->comms.assign(ndev, nullptr);
    const ncclResult_t r = rccl().init_all(g->comms.data(), ndev, g->devices.data());
    if (r != ncclSuccess) {
        g->comms.clear();
        g->exchange = std::string("host (ncclCommInitAll failed: ") + rccl().error_string(r) + ")";
        return;
    }
    g->exchange = "rccl allgather (" + std::to_string(ndev) + (ndev == 1 ? " rank)" : " ranks)");
}

}  // namespace

extern "C" {

int sw_group_create(const int32_t* devices, int32_t ndev, sw_group** out) {
    if (!out || ndev <= 0 || !devices) return gfail(SW_E_INVALID, "null argument / no devices");
    *out = nullptr;
    auto* g = new (std::nothrow) sw_group();
    if (!g) return gfail(SW_E_NOMEM, "out of host memory");
    g->devices.assign(devices, devices + ndev);
    g->h.assign(ndev, nullptr);
    g->d_keys.assign(ndev, nullptr);
    g->d_all.assign(ndev, nullptr);
    for (int d = 0; d < ndev; ++d) {
        const int rc = sw_create(devices[d], &g->h[d]);
        if (rc) {
            const std::string e = sw_last_error();
            sw_group_destroy(g);
            return gfail(rc, e);
        }
    }
    std::vector<int32_t> sorted(g->devices);
    std::sort(sorted.begin(), sorted.end());
    g->distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
    g->exchange = g->distinct ? "rccl allgather (communicators created by the first top-K)"
                              : "host (a device appears twice: no RCCL communicator)";
    *out = g;
    return SW_OK;
}

int sw_group_destroy(sw_group* g) {
    if (!g) return SW_OK;
    for (auto c : g->comms)
        if (c) rccl().destroy(c);
    for (size_t d = 0; d < g->devices.size(); ++d) {
        (void)hipSetDevice(g->devices[d]);
        if (g->d_keys[d]) (void)hipFree(g->d_keys[d]);
        if (g->d_all[d]) (void)hipFree(g->d_all[d]);
        if (d == 0 && g->d_final) (void)hipFree(g->d_final);
        if (g->h[d]) sw_destroy(g->h[d]);
    }
    delete g;
    return SW_OK;
}

const char* sw_group_info(const sw_group* g) { return g ? g->exchange.c_str() : ""; }

int sw_group_handle(sw_group* g, int32_t d, sw_handle** out) {
    if (!g || !out || d < 0 || d >= static_cast<int32_t>(g->h.size())) return gfail(SW_E_INVALID, "bad device slot");
    *out = g->h[d];
    return SW_OK;
}

int sw_group_db_create(sw_group* g, const uint8_t* residues, const int64_t* offsets, int64_t n, const int32_t* ids,
                       sw_gdb** out) {
    if (!g || !out || n < 0 || (n > 0 && !offsets)) return gfail(SW_E_INVALID, "null argument");
    *out = nullptr;
    const int G = static_cast<int>(g->devices.size());
    auto* gd = new (std::nothrow) sw_gdb();
    if (!gd) return gfail(SW_E_NOMEM, "out of host memory");
    gd->g = g;
    gd->n = n;
    gd->db.assign(G, nullptr);
    gd->ids.assign(G, {});
    gd->d_ids.assign(G, nullptr);
    gd->d_scores.assign(G, nullptr);
    // LPT deal: longest first, each to the lightest shard (lowest index on ties)
    std::vector<int64_t> order(n);
    for (int64_t k = 0; k < n; ++k) order[k] = k;
    auto len = [&](int64_t k) { return offsets[k + 1] - offsets[k]; };
    std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) { return len(a) > len(b); });
    std::vector<int> owner(n);
    using Load = std::pair<int64_t, int>;
    std::priority_queue<Load, std::vector<Load>, std::greater<Load>> heap;
    for (int d = 0; d < G; ++d) heap.push({0, d});
    for (int64_t k : order) {
        Load l = heap.top();
        heap.pop();
        owner[k] = l.second;
        l.first += len(k);
        heap.push(l);
    }
    std::vector<std::vector<int64_t>> offs(G, std::vector<int64_t>(1, 0));
    std::vector<std::vector<uint8_t>> res(G);
    for (int64_t k = 0; k < n; ++k) {  // shards keep file (id) order
        const int d = owner[k];
        const int32_t id = ids ? ids[k] : static_cast<int32_t>(k);
        if (id < 0) {
            sw_group_db_free(gd);
            return gfail(SW_E_INVALID, "ids must be >= 0");
        }
        gd->max_id = std::max(gd->max_id, id);
        gd->ids[d].push_back(id);
        res[d].insert(res[d].end(), residues + offsets[k], residues + offsets[k + 1]);
        offs[d].push_back(static_cast<int64_t>(res[d].size()));
    }
    const int rc = for_each_device(G, [&](int d) {
        const int64_t nd = static_cast<int64_t>(gd->ids[d].size());
        int r = sw_db_create(g->h[d], res[d].data(), offs[d].data(), nd, nullptr, &gd->db[d]);
        if (r) return r;
        GHIP(hipSetDevice(g->devices[d]));
        if (nd) {
            GHIP(hipMalloc(reinterpret_cast<void**>(&gd->d_ids[d]), sizeof(int32_t) * nd));
            GHIP(hipMalloc(reinterpret_cast<void**>(&gd->d_scores[d]), sizeof(int32_t) * nd));
            GHIP(hipMemcpy(gd->d_ids[d], gd->ids[d].data(), sizeof(int32_t) * nd, hipMemcpyHostToDevice));
        }
        return SW_OK;
    });
    if (rc) {
        const std::string e = sw_last_error();
        sw_group_db_free(gd);
        return gfail(rc, e);
    }
    *out = gd;
    return SW_OK;
}

int sw_group_db_free(sw_gdb* gd) {
    if (!gd) return SW_OK;
    for (size_t d = 0; d < gd->db.size(); ++d) {
        (void)hipSetDevice(gd->g->devices[d]);
        if (gd->db[d]) sw_db_free(gd->db[d]);
        if (gd->d_ids[d]) (void)hipFree(gd->d_ids[d]);
        if (gd->d_scores[d]) (void)hipFree(gd->d_scores[d]);
    }
    delete gd;
    return SW_OK;
}

int sw_group_db_shard(const sw_gdb* gd, int32_t d, int64_t* n_subjects, int64_t* residues) {
    if (!gd || d < 0 || d >= static_cast<int32_t>(gd->db.size())) return gfail(SW_E_INVALID, "bad shard");
    sw_db_stats st;
    const int rc = sw_db_get_stats(gd->db[d], &st);
    if (rc) return rc;
    if (n_subjects) *n_subjects = st.n_subjects;
    if (residues) *residues = st.residues;
    return SW_OK;
}

int sw_group_scan(sw_group* g, const sw_gdb* gd, const uint8_t* query, int32_t qlen, const sw_scoring* sc,
                  int32_t* scores_host) {
    if (!g || !gd || gd->g != g || (!scores_host && gd->n > 0)) return gfail(SW_E_INVALID, "null argument");
    const int G = static_cast<int>(g->devices.size());
    if (gd->max_id >= 0) std::memset(scores_host, 0, sizeof(int32_t) * (static_cast<size_t>(gd->max_id) + 1));
    return for_each_device(G, [&](int d) {
        const size_t nd = gd->ids[d].size();
        if (!nd) return static_cast<int>(SW_OK);
        std::vector<int32_t> local(nd);
        const int r = sw_scan(g->h[d], gd->db[d], query, qlen, sc, local.data());
        if (r) return r;
        for (size_t k = 0; k < nd; ++k) scores_host[gd->ids[d][k]] = local[k];  // disjoint ids per shard
        return static_cast<int>(SW_OK);
    });
}

int sw_group_topk(sw_group* g, const sw_gdb* gd, const uint8_t* query, int32_t qlen, const sw_scoring* sc,
                  int32_t k, int64_t* keys_host) {
    if (!g || !gd || gd->g != g || !keys_host || k <= 0 || k > 4096)
        return gfail(SW_E_INVALID, "bad top-k arguments (1 <= k <= 4096)");
    const int G = static_cast<int>(g->devices.size());
    int rc = ensure_keys(g, k);
    if (rc) return rc;
    // 1. every device: scan its shard, rank it (global ids), asynchronously
    rc = for_each_device(G, [&](int d) {
        const int64_t nd = static_cast<int64_t>(gd->ids[d].size());
        if (nd)  // the shard's scores ranked with global ids, in the scan's launch when it is merged
            return sw_scan_rank_device(g->h[d], gd->db[d], query, qlen, sc, gd->d_scores[d], k, gd->d_ids[d], 0,
                                       g->d_keys[d]);
        return sw_topk_device_ids(g->h[d], gd->d_scores[d], nd, gd->d_ids[d], k, g->d_keys[d]);
    });
    if (rc) return rc;
    // 2. exchange: every device receives all G x k keys
    ensure_comms(g);
    if (!g->comms.empty()) {
        ncclResult_t r = rccl().group_start();
        for (int d = 0; d < G && r == ncclSuccess; ++d) {
            GHIP(hipSetDevice(g->devices[d]));
            r = rccl().all_gather(g->d_keys[d], g->d_all[d], static_cast<size_t>(k), ncclInt64, g->comms[d],
                                  static_cast<hipStream_t>(sw_stream(g->h[d])));
        }
        const ncclResult_t e = rccl().group_end();
        if (r == ncclSuccess) r = e;
        if (r != ncclSuccess) return gfail(SW_E_HIP, std::string("ncclAllGather: ") + rccl().error_string(r));
    } else {
        std::vector<int64_t> all(static_cast<size_t>(k) * G);
        for (int d = 0; d < G; ++d) {
            GHIP(hipSetDevice(g->devices[d]));
            GHIP(hipStreamSynchronize(static_cast<hipStream_t>(sw_stream(g->h[d]))));
            GHIP(hipMemcpy(all.data() + static_cast<size_t>(k) * d, g->d_keys[d], sizeof(int64_t) * k,
                           hipMemcpyDeviceToHost));
        }
        GHIP(hipSetDevice(g->devices[0]));
        GHIP(hipMemcpy(g->d_all[0], all.data(), sizeof(int64_t) * all.size(), hipMemcpyHostToDevice));
    }
    // 3. device 0 merges (score desc, global id asc) and returns k keys
    if ((rc = sw_topk_keys_device(g->h[0], g->d_all[0], static_cast<int64_t>(k) * G, k, g->d_final))) return rc;
    GHIP(hipSetDevice(g->devices[0]));
    hipStream_t s0 = static_cast<hipStream_t>(sw_stream(g->h[0]));
    GHIP(hipMemcpyAsync(keys_host, g->d_final, sizeof(int64_t) * k, hipMemcpyDeviceToHost, s0));
    GHIP(hipStreamSynchronize(s0));
    return SW_OK;
}

}  // extern "C"
