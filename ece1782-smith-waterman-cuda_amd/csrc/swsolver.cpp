// swsolver.cpp — the reference's C++ solver entry points over the C ABI.
//
//   smith_waterman_cuda       (reference SWSolver.h:9,  SWSolver.cu:266-404)
//   smith_waterman_cuda_char  (reference SWSolver_char.h:9, SWSolver_char.cu:193-280)
//
// One process-wide handle on device $SW_DEVICE (default 0), created on first
// use.  With $SW_GPUS = N > 1 (or sw_solver_set_gpus, `main --gpus N`) the
// database is sharded over devices 0..N-1 (or the list in $SW_DEVICES) by a
// process-wide sw_group (sw_amd.h: residue-balanced shards, one host thread
// per device); the result vector is identical to the one-GPU path.  The
// database is flattened in the order the reference reports results
// (descending padded length, file order within a length: SWSolver.cu:309,
// 384-390), uploaded, scanned and freed per call, like the reference does
// (it re-packs per call too, SWSolver.cu:301-371).  Flattening + encoding
// runs on the host's cores; sw_solver_last_timing() splits the call into
// flatten / device start-up (first call only) / upload (pack + H2D) / scan.
#include <sys/time.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "SWSolver.h"
#include "SWSolver_char.h"
#include "sw_amd.h"
#include "sw_solver_ext.h"

namespace {

std::mutex g_mu;
sw_handle* g_handle = nullptr;
sw_group* g_group = nullptr;
int g_gpus = 0;  // 0: $SW_GPUS or 1
sw_solver_timing g_timing = {};

void check(int rc, const char* what) {
    if (rc != SW_OK) throw std::runtime_error(std::string(what) + ": " + sw_last_error());
}

double now_s() {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return static_cast<double>(tv.tv_usec) / 1000000 + tv.tv_sec;
}

int gpus() {
    if (g_gpus > 0) return g_gpus;
    const char* e = std::getenv("SW_GPUS");
    const int n = e ? std::atoi(e) : 1;
    return n > 0 ? n : 1;
}

sw_handle* handle() {
    if (!g_handle) {
        const char* dev = std::getenv("SW_DEVICE");
        check(sw_create(dev ? std::atoi(dev) : 0, &g_handle), "sw_create");
    }
    return g_handle;
}

// The group over the first gpus() devices ($SW_DEVICES="a,b,..." overrides
// the list, e.g. "0,0" to run the sharded path on a one-GPU machine).
sw_group* group() {
    const int n = gpus();
    if (g_group) return g_group;
    std::vector<int32_t> devs;
    if (const char* e = std::getenv("SW_DEVICES")) {
        std::string s(e);
        size_t at = 0;
        while (at <= s.size() && static_cast<int>(devs.size()) < n) {
            const size_t c = s.find(',', at);
            devs.push_back(std::atoi(s.substr(at, c == std::string::npos ? std::string::npos : c - at).c_str()));
            if (c == std::string::npos) break;
            at = c + 1;
        }
    }
    for (int d = static_cast<int>(devs.size()); d < n; ++d) devs.push_back(d);
    check(sw_group_create(devs.data(), n, &g_group), "sw_group_create");
    return g_group;
}

struct Flat {
    std::vector<uint8_t> residues;
    std::vector<int64_t> offsets{0};
    std::vector<int> record_ids;  // FASTA record id of each flattened subject
};

// Flatten in the reference's reporting order; the encoding (SWSolver.cu:91-
// 120) of the concatenated residues is split over the host's cores.
Flat flatten(FASTADatabase& db) {
    Flat f;
    std::vector<const subject_sequence*> subj;
    subj.reserve(db.numSubjects > 0 ? static_cast<size_t>(db.numSubjects) : 0);
    for (auto it = db.parsedDB.rbegin(); it != db.parsedDB.rend(); ++it)
        for (const subject_sequence& s : it->second) subj.push_back(&s);
    const size_t n = subj.size();
    f.offsets.resize(n + 1);
    f.record_ids.resize(n);
    f.offsets[0] = 0;
    for (size_t k = 0; k < n; ++k) {
        f.offsets[k + 1] = f.offsets[k] + static_cast<int64_t>(subj[k]->sequence.size());
        f.record_ids[k] = subj[k]->id;
    }
    f.residues.resize(static_cast<size_t>(f.offsets[n]));
    uint8_t probe;
    check(sw_encode("A", 1, &probe), "sw_encode");  // the code table exists before the threads start
    unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (n < 4096) nt = 1;
    std::vector<std::thread> th;
    std::vector<int> rc(nt, SW_OK);
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (size_t k = t; k < n; k += nt) {
                const std::string& s = subj[k]->sequence;
                const int r = sw_encode(s.data(), static_cast<int64_t>(s.size()), f.residues.data() + f.offsets[k]);
                if (r) rc[t] = r;
            }
        });
    for (auto& x : th) x.join();
    for (int r : rc) check(r, "sw_encode");
    return f;
}

// Scores of the flattened subjects (index k), reference scoring:
// BLOSUM50 of SWSolver.cu:54-81 with linear gap 2 (SWSolver.cu:7).
// char_compat: the _char path's scoring (SW_MATRIX_BLOSUM50_CHAR, no query
// padding: SWSolver_char.cu:195-198 copies the query as is).
std::vector<int32_t> score_all(FASTAQuery& query, const Flat& f, bool char_compat = false) {
    std::string q = query.get_buffer();
    while (!char_compat && q.size() % TILE_SIZE != 0) q += "/";  // SWSolver.cu:267-269
    std::vector<uint8_t> qc(q.size());
    check(sw_encode(q.data(), static_cast<int64_t>(q.size()), qc.data()), "sw_encode");
    const int64_t n = static_cast<int64_t>(f.record_ids.size());
    std::vector<int32_t> scores(static_cast<size_t>(n), 0);
    g_timing.gpus = gpus();
    if (n == 0) return scores;
    int8_t mat[625];
    if (char_compat) check(sw_builtin_matrix(SW_MATRIX_BLOSUM50_CHAR, mat), "sw_builtin_matrix");
    const sw_scoring sc = {char_compat ? mat : nullptr, 2, 2};
    // device start-up (HIP runtime, handle or group) is timed on its own
    double t0 = now_s();
    sw_handle* h = gpus() == 1 ? handle() : nullptr;
    sw_group* g = gpus() == 1 ? nullptr : group();
    g_timing.init_s = now_s() - t0;
    t0 = now_s();
    if (h) {
        sw_db* db = nullptr;
        check(sw_db_create(h, f.residues.data(), f.offsets.data(), n, nullptr, &db), "sw_db_create");
        g_timing.upload_s = now_s() - t0;
        t0 = now_s();
        const int rc = sw_scan(h, db, qc.data(), static_cast<int32_t>(qc.size()), &sc, scores.data());
        g_timing.scan_s = now_s() - t0;
        sw_db_free(db);
        check(rc, "sw_scan");
    } else {
        sw_gdb* db = nullptr;
        check(sw_group_db_create(g, f.residues.data(), f.offsets.data(), n, nullptr, &db), "sw_group_db_create");
        g_timing.upload_s = now_s() - t0;
        t0 = now_s();
        const int rc = sw_group_scan(g, db, qc.data(), static_cast<int32_t>(qc.size()), &sc, scores.data());
        g_timing.scan_s = now_s() - t0;
        sw_group_db_free(db);
        check(rc, "sw_group_scan");
    }
    return scores;
}

Flat timed_flatten(FASTADatabase& db) {
    g_timing = sw_solver_timing{};
    const double t0 = now_s();
    Flat f = flatten(db);
    g_timing.flatten_s = now_s() - t0;
    return f;
}

}  // namespace

void smith_waterman_cuda(FASTAQuery& query, FASTADatabase& db, std::vector<seqid_score>& result) {
    std::lock_guard<std::mutex> lock(g_mu);  // the reference is not re-entrant either
    const Flat f = timed_flatten(db);
    const std::vector<int32_t> scores = score_all(query, f);
    for (size_t k = 0; k < scores.size(); ++k) result.push_back(std::make_pair(f.record_ids[k], scores[k]));
}

void sw_save_fasta_db(FASTADatabase& fdb, const std::string& path) {
    std::lock_guard<std::mutex> lock(g_mu);
    const Flat f = flatten(fdb);
    const int64_t n = static_cast<int64_t>(f.record_ids.size());
    std::vector<int32_t> ids(f.record_ids.begin(), f.record_ids.end());
    sw_db* db = nullptr;
    check(sw_db_create(handle(), f.residues.data(), f.offsets.data(), n, n ? ids.data() : nullptr, &db),
          "sw_db_create");
    const int rc = sw_db_save(db, path.c_str());
    sw_db_free(db);
    check(rc, "sw_db_save");
}

void sw_solver_set_gpus(int n) {
    std::lock_guard<std::mutex> lock(g_mu);
    if (n != g_gpus && g_group) {
        sw_group_destroy(g_group);
        g_group = nullptr;
    }
    g_gpus = n;
}

sw_group* sw_solver_group() {
    std::lock_guard<std::mutex> lock(g_mu);
    return gpus() > 1 ? group() : nullptr;
}

sw_solver_timing sw_solver_last_timing() { return g_timing; }

// Scores equal smith_waterman_cuda's (golden-pinned), returned in file order;
// SW_CHAR_COMPAT=1 scores with the _char path's own table instead
// (SW_MATRIX_BLOSUM50_CHAR).
std::vector<seqid_score> smith_waterman_cuda_char(FASTAQuery& query, FASTADatabase& db) {
    std::lock_guard<std::mutex> lock(g_mu);
    const Flat f = timed_flatten(db);
    const char* cc = std::getenv("SW_CHAR_COMPAT");
    const std::vector<int32_t> scores = score_all(query, f, cc && cc[0] == '1');
    std::vector<seqid_score> out(scores.size());
    for (size_t k = 0; k < scores.size(); ++k) out[k] = std::make_pair(f.record_ids[k], scores[k]);
    std::stable_sort(out.begin(), out.end(),
                     [](const seqid_score& a, const seqid_score& b) { return a.first < b.first; });
    return out;
}
