// swsolver.cpp — the reference's C++ solver entry points over the C ABI.
//
//   smith_waterman_cuda       (reference SWSolver.h:9,  SWSolver.cu:266-404)
//   smith_waterman_cuda_char  (reference SWSolver_char.h:9, SWSolver_char.cu:193-280)
//
// One process-wide handle on device $SW_DEVICE (default 0), created on first
// use.  The database is flattened in the order the reference reports results
// (descending padded length, file order within a length: SWSolver.cu:309,
// 384-390), uploaded, scanned and freed per call, like the reference does
// (it re-packs per call too, SWSolver.cu:301-371).
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#include "SWSolver.h"
#include "SWSolver_char.h"
#include "sw_amd.h"

namespace {

std::mutex g_mu;
sw_handle* g_handle = nullptr;

void check(int rc, const char* what) {
    if (rc != SW_OK) throw std::runtime_error(std::string(what) + ": " + sw_last_error());
}

sw_handle* handle() {
    if (!g_handle) {
        const char* dev = std::getenv("SW_DEVICE");
        check(sw_create(dev ? std::atoi(dev) : 0, &g_handle), "sw_create");
    }
    return g_handle;
}

struct Flat {
    std::vector<uint8_t> residues;
    std::vector<int64_t> offsets{0};
    std::vector<int> record_ids;  // FASTA record id of each flattened subject
};

// Flatten in the reference's reporting order.
Flat flatten(FASTADatabase& db) {
    Flat f;
    f.offsets.reserve(static_cast<size_t>(db.numSubjects) + 1);
    for (auto it = db.parsedDB.rbegin(); it != db.parsedDB.rend(); ++it)
        for (const subject_sequence& s : it->second) {
            const size_t at = f.residues.size();
            f.residues.resize(at + s.sequence.size());
            check(sw_encode(s.sequence.data(), static_cast<int64_t>(s.sequence.size()), f.residues.data() + at),
                  "sw_encode");
            f.offsets.push_back(static_cast<int64_t>(f.residues.size()));
            f.record_ids.push_back(s.id);
        }
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
    if (n == 0) return scores;
    sw_handle* h = handle();
    sw_db* db = nullptr;
    check(sw_db_create(h, f.residues.data(), f.offsets.data(), n, nullptr, &db), "sw_db_create");
    int8_t mat[625];
    if (char_compat) check(sw_builtin_matrix(SW_MATRIX_BLOSUM50_CHAR, mat), "sw_builtin_matrix");
    const sw_scoring sc = {char_compat ? mat : nullptr, 2, 2};
    const int rc = sw_scan(h, db, qc.data(), static_cast<int32_t>(qc.size()), &sc, scores.data());
    sw_db_free(db);
    check(rc, "sw_scan");
    return scores;
}

}  // namespace

void smith_waterman_cuda(FASTAQuery& query, FASTADatabase& db, std::vector<seqid_score>& result) {
    std::lock_guard<std::mutex> lock(g_mu);  // the reference is not re-entrant either
    const Flat f = flatten(db);
    const std::vector<int32_t> scores = score_all(query, f);
    for (size_t k = 0; k < scores.size(); ++k) result.push_back(std::make_pair(f.record_ids[k], scores[k]));
}

// Not part of the reference interface: writes the flattened database (the
// reference's reporting order, record ids as result ids) as a sw_db_save
// file, for `main --make-db`.
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

// Scores equal smith_waterman_cuda's (golden-pinned), returned in file order;
// SW_CHAR_COMPAT=1 scores with the _char path's own table instead
// (SW_MATRIX_BLOSUM50_CHAR).
std::vector<seqid_score> smith_waterman_cuda_char(FASTAQuery& query, FASTADatabase& db) {
    std::lock_guard<std::mutex> lock(g_mu);
    const Flat f = flatten(db);
    const char* cc = std::getenv("SW_CHAR_COMPAT");
    const std::vector<int32_t> scores = score_all(query, f, cc && cc[0] == '1');
    std::vector<seqid_score> out(scores.size());
    for (size_t k = 0; k < scores.size(); ++k) out[k] = std::make_pair(f.record_ids[k], scores[k]);
    std::stable_sort(out.begin(), out.end(),
                     [](const seqid_score& a, const seqid_score& b) { return a.first < b.first; });
    return out;
}
