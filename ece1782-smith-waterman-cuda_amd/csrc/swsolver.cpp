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
//
// Scoring: the reference's (BLOSUM50 of SWSolver.cu:54-81, linear gap 2 of
// SWSolver.cu:7) unless sw_solver_set_scoring chose another matrix / gap
// model (`main --matrix --gap-open --gap-extend`); smith_waterman_cuda_topk
// returns only the k best subjects, ranked on the device (`main --topk`).
#include <sys/time.h>

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <sstream>
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
// the scoring of smith_waterman_cuda[_topk]; custom = false: the reference's
struct SolverScoring {
    bool custom = false;
    bool has_matrix = false;
    int8_t mat[625] = {};
    int go = 2, ge = 2;
} g_sc;

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
// strip_pad: without the parser's '/' padding (FASTAParsers.h pads every
// subject to a multiple of TILE_SIZE; '/' encodes as '*'): the subjects as
// written.  Under the reference's BLOSUM50 the pad scores 0 and changes no
// score, so it is kept there; other scorings (BLOSUM62: '*' +1 against '*')
// and the binary database files get the subjects as written.
Flat flatten(FASTADatabase& db, bool strip_pad = false) {
    Flat f;
    std::vector<const subject_sequence*> subj;
    subj.reserve(db.numSubjects > 0 ? static_cast<size_t>(db.numSubjects) : 0);
    for (auto it = db.parsedDB.rbegin(); it != db.parsedDB.rend(); ++it)
        for (const subject_sequence& s : it->second) subj.push_back(&s);
    const size_t n = subj.size();
    f.offsets.resize(n + 1);
    f.record_ids.resize(n);
    f.offsets[0] = 0;
    auto len_of = [&](size_t k) {
        const std::string& s = subj[k]->sequence;
        size_t m = s.size();
        while (strip_pad && m > 0 && s[m - 1] == '/') --m;
        return m;
    };
    for (size_t k = 0; k < n; ++k) {
        f.offsets[k + 1] = f.offsets[k] + static_cast<int64_t>(len_of(k));
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
                const int r = sw_encode(s.data(), f.offsets[k + 1] - f.offsets[k], f.residues.data() + f.offsets[k]);
                if (r) rc[t] = r;
            }
        });
    for (auto& x : th) x.join();
    for (int r : rc) check(r, "sw_encode");
    return f;
}

// The encoded query.  The reference pads it with '/' to a multiple of
// TILE_SIZE (SWSolver.cu:267-269); '/' encodes as '*', whose BLOSUM50 row is
// all zero, so under the reference's scoring the padding cannot change a
// score and is kept for the literal drop-in.  Other scorings (BLOSUM62 scores
// '*' -4 / +1) get the query as written, and so does the _char path
// (SWSolver_char.cu:195-198 copies it as is).
std::vector<uint8_t> encode_query(FASTAQuery& query, bool pad) {
    std::string q = query.get_buffer();
    while (pad && q.size() % TILE_SIZE != 0) q += "/";
    std::vector<uint8_t> qc(q.size());
    check(sw_encode(q.data(), static_cast<int64_t>(q.size()), qc.data()), "sw_encode");
    return qc;
}

// Scores of the flattened subjects (index k), under g_sc (by default the
// reference's: BLOSUM50 of SWSolver.cu:54-81 with linear gap 2, SWSolver.cu:7).
// char_compat: the _char path's scoring (SW_MATRIX_BLOSUM50_CHAR, no query
// padding).
std::vector<int32_t> score_all(FASTAQuery& query, const Flat& f, bool char_compat = false) {
    const std::vector<uint8_t> qc = encode_query(query, !char_compat && !g_sc.custom);
    const int64_t n = static_cast<int64_t>(f.record_ids.size());
    std::vector<int32_t> scores(static_cast<size_t>(n), 0);
    g_timing.gpus = gpus();
    if (n == 0) return scores;
    int8_t mat[625];
    if (char_compat) check(sw_builtin_matrix(SW_MATRIX_BLOSUM50_CHAR, mat), "sw_builtin_matrix");
    const sw_scoring sc = char_compat ? sw_scoring{mat, 2, 2}
                                      : sw_scoring{g_sc.has_matrix ? g_sc.mat : nullptr, g_sc.go, g_sc.ge};
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

Flat timed_flatten(FASTADatabase& db, bool strip_pad) {
    g_timing = sw_solver_timing{};
    const double t0 = now_s();
    Flat f = flatten(db, strip_pad);
    g_timing.flatten_s = now_s() - t0;
    return f;
}

// One matrix entry of a text matrix file.
bool parse_int(const std::string& tok, int* v) {
    char* end = nullptr;
    const long x = std::strtol(tok.c_str(), &end, 10);
    if (tok.empty() || *end != '\0' || x < -100 || x > 100) return false;
    *v = static_cast<int>(x);
    return true;
}

}  // namespace

bool sw_solver_read_matrix(const std::string& spec, int8_t out[625], std::string* err) {
    std::string low(spec);
    for (char& c : low) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
    if (low == "blosum50") return sw_builtin_matrix(SW_MATRIX_BLOSUM50_REF, out) == SW_OK;
    if (low == "blosum62") return sw_builtin_matrix(SW_MATRIX_BLOSUM62, out) == SW_OK;
    auto bad = [&](const std::string& why) {
        if (err) *err = spec + ": " + why;
        return false;
    };
    std::ifstream in(spec.c_str());
    if (!in) return bad("cannot open matrix file (or use blosum50 / blosum62)");
    static const char kLetters[] = "ARNDCQEGHILKMFPSTWYVBJZX*";  // code order (SWSolver.cu:17-41)
    auto code_of = [&](const std::string& t) -> int {
        if (t.size() != 1) return -1;
        const char* p = std::strchr(kLetters, std::toupper(static_cast<unsigned char>(t[0])));
        return p && *p ? static_cast<int>(p - kLetters) : -1;
    };
    std::vector<std::vector<std::string>> rows;
    std::string line;
    while (std::getline(in, line)) {
        const size_t h = line.find('#');
        if (h != std::string::npos) line.erase(h);
        std::istringstream ls(line);
        std::vector<std::string> tok;
        for (std::string t; ls >> t;) tok.push_back(t);
        if (!tok.empty()) rows.push_back(tok);
    }
    if (rows.empty()) return bad("empty matrix file");
    int v = 0;
    if (parse_int(rows[0][0], &v)) {  // 25 rows of 25 numbers in code order
        if (rows.size() != 25) return bad("expected 25 rows of 25 numbers (code order ARNDCQEGHILKMFPSTWYVBJZX*)");
        for (int a = 0; a < 25; ++a) {
            if (rows[a].size() != 25) return bad("expected 25 numbers in row " + std::to_string(a + 1));
            for (int b = 0; b < 25; ++b) {
                if (!parse_int(rows[a][b], &v)) return bad("bad entry '" + rows[a][b] + "' (integers in -100..100)");
                out[a * 25 + b] = static_cast<int8_t>(v);
            }
        }
        return true;
    }
    // NCBI layout: a header row of residue letters, then one row per letter
    std::vector<int> col;
    for (const std::string& t : rows[0]) {
        const int c = code_of(t);
        if (c < 0) return bad("unknown residue letter '" + t + "' in the header row");
        col.push_back(c);
    }
    int16_t m[25][25];
    bool have[25] = {};
    for (size_t r = 1; r < rows.size(); ++r) {
        const int a = code_of(rows[r][0]);
        if (a < 0) return bad("unknown residue letter '" + rows[r][0] + "'");
        if (rows[r].size() != col.size() + 1) return bad("row '" + rows[r][0] + "' does not match the header");
        if (have[a]) return bad("row '" + rows[r][0] + "' given twice");
        for (size_t j = 0; j < col.size(); ++j) {
            if (!parse_int(rows[r][j + 1], &v)) return bad("bad entry '" + rows[r][j + 1] + "' (integers in -100..100)");
            m[a][col[j]] = static_cast<int16_t>(v);
        }
        have[a] = true;
    }
    bool in_cols[25] = {};
    for (int c : col) in_cols[c] = true;
    for (int a = 0; a < 25; ++a)
        if (have[a] != in_cols[a]) return bad(std::string("letter '") + kLetters[a] + "' is a row or a column, not both");
    // letters the file leaves out (e.g. J in NCBI BLOSUM62) score as X
    constexpr int X = 23;
    for (int a = 0; a < 25; ++a)
        if (!have[a] && !have[X]) return bad(std::string("no row for '") + kLetters[a] + "' and no X row to stand in");
    for (int a = 0; a < 25; ++a)
        for (int b = 0; b < 25; ++b) out[a * 25 + b] = static_cast<int8_t>(m[have[a] ? a : X][have[b] ? b : X]);
    return true;
}

void sw_solver_set_scoring(const int8_t* matrix625, int gap_open, int gap_extend) {
    if (gap_open < 1 || gap_open > 1000 || gap_extend < 1 || gap_extend > 1000)
        throw std::invalid_argument("gap penalties must be in 1..1000");
    if (matrix625)
        for (int k = 0; k < 625; ++k)
            if (matrix625[k] < -100 || matrix625[k] > 100)
                throw std::invalid_argument("matrix entries must be in -100..100");
    std::lock_guard<std::mutex> lock(g_mu);
    g_sc = SolverScoring{};
    g_sc.custom = true;
    g_sc.has_matrix = matrix625 != nullptr;
    if (matrix625) std::memcpy(g_sc.mat, matrix625, 625);
    g_sc.go = gap_open;
    g_sc.ge = gap_extend;
}

void sw_solver_reset_scoring() {
    std::lock_guard<std::mutex> lock(g_mu);
    g_sc = SolverScoring{};
}

std::vector<seqid_score> smith_waterman_cuda_topk(FASTAQuery& query, FASTADatabase& db, int k) {
    if (k < 1) throw std::invalid_argument("top-k needs k >= 1");
    std::lock_guard<std::mutex> lock(g_mu);
    const Flat f = timed_flatten(db, g_sc.custom);
    const int64_t n = static_cast<int64_t>(f.record_ids.size());
    std::vector<seqid_score> out;
    bool ids_ok = n > 0;
    for (int id : f.record_ids) ids_ok = ids_ok && id >= 0;
    if (k > 4096 || !ids_ok) {
        // beyond the device top-K's k (or a headerless file's id -1): every
        // score to the host, ranked there (score desc, id asc)
        const std::vector<int32_t> scores = score_all(query, f);
        for (int64_t i = 0; i < n; ++i) out.push_back(std::make_pair(f.record_ids[i], scores[i]));
        const size_t kk = std::min<size_t>(out.size(), static_cast<size_t>(k));
        std::partial_sort(out.begin(), out.begin() + kk, out.end(), [](const seqid_score& a, const seqid_score& b) {
            return a.second != b.second ? a.second > b.second : a.first < b.first;
        });
        out.resize(kk);
        return out;
    }
    const std::vector<uint8_t> qc = encode_query(query, !g_sc.custom);
    const sw_scoring sc = {g_sc.has_matrix ? g_sc.mat : nullptr, g_sc.go, g_sc.ge};
    std::vector<int32_t> ids(f.record_ids.begin(), f.record_ids.end());
    std::vector<int64_t> keys(static_cast<size_t>(k));
    g_timing.gpus = gpus();
    double t0 = now_s();
    sw_handle* h = gpus() == 1 ? handle() : nullptr;
    sw_group* g = gpus() == 1 ? nullptr : group();
    g_timing.init_s = now_s() - t0;
    t0 = now_s();
    const int32_t ql = static_cast<int32_t>(qc.size());
    if (h) {
        sw_db* sdb = nullptr;
        check(sw_db_create(h, f.residues.data(), f.offsets.data(), n, ids.data(), &sdb), "sw_db_create");
        g_timing.upload_s = now_s() - t0;
        t0 = now_s();
        const int rc = sw_scan_topk(h, sdb, qc.data(), ql, &sc, k, keys.data());
        g_timing.scan_s = now_s() - t0;
        sw_db_free(sdb);
        check(rc, "sw_scan_topk");
    } else {
        sw_gdb* gdb = nullptr;
        check(sw_group_db_create(g, f.residues.data(), f.offsets.data(), n, ids.data(), &gdb), "sw_group_db_create");
        g_timing.upload_s = now_s() - t0;
        t0 = now_s();
        const int rc = sw_group_topk(g, gdb, qc.data(), ql, &sc, k, keys.data());
        g_timing.scan_s = now_s() - t0;
        sw_group_db_free(gdb);
        check(rc, "sw_group_topk");
    }
    for (int64_t key : keys) {
        if (key == INT64_MIN) break;  // fewer subjects than k
        out.push_back(std::make_pair(static_cast<int>((int64_t{1} << 31) - 1 - (key & 0xffffffff)),
                                     static_cast<int>(key >> 32)));
    }
    return out;
}

void smith_waterman_cuda(FASTAQuery& query, FASTADatabase& db, std::vector<seqid_score>& result) {
    std::lock_guard<std::mutex> lock(g_mu);  // the reference is not re-entrant either
    const Flat f = timed_flatten(db, g_sc.custom);
    const std::vector<int32_t> scores = score_all(query, f);
    for (size_t k = 0; k < scores.size(); ++k) result.push_back(std::make_pair(f.record_ids[k], scores[k]));
}

void sw_save_fasta_db(FASTADatabase& fdb, const std::string& path) {
    std::lock_guard<std::mutex> lock(g_mu);
    const Flat f = flatten(fdb, true);  // as written; main's METRICS restore the padded sizes
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
    const Flat f = timed_flatten(db, false);
    const char* cc = std::getenv("SW_CHAR_COMPAT");
    const std::vector<int32_t> scores = score_all(query, f, cc && cc[0] == '1');
    std::vector<seqid_score> out(scores.size());
    for (size_t k = 0; k < scores.size(); ++k) out[k] = std::make_pair(f.record_ids[k], scores[k]);
    std::stable_sort(out.begin(), out.end(),
                     [](const seqid_score& a, const seqid_score& b) { return a.first < b.first; });
    return out;
}
