// main.cpp — the FASTA scan CLI, a drop-in for the reference's bin/main
// (src/main.cpp:19-74) without boost: same flags (--help, --query, --db,
// "--opt value" or "--opt=value"), same output (the query echo, one
// "id:score" line per subject in the solver's order, the METRICS block with
// the reference's GCUPS formula: 1e-9 * |query| * sum(padded subject
// lengths) / wall seconds, wall time from program start, parsing included,
// main.cpp:20,62-72).
//
// Extra, optional: --metrics-json prints one JSON line after the METRICS
// block with the wall-clock split (FASTA parse, flatten + encode, upload =
// pack + H2D, scan); --gpus N shards the database over N GPUs (sw_group:
// residue-balanced shards, one host thread per device; same output).
// Binary databases: --make-db OUT with --db FASTA
// writes OUT (sw_db_save) and exits; --db X.swdb scans such a file with the
// same output (same ids, same order) as the FASTA it came from, without
// parsing FASTA.
// Scoring (the reference hard-wires BLOSUM50 and a linear gap of 2,
// SWSolver.cu:7-8,54-81): --matrix blosum50|blosum62|FILE, --gap-open G,
// --gap-extend E (a k-residue gap costs G + (k-1) E; E defaults to G, i.e.
// linear, G to the reference's 2).  --topk K prints only the K best subjects
// (score descending, record id ascending), ranked on the device.  Without
// these flags the output is the reference's, byte for byte.
#include <sys/time.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "FASTAParsers.h"
#include "SWSolver.h"
#include "sw_amd.h"
#include "sw_solver_ext.h"

namespace {

double now_s() {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return static_cast<double>(tv.tv_usec) / 1000000 + tv.tv_sec;
}

void usage() {
    std::cout << "Smith-Waterman MI355X Usage:\n"
              << "  --help                Display this help message\n"
              << "  --query arg           Path to query file (required)\n"
              << "  --db arg              Path to database file (required; FASTA, or a .swdb file)\n"
              << "  --make-db arg         Write the FASTA --db as a binary .swdb database and exit\n"
              << "  --gpus arg            Shard the FASTA database over this many GPUs (default 1)\n"
              << "  --matrix arg          blosum50 (default, the reference's), blosum62, or a matrix file\n"
              << "  --gap-open arg        Cost of a gap's first residue (default 2)\n"
              << "  --gap-extend arg      Cost of each further gap residue (default: --gap-open, linear)\n"
              << "  --topk arg            Print only the arg best subjects (score desc, id asc)\n";
}

// a whole-string integer in [lo, hi]
bool parse_int(const std::string& s, long lo, long hi, int* out) {
    char* end = nullptr;
    const long v = std::strtol(s.c_str(), &end, 10);
    if (s.empty() || *end != '\0' || v < lo || v > hi) return false;
    *out = static_cast<int>(v);
    return true;
}

}  // namespace

int main(int argc, char* argv[]) {
    const double time_start = now_s();

    std::map<std::string, std::string> opt;
    bool help = false;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        if (a == "--help") { help = true; continue; }
        if (a.rfind("--", 0) != 0) { usage(); return 1; }
        std::string key = a.substr(2), val;
        const size_t eq = key.find('=');
        if (eq != std::string::npos) {
            val = key.substr(eq + 1);
            key = key.substr(0, eq);
        } else if (key != "metrics-json") {
            if (i + 1 >= argc) { usage(); return 1; }
            val = argv[++i];
        }
        if (key != "query" && key != "db" && key != "metrics-json" && key != "make-db" && key != "gpus" &&
            key != "matrix" && key != "gap-open" && key != "gap-extend" && key != "topk") {
            std::cerr << "unrecognised option '--" << key << "'\n";
            return 1;
        }
        opt[key] = val;
    }
    // reference: a missing required option prints the description and exits 1
    // (main.cpp:38-41), --help likewise (main.cpp:33-36)
    if (opt.count("make-db") && opt.count("db") && !help) {
        FASTADatabase fdb(opt["db"]);
        try {
            sw_save_fasta_db(fdb, opt["make-db"]);
        } catch (const std::exception& e) {
            std::cerr << e.what() << "\n";
            return 1;
        }
        cout << "Wrote " << opt["make-db"] << ": " << fdb.numSubjects << " subjects, " << fdb.subjectLengthSum
             << " padded residues." << endl;
        return 0;
    }
    if (!opt.count("query") || !opt.count("db") || help || argc <= 1) {
        usage();
        return 1;
    }
    if (opt.count("gpus")) {
        const int n = std::atoi(opt["gpus"].c_str());
        if (n < 1) { usage(); return 1; }
        sw_solver_set_gpus(n);
    }
    // scoring: the reference's unless a scoring flag is given
    const bool custom = opt.count("matrix") || opt.count("gap-open") || opt.count("gap-extend");
    int8_t mat[625];
    int gap_open = 2, gap_extend = 2, topk = 0;
    if (custom) {
        std::string err;
        if (!sw_solver_read_matrix(opt.count("matrix") ? opt["matrix"] : "blosum50", mat, &err)) {
            std::cerr << "--matrix " << err << "\n";
            return 1;
        }
        if (opt.count("gap-open") && !parse_int(opt["gap-open"], 1, 1000, &gap_open)) {
            std::cerr << "--gap-open must be an integer in 1..1000\n";
            return 1;
        }
        gap_extend = gap_open;
        if (opt.count("gap-extend") && !parse_int(opt["gap-extend"], 1, 1000, &gap_extend)) {
            std::cerr << "--gap-extend must be an integer in 1..1000\n";
            return 1;
        }
        sw_solver_set_scoring(mat, gap_open, gap_extend);
    }
    if (opt.count("topk") && !parse_int(opt["topk"], 1, INT32_MAX, &topk)) {
        std::cerr << "--topk must be a positive integer\n";
        return 1;
    }
    const std::string& dbpath = opt["db"];
    const bool binary = dbpath.size() > 5 && dbpath.compare(dbpath.size() - 5, 5, ".swdb") == 0;

    FASTAQuery query(opt["query"], true);
    cout << "Input buffer:";
    query.print_buffer();
    cout << endl;
    string querySequence = query.get_buffer();

    vector<seqid_score> result;
    result.reserve(600000);
    int64_t num_subjects = 0, length_sum = 0;
    double solve_s = 0, parse_s = 0;
    if (!binary) {
        const double t_parse = now_s();
        FASTADatabase db(dbpath);
        parse_s = now_s() - t_parse;
        const double t_solve = now_s();
        try {
            if (topk) result = smith_waterman_cuda_topk(query, db, topk);
            else smith_waterman_cuda(query, db, result);
        } catch (const std::exception& e) {
            std::cerr << e.what() << "\n";
            return 1;
        }
        solve_s = now_s() - t_solve;
        num_subjects = db.numSubjects;
        length_sum = db.subjectLengthSum;
    } else {
        // the file holds the reference's order and record ids (sw_save_fasta_db)
        auto die = [](const char* what) {
            std::cerr << what << ": " << sw_last_error() << "\n";
            return 1;
        };
        sw_handle* h = nullptr;
        const char* dev = std::getenv("SW_DEVICE");
        if (sw_create(dev ? std::atoi(dev) : 0, &h)) return die("sw_create");
        sw_db* sdb = nullptr;
        if (sw_db_load(h, dbpath.c_str(), &sdb)) return die("sw_db_load");
        sw_db_stats st;
        sw_db_get_stats(sdb, &st);
        std::vector<int64_t> lens(static_cast<size_t>(st.n_subjects));
        std::vector<int32_t> ids(static_cast<size_t>(st.n_subjects));
        sw_db_subjects(sdb, lens.data(), ids.data());
        std::string q = query.get_buffer();
        // the reference pads the query (SWSolver.cu:267-269); its pad rows
        // score 0 only under its own table (see swsolver.cpp encode_query)
        while (!custom && q.size() % 8 != 0) q += "/";
        std::vector<uint8_t> qc(q.size());
        sw_encode(q.data(), static_cast<int64_t>(q.size()), qc.data());
        // BLOSUM50 (SWSolver.cu:54-81), gap 2 (:7), unless chosen
        const sw_scoring sc = {custom ? mat : nullptr, gap_open, gap_extend};
        const double t_solve = now_s();
        if (topk && topk <= 4096) {
            std::vector<int64_t> keys(static_cast<size_t>(topk));
            if (sw_scan_topk(h, sdb, qc.data(), static_cast<int32_t>(qc.size()), &sc, topk, keys.data()))
                return die("sw_scan_topk");
            for (int64_t key : keys) {
                if (key == INT64_MIN) break;
                result.push_back(std::make_pair(static_cast<int>((int64_t{1} << 31) - 1 - (key & 0xffffffff)),
                                                static_cast<int>(key >> 32)));
            }
        } else {
            std::vector<int32_t> scores(static_cast<size_t>(st.max_id + 1), 0);
            if (st.n_subjects && sw_scan(h, sdb, qc.data(), static_cast<int32_t>(qc.size()), &sc, scores.data()))
                return die("sw_scan");
            // the reference's report order: padded length descending, file
            // (= record id) order within a length (SWSolver.cu:309,384-390)
            std::vector<int64_t> order(static_cast<size_t>(st.n_subjects));
            for (int64_t k = 0; k < st.n_subjects; ++k) order[k] = k;
            std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
                const int pa = roundUp(static_cast<int>(lens[a]), TILE_SIZE), pb = roundUp(static_cast<int>(lens[b]), TILE_SIZE);
                return pa != pb ? pa > pb : ids[a] < ids[b];
            });
            for (int64_t k : order) result.push_back(std::make_pair(static_cast<int>(ids[k]), scores[ids[k]]));
            if (topk) {  // beyond the device top-K's 4096: ranked here
                const size_t kk = std::min<size_t>(result.size(), static_cast<size_t>(topk));
                std::partial_sort(result.begin(), result.begin() + kk, result.end(),
                                  [](const seqid_score& a, const seqid_score& b) {
                                      return a.second != b.second ? a.second > b.second : a.first < b.first;
                                  });
                result.resize(kk);
            }
        }
        solve_s = now_s() - t_solve;
        // the FASTA parser's padded sizes (TILE_SIZE, FASTAParsers.h): files
        // hold the subjects as written (older ones '/'-padded: the same sums)
        for (int64_t k = 0; k < st.n_subjects; ++k) length_sum += roundUp(static_cast<int>(lens[k]), TILE_SIZE);
        num_subjects = st.n_subjects;
        sw_db_free(sdb);
        sw_destroy(h);
    }

    for (vector<seqid_score>::iterator it = result.begin(); it != result.end(); ++it)
        cout << (*it).first << ":" << (*it).second << "\n";

    const double seconds_elapsed = now_s() - time_start;
    cout << std::string(80, '=') << endl;
    cout << "METRICS:" << endl;
    cout << "Query length: " << querySequence.length() << " chars." << endl;
    cout << "Num subjects: " << num_subjects << endl;
    cout << "Sum of DB length: " << length_sum << " chars." << endl;
    cout << "Time elapsed: " << seconds_elapsed << " seconds." << endl;
    cout << "Performance: " << 1E-9 * (querySequence.length() * static_cast<double>(length_sum)) / seconds_elapsed
         << " GCUPS." << endl;
    if (opt.count("metrics-json")) {
        const sw_solver_timing t = sw_solver_last_timing();
        cout << "{\"query_len\": " << querySequence.length() << ", \"subjects\": " << num_subjects
             << ", \"padded_residues\": " << length_sum << ", \"wall_s\": " << seconds_elapsed
             << ", \"parse_s\": " << parse_s << ", \"solve_s\": " << solve_s << ", \"flatten_s\": " << t.flatten_s
             << ", \"init_s\": " << t.init_s << ", \"upload_s\": " << t.upload_s << ", \"scan_s\": " << t.scan_s
             << ", \"gpus\": " << t.gpus
             << "}" << endl;
    }
    return 0;
}
