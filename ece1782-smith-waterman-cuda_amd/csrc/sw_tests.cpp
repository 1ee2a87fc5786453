// sw_tests.cpp — the reference's Boost.Test harness (test/swissprot_tests.cpp)
// restated without boost, over the drop-in C++ interface (SWSolver.h).
//
//   Comparison/<Q>          every (id, score) of smith_waterman_cuda checked
//                           against a golden file keyed by record index
//                           (swissprot_tests.cpp:20-38, 60-75, 89-95)
//   Performance/<Q>         parse + solve wall-clock GCUPS per query, printed
//                           like swissprot_tests.cpp:40-58,98-116
//
// usage: sw_tests --queries DIR --db FASTA --golden-dir DIR [--suite S] [--golden-suffix .txt]
//   Comparison runs for every <Q> with DIR/<Q><suffix> present.
//   In this repo: --db tests/golden/subset111.fasta --golden-dir tests/golden
//   --golden-suffix .subset111.scores (the 111 Swiss-Prot records that ship
//   with the reference); with a full uniprot_sprot.fasta, point --db at it
//   and --golden-dir at the unzipped test/reference files.
#include <sys/time.h>

#include <cstdio>
#include <fstream>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "FASTAParsers.h"
#include "SWSolver.h"
#include "SWSolver_char.h"

namespace {

double stamp() {
    struct timeval tv;
    gettimeofday(&tv, nullptr);
    return static_cast<double>(tv.tv_usec) / 1000000 + tv.tv_sec;
}

std::map<int, int> parse_golden_results(const std::string& path) {
    std::ifstream in(path.c_str());
    std::map<int, int> out;
    std::string line;
    int idx = 0, score = 0;
    while (std::getline(in, line)) {
        std::istringstream(line) >> score;
        out[idx++] = score;
    }
    return out;
}

bool file_exists(const std::string& p) { return std::ifstream(p.c_str()).good(); }

int run_query_against_reference(const std::string& qpath, const std::string& dbpath, const std::string& refpath) {
    FASTAQuery query(qpath, true);
    FASTADatabase db(dbpath);
    std::vector<seqid_score> result;
    result.reserve(600000);
    smith_waterman_cuda(query, db, result);
    std::map<int, int> ref = parse_golden_results(refpath);
    int failures = 0;
    for (const seqid_score& r : result) {
        if (r.second != ref[r.first]) {
            if (failures < 10)
                std::cout << "  " << r.first << ": Ours: " << r.second << " | Theirs: " << ref[r.first] << "\n";
            ++failures;
        }
    }
    // the char entry point must agree too (file order)
    std::vector<seqid_score> chars = smith_waterman_cuda_char(query, db);
    for (const seqid_score& r : chars)
        if (r.second != ref[r.first]) ++failures;
    std::cout << "  Number of subjects scored: " << result.size() << "\n";
    return failures;
}

void run_query_performance(const std::string& qpath, const std::string& dbpath) {
    const double t0 = stamp();
    FASTAQuery query(qpath, true);
    FASTADatabase db(dbpath);
    std::vector<seqid_score> result;
    result.reserve(600000);
    smith_waterman_cuda(query, db, result);
    const double secs = stamp() - t0;
    std::cout << "Query " << qpath << " length " << query.get_buffer().length() << ", Performance: "
              << 1E-9 * (query.get_buffer().length() * static_cast<double>(db.subjectLengthSum)) / secs
              << " GCUPS, Time: " << secs << std::endl;
}

}  // namespace

int main(int argc, char** argv) {
    std::map<std::string, std::string> o;
    for (int i = 1; i + 1 < argc; i += 2) o[std::string(argv[i]).substr(2)] = argv[i + 1];
    const std::string qdir = o.count("queries") ? o["queries"] : "tests/golden/queries";
    const std::string dbp = o.count("db") ? o["db"] : "tests/golden/subset111.fasta";
    const std::string gdir = o.count("golden-dir") ? o["golden-dir"] : "tests/golden";
    const std::string suffix = o.count("golden-suffix") ? o["golden-suffix"] : ".subset111.scores";
    const std::string suite = o.count("suite") ? o["suite"] : "Comparison";

    int failed_cases = 0, cases = 0;
    if (suite == "Comparison" || suite == "all") {
        for (const char* q : {"P01008", "P02232"}) {
            const std::string ref = gdir + "/" + q + suffix;
            if (!file_exists(ref)) continue;
            ++cases;
            std::cout << "Comparison/" << q << "\n";
            const int f = run_query_against_reference(qdir + "/" + q + ".fasta", dbp, ref);
            if (f) { ++failed_cases; std::cout << "  FAILED: " << f << " mismatches\n"; }
            else std::cout << "  ok\n";
        }
    }
    if (suite == "Performance" || suite == "all") {
        // swissprot_tests.cpp:99-115
        for (const char* q : {"P02232", "P05013", "P14942", "P07327", "P01008", "P03435", "P42357", "P21177",
                              "P27895", "P07756", "P04775", "P19096", "P28167", "P0C6B8", "P20930", "P08519",
                              "P33450"}) {
            ++cases;
            run_query_performance(qdir + "/" + q + ".fasta", dbp);
        }
    }
    std::cout << (failed_cases ? "*** " : "") << failed_cases << " failure(s) in " << cases << " test case(s)\n";
    return failed_cases ? 1 : 0;
}
