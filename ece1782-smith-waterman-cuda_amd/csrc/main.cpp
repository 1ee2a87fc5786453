// main.cpp — the FASTA scan CLI, a drop-in for the reference's bin/main
// (src/main.cpp:19-74) without boost: same flags (--help, --query, --db,
// "--opt value" or "--opt=value"), same output (the query echo, one
// "id:score" line per subject in the solver's order, the METRICS block with
// the reference's GCUPS formula: 1e-9 * |query| * sum(padded subject
// lengths) / wall seconds, wall time from program start, parsing included,
// main.cpp:20,62-72).
//
// Extra, optional: --metrics-json prints one JSON line after the METRICS
// block with the kernel-only time and algorithmic GCUPS (unpadded cells).
#include <sys/time.h>

#include <cstring>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#include "FASTAParsers.h"
#include "SWSolver.h"

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
              << "  --db arg              Path to database file (required)\n";
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
        if (key != "query" && key != "db" && key != "metrics-json") {
            std::cerr << "unrecognised option '--" << key << "'\n";
            return 1;
        }
        opt[key] = val;
    }
    // reference: a missing required option prints the description and exits 1
    // (main.cpp:38-41), --help likewise (main.cpp:33-36)
    if (!opt.count("query") || !opt.count("db") || help || argc <= 1) {
        usage();
        return 1;
    }

    FASTAQuery query(opt["query"], true);
    cout << "Input buffer:";
    query.print_buffer();
    cout << endl;
    string querySequence = query.get_buffer();

    FASTADatabase db(opt["db"]);

    vector<seqid_score> result;
    result.reserve(600000);
    const double t_solve = now_s();
    smith_waterman_cuda(query, db, result);
    const double solve_s = now_s() - t_solve;

    for (vector<seqid_score>::iterator it = result.begin(); it != result.end(); ++it)
        cout << (*it).first << ":" << (*it).second << "\n";

    const double seconds_elapsed = now_s() - time_start;
    cout << std::string(80, '=') << endl;
    cout << "METRICS:" << endl;
    cout << "Query length: " << querySequence.length() << " chars." << endl;
    cout << "Num subjects: " << db.numSubjects << endl;
    cout << "Sum of DB length: " << db.subjectLengthSum << " chars." << endl;
    cout << "Time elapsed: " << seconds_elapsed << " seconds." << endl;
    cout << "Performance: " << 1E-9 * (querySequence.length() * static_cast<double>(db.subjectLengthSum)) / seconds_elapsed
         << " GCUPS." << endl;
    if (opt.count("metrics-json")) {
        cout << "{\"query_len\": " << querySequence.length() << ", \"subjects\": " << db.numSubjects
             << ", \"padded_residues\": " << db.subjectLengthSum << ", \"wall_s\": " << seconds_elapsed
             << ", \"solve_s\": " << solve_s << "}" << endl;
    }
    return 0;
}
