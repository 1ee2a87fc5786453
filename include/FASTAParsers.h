/*
 * FASTAParsers.h — the FASTA input contract of the scan path.
 *
 * Same classes, fields and behaviour as the reference's src/FASTAParsers.h
 * (which BASELINE.json's north_star keeps "unchanged"), written for this
 * build:
 *   FASTAQuery(path, isQuery)   first line skipped, the rest concatenated
 *                               verbatim (reference FASTAParsers.h:38-51)
 *   FASTADatabase(path)         '>' starts a record; id = 0-based record
 *                               index; sequences padded with '/' to a multiple
 *                               of TILE_SIZE; bucketed by padded length in
 *                               parsedDB; subjectLengthSum sums PADDED lengths
 *                               (reference FASTAParsers.h:65-138)
 * Edge cases kept: lines before the first '>' are dropped; a file without
 * '>' is one subject with id -1; the last record is always added, so an
 * empty file gives one empty subject with id -1.
 *
 * Like the reference header it exports `using namespace std;` — the
 * reference's main.cpp and swissprot_tests.cpp rely on it.
 */
#ifndef FASTAPARSERS_H
#define FASTAPARSERS_H

#include <fstream>
#include <iostream>
#include <map>
#include <string>
#include <vector>

#ifndef TILE_SIZE
#define TILE_SIZE 8
#endif

using namespace std;

struct subject_sequence {
    int id;
    string sequence;
};

static inline int roundUp(int numToRound, int multiple) {
    if (multiple == 0) return numToRound;
    const int over = numToRound % multiple;
    return over == 0 ? numToRound : numToRound + (multiple - over);
}

class FASTAQuery {
  private:
    bool isQuery;
    string buffer;

  public:
    FASTAQuery(std::string filepath, bool _isQuery) : isQuery(_isQuery) {
        ifstream in(filepath.c_str());
        string line;
        buffer.reserve(10000);
        if (!getline(in, line)) return;  // header line
        while (getline(in, line)) buffer += line;
    }

    ~FASTAQuery() {}

    void print_buffer() { cout << buffer << endl; }

    string get_buffer() { return buffer; }
};

class FASTADatabase {
  public:
    // key: padded sequence length; value: the subjects of that length, in file order
    map<int, vector<subject_sequence> > parsedDB;
    int largestSubjectLength;
    int numSubjects;
    int subjectLengthSum;

    FASTADatabase(std::string filepath) : largestSubjectLength(0), numSubjects(0), subjectLengthSum(0) {
        ifstream in(filepath.c_str());
        string line, current;
        int record = -1;
        bool seen_header = false;
        while (getline(in, line)) {
            if (!line.empty() && line[0] == '>') {
                if (seen_header) finish(record, current);
                seen_header = true;
                current.clear();
                ++record;
            } else {
                current += line;
            }
        }
        finish(record, current);
    }

  private:
    void finish(int id, string& seq) {
        const int len = static_cast<int>(seq.size());
        seq.append(static_cast<size_t>(roundUp(len, TILE_SIZE) - len), '/');
        subject_sequence s;
        s.id = id;
        s.sequence = seq;
        const int padded = static_cast<int>(s.sequence.size());
        parsedDB[padded].push_back(s);
        subjectLengthSum += padded;
        if (padded > largestSubjectLength) largestSubjectLength = padded;
        ++numSubjects;
    }
};

#endif /* FASTAPARSERS_H */
