// bt2g_client.cpp -- the alignment server's client, many connections per process.
//
// Row (f)-4 of SURVEY.md section 8: the wire side of the north-star path.  The
// reference's client (bowtie2-align-l, PatternSourceWebClient, pat.cpp:2219-2789
// and bt2_search.cpp:4555-4617, 4958-5019) is one connection per process with
// a reader thread, a sender thread and a receiver thread per connection and
// three heap objects per read.  This client speaks the same protocol with the
// same bytes on the wire and the same SAM out, but drives many connections from
// a few threads (one epoll loop per thread), parses FASTQ straight from memory
// and keeps each connection's reads in one arena:
//
//   * FASTQ: the light parser of FastqPatternSource::nextBatchFromFile
//     (pat.cpp:1066-1142: records of four newlines, blank lines skipped, a
//     partial record ends at a line starting with '@') and its parse()
//     (pat.cpp:1147-1258: name up to the line end, sequence letters through
//     asc2dna, alphabet.cpp:142-160, '.' as N, --trim5/--trim3, Phred+33 or +64
//     qualities, qual.h:105-146, the reference's error messages);
//   * TAB6 out (readPair2Tab6, pat.cpp:2341-2374): "XXXX/1\tSEQ\tQUAL[\tXXXX/2
//     \tSEQ\tQUAL]\n", XXXX the read's slot in the two 10 000-entry name maps
//     of LockedOrigBufMap (pat.h:2464-2550): slots handed out in read order from
//     map 0, then map 1, a map reused from slot 0 once every read in it ended;
//     lines go out in HTTP chunks of at most 40 lines (RE_PER_PACKET,
//     pat.h:2451; write_chunked_str, pat.h:2686-2695), then the 0-size chunk and
//     shutdown(SHUT_WR) (pat.cpp:2488-2568);
//   * the handshake (pat.cpp:2395-2436): PUT /BT2SRV/<index>/align with
//     X-BT2SRV-Request-Terminator, "HTTP/1.1 200 OK" and X-BT2SRV-Terminator
//     required in the answer;
//   * SAM in (process_read_buffer / process_read_line / process_end_read,
//     pat.cpp:2570-2754): the 4-hex slot id of every record replaced by the
//     saved read name (its trailing "/1" dropped, OrigBuf::saveOrigBufs,
//     pat.cpp:2286-2336), other '@' lines passed through, "@CO END READ\t<id>"
//     frees the slot, "@CO BT2SRV All Done" ends the connection; --passthrough appends
//     the read's original FASTQ record, %-escaped (copyOptFieldNewlineEscaped,
//     pat.cpp:2258-2284).
//
// Other inputs (round 6), as the reference client's PatternSource family
// (pat.h:878-1232) parses them before readPair2Tab6:
//
//   * -f FASTA: FastaPatternSource (pat.cpp:790-912): a record is '>' and every
//     byte up to the next '>', the name its first line, the sequence every
//     letter ('.' as N) after it except the record's last byte, qualities 'I';
//   * --tab5 / --12 / --tab6 (files of one read or pair per line):
//     TabbedPatternSource (pat.cpp:1524-1661, tabbed_parse): NAME\tSEQ\tQUAL,
//     then \tSEQ\tQUAL (tab5, the mate named as the first) or \tNAME\tSEQ\tQUAL
//     (tab6) for a pair -- unpaired and paired lines may mix in one file;
//   * -r raw (RawPatternSource, pat.cpp:1743-1817): one sequence a line, named
//     by its read number, qualities 'I';
//   * -c: the -U / -1 / -2 arguments are the reads themselves, SEQ[:QUALS]
//     comma-separated (VectorPatternSource, pat.cpp:614-700: named by their
//     index, parsed as tab5 lines).
// A read that does not parse is skipped, its read number spent (the client
// loop of bt2_search.cpp:4578-4586).
//
// Per connection the SAM bytes are those of the reference client given the
// same reads (tests/test_client.py diffs the two on the same server).  What
// differs is packaging: the reference prints "Read name does not end in /1!"
// once per read, this client once per connection with a count.
//
// Usage:
//   bt2g-client -x <index> (-U f[,f...] | -1 f1 -2 f2) [-k K] [-R N] [-p T]
//               [-S out.sam] [--server-host H] [--server-port P] [--passthrough]
//               [-3 n] [-5 n] [--phred33|--phred64] [--no-hd] [-q]
//   bt2g-client -x <index> --chunks LIST [-k K] [-p T] [--out-dir D | -S out]
// -k: connections open at once (default 1); -R: reads (pairs) per connection
// (default: all, one connection, as the reference client); --chunks: one
// connection per line of LIST ("U f[,f...]" or "P f1 f2"), the way bench.py
// ran one reference client per chunk file; --out-dir: the SAM of chunk i in
// D/chunkNNNNN.sam, else all of it on -S / stdout in chunk order (with
// --mark-chunks each chunk after a line "@CO BT2G-CLIENT CHUNK <i>").  Host and
// port also from $BT2CLT_SERVER_HOST / $BT2CLT_SERVER_PORT, as the reference.
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <zlib.h>

#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------- options

struct Opts {
    std::string index, host = "localhost", out, out_dir, chunks;
    int port = 0, conns = 1, threads = 0, trim5 = 0, trim3 = 0;
    long long per_conn = 0;                 // 0: every read over one connection
    long long skip = 0, upto = -1;          // -s / -u: reads [skip, upto) of the input (rdid)
    bool phred64 = false, xr = false, stats = false, mark = false, count = false;
    enum Fmt { FASTQ, FASTA, TAB5, TAB6, RAW, CMDLINE } fmt = FASTQ;
    std::vector<std::string> U, m1, m2;
};

struct Fail : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// asc2dna (alphabet.cpp:142-160): A/a 0, C/c 1, G/g 2, T/t 3, every other byte 4
inline char dna_char(unsigned char c) {
    switch (c) {
        case 'A': case 'a': return 'A';
        case 'C': case 'c': return 'C';
        case 'G': case 'g': return 'G';
        case 'T': case 't': return 'T';
        default: return 'N';
    }
}

// ---------------------------------------------------------------- reads

struct Rec {                 // one mate, offsets into Input::arena
    uint32_t name, name_len;   // the name to restore, "/1" dropped
    uint32_t tab, tab_len;     // "\tSEQ\tQUAL"
    uint32_t orig, orig_len;   // %-escaped FASTQ record (--passthrough only)
};

struct Input {
    std::string arena;        // names and TAB6 fields; the first `used` bytes are taken
    size_t used = 0;
    std::vector<Rec> a, b;    // b empty: unpaired; else b[i].tab_len == 0 for an unpaired read i (tabbed input)
    long long bad_names = 0;  // names of mate 1 without "/1" (pat.cpp:2289-2291)
    bool paired() const { return !b.empty(); }
    bool pair(size_t i) const { return !b.empty() && b[i].tab_len != 0; }
};

std::string slurp(const std::string& path) {
    std::string s;
    {   // plain files straight in; gzip (1f 8b) through zlib, as the reference's reader
        int fd = open(path.c_str(), O_RDONLY);
        if (fd < 0) throw Fail("Error: could not open " + path);
        struct stat st;
        unsigned char mg[2] = {0, 0};
        bool gz = pread(fd, mg, 2, 0) == 2 && mg[0] == 0x1f && mg[1] == 0x8b;
        if (!gz && fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
            s.resize((size_t)st.st_size);
            size_t n = 0;
            while (n < s.size()) {
                ssize_t k = read(fd, &s[n], s.size() - n);
                if (k <= 0) break;
                n += (size_t)k;
            }
            close(fd);
            s.resize(n);
            return s;
        }
        close(fd);
    }
    gzFile f = gzopen(path.c_str(), "rb");
    if (!f) throw Fail("Error: could not open " + path);
    gzbuffer(f, 1 << 20);
    size_t n = 0;
    s.resize(1 << 22);
    for (;;) {
        if (s.size() - n < (1 << 20)) s.resize(s.size() * 2);
        int got = gzread(f, &s[n], (unsigned)(s.size() - n));
        if (got < 0) {
            gzclose(f);
            throw Fail("Error: could not read " + path);
        }
        if (got == 0) break;
        n += (size_t)got;
    }
    gzclose(f);
    s.resize(n);
    return s;
}

// FastqPatternSource::nextBatchFromFile over a whole file held in memory:
// record i's bytes (as the light parser appends them) go to `recs`.
struct RecSpan { size_t off, len; };

void light_parse(const std::string& s, std::string& scratch, std::vector<RecSpan>& out) {
    const char* p = s.data();
    const size_t n = s.size();
    size_t i = 0;
    while (i < n && (p[i] == '\r' || p[i] == '\n')) i++;
    if (i == n) return;
    if (p[i] != '@') throw Fail("Error: reads file does not look like a FASTQ file");
    bool first = true;
    for (;;) {
        // record start: blank lines skipped (buf.length() == 0)
        if (!first) {
            while (i < n && (p[i] == '\r' || p[i] == '\n')) i++;
            if (i >= n) return;                         // EOF: nothing appended, record not counted
        }
        first = false;
        const size_t start = i;
        bool contiguous = true;
        size_t sc0 = scratch.size();
        int newlines = 4;
        bool eof = false;
        while (newlines) {
            const char* nl = (const char*)memchr(p + i, '\n', n - i);
            size_t end = nl ? (size_t)(nl - p) : n;
            if (!contiguous) scratch.append(p + i, end - i);
            if (!nl) {                                   // EOF inside a line
                if (newlines == 1) newlines = 0;         // read as the final newline, not appended
                i = n;
                eof = true;
                break;
            }
            if (!contiguous) scratch.push_back('\n');
            i = end + 1;
            newlines--;
            if (!newlines) break;
            size_t j = i;                                // after a newline: \r and \n skipped
            while (j < n && (p[j] == '\r' || p[j] == '\n')) j++;
            if (j != i && contiguous) {                  // bytes dropped: copy from here on
                scratch.append(p + start, i - start);
                contiguous = false;
            }
            i = j;
            if (i >= n) {
                if (newlines == 1) newlines = 0;
                eof = true;
                break;
            }
            if (p[i] == '@' && newlines > 1 && newlines < 4) break;   // partial record
        }
        if (newlines < 4) {
            if (contiguous) out.push_back({start, i - start});
            else out.push_back({(size_t)1 << 62 | sc0, scratch.size() - sc0});
        }
        if (eof || i >= n) return;
    }
}

// sequence bytes (pat.cpp:1174-1186): letters through asc2dna printed back
// ("ACGTN"[code]), '.' as N, every other byte skipped
struct SeqTable {
    char t[256];
    SeqTable() {
        for (int c = 0; c < 256; c++) t[c] = isalpha(c) ? dna_char((unsigned char)c) : 0;
        t[(unsigned char)'.'] = 'N';
    }
};
const SeqTable kSeq;

// FastqPatternSource::parse (pat.cpp:1147-1258) of one record; appends the
// name and the TAB6 fields to in.arena (in.used bytes of it are taken).
void parse_rec(const char* r, size_t len, long long rdid, const Opts& o, Input& in, Rec& rec, bool mate1) {
    size_t need = in.used + 3 * len + 64 + (o.xr ? 3 * len : 0);
    if (need > in.arena.size()) in.arena.resize(std::max(need, in.arena.size() * 2));
    char* A = &in.arena[0];
    size_t w = in.used;
    size_t cur = 1;
    auto at = [&](size_t k) -> int {
        if (k >= len) throw Fail("Error: reads file contained a truncated record");
        return (unsigned char)r[k];
    };
    int c;
    size_t name_end = 1;
    for (;;) {
        c = at(cur++);
        if (c == '\n' || c == '\r') {
            name_end = cur - 1;
            do { c = at(cur++); } while (c == '\n' || c == '\r');
            break;
        }
    }
    std::string dflt;
    const char* name = r + 1;
    size_t name_len = name_end - 1;
    if (name_len == 0) {                      // a default name: the read's number (pat.cpp:1246-1251)
        dflt = std::to_string(rdid);
        name = dflt.data();
        name_len = dflt.size();
    }
    // the name kept for the SAM: mate 1's name without its "/1" (pat.cpp:2289-2297)
    size_t keep = name_len;
    if (mate1) {
        if (name_len < 3 || memcmp(name + name_len - 2, "/1", 2) != 0) in.bad_names++;
        else keep -= 2;
    }
    memcpy(A + w, name, keep);
    rec.name = (uint32_t)w;
    rec.name_len = (uint32_t)keep;
    w += keep;
    rec.tab = (uint32_t)w;
    A[w++] = '\t';
    // sequence
    const size_t seq0 = w;
    int nchar = 0;
    while (c != '+') {
        char b = kSeq.t[c];
        if (b && nchar++ >= o.trim5) A[w++] = b;
        c = at(cur++);
    }
    const int seqlen = (int)(w - seq0);
    const int trimmed5 = nchar - seqlen;
    const int trimmed3 = std::min<int>(o.trim3, seqlen);
    w -= trimmed3;
    do { c = at(cur++); } while (c != '\n' && c != '\r');
    while (cur < len && (c == '\n' || c == '\r')) c = (unsigned char)r[cur++];
    A[w++] = '\t';
    const size_t q0 = w;
    auto conv = [&](int ch) -> int {
        if (ch == ' ')
            throw Fail("Saw a space but expected an ASCII-encoded quality value.\n"
                       "Are quality values formatted as integers?  If so, try --integer-quals.");
        if (o.phred64) {
            if (ch < 64)
                throw Fail("Saw ASCII character " + std::to_string(ch) + " but expected 64-based Phred qual.\n"
                           "Try not specifying --solexa1.3-quals/--phred64-quals.");
            return ch - (64 - 33);
        }
        if (ch < 33) throw Fail("Saw ASCII character " + std::to_string(ch) + " but expected 33-based Phred qual.");
        return ch;
    };
    if (nchar > 0) {
        int nqual = 0;
        c = conv(c);
        if (nqual++ >= trimmed5) A[w++] = (char)c;
        while (cur < len) {
            c = (unsigned char)r[cur++];
            if (c == ' ')
                throw Fail("Error: Encountered one or more spaces while parsing the quality string for read " +
                           std::string(name, name_len) +
                           ".  If this is a FASTQ file with integer (non-ASCII-encoded) qualities, try re-running "
                           "with the --integer-quals option.");
            if (c == '\r' || c == '\n') break;
            c = conv(c);
            if (nqual++ >= trimmed5) A[w++] = (char)c;
        }
        size_t ql = w - q0;
        w -= std::min<size_t>(ql, (size_t)trimmed3);
        ql = w - q0;
        if ((int)ql < seqlen - trimmed3)
            throw Fail("Error: Read " + std::string(name, name_len) + " has more read characters than quality values.");
        if ((int)ql > seqlen - trimmed3)
            throw Fail("Error: Read " + std::string(name, name_len) + " has more quality values than read characters.");
    }
    rec.tab_len = (uint32_t)(w - rec.tab);
    rec.orig = (uint32_t)w;
    if (o.xr) {
        static const char hex[] = "0123456789ABCDEF";
        for (size_t k = 0; k < len; k++) {
            unsigned char s = (unsigned char)r[k];
            if (s == 10 || s == 13 || s == '%') {
                A[w++] = '%';
                A[w++] = hex[s >> 4];
                A[w++] = hex[s & 15];
            } else {
                A[w++] = (char)s;
            }
        }
    }
    rec.orig_len = (uint32_t)(w - rec.orig);
    in.used = w;
    if (w > 0xF0000000u) throw Fail("Error: input of one connection over 3.7 GB");
}

// A parsed read into in.arena: its name (mate 1: without a final "/1",
// saveOrigBufs), "\tSEQ\tQUAL" and the %-escaped original bytes (--passthrough).
void emit(Input& in, const Opts& o, Rec& rec, const char* name, size_t name_len, const std::string& seq,
          const std::string& qual, const char* orig, size_t orig_len, bool mate1) {
    size_t need = in.used + name_len + seq.size() + qual.size() + 3 * orig_len + 16;
    if (need > in.arena.size()) in.arena.resize(std::max(need, in.arena.size() * 2));
    char* A = &in.arena[0];
    size_t w = in.used;
    size_t keep = name_len;
    if (mate1) {
        if (name_len < 3 || memcmp(name + name_len - 2, "/1", 2) != 0) in.bad_names++;
        else keep -= 2;
    }
    memcpy(A + w, name, keep);
    rec.name = (uint32_t)w;
    rec.name_len = (uint32_t)keep;
    w += keep;
    rec.tab = (uint32_t)w;
    A[w++] = '\t';
    memcpy(A + w, seq.data(), seq.size());
    w += seq.size();
    A[w++] = '\t';
    memcpy(A + w, qual.data(), qual.size());
    w += qual.size();
    rec.tab_len = (uint32_t)(w - rec.tab);
    rec.orig = (uint32_t)w;
    if (o.xr) {
        static const char hex[] = "0123456789ABCDEF";
        for (size_t k = 0; k < orig_len; k++) {
            unsigned char c = (unsigned char)orig[k];
            if (c == 10 || c == 13 || c == '%') {
                A[w++] = '%';
                A[w++] = hex[c >> 4];
                A[w++] = hex[c & 15];
            } else {
                A[w++] = (char)c;
            }
        }
    }
    rec.orig_len = (uint32_t)(w - rec.orig);
    in.used = w;
    if (w > 0xF0000000u) throw Fail("Error: input of one connection over 3.7 GB");
}

// --trim5 / --trim3 of a parsed sequence and its qualities (Read::patFw /
// qual trimEnd; the 5' letters were dropped while parsing)
void trim3(std::string& seq, std::string& qual, int t3) {
    const size_t k = std::min(seq.size(), (size_t)std::max(0, t3));
    seq.resize(seq.size() - k);
    qual.resize(qual.size() - std::min(qual.size(), (size_t)std::max(0, t3)));
}

// Phred+33 of a quality character (charToPhred33, qual.h:105-146; FASTQ's rules)
int qual33(int ch, const Opts& o) {
    if (ch == ' ')
        throw Fail("Saw a space but expected an ASCII-encoded quality value.\n"
                   "Are quality values formatted as integers?  If so, try --integer-quals.");
    if (o.phred64) {
        if (ch < 64)
            throw Fail("Saw ASCII character " + std::to_string(ch) + " but expected 64-based Phred qual.\n"
                       "Try not specifying --solexa1.3-quals/--phred64-quals.");
        return ch - (64 - 33);
    }
    if (ch < 33) throw Fail("Saw ASCII character " + std::to_string(ch) + " but expected 33-based Phred qual.");
    return ch;
}

// FastaPatternSource::nextBatchFromFile + parse (pat.cpp:790-912) over a file
// in memory: every record of `s` into dst (rdid counts every record, parsed
// or not).
void load_fasta(const std::string& s, const Opts& o, Input& in, std::vector<Rec>& dst, long long& rdid, bool mate1) {
    const char* p = s.data();
    const size_t n = s.size();
    size_t i = 0;
    while (i < n && (p[i] == '\r' || p[i] == '\n')) i++;
    if (i >= n) return;
    if (p[i] != '>') throw Fail("Error: reads file does not look like a FASTA file");
    std::string seq, qual;
    while (i < n) {
        // the record: '>' and every byte up to the next '>'
        const size_t start = i;
        const char* nx = (const char*)memchr(p + i + 1, '>', n - i - 1);
        const size_t end = nx ? (size_t)(nx - p) : n;
        i = end;
        const char* r = p + start;
        const size_t len = end - start;
        const long long id = rdid++;
        if (len == 1 && !nx) break;                 // a lone '>' at EOF: no record (pat.cpp:836-838)
        size_t cur = 1;
        int c = -1;
        size_t name_end = 1;
        bool ended = false;
        while (cur < len) {                          // the name: the first line
            c = (unsigned char)r[cur++];
            if (c == '\n' || c == '\r') {
                name_end = cur - 1;
                do {
                    c = cur < len ? (unsigned char)r[cur] : 0;
                    cur++;
                } while ((c == '\n' || c == '\r') && cur < len);
                ended = true;
                break;
            }
        }
        if (!ended) name_end = cur;
        if (cur >= len) continue;                    // "FASTA ended prematurely": not parsed
        seq.clear();
        int nchar = 0;
        while (cur < len) {                          // the record's last byte is never a base
            if (c == '.') c = 'N';
            if (isalpha(c) && nchar++ >= o.trim5) seq.push_back(dna_char((unsigned char)c));
            c = (unsigned char)r[cur++];
            if ((c == '\n' || c == '\r') && cur < len && r[cur] != '>') c = (unsigned char)r[cur++];
        }
        qual.assign(seq.size(), 'I');
        trim3(seq, qual, o.trim3);
        std::string dflt;
        const char* name = r + 1;
        size_t name_len = name_end - 1;
        if (name_len == 0) {
            dflt = std::to_string(id);
            name = dflt.data();
            name_len = dflt.size();
        }
        Rec rec;
        emit(in, o, rec, name, name_len, seq, qual, r, len, mate1);
        dst.push_back(rec);
    }
}

// tabbed_parse (pat.cpp:1550-1654) of one line: false when it does not parse;
// pb true when it held a pair.
bool tab_line(const char* r, size_t len, bool tab6, const Opts& o, std::string nm[2], std::string sq[2],
              std::string ql[2], bool& pb) {
    int c = '\t';
    size_t cur = 0;
    pb = false;
    auto at = [&](size_t k) -> int { return k < len ? (unsigned char)r[k] : 0; };
    for (int e = 0; e < 2 && c == '\t'; e++) {
        nm[e].clear();
        sq[e].clear();
        ql[e].clear();
        if (e == 0 || tab6) {
            c = at(cur++);
            while (c != '\t' && cur < len) {
                nm[e].push_back((char)c);
                c = at(cur++);
            }
            if (c != '\t' || cur >= len) return false;
        } else {
            nm[1] = nm[0];
        }
        c = at(cur++);
        int nchar = 0;
        while (c != '\t' && cur < len) {
            if (isalpha(c) && nchar++ >= o.trim5) sq[e].push_back(dna_char((unsigned char)c));
            c = at(cur++);
        }
        if (c != '\t' || cur >= len) return false;
        c = at(cur++);
        int nqual = 0;
        while (c != '\t' && c != '\n' && c != '\r') {
            if (c == ' ')                            // wrongQualityFormat (pat.cpp:2199-2205)
                throw Fail("Error: Encountered one or more spaces while parsing the quality string for read " + nm[e] +
                           ".  If this is a FASTQ file with integer (non-ASCII-encoded) qualities, try re-running "
                           "with the --integer-quals option.");
            const int q = qual33(c, o);
            if (++nqual > o.trim5) ql[e].push_back((char)q);
            if (cur >= len) break;
            c = at(cur++);
        }
        if (nchar > nqual)
            throw Fail("Error: Read " + nm[e] + " has more read characters than quality values.");
        if (nqual > nchar)
            throw Fail("Error: Read " + nm[e] + " has more quality values than read characters.");
        trim3(sq[e], ql[e], o.trim3);
        if (e == 1) pb = true;
    }
    return true;
}

// Lines of a tabbed (or raw) file in memory, as their light parsers split
// them: blank lines skipped.
void lines_of(const std::string& s, std::vector<RecSpan>& out) {
    const char* p = s.data();
    const size_t n = s.size();
    size_t i = 0;
    while (i < n) {
        while (i < n && (p[i] == '\n' || p[i] == '\r')) i++;
        if (i >= n) break;
        const size_t st = i;
        while (i < n && p[i] != '\n' && p[i] != '\r') i++;
        out.push_back({st, i - st});
    }
}

// --tab5 / --tab6 / --12 (and -c, as tab5 lines): pairs and unpaired reads
// may mix; a[i], b[i] (b[i].tab_len == 0: read i unpaired)
void load_tabbed(const std::vector<std::string>& lines_src, bool from_files, bool tab6, const Opts& o, Input& in) {
    std::vector<Rec> a, b;
    bool any_pair = false;
    long long rdid = 0;
    std::string nm[2], sq[2], ql[2];
    auto one = [&](const char* r, size_t len) {
        bool pb = false;
        rdid++;
        if (!tab_line(r, len, tab6, o, nm, sq, ql, pb)) return;
        Rec ra, rb{};
        emit(in, o, ra, nm[0].data(), nm[0].size(), sq[0], ql[0], r, len, true);
        if (pb) {
            emit(in, o, rb, nm[1].data(), nm[1].size(), sq[1], ql[1], r, 0, false);
            any_pair = true;
        }
        a.push_back(ra);
        b.push_back(rb);
    };
    if (from_files) {
        for (const auto& f : lines_src) {
            std::string s = slurp(f);
            std::vector<RecSpan> ls;
            lines_of(s, ls);
            for (const auto& l : ls) one(s.data() + l.off, l.len);
        }
    } else {
        for (const auto& l : lines_src) one(l.data(), l.size());
    }
    in.a.swap(a);
    if (any_pair) in.b.swap(b);
}

// -r: RawPatternSource (pat.cpp:1743-1817)
void load_raw(const std::string& s, const Opts& o, Input& in, std::vector<Rec>& dst, long long& rdid, bool mate1) {
    std::vector<RecSpan> ls;
    lines_of(s, ls);
    std::string seq, qual;
    for (const auto& l : ls) {
        const char* r = s.data() + l.off;
        const long long id = rdid++;
        seq.clear();
        int nchar = 0;
        for (size_t k = 0; k < l.len; k++)
            if (isalpha((unsigned char)r[k]) && nchar++ >= o.trim5) seq.push_back(dna_char((unsigned char)r[k]));
        qual.assign(seq.size(), 'I');
        trim3(seq, qual, o.trim3);
        const std::string name = std::to_string(id);
        Rec rec;
        emit(in, o, rec, name.data(), name.size(), seq, qual, r, l.len, mate1);
        dst.push_back(rec);
    }
}

void load_mate(const std::vector<std::string>& files, const Opts& o, Input& in, std::vector<Rec>& dst, bool mate1) {
    long long rdid = 0;
    if (o.fmt == Opts::FASTA || o.fmt == Opts::RAW) {
        for (const auto& f : files) {
            std::string s = slurp(f);
            if (o.fmt == Opts::FASTA) load_fasta(s, o, in, dst, rdid, mate1);
            else load_raw(s, o, in, dst, rdid, mate1);
        }
        return;
    }
    if (o.fmt == Opts::CMDLINE) {
        // VectorPatternSource: "i\tSEQ\tQUALS" (QUALS 'I' when not given)
        Input tmp;
        std::vector<std::string> lines;
        for (size_t i = 0; i < files.size(); i++) {
            const std::string& t = files[i];
            const size_t k = t.find(':');
            const std::string sq = t.substr(0, k);
            lines.push_back(std::to_string(i) + "\t" + sq + "\t" +
                            (k == std::string::npos ? std::string(sq.size(), 'I') : t.substr(k + 1)));
        }
        tmp.arena.swap(in.arena);
        tmp.used = in.used;
        tmp.bad_names = in.bad_names;
        load_tabbed(lines, false, false, o, tmp);
        in.arena.swap(tmp.arena);
        in.used = tmp.used;
        in.bad_names = tmp.bad_names;
        for (const Rec& r : tmp.a) dst.push_back(r);
        return;
    }
    for (const auto& f : files) {
        std::string s = slurp(f);
        std::string scratch;
        std::vector<RecSpan> spans;
        light_parse(s, scratch, spans);
        if (in.arena.size() < in.used + s.size() + 32 * spans.size())
            in.arena.resize(in.used + s.size() + 32 * spans.size());
        for (const auto& sp : spans) {
            const char* base = (sp.off >> 62) ? scratch.data() + (sp.off & ((1ull << 62) - 1)) : s.data() + sp.off;
            Rec rec;
            parse_rec(base, sp.len, rdid++, o, in, rec, mate1);
            dst.push_back(rec);
        }
    }
}

std::unique_ptr<Input> load_input(const std::vector<std::string>& U, const std::vector<std::string>& m1,
                                   const std::vector<std::string>& m2, const Opts& o) {
    std::unique_ptr<Input> in(new Input);
    if (o.fmt == Opts::TAB5 || o.fmt == Opts::TAB6) {
        // (the files of --tab5 / --tab6 / --12 come in U: one read or pair a line)
        load_tabbed(U, true, o.fmt == Opts::TAB6, o, *in);
    } else if (!m1.empty() || !m2.empty()) {
        load_mate(m1, o, *in, in->a, true);
        load_mate(m2, o, *in, in->b, false);
        if (in->a.size() < in->b.size())
            throw Fail("Error, fewer reads in file specified with -1 than in file specified with -2");
        if (in->a.size() > in->b.size())
            throw Fail("Error, fewer reads in file specified with -2 than in file specified with -1");
        if (in->a.empty()) in->b.clear();
    } else {
        load_mate(U, o, *in, in->a, true);
    }
    // rdid >= skipReads && rdid < qUpto (bt2_search.cpp:4594-4603), qUpto
    // counted after the skipped reads (bt2_search.cpp:1801-1806)
    size_t hi = o.upto >= 0 ? std::min(in->a.size(), (size_t)(o.upto + std::max(0LL, o.skip))) : in->a.size();
    size_t lo = std::min(hi, (size_t)std::max(0LL, o.skip));
    if (lo > 0 || hi < in->a.size()) {
        in->a = std::vector<Rec>(in->a.begin() + lo, in->a.begin() + hi);
        if (in->paired()) in->b = std::vector<Rec>(in->b.begin() + lo, in->b.begin() + hi);
    }
    return in;
}

// ---------------------------------------------------------------- one connection

constexpr int BUF_CAPACITY = 10000;   // LockedOrigBufMap::BUF_CAPACITY
constexpr int RE_PER_PACKET = 40;     // PatternSourceWebClient::RE_PER_PACKET
constexpr uint32_t NO_READ = 0xFFFFFFFFu;

struct Job {
    std::shared_ptr<const Input> in;   // null: loaded by the worker (chunk mode)
    std::vector<std::string> U, m1, m2;
    size_t lo = 0, hi = 0;             // reads [lo, hi) of `in`
};

struct Conn {
    int fd = -1;
    size_t job = 0;
    std::shared_ptr<const Input> in;
    size_t lo = 0, hi = 0, next = 0;
    // LockedOrigBufMap: two maps of BUF_CAPACITY slots
    uint16_t used_idx[2] = {0, 0}, used_cnt[2] = {0, 0};
    std::vector<uint32_t> slot[2];           // read index, NO_READ when free
    std::vector<uint8_t> present[2];         // bit 0 mate 1, bit 1 mate 2 (OrigBuf::readaPresent/readbPresent)
    std::string out;                         // bytes to send
    size_t out_pos = 0;
    bool end_queued = false, shut = false, header = false, finished = false;
    std::string in_buf;                      // received, not yet processed
    std::string sam;
    long long warned_lines = 0;
    // --count-aligned: reads (pairs) with an alignment among the records received,
    // counted as bench.py's count_aligned does (primary records without 0x4; a
    // pair by its first mate's record, 0x4 and 0x8 not both set)
    bool count = false;
    long long aligned = 0;
};

// LockedOrigBufMap::take_ownership (pat.h:2519-2538); -1 when both maps are full
inline int take_slot(Conn& c, uint32_t read) {
    for (int m = 0; m < 2; m++) {
        if (c.used_idx[m] < BUF_CAPACITY) {
            int id = c.used_idx[m]++;
            c.used_cnt[m]++;
            c.slot[m][id] = read;
            c.present[m][id] = c.in->pair(read) ? 3 : 1;
            return id + m * BUF_CAPACITY;
        }
    }
    return -1;
}

// LockedOrigBufMap::release (pat.h:2497-2516)
inline void release_slot(Conn& c, int id) {
    int m = id >= BUF_CAPACITY;
    int k = id - m * BUF_CAPACITY;
    c.slot[m][k] = NO_READ;
    if (--c.used_cnt[m] == 0) c.used_idx[m] = 0;
}

inline uint32_t lookup(const Conn& c, unsigned long id) {
    if (id >= 2 * (unsigned long)BUF_CAPACITY) return NO_READ;
    int m = id >= (unsigned long)BUF_CAPACITY;
    return c.slot[m][id - m * BUF_CAPACITY];
}

inline void hex4(char* d, int id) {
    static const char hx[] = "0123456789ABCDEF";
    d[0] = hx[(id >> 12) & 15];
    d[1] = hx[(id >> 8) & 15];
    d[2] = hx[(id >> 4) & 15];
    d[3] = hx[id & 15];
}

// sendDataWorker (pat.cpp:2488-2568): packets of <= 40 TAB6 lines as HTTP
// chunks; ids are taken as the lines are made, so a full pair of maps waits
// for the server's END READ lines as addReadPair does.  Fills c.out up to
// ~256 KB; returns whether anything was added.
bool fill_out(Conn& c) {
    if (c.end_queued) return false;
    if (c.out_pos == c.out.size()) {
        c.out.clear();
        c.out_pos = 0;
    }
    bool added = false;
    const Input& in = *c.in;
    const char* A = in.arena.data();
    while (c.out.size() < (256u << 10) && c.next < c.hi) {
        size_t hdr = c.out.size();
        c.out.append("00000000\r\n");            // chunk-size line, patched below
        size_t body = c.out.size();
        int nre = 0;
        while (nre < RE_PER_PACKET && c.next < c.hi) {
            int id = take_slot(c, (uint32_t)c.next);
            if (id < 0) break;
            const Rec& a = in.a[c.next];
            char nm[6] = {0, 0, 0, 0, '/', '1'};
            hex4(nm, id);
            c.out.append(nm, 6);
            c.out.append(A + a.tab, a.tab_len);
            if (in.pair(c.next)) {
                const Rec& b = in.b[c.next];
                nm[5] = '2';
                c.out.push_back('\t');
                c.out.append(nm, 6);
                c.out.append(A + b.tab, b.tab_len);
            }
            c.out.push_back('\n');
            c.next++;
            nre++;
        }
        if (nre == 0) {
            c.out.resize(hdr);
            break;
        }
        char hx[16];
        int hl = snprintf(hx, sizeof hx, "%zx\r\n", c.out.size() - body);
        // move the body to sit right after the real size line
        c.out.replace(hdr, body - hdr, hx, (size_t)hl);
        c.out.append("\r\n");
        added = true;
    }
    if (c.next == c.hi) {
        c.out.append("0\r\n\r\n");                 // write_chunked_str(fd, send_str, 0)
        c.end_queued = true;
        added = true;
    }
    return added;
}

// process_read_line (pat.cpp:2570-2646)
void read_line(Conn& c, const char* line, size_t n, bool xr) {
    const char* tab = (const char*)memchr(line, '\t', n);
    auto pass = [&](const char* w) {
        if (c.warned_lines++ < 4) fprintf(stderr, "%s", w);
        c.sam.append(line, n);
    };
    if (!tab) return pass("WARNING: Malformed line found, no tab\n");
    size_t tl = (size_t)(tab - line);
    if (tl != 4 && tl != 6) return pass("WARNING: Malformed line found, read index string too long\n");
    if (tl == 6 && line[4] != '/') return pass("WARNING: Malformed line found, invalid paired read index string\n");
    unsigned long id = 0;
    size_t k = 0;
    for (; k < tl && isxdigit((unsigned char)line[k]); k++)
        id = id * 16 + (unsigned long)(isdigit((unsigned char)line[k]) ? line[k] - '0' : (line[k] | 32) - 'a' + 10);
    if (k != 4) return pass("WARNING: Malformed line found, not valid read index\n");
    uint32_t r = lookup(c, id);
    if (r == NO_READ) return pass("WARNING: Malformed line found, invalid read index found\n");
    const Input& in = *c.in;
    const Rec& a = in.a[r];
    c.sam.append(in.arena.data() + a.name, a.name_len);
    c.sam.append(line + 4, n - 4);
    if (c.count) {
        const unsigned long f = strtoul(tab + 1, nullptr, 10);
        if (!(f & 0x900)) {
            if (f & 0x1) c.aligned += (f & 0x40) && (f & 0xC) != 0xC;
            else c.aligned += !(f & 0x4);
        }
    }
    if (xr) {
        unsigned long flags = strtoul(tab + 1, nullptr, 10);
        bool mate2 = (flags & 0x1) && (flags & 0x80);
        if (!mate2) c.sam.append(in.arena.data() + a.orig, a.orig_len);
        else if (in.pair(r)) c.sam.append(in.arena.data() + in.b[r].orig, in.b[r].orig_len);
        c.sam.push_back('\n');
    }
}

// process_end_read (pat.cpp:2648-2708)
void end_read(Conn& c, const char* id, size_t n) {
    if (n != 4 && n != 6) {
        fprintf(stderr, "WARNING: Malformed end line found, read index string too long (%zu)\n", n);
        return;
    }
    unsigned long v = 0;
    size_t k = 0;
    for (; k < n && isxdigit((unsigned char)id[k]); k++)
        v = v * 16 + (unsigned long)(isdigit((unsigned char)id[k]) ? id[k] - '0' : (id[k] | 32) - 'a' + 10);
    if (k != 4) {
        fprintf(stderr, "WARNING: Malformed end line found, not valid read index (len %zu)\n", k);
        return;
    }
    if (lookup(c, v) == NO_READ) {
        fprintf(stderr, "WARNING: Malformed end line found, invalid read index found\n");
        return;
    }
    int m = v >= (unsigned long)BUF_CAPACITY;
    size_t s = v - m * BUF_CAPACITY;
    if (n == 4) {
        release_slot(c, (int)v);
    } else {
        c.present[m][s] &= (uint8_t)~(id[5] == '2' ? 2 : 1);
        if (!c.present[m][s]) release_slot(c, (int)v);
    }
}

// process_read_buffer (pat.cpp:2712-2754): complete lines of c.in_buf;
// returns true at "@CO BT2SRV All Done".
bool take_lines(Conn& c, bool xr) {
    static const char done[] = "@CO BT2SRV All Done\n";
    static const char endr[] = "@CO END READ\t";
    const char* p = c.in_buf.data();
    size_t n = c.in_buf.size(), i = 0;
    bool end = false;
    while (n - i >= 20) {
        if (memcmp(p + i, done, 20) == 0) {
            end = true;
            break;
        }
        const char* nl = (const char*)memchr(p + i, '\n', n - i);
        if (!nl) break;
        size_t ll = (size_t)(nl - (p + i)) + 1;
        if (ll >= 13 && memcmp(p + i, endr, 13) == 0) end_read(c, p + i + 13, ll - 14);
        else if (p[i] == '@') c.sam.append(p + i, ll);
        else read_line(c, p + i, ll, xr);
        i += ll;
    }
    if (end) c.in_buf.clear();
    else c.in_buf.erase(0, i);
    return end;
}

// the answer's header (initialHandshake + parseHeader, pat.cpp:2395-2436,
// pat_read_header pat.cpp:1901-1950: it ends at two newlines, \r ignored)
int take_header(Conn& c) {
    const std::string& b = c.in_buf;
    int nnl = 0;
    size_t i = 0;
    for (; i < b.size(); i++) {
        char ch = b[i];
        if (ch == '\r') continue;
        nnl = ch == '\n' ? nnl + 1 : 0;
        if (nnl == 2) break;
    }
    if (nnl < 2) return b.size() > 64 * 1024 ? -1 : 0;
    std::string h = b.substr(0, i + 1);
    if (h.size() < 15 || memcmp(h.data(), "HTTP/1.1 200 OK", 15) != 0) return -1;
    if (h.find("\nX-BT2SRV-Terminator: 1") == std::string::npos &&
        h.find("\nx-bt2srv-terminator: 1") == std::string::npos) {
        fprintf(stderr, "ERROR: Server does not appear to be valid BT2SRV\n");
        return -1;
    }
    c.in_buf.erase(0, i + 1);
    c.header = true;
    return 1;
}

int connect_to(const Opts& o) {
    struct addrinfo hints;
    memset(&hints, 0, sizeof hints);
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    struct addrinfo* res = nullptr;
    if (getaddrinfo(o.host.c_str(), nullptr, &hints, &res) != 0) return -1;
    int fd = socket(AF_INET, SOCK_STREAM, 0);
    bool ok = false;
    for (struct addrinfo* r = res; fd >= 0 && r; r = r->ai_next) {
        struct sockaddr_in a;
        memset(&a, 0, sizeof a);
        a.sin_family = AF_INET;
        a.sin_addr = ((struct sockaddr_in*)r->ai_addr)->sin_addr;
        a.sin_port = htons((uint16_t)o.port);
        if (connect(fd, (struct sockaddr*)&a, sizeof a) == 0) {
            ok = true;
            break;
        }
    }
    freeaddrinfo(res);
    if (!ok) {
        if (fd >= 0) close(fd);
        return -1;
    }
    std::string req = "PUT /BT2SRV/" + o.index + "/align HTTP/1.1\r\nHost: " + o.host + ":" + std::to_string(o.port) +
                      "\r\nUser-Agent: BT2CLT\r\nAccept: */*\r\nTransfer-Encoding: chunked\r\n"
                      "X-BT2SRV-Request-Terminator: 1\r\n\r\n";
    size_t w = 0;
    while (w < req.size()) {
        ssize_t k = write(fd, req.data() + w, req.size() - w);
        if (k <= 0) {
            close(fd);
            return -1;
        }
        w += (size_t)k;
    }
    fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK);
    return fd;
}

// ---------------------------------------------------------------- output

struct Sink {
    const Opts& o;
    FILE* f = nullptr;
    std::mutex m;
    std::vector<std::string> pending;
    std::vector<char> ready;
    size_t next = 0;
    explicit Sink(const Opts& opts, size_t njobs) : o(opts), pending(njobs), ready(njobs, 0) {
        if (o.out_dir.empty()) {
            f = o.out.empty() ? stdout : fopen(o.out.c_str(), "wb");
            if (!f) throw Fail("Error: could not open " + o.out);
        }
    }
    void put(size_t job, std::string&& sam) {
        if (!o.out_dir.empty()) {
            char nm[32];
            snprintf(nm, sizeof nm, "/chunk%05zu.sam", job);
            std::string path = o.out_dir + nm;
            FILE* g = fopen(path.c_str(), "wb");
            if (!g || fwrite(sam.data(), 1, sam.size(), g) != sam.size() || fclose(g) != 0)
                throw Fail("Error: could not write " + path);
            return;
        }
        std::lock_guard<std::mutex> lk(m);
        pending[job] = std::move(sam);
        ready[job] = 1;
        while (next < ready.size() && ready[next]) {   // chunk order
            if (o.mark) fprintf(f, "@CO BT2G-CLIENT CHUNK %zu\n", next);
            fwrite(pending[next].data(), 1, pending[next].size(), f);
            std::string().swap(pending[next]);
            next++;
        }
    }
    void close_out() {
        if (f && f != stdout) fclose(f);
        else if (f) fflush(f);
    }
};

// ---------------------------------------------------------------- the loops

struct Shared {
    const Opts& o;
    std::vector<Job>& jobs;
    Sink& sink;
    std::atomic<size_t> next_job{0};
    std::atomic<int> failed{0};
    std::atomic<long long> reads{0}, bad_names{0}, bytes_out{0}, bytes_in{0}, aligned{0};
};

void worker(Shared& S, int cap) {
    const Opts& o = S.o;
    int ep = epoll_create1(0);
    std::vector<std::unique_ptr<Conn>> live;
    std::vector<char> rb(1 << 18);
    auto open_next = [&]() -> bool {
        size_t j = S.next_job.fetch_add(1);
        if (j >= S.jobs.size()) return false;
        Job& jb = S.jobs[j];
        std::unique_ptr<Conn> c(new Conn);
        c->job = j;
        if (jb.in) {
            c->in = jb.in;
            c->lo = jb.lo;
            c->hi = jb.hi;
        } else {
            std::shared_ptr<Input> in(load_input(jb.U, jb.m1, jb.m2, o).release());
            c->in = in;
            c->lo = 0;
            c->hi = in->a.size();
            if (in->bad_names) S.bad_names += in->bad_names;
        }
        c->next = c->lo;
        c->count = o.count;
        for (int m = 0; m < 2; m++) {
            c->slot[m].assign(BUF_CAPACITY, NO_READ);
            c->present[m].assign(BUF_CAPACITY, 0);
        }
        c->fd = connect_to(o);
        if (c->fd < 0) throw Fail("ERROR: Failed to connect to " + o.host + ":" + std::to_string(o.port) + "!");
        struct epoll_event ev;
        memset(&ev, 0, sizeof ev);
        ev.events = EPOLLIN | EPOLLOUT | EPOLLET | EPOLLRDHUP;
        ev.data.ptr = c.get();
        epoll_ctl(ep, EPOLL_CTL_ADD, c->fd, &ev);
        live.push_back(std::move(c));
        return true;
    };
    bool more = true;
    try {
        while (more && (int)live.size() < cap) more = open_next();
        std::vector<struct epoll_event> evs(64);
        while (!live.empty()) {
            int ne = epoll_wait(ep, evs.data(), (int)evs.size(), 1000);
            if (ne < 0 && errno != EINTR) throw Fail("ERROR: epoll_wait failed");
            for (int e = 0; e < ne; e++) {
                Conn& c = *(Conn*)evs[e].data.ptr;
                bool progress = true;
                while (progress && !c.finished) {
                    progress = false;
                    // receive
                    for (;;) {
                        ssize_t k = read(c.fd, rb.data(), rb.size());
                        if (k > 0) {
                            S.bytes_in += k;
                            c.in_buf.append(rb.data(), (size_t)k);
                            progress = true;
                            continue;
                        }
                        if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
                        if (k < 0 && errno == EINTR) continue;
                        // EOF or error before the terminator
                        if (!c.header || !take_lines(c, o.xr)) throw Fail("ERROR: Read from server failed, aborting");
                        c.finished = true;
                        break;
                    }
                    if (c.finished) break;
                    if (!c.header) {
                        int h = take_header(c);
                        if (h < 0) throw Fail("ERROR: Failed to connect to " + o.host + ":" + std::to_string(o.port) + "!");
                        if (h == 0) break;
                        progress = true;
                    }
                    if (take_lines(c, o.xr)) {
                        c.finished = true;
                        break;
                    }
                    // send
                    for (;;) {
                        if (c.out_pos == c.out.size() && !fill_out(c)) break;
                        if (c.out_pos == c.out.size()) break;
                        ssize_t k = write(c.fd, c.out.data() + c.out_pos, c.out.size() - c.out_pos);
                        if (k > 0) {
                            S.bytes_out += k;
                            c.out_pos += (size_t)k;
                            progress = true;
                            continue;
                        }
                        if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
                        if (k < 0 && errno == EINTR) continue;
                        throw Fail("ERROR: Write to server failed, aborting");
                    }
                    if (c.end_queued && c.out_pos == c.out.size() && !c.shut) {
                        shutdown(c.fd, SHUT_WR);
                        c.shut = true;
                    }
                }
                if (c.finished) {
                    epoll_ctl(ep, EPOLL_CTL_DEL, c.fd, nullptr);
                    close(c.fd);
                    S.reads += (long long)(c.hi - c.lo);
                    S.aligned += c.aligned;
                    if (c.used_cnt[0] || c.used_cnt[1]) {
                        fprintf(stderr, "ERROR: Did not process all the input file\n");
                        S.failed = 1;
                    }
                    S.sink.put(c.job, std::move(c.sam));
                    for (size_t k = 0; k < live.size(); k++)
                        if (live[k].get() == &c) {
                            live[k].swap(live.back());
                            live.pop_back();
                            break;
                        }
                    if (more) more = open_next();
                }
            }
        }
    } catch (const std::exception& ex) {
        fprintf(stderr, "%s\n", ex.what());
        S.failed = 1;
        for (auto& c : live)
            if (c->fd >= 0) close(c->fd);
    }
    close(ep);
}

void split_commas(const char* s, std::vector<std::string>& v) {
    std::string cur;
    for (; *s; s++) {
        if (*s == ',') {
            if (!cur.empty()) v.push_back(cur);
            cur.clear();
        } else {
            cur.push_back(*s);
        }
    }
    if (!cur.empty()) v.push_back(cur);
}

void usage() {
    fprintf(stderr,
            "Usage: bt2g-client -x <index> (-U f[,f..] | -1 f1 -2 f2) [-k conns] [-R reads/conn] [-p threads]\n"
            "                   [-S out.sam] [--server-host H] [--server-port P] [--passthrough] [-3 n] [-5 n]\n"
            "                   [--phred33|--phred64] [-s skip] [-u upto] [--no-hd] [--stats]\n"
            "                   [-q | -f | -r | -c | --tab5 f | --12 f | --tab6 f]\n"
            "       bt2g-client -x <index> --chunks LIST [-k conns] [-p threads] [--out-dir D | -S out.sam]\n"
            "                   [--mark-chunks] [--count-aligned]\n");
}

}  // namespace

int main(int argc, char** argv) {
    signal(SIGPIPE, SIG_IGN);
    Opts o;
    if (const char* e = getenv("BT2CLT_SERVER_PORT")) o.port = atoi(e);
    if (const char* e = getenv("BT2CLT_SERVER_HOST")) o.host = e;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto val = [&]() -> const char* {
            if (i + 1 >= argc) {
                fprintf(stderr, "Error: %s needs a value\n", a.c_str());
                exit(1);
            }
            return argv[++i];
        };
        if (a == "-x") o.index = val();
        else if (a == "-U" || a == "--unpaired") split_commas(val(), o.U);
        else if (a == "-1") split_commas(val(), o.m1);
        else if (a == "-2") split_commas(val(), o.m2);
        else if (a == "-S" || a == "--output") o.out = val();
        else if (a == "--server-host") o.host = val();
        else if (a == "--server-port") o.port = atoi(val());
        else if (a == "-k" || a == "--connections") o.conns = atoi(val());
        else if (a == "-R" || a == "--reads-per-connection") o.per_conn = atoll(val());
        else if (a == "-p" || a == "--threads") o.threads = atoi(val());
        else if (a == "--chunks") o.chunks = val();
        else if (a == "--out-dir") o.out_dir = val();
        else if (a == "-s" || a == "--skip") o.skip = atoll(val());
        else if (a == "-u" || a == "--qupto" || a == "--upto") o.upto = atoll(val());
        else if (a == "-3" || a == "--trim3") o.trim3 = atoi(val());
        else if (a == "-5" || a == "--trim5") o.trim5 = atoi(val());
        else if (a == "--phred64" || a == "--phred64-quals" || a == "--solexa1.3-quals") o.phred64 = true;
        else if (a == "--phred33" || a == "--phred33-quals") o.phred64 = false;
        else if (a == "--passthrough" || a == "--xr") o.xr = true;
        else if (a == "--stats") o.stats = true;
        else if (a == "--mark-chunks") o.mark = true;
        else if (a == "--count-aligned") o.count = true;
        else if (a == "-f" || a == "--fasta") o.fmt = Opts::FASTA;
        else if (a == "-q" || a == "--fastq") o.fmt = Opts::FASTQ;
        else if (a == "-r" || a == "--raw") o.fmt = Opts::RAW;
        else if (a == "-c") o.fmt = Opts::CMDLINE;
        else if (a == "--tab5" || a == "--12") { o.fmt = Opts::TAB5; split_commas(val(), o.U); }
        else if (a == "--tab6") { o.fmt = Opts::TAB6; split_commas(val(), o.U); }
        else if (a == "--no-hd" || a == "--quiet" || a == "-t") {
        } else if (a == "-h" || a == "--help") {
            usage();
            return 0;
        } else {
            fprintf(stderr, "Error: unsupported option %s\n", a.c_str());
            usage();
            return 1;
        }
    }
    if (o.index.empty() || (o.U.empty() && o.m1.empty() && o.chunks.empty()) || (o.m1.empty() != o.m2.empty())) {
        usage();
        return 1;
    }
    {   // logical index name: basename (bt2_search.cpp:5419-5424)
        size_t s = o.index.find_last_of('/');
        if (s != std::string::npos) o.index = o.index.substr(s + 1);
    }
    if (o.conns < 1) o.conns = 1;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    std::vector<Job> jobs;
    long long bad = 0;
    try {
        if (!o.chunks.empty()) {
            FILE* f = fopen(o.chunks.c_str(), "r");
            if (!f) throw Fail("Error: could not open " + o.chunks);
            char line[8192];
            while (fgets(line, sizeof line, f)) {
                char kind[4], p1[4096], p2[4096];
                int n = sscanf(line, "%3s %4095s %4095s", kind, p1, p2);
                if (n < 2) continue;
                Job j;
                if (kind[0] == 'P' && n == 3) {
                    split_commas(p1, j.m1);
                    split_commas(p2, j.m2);
                } else {
                    split_commas(p1, j.U);
                }
                jobs.push_back(std::move(j));
            }
            fclose(f);
        } else {
            std::shared_ptr<Input> in(load_input(o.U, o.m1, o.m2, o).release());
            bad = in->bad_names;
            size_t n = in->a.size();
            size_t per = o.per_conn > 0 ? (size_t)o.per_conn : std::max<size_t>(n, 1);
            for (size_t lo = 0; lo < std::max<size_t>(n, 1); lo += per) {
                Job j;
                j.in = in;
                j.lo = lo;
                j.hi = std::min(n, lo + per);
                jobs.push_back(std::move(j));
            }
        }
    } catch (const std::exception& ex) {
        fprintf(stderr, "%s\n", ex.what());
        return 1;
    }
    if (!o.out_dir.empty()) mkdir(o.out_dir.c_str(), 0755);
    int ret = 0;
    try {
        Sink sink(o, jobs.size());
        Shared S{o, jobs, sink};
        S.bad_names = bad;
        int conns = (int)std::min<size_t>((size_t)o.conns, std::max<size_t>(jobs.size(), 1));
        int nt = o.threads > 0 ? o.threads : std::min(conns, 4);
        nt = std::max(1, std::min(nt, conns));
        std::vector<std::thread> th;
        for (int t = 0; t < nt; t++) {
            int cap = conns / nt + (t < conns % nt ? 1 : 0);
            th.emplace_back(worker, std::ref(S), cap);
        }
        for (auto& t : th) t.join();
        sink.close_out();
        if (S.bad_names)
            fprintf(stderr, "WARNING: Read name does not end in /1! Results likely invalid (%lld reads)\n",
                    (long long)S.bad_names);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if (o.stats)
            fprintf(stderr, "bt2g-client: %lld reads over %zu connections (%d at a time, %d threads), %.3f s, "
                            "%.1f MB out, %.1f MB in\n",
                    (long long)S.reads, jobs.size(), conns, nt,
                    (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec), S.bytes_out / 1e6,
                    S.bytes_in / 1e6);
        if (o.count)
            fprintf(stderr, "bt2g-client: aligned %lld of %lld\n", (long long)S.aligned, (long long)S.reads);
        ret = S.failed ? 1 : 0;
    } catch (const std::exception& ex) {
        fprintf(stderr, "%s\n", ex.what());
        ret = 1;
    }
    return ret;
}
