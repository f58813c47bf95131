// ingest.cpp — native input conversion: the SPMFBuilder
// formats (/root/reference/src/main/scala/de/kp/spark/fsm/util/SPMFBuilder.scala)
// parsed straight from a file image into the token arrays fsm_db_from_tokens
// takes (and so into K0 on the GPU), instead of building "idx|seq" strings
// that the miners then parse again.
//
// Per format, restating SPMFBuilder.scala (every input item becomes an
// itemset of its own, each sequence ends with -2; `index` numbers the
// sequences 0, 1, 2 ... in file order and keeps the first `limit`; its
// file.count (:192) runs the conversion over EVERY line, so a malformed line
// past the limit still fails the build, except for SPMF, whose lines are not
// parsed until the miner reads the kept ones):
//   BMS      :66-93   "uid<TAB>pid" lines grouped by uid; Spark's groupBy
//                     order is unspecified: here groups in order of the uid's
//                     first line, items in line order [documented choice]
//   CSV      :95-116  "i,j,k" -> i -1 j -1 k -1 -2
//   KOSARAK  :118-139 "i j k"  -> i -1 j -1 k -1 -2
//   SNAKE    :141-176 lines of >= 11 chars, every char c -> item (c - 65)
//   SPMF     :178-183 the lines as they are (SPMF token lines, no <t>)
//   INDEXED  (the builder's own output) "idx|seq": sid = idx, seq as SPMF
// Java semantics kept: String.split (trailing empty strings dropped, inner
// ones kept), Integer.parseInt (strict, so an empty or padded field fails),
// .trim() where the reference trims (BMS fields).  Lines end at \n, \r\n or
// \r (Hadoop's LineRecordReader).  Failures return FSM_EPARSE with the line.
#include <algorithm>
#include <climits>
#include <string>
#include <unordered_map>

#include "fsm_internal.h"

namespace fsm {
namespace {

struct Line {
    const char* p;
    int64_t n;
};

void split_lines(const char* d, int64_t len, std::vector<Line>& out) {
    int64_t s = 0;
    for (int64_t i = 0; i < len; ++i) {
        if (d[i] == '\n' || d[i] == '\r') {
            out.push_back({d + s, i - s});
            if (d[i] == '\r' && i + 1 < len && d[i + 1] == '\n') ++i;
            s = i + 1;
        }
    }
    if (s < len) out.push_back({d + s, len - s});
}

// java.lang.String.split(sep) for a one-char separator (limit 0)
void jsplit(const char* p, int64_t n, char sep, std::vector<Line>& out) {
    out.clear();
    if (n == 0) {
        out.push_back({p, 0});
        return;
    }
    int64_t s = 0;
    for (int64_t i = 0; i < n; ++i)
        if (p[i] == sep) {
            out.push_back({p + s, i - s});
            s = i + 1;
        }
    out.push_back({p + s, n - s});
    while (!out.empty() && out.back().n == 0) out.pop_back();
}

// java.lang.Integer.parseInt
bool jint(const char* p, int64_t n, int32_t& v) {
    if (n <= 0) return false;
    int64_t i = 0;
    bool neg = false;
    if (p[0] == '-' || p[0] == '+') {
        neg = p[0] == '-';
        if (n == 1) return false;
        i = 1;
    }
    int64_t acc = 0;
    for (; i < n; ++i) {
        const unsigned d = unsigned(uint8_t(p[i])) - unsigned('0');
        if (d > 9) return false;
        acc = acc * 10 + d;
        if (acc > int64_t(INT32_MAX) + 1) return false;
    }
    if (!neg && acc > INT32_MAX) return false;
    v = int32_t(neg ? -acc : acc);
    return true;
}

// String.trim(): strips chars <= ' ' at both ends
Line jtrim(Line l) {
    while (l.n > 0 && uint8_t(l.p[0]) <= ' ') {
        ++l.p;
        --l.n;
    }
    while (l.n > 0 && uint8_t(l.p[l.n - 1]) <= ' ') --l.n;
    return l;
}

std::string quote(const Line& l) { return std::string(l.p, size_t(std::min<int64_t>(l.n, 60))); }

struct Out {
    std::vector<int32_t> sids;
    std::vector<int64_t> off{0};
    std::vector<int64_t> tok;
    int64_t limit;
    int64_t seen = 0;  // sequences converted, kept or not
    bool full() const { return limit >= 0 && int64_t(sids.size()) >= limit; }
    // keep the sequence built since the last end_seq, or drop it past the limit
    void end_seq() {
        const int32_t sid = int32_t(seen++);
        if (full()) {
            tok.resize(size_t(off.back()));
            return;
        }
        tok.push_back(-2);
        sids.push_back(sid);
        off.push_back(int64_t(tok.size()));
    }
};

[[noreturn]] void bad(const char* fmt, int64_t line, const std::string& what) {
    throw Error(FSM_EPARSE, std::string("SPMFBuilder ") + fmt + ": line " + std::to_string(line + 1) + ": " + what);
}

}  // namespace

void ingest(int32_t format, const char* data, int64_t len, int64_t limit, Out& o) {
    o.limit = limit;
    std::vector<Line> lines, parts;
    split_lines(data, len, lines);
    switch (format) {
        case FSM_FMT_BMS: {
            // groupBy uid: groups in order of first appearance, items in line order
            std::unordered_map<int32_t, size_t> gidx;
            std::vector<std::vector<int32_t>> groups;
            for (size_t r = 0; r < lines.size(); ++r) {
                jsplit(lines[r].p, lines[r].n, '\t', parts);
                if (parts.size() < 2) bad("BMS", int64_t(r), "expected uid<TAB>pid, got '" + quote(lines[r]) + "'");
                int32_t uid, pid;
                const Line a = jtrim(parts[0]), b = jtrim(parts[1]);
                if (!jint(a.p, a.n, uid) || !jint(b.p, b.n, pid))
                    bad("BMS", int64_t(r), "NumberFormatException in '" + quote(lines[r]) + "'");
                auto it = gidx.find(uid);
                if (it == gidx.end()) {
                    it = gidx.emplace(uid, groups.size()).first;
                    groups.emplace_back();
                }
                groups[it->second].push_back(pid);
            }
            for (size_t g = 0; g < groups.size() && !o.full(); ++g) {
                for (int32_t it : groups[g]) {
                    o.tok.push_back(it);
                    o.tok.push_back(-1);
                }
                o.end_seq();
            }
            break;
        }
        case FSM_FMT_CSV:
        case FSM_FMT_KOSARAK: {
            const char sep = format == FSM_FMT_CSV ? ',' : ' ';
            const char* name = format == FSM_FMT_CSV ? "CSV" : "KOSARAK";
            for (size_t r = 0; r < lines.size(); ++r) {
                jsplit(lines[r].p, lines[r].n, sep, parts);
                for (const Line& t : parts) {
                    int32_t v;
                    if (!jint(t.p, t.n, v)) bad(name, int64_t(r), "NumberFormatException for '" + quote(t) + "'");
                    if (!o.full()) {
                        o.tok.push_back(v);
                        o.tok.push_back(-1);
                    }
                }
                o.end_seq();
            }
            break;
        }
        case FSM_FMT_SNAKE: {
            // String.length counts UTF-16 units and toCharArray yields them; ASCII input assumed
            for (size_t r = 0; r < lines.size() && !o.full(); ++r) {
                if (lines[r].n < 11) continue;
                for (int64_t i = 0; i < lines[r].n; ++i) {
                    o.tok.push_back(int64_t(uint8_t(lines[r].p[i])) - 65);
                    o.tok.push_back(-1);
                }
                o.end_seq();
            }
            break;
        }
        case FSM_FMT_SPMF:
        case FSM_FMT_INDEXED: {
            for (size_t r = 0; r < lines.size() && !o.full(); ++r) {
                Line l = lines[r];
                int32_t sid = int32_t(o.sids.size());
                if (format == FSM_FMT_INDEXED) {
                    int64_t bar = 0;
                    while (bar < l.n && l.p[bar] != '|') ++bar;
                    if (bar == l.n || !jint(l.p, bar, sid))
                        bad("INDEXED", int64_t(r), "expected idx|sequence, got '" + quote(l) + "'");
                    l.p += bar + 1;
                    l.n -= bar + 1;
                }
                jsplit(l.p, l.n, ' ', parts);
                for (const Line& t : parts) {
                    int32_t v;
                    if (t.n > 0 && t.p[0] == '<')
                        bad("SPMF", int64_t(r), "timestamped itemsets ('" + quote(t) +
                                                    "') take fsm_db_from_spmf, not the token path");
                    if (!jint(t.p, t.n, v)) bad("SPMF", int64_t(r), "NumberFormatException for '" + quote(t) + "'");
                    // the miners' parsers compare the TEXT with "-1" / "-2" (SPADE.scala:171,185):
                    // "-01" is an item there, a separator as a token
                    if ((v == -1 || v == -2) && !(t.n == 2 && t.p[0] == '-'))
                        bad("SPMF", int64_t(r), "token '" + quote(t) + "' reads as an item in the reference; "
                                                "take fsm_db_from_spmf for such input");
                    o.tok.push_back(v);
                }
                o.sids.push_back(sid);  // the tokens as they are (the miners' parsers apply -1 / -2)
                o.off.push_back(int64_t(o.tok.size()));
            }
            break;
        }
        default:
            throw Error(FSM_EINVAL, "fsm_ingest: unknown format " + std::to_string(format));
    }
}

}  // namespace fsm

using fsm::Error;

extern "C" int fsm_ingest(int32_t format, const char* data, int64_t len, int64_t limit, fsm_token_db** out) {
    if (!out || (len > 0 && !data) || len < 0) return FSM_EINVAL;
    *out = nullptr;
    try {
        fsm::Out o;
        fsm::ingest(format, data, len, limit, o);
        auto* t = static_cast<fsm_token_db*>(std::calloc(1, sizeof(fsm_token_db)));
        if (!t) return FSM_ENOMEM;
        t->n = int64_t(o.sids.size());
        t->n_tokens = int64_t(o.tok.size());
        t->sids = static_cast<int32_t*>(std::malloc(std::max<size_t>(o.sids.size(), 1) * 4));
        t->seq_off = static_cast<int64_t*>(std::malloc(o.off.size() * 8));
        t->tokens = static_cast<int64_t*>(std::malloc(std::max<size_t>(o.tok.size(), 1) * 8));
        if (!t->sids || !t->seq_off || !t->tokens) {
            fsm_token_db_free(t);
            return FSM_ENOMEM;
        }
        // empty vectors may hand out a null data(): memcpy from null is undefined even for 0 bytes
        if (!o.sids.empty()) std::memcpy(t->sids, o.sids.data(), o.sids.size() * 4);
        if (!o.off.empty()) std::memcpy(t->seq_off, o.off.data(), o.off.size() * 8);
        if (!o.tok.empty()) std::memcpy(t->tokens, o.tok.data(), o.tok.size() * 8);
        *out = t;
        return FSM_OK;
    } catch (const Error& e) {
        fsm::set_thread_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        fsm::set_thread_error("host allocation failed");
        return FSM_ENOMEM;
    }
}

extern "C" void fsm_token_db_free(fsm_token_db* t) {
    if (!t) return;
    std::free(t->sids);
    std::free(t->seq_off);
    std::free(t->tokens);
    std::free(t);
}
