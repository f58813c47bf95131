// parsers_harness.cpp — CPU sanitizer harness for libfsm's host parsers
// (TEST INFRASTRUCTURE; VERDICT r2 "weak" 11 / "next round" 8).
//
// flatten.cpp (SPADE.scala:145-212 / TSR.scala:109-143 line and token parsing),
// ingest.cpp (util/SPMFBuilder.scala formats) and results.cpp (result documents
// and rule queries) take untrusted input.  tests/fuzz/Makefile compiles those
// three sources unchanged, with g++ -fsanitize=address,undefined (host code
// only: no GPU code is involved), into this driver; tests/test_fuzz.py feeds it
// hypothesis-generated malformed input and requires a clean exit: every bad
// input must come back as an fsm error, never as a sanitizer report.
//
// Input (stdin): a sequence of cases, each  u8 kind | u32 payload length | payload
//   kind 0 / 1  SPADE / TSR lines:  u32 n, then n x (i32 sid, u32 len, bytes)
//   kind 2 / 3  SPADE / TSR tokens: u32 n, then n x (i32 sid, u32 ntok, i64 tokens[ntok])
//   kind 4      ingest:             i32 format, i64 limit, then the file image
//   kind 5      result documents:   u32 n patterns / rules made from the payload ints
// Output: one line per case, "<kind> ok|err <code>".
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../spark-fsm_amd/csrc/fsm_internal.h"

namespace fsm {
// fsm_api.cpp (not linked here) keeps the context-free error message
void set_thread_error(const std::string&) {}
}  // namespace fsm

namespace {

struct Reader {
    const uint8_t* p;
    size_t n, at = 0;
    bool ok = true;
    template <class T> T get() {
        T v{};
        if (at + sizeof(T) > n) {
            ok = false;
            return v;
        }
        std::memcpy(&v, p + at, sizeof(T));
        at += sizeof(T);
        return v;
    }
    const char* bytes(size_t k) {
        if (at + k > n) {
            ok = false;
            return nullptr;
        }
        const char* q = reinterpret_cast<const char*>(p + at);
        at += k;
        return q;
    }
};

int run_lines(Reader& r, bool tsr) {
    const uint32_t n = r.get<uint32_t>();
    std::vector<int32_t> sids;
    std::vector<std::string> text;
    for (uint32_t i = 0; i < n && r.ok; ++i) {
        sids.push_back(r.get<int32_t>());
        const uint32_t len = r.get<uint32_t>();
        const char* b = r.bytes(len);
        text.emplace_back(b ? b : "", b ? len : 0);
    }
    if (!r.ok) return -1;
    // each line in its own exact-size heap block: an overread of a line is a sanitizer report
    std::vector<std::unique_ptr<char[]>> own;
    std::vector<const char*> lines;
    std::vector<int64_t> lens;
    for (const std::string& t : text) {
        own.emplace_back(new char[t.size() ? t.size() : 1]);
        if (!t.empty()) std::memcpy(own.back().get(), t.data(), t.size());
        lines.push_back(own.back().get());
        lens.push_back(int64_t(t.size()));
    }
    fsm::Source src;
    src.sids = sids.data();
    src.lines = lines.data();
    src.lens = lens.data();
    src.n = int64_t(n);
    try {
        if (tsr) {
            fsm::FlatTsr f;
            fsm::flatten_tsr(src, f);
        } else {
            fsm::FlatSpade f;
            fsm::flatten_spade(src, f);
        }
    } catch (const fsm::Error& e) {
        return e.code;
    }
    return 0;
}

int run_tokens(Reader& r, bool tsr) {
    const uint32_t n = r.get<uint32_t>();
    std::vector<int32_t> sids;
    std::vector<int64_t> off{0}, tok;
    for (uint32_t i = 0; i < n && r.ok; ++i) {
        sids.push_back(r.get<int32_t>());
        const uint32_t k = r.get<uint32_t>();
        for (uint32_t j = 0; j < k && r.ok; ++j) tok.push_back(r.get<int64_t>());
        off.push_back(int64_t(tok.size()));
    }
    if (!r.ok) return -1;
    std::unique_ptr<int64_t[]> tk(new int64_t[tok.empty() ? 1 : tok.size()]);
    if (!tok.empty()) std::memcpy(tk.get(), tok.data(), tok.size() * 8);
    fsm::Source src;
    src.sids = sids.data();
    src.seq_off = off.data();
    src.tokens = tk.get();
    src.n = int64_t(n);
    try {
        if (tsr) {
            fsm::FlatTsr f;
            fsm::flatten_tsr(src, f);
        } else {
            fsm::FlatSpade f;
            fsm::flatten_spade(src, f);
        }
    } catch (const fsm::Error& e) {
        return e.code;
    }
    return 0;
}

int run_ingest(Reader& r) {
    const int32_t fmt = r.get<int32_t>();
    const int64_t limit = r.get<int64_t>();
    if (!r.ok) return -1;
    const size_t len = r.n - r.at;
    std::unique_ptr<char[]> img(new char[len ? len : 1]);  // exact size, no terminator
    if (len) std::memcpy(img.get(), r.bytes(len), len);
    fsm_token_db* t = nullptr;
    const int rc = fsm_ingest(fmt, img.get(), int64_t(len), limit, &t);
    if (rc == 0) fsm_token_db_free(t);
    return rc;
}

// patterns and rules made from the payload ints (structurally valid CSR, arbitrary values)
int run_results(Reader& r) {
    const uint32_t n = r.get<uint32_t>() % 64;
    std::vector<int32_t> v;
    while (r.ok && r.at + 4 <= r.n) v.push_back(r.get<int32_t>());
    if (v.empty()) v.push_back(0);
    size_t at = 0;
    auto next = [&] { return v[at++ % v.size()]; };
    std::vector<int32_t> sup, items, ante, cons;
    std::vector<int64_t> pat_off{0}, set_off{0}, aoff{0}, coff{0};
    std::vector<double> conf;
    for (uint32_t i = 0; i < n; ++i) {
        const int ns = 1 + (next() & 3);
        for (int s = 0; s < ns; ++s) {
            const int ni = 1 + (next() & 3);
            for (int k = 0; k < ni; ++k) items.push_back(next());
            set_off.push_back(int64_t(items.size()));
        }
        pat_off.push_back(int64_t(set_off.size()) - 1);
        sup.push_back(next());
        for (int k = 0, m = 1 + (next() & 3); k < m; ++k) ante.push_back(next());
        for (int k = 0, m = 1 + (next() & 3); k < m; ++k) cons.push_back(next());
        aoff.push_back(int64_t(ante.size()));
        coff.push_back(int64_t(cons.size()));
        const int32_t a = next(), b = next();
        conf.push_back(b ? double(a) / double(b) : 0.5);
    }
    fsm_patterns p{};
    p.n = int64_t(n);
    p.support = sup.data();
    p.pat_off = pat_off.data();
    p.set_off = set_off.data();
    p.items = items.data();
    p.n_sets = int64_t(set_off.size()) - 1;
    p.n_items = int64_t(items.size());
    fsm_rules q{};
    q.n = int64_t(n);
    q.support = sup.data();
    q.confidence = conf.data();
    q.ante_off = aoff.data();
    q.ante = ante.data();
    q.cons_off = coff.data();
    q.cons = cons.data();
    q.total = next();
    char* out = nullptr;
    int64_t len = 0;
    int rc = fsm_patterns_serialize(&p, &out, &len);
    if (rc == 0) fsm_buffer_free(out);
    if (rc == 0 && (rc = fsm_patterns_json(&p, &out, &len)) == 0) fsm_buffer_free(out);
    if (rc == 0 && (rc = fsm_rules_json(&q, &out, &len)) == 0) fsm_buffer_free(out);
    std::vector<int64_t> idx(n + 1);
    int64_t nq = 0;
    std::vector<int32_t> probe(v.begin(), v.begin() + std::min<size_t>(v.size(), 8));
    if (rc == 0) rc = fsm_rules_query(&q, next() & 1, probe.data(), int64_t(probe.size()), idx.data(), &nq);
    return rc;
}

}  // namespace


int main() {
    std::vector<uint8_t> in;
    uint8_t buf[65536];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, stdin)) > 0) in.insert(in.end(), buf, buf + k);
    Reader all{in.data(), in.size()};
    while (all.at < all.n) {
        const uint8_t kind = all.get<uint8_t>();
        const uint32_t plen = all.get<uint32_t>();
        const char* pl = all.bytes(plen);
        if (!all.ok) return 2;
        Reader r{reinterpret_cast<const uint8_t*>(pl), plen};
        int rc = -1;
        switch (kind) {
            case 0: rc = run_lines(r, false); break;
            case 1: rc = run_lines(r, true); break;
            case 2: rc = run_tokens(r, false); break;
            case 3: rc = run_tokens(r, true); break;
            case 4: rc = run_ingest(r); break;
            case 5: rc = run_results(r); break;
            default: return 2;
        }
        std::printf("%u %s %d\n", unsigned(kind), rc == 0 ? "ok" : "err", rc);
    }
    return 0;
}
