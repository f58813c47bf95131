// flatten.cpp — host-side "flatten once" of the SPMF dataset (SURVEY §8a rows
// a1, a2, a6, a7, a8).  Parses every record exactly once with the reference's
// tokenizer rules and produces the row layout that is uploaded to HBM:
//
//   SPADE  SPADE.newSequence (SPADE.scala:145-212) + the seqOp bit
//          registrations (SPADE.scala:53-102): per sequence id, the distinct
//          items with the bitmask of rank-compressed timestamps (eids).
//   TSR    TSR.scala:41 (every token toInt), TSR.newSequence (:109-143) and
//          the Vertical first/last maps (:52-94): per sequence, the distinct
//          items with first/last 0-based itemset index.
//
// Records are parsed in parallel on host threads; errors are reported for the
// lowest failing record index so the outcome does not depend on scheduling.
#include <algorithm>
#include <atomic>
#include <climits>
#include <thread>
#include <unordered_map>

#include "fsm_internal.h"

namespace fsm {
namespace {

struct Tok {
    const char* p;
    int64_t n;
};

// java.lang.String.split(" ") (limit 0): "" -> [""], " " -> [], trailing
// empty strings dropped, leading / inner empty strings kept.
void split_space(const char* s, int64_t len, std::vector<Tok>& out) {
    out.clear();
    if (len == 0) {
        out.push_back({s, 0});
        return;
    }
    int64_t start = 0;
    for (int64_t i = 0; i < len; ++i) {
        if (s[i] == ' ') {
            out.push_back({s + start, i - start});
            start = i + 1;
        }
    }
    out.push_back({s + start, len - start});
    while (!out.empty() && out.back().n == 0) out.pop_back();
}

// java.lang.Long.parseLong(s, 10) over ASCII digits.
bool jparse_long(const char* p, int64_t n, int64_t& v) {
    if (n <= 0) return false;
    bool neg = false;
    int64_t i = 0;
    if (p[0] == '-' || p[0] == '+') {
        neg = p[0] == '-';
        if (n == 1) return false;
        i = 1;
    }
    const uint64_t lim = neg ? uint64_t(INT64_MAX) + 1u : uint64_t(INT64_MAX);
    uint64_t acc = 0;
    for (; i < n; ++i) {
        unsigned d = unsigned(uint8_t(p[i])) - unsigned('0');
        if (d > 9) return false;
        if (acc > (lim - d) / 10u) return false;
        acc = acc * 10u + d;
    }
    v = neg ? int64_t(0u - acc) : int64_t(acc);
    return true;
}

bool jparse_int(const char* p, int64_t n, int32_t& v) {
    int64_t w;
    if (!jparse_long(p, n, w) || w < INT32_MIN || w > INT32_MAX) return false;
    v = int32_t(w);
    return true;
}

inline bool is_lit(const Tok& t, char a, char b) { return t.n == 2 && t.p[0] == a && t.p[1] == b; }

std::string clip(const Tok& t) { return std::string(t.p, size_t(t.n > 40 ? 40 : t.n)); }

struct RecErr {
    int64_t rec = INT64_MAX;
    int code = FSM_OK;
    std::string msg;
    void set(int64_t r, int c, std::string m) {
        if (r < rec) { rec = r; code = c; msg = std::move(m); }
    }
};

int nthreads_for(int64_t n) {
    unsigned hc = std::thread::hardware_concurrency();
    int t = int(hc ? hc : 4);
    if (t > 32) t = 32;
    int64_t by_work = n / 20000 + 1;
    return int(std::min<int64_t>(t, by_work));
}

template <class F> void parallel_chunks(int64_t n, int T, F&& f) {
    if (T <= 1) { f(0, int64_t(0), n); return; }
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
        int64_t a = n * t / T, b = n * (t + 1) / T;
        th.emplace_back([&, t, a, b] { f(t, a, b); });
    }
    for (auto& x : th) x.join();
}

// SPADE record state machine (SPADE.scala:151-210). Emits (ts32, item) for
// every item of every closed itemset.
struct SpadeRec {
    int64_t ts_state = -1;  // var timestamp:Long = -1
    int64_t cur_ts = 0;     // Itemset default timestamp [EXT; 0 assumed]
    std::vector<int32_t> cur;
    void begin() { ts_state = -1; cur_ts = 0; cur.clear(); }
    void timestamp(int64_t v) { ts_state = v; cur_ts = v; }
    bool end_itemset(std::vector<uint64_t>& out) {  // false: negative ts32
        const int32_t ts32 = int32_t(uint32_t(uint64_t(cur_ts)));
        if (!cur.empty() && ts32 < 0) return false;
        for (int32_t it : cur) out.push_back((uint64_t(uint32_t(ts32)) << 32) | uint32_t(it));
        cur.clear();
        cur_ts = int64_t(uint64_t(cur_ts) + 1u);
        ts_state = int64_t(uint64_t(ts_state) + 1u);
        return true;
    }
    void item(int32_t v) {
        cur.push_back(v);
        if (ts_state < 0) { ts_state = 1; cur_ts = 1; }
    }
};

// dense remap of item values (ascending); returns value table
struct ItemMap {
    int32_t lo = 0;
    std::vector<uint32_t> direct;           // value - lo -> dense
    std::unordered_map<int32_t, uint32_t> hashed;
    std::vector<int32_t> vals;
    bool use_direct = true;
    uint32_t operator()(int32_t v) const {
        if (use_direct) return direct[size_t(int64_t(v) - lo)];
        return hashed.find(v)->second;
    }
};

void build_item_map(const std::vector<std::vector<int32_t>>& parts, ItemMap& m) {
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (auto& p : parts)
        for (int32_t v : p) { lo = std::min<int64_t>(lo, v); hi = std::max<int64_t>(hi, v); }
    if (lo > hi) { m.vals.clear(); return; }
    if (hi - lo < (int64_t(1) << 26)) {
        m.use_direct = true;
        m.lo = int32_t(lo);
        m.direct.assign(size_t(hi - lo + 1), 0);
        for (auto& p : parts)
            for (int32_t v : p) m.direct[size_t(int64_t(v) - lo)] = 1;
        uint32_t k = 0;
        for (size_t i = 0; i < m.direct.size(); ++i)
            if (m.direct[i]) { m.direct[i] = k++; m.vals.push_back(int32_t(lo + int64_t(i))); }
    } else {
        m.use_direct = false;
        std::vector<int32_t> all;
        for (auto& p : parts) all.insert(all.end(), p.begin(), p.end());
        std::sort(all.begin(), all.end());
        all.erase(std::unique(all.begin(), all.end()), all.end());
        m.vals = all;
        for (size_t i = 0; i < all.size(); ++i) m.hashed.emplace(all[i], uint32_t(i));
    }
}

}  // namespace

// --------------------------------------------------------------- SPADE
void flatten_spade(const Source& src, FlatSpade& out) {
    const int64_t n = src.n;
    out = FlatSpade();
    out.total = n;
    const int T = nthreads_for(n);
    // 1. parse every record -> packed (ts32 << 32 | item) of closed itemsets
    std::vector<std::vector<uint64_t>> pairs(static_cast<size_t>(T));
    std::vector<int64_t> rec_beg(size_t(n), 0);  // offset within its thread buffer
    std::vector<int64_t> rec_cnt(size_t(n), 0);
    std::vector<int32_t> rec_thr(size_t(n), 0);
    std::vector<RecErr> errs(static_cast<size_t>(T));
    parallel_chunks(n, T, [&](int t, int64_t a, int64_t b) {
        std::vector<Tok> toks;
        SpadeRec st;
        auto& buf = pairs[size_t(t)];
        for (int64_t r = a; r < b; ++r) {
            rec_thr[size_t(r)] = t;
            rec_beg[size_t(r)] = int64_t(buf.size());
            const int32_t sid = src.sids[r];
            if (sid < 0) {
                errs[size_t(t)].set(r, FSM_EPARSE, "SPADE: negative sequence id " + std::to_string(sid) +
                                                        " (IDListBitmap sid index)");
                break;
            }
            st.begin();
            bool ok = true;
            if (src.lines) {
                split_space(src.lines[r], src.lens[r], toks);
                for (const Tok& tk : toks) {
                    if (tk.n == 0) {
                        errs[size_t(t)].set(r, FSM_EPARSE, "SPADE parse: empty token in sid=" + std::to_string(sid) +
                                            " (StringIndexOutOfBoundsException, SPADE.scala:161)");
                        ok = false;
                        break;
                    }
                    if (tk.p[0] == '<') {
                        int64_t v;
                        if (tk.n < 2 || !jparse_long(tk.p + 1, tk.n - 2, v)) {
                            errs[size_t(t)].set(r, FSM_EPARSE, "SPADE parse: bad timestamp token '" + clip(tk) +
                                                "' in sid=" + std::to_string(sid) + " (SPADE.scala:166-168)");
                            ok = false;
                            break;
                        }
                        st.timestamp(v);
                    } else if (is_lit(tk, '-', '1')) {
                        if (!st.end_itemset(buf)) {
                            errs[size_t(t)].set(r, FSM_EPARSE, "SPADE: negative timestamp in sid=" +
                                                std::to_string(sid) + " (IDListBitmap.registerBit, SPADE.scala:74,90)");
                            ok = false;
                            break;
                        }
                    } else if (is_lit(tk, '-', '2')) {
                    } else {
                        int32_t v;
                        if (!jparse_int(tk.p, tk.n, v)) {
                            errs[size_t(t)].set(r, FSM_EPARSE, "SPADE parse: bad item token '" + clip(tk) +
                                                "' in sid=" + std::to_string(sid) + " (NumberFormatException, SPADE.scala:194)");
                            ok = false;
                            break;
                        }
                        st.item(v);
                    }
                }
            } else {
                for (int64_t q = src.seq_off[r]; q < src.seq_off[r + 1]; ++q) {
                    const int64_t v = src.tokens[q];
                    if (v == -1) {
                        st.end_itemset(buf);  // implicit timestamps are never negative
                    } else if (v == -2) {
                    } else if (v < INT32_MIN || v > INT32_MAX) {
                        errs[size_t(t)].set(r, FSM_EPARSE, "SPADE: token " + std::to_string(v) +
                                            " does not fit an Int item (sid=" + std::to_string(sid) + ")");
                        ok = false;
                        break;
                    } else {
                        st.item(int32_t(v));
                    }
                }
            }
            if (!ok) break;
            rec_cnt[size_t(r)] = int64_t(buf.size()) - rec_beg[size_t(r)];
        }
    });
    RecErr first;
    for (auto& e : errs) if (e.rec < first.rec) first = e;
    if (first.rec != INT64_MAX) throw Error(first.code, first.msg);

    // 2. group records by sid (stable); equal sids share one id-list row
    std::vector<int64_t> order(static_cast<size_t>(n));
    for (int64_t r = 0; r < n; ++r) order[size_t(r)] = r;
    bool sorted = true;
    for (int64_t r = 1; r < n && sorted; ++r) sorted = src.sids[r] > src.sids[r - 1];
    if (!sorted)
        std::stable_sort(order.begin(), order.end(),
                         [&](int64_t a, int64_t b) { return src.sids[a] < src.sids[b]; });
    std::vector<int64_t> grp;  // start positions in order[] of each distinct sid
    for (int64_t q = 0; q < n; ++q)
        if (q == 0 || src.sids[order[size_t(q)]] != src.sids[order[size_t(q - 1)]]) grp.push_back(q);
    const int64_t R = int64_t(grp.size());
    grp.push_back(n);

    // 3. per row: eid ranks by distinct timestamp, distinct items with masks
    const int T2 = nthreads_for(R);
    std::vector<std::vector<int32_t>> ent_val(static_cast<size_t>(T2));
    std::vector<std::vector<uint64_t>> ent_msk(static_cast<size_t>(T2));   // row_words words per entry
    std::vector<std::vector<uint32_t>> row_len(static_cast<size_t>(T2));
    std::vector<std::vector<uint16_t>> row_words(static_cast<size_t>(T2));
    std::vector<int> maxE(size_t(T2), 0);
    std::vector<int64_t> maxOcc(size_t(T2), 0);
    parallel_chunks(R, T2, [&](int t, int64_t a, int64_t b) {
        std::vector<uint64_t> buf, m;
        std::vector<std::pair<int32_t, int32_t>> ie;  // (item, eid)
        auto& ev = ent_val[size_t(t)];
        auto& em = ent_msk[size_t(t)];
        auto& rl = row_len[size_t(t)];
        auto& rw = row_words[size_t(t)];
        for (int64_t g = a; g < b; ++g) {
            buf.clear();
            for (int64_t q = grp[size_t(g)]; q < grp[size_t(g + 1)]; ++q) {
                const int64_t r = order[size_t(q)];
                const auto& pb = pairs[size_t(rec_thr[size_t(r)])];
                buf.insert(buf.end(), pb.begin() + rec_beg[size_t(r)],
                           pb.begin() + rec_beg[size_t(r)] + rec_cnt[size_t(r)]);
            }
            std::sort(buf.begin(), buf.end());  // by ts (non-negative), then item bits
            ie.clear();
            int32_t e = -1;
            uint32_t last_ts = 0;
            for (size_t q = 0; q < buf.size(); ++q) {
                const uint32_t ts = uint32_t(buf[q] >> 32);
                if (q == 0 || ts != last_ts) ++e;
                last_ts = ts;
                ie.push_back({int32_t(uint32_t(buf[q])), e});
            }
            maxE[size_t(t)] = std::max(maxE[size_t(t)], e + 1);
            maxOcc[size_t(t)] = std::max<int64_t>(maxOcc[size_t(t)], int64_t(ie.size()));
            const int wr = std::max(1, std::min(int(kMaxMaskWords), (e + 1 + 63) / 64));
            std::sort(ie.begin(), ie.end());
            uint32_t len = 0;
            for (size_t q = 0; q < ie.size();) {
                size_t s = q;
                m.assign(size_t(wr), 0);
                while (q < ie.size() && ie[q].first == ie[s].first) {
                    const int32_t ee = ie[q].second;
                    if (ee < int32_t(64 * kMaxMaskWords)) m[size_t(ee >> 6)] |= 1ull << (ee & 63);
                    ++q;
                }
                ev.push_back(ie[s].first);
                em.insert(em.end(), m.begin(), m.end());
                ++len;
            }
            rl.push_back(len);
            rw.push_back(uint16_t(wr - 1));
        }
    });
    int mE = 0;
    for (int v : maxE) mE = std::max(mE, v);
    for (int64_t v : maxOcc) out.max_occ = std::max(out.max_occ, v);
    if (mE > int(64 * kMaxMaskWords))
        throw Error(FSM_ELIMIT, "SPADE: a sequence has " + std::to_string(mE) +
                                    " distinct timestamps; the engine supports up to " +
                                    std::to_string(64 * kMaxMaskWords));
    int W = 1;
    while (W * 64 < mE) W *= 2;
    out.W = W;

    ItemMap imap;
    build_item_map(ent_val, imap);
    out.item_val = imap.vals;
    int64_t E = 0;
    for (auto& v : ent_val) E += int64_t(v.size());
    if (E >= (int64_t(1) << 32)) throw Error(FSM_ELIMIT, "SPADE: more than 2^32 (item, sid) entries");
    out.row_off.resize(size_t(R) + 1);
    out.ent_item.resize(size_t(E));
    out.ent_mask.assign(size_t(E) * size_t(W), 0);
    int64_t row = 0, e = 0;
    out.row_off[0] = 0;
    for (int t = 0; t < T2; ++t) {
        const auto& ev = ent_val[size_t(t)];
        const auto& em = ent_msk[size_t(t)];
        size_t q = 0, mo = 0;
        for (size_t k = 0; k < row_len[size_t(t)].size(); ++k) {
            const uint32_t len = row_len[size_t(t)][k];
            const size_t wr = size_t(row_words[size_t(t)][k]) + 1;
            out.row_off[size_t(row + 1)] = out.row_off[size_t(row)] + len;
            ++row;
            for (uint32_t x = 0; x < len; ++x, ++q, ++e, mo += wr) {
                out.ent_item[size_t(e)] = imap(ev[q]);
                std::memcpy(&out.ent_mask[size_t(e) * size_t(W)], &em[mo], sizeof(uint64_t) * wr);
            }
        }
    }
}

// ----------------------------------------------------------------- TSR
void flatten_tsr(const Source& src, FlatTsr& out) {
    const int64_t n = src.n;
    out = FlatTsr();
    out.total = n;
    const int T = nthreads_for(n);
    std::vector<std::vector<int32_t>> ent_val(static_cast<size_t>(T));
    std::vector<std::vector<uint32_t>> ent_f(static_cast<size_t>(T)), ent_l(static_cast<size_t>(T)), row_len(static_cast<size_t>(T));
    std::vector<RecErr> errs(static_cast<size_t>(T));
    std::vector<char> any(size_t(T), 0);
    parallel_chunks(n, T, [&](int t, int64_t a, int64_t b) {
        std::vector<Tok> toks;
        std::vector<int32_t> vals;
        std::vector<std::pair<int32_t, uint32_t>> ip;  // (item, itemset index)
        auto& er = errs[size_t(t)];
        for (int64_t r = a; r < b; ++r) {
            if (src.sids[r] != int32_t(r)) {
                er.set(r, FSM_EPARSE, "TSR: sequence ids must be dense 0..N-1 in input order "
                                      "(TSR.scala:95,103 index sequences by sid); record " +
                                          std::to_string(r) + " has sid " + std::to_string(src.sids[r]));
                break;
            }
            ip.clear();
            uint32_t pos = 0;
            size_t open_from = 0;  // ip index where the open itemset starts
            bool ok = true;
            // negative items are checked once the trailing itemset is dropped: only those of
            // closed itemsets index the Vertical arrays (TSR.scala:63-75)
            auto item = [&](int64_t v, const std::string&) {
                ip.push_back({int32_t(v), pos});
                return true;
            };
            if (src.lines) {
                split_space(src.lines[r], src.lens[r], toks);
                vals.resize(toks.size());
                for (size_t q = 0; q < toks.size(); ++q) {  // TSR.scala:41: every token toInt
                    if (!jparse_int(toks[q].p, toks[q].n, vals[q])) {
                        er.set(r, FSM_EPARSE, "TSR parse: bad token '" + clip(toks[q]) + "' in sid=" +
                                                  std::to_string(r) + " (NumberFormatException, TSR.scala:41)");
                        ok = false;
                        break;
                    }
                    if (vals[q] > -1) any[size_t(t)] = 1;
                }
                for (size_t q = 0; ok && q < toks.size(); ++q) {
                    if (is_lit(toks[q], '-', '1')) { ++pos; open_from = ip.size(); }
                    else if (is_lit(toks[q], '-', '2')) {}
                    else ok = item(vals[q], clip(toks[q]));
                }
            } else {
                for (int64_t q = src.seq_off[r]; ok && q < src.seq_off[r + 1]; ++q) {
                    const int64_t v = src.tokens[q];
                    if (v < INT32_MIN || v > INT32_MAX) {
                        er.set(r, FSM_EPARSE, "TSR: token " + std::to_string(v) + " does not fit an Int");
                        ok = false;
                    } else if (v == -1) { ++pos; open_from = ip.size(); }
                    else if (v == -2) {}
                    else { if (v > -1) any[size_t(t)] = 1; ok = item(v, std::to_string(v)); }
                }
            }
            if (!ok) break;
            ip.resize(open_from);  // items after the last -1 are dropped
            for (const auto& x : ip)
                if (x.first < 0) {
                    er.set(r, FSM_EPARSE, "TSR: negative item " + std::to_string(x.first) + " in sid=" +
                                              std::to_string(r) + " (Vertical array index)");
                    ok = false;
                    break;
                }
            if (!ok) break;
            std::sort(ip.begin(), ip.end());
            uint32_t len = 0;
            for (size_t q = 0; q < ip.size();) {
                size_t s = q;
                while (q < ip.size() && ip[q].first == ip[s].first) ++q;
                ent_val[size_t(t)].push_back(ip[s].first);
                ent_f[size_t(t)].push_back(ip[s].second);
                ent_l[size_t(t)].push_back(ip[q - 1].second);
                ++len;
            }
            row_len[size_t(t)].push_back(len);
        }
    });
    RecErr first;
    for (auto& e : errs) if (e.rec < first.rec) first = e;
    if (first.rec != INT64_MAX) throw Error(first.code, first.msg);
    bool anyi = false;
    for (char c : any) anyi |= c != 0;
    if (!anyi) throw Error(FSM_EPARSE, "TSR: no items in dataset (empty.max at TSR.scala:43)");

    ItemMap imap;
    build_item_map(ent_val, imap);
    out.item_val = imap.vals;
    int64_t E = 0;
    for (auto& v : ent_val) E += int64_t(v.size());
    if (E >= (int64_t(1) << 32)) throw Error(FSM_ELIMIT, "TSR: more than 2^32 (item, sid) entries");
    out.row_off.assign(size_t(n) + 1, 0);
    out.ent_item.resize(size_t(E));
    out.ent_first.resize(size_t(E));
    out.ent_last.resize(size_t(E));
    int64_t row = 0, e = 0;
    for (int t = 0; t < T; ++t) {
        for (uint32_t len : row_len[size_t(t)]) {
            out.row_off[size_t(row + 1)] = out.row_off[size_t(row)] + len;
            ++row;
        }
        for (size_t q = 0; q < ent_val[size_t(t)].size(); ++q, ++e) {
            out.ent_item[size_t(e)] = imap(ent_val[size_t(t)][q]);
            out.ent_first[size_t(e)] = ent_f[size_t(t)][q];
            out.ent_last[size_t(e)] = ent_l[size_t(t)][q];
        }
    }
}

}  // namespace fsm
