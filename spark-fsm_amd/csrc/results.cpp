// results.cpp — what happens to the mined results after the hot path
// (SURVEY §8f rows 3 and 4), done in bulk straight from the result CSR.
//
// Persistence (row 3).  SPADEActor maps every pattern through serialize() and
// stores Patterns(List[Pattern(support, itemsets)]) (SPADEActor.scala:47-68);
// TSRActor stores Rules(List[Rule(antecedent, consequent, support, total,
// confidence)]) (TSRActor.scala:52-71).  Both go to Redis through the
// unvendored de.kp.spark.core RedisDB, whose documents are json4s
// Serialization.write of those case classes (model/Model.scala:20-24 imports
// it): fields in constructor order, doubles as java.lang.Double.toString.
//   fsm_patterns_serialize  one serialize() line per pattern ("1 2 -1 3 -1 | 42")
//   fsm_patterns_json       {"items":[{"support":42,"itemsets":[[1,2],[3]]},...]}
//   fsm_rules_json          {"items":[{"antecedent":[1],"consequent":[2],"support":2,
//                            "total":3,"confidence":0.6666666666666666},...]}
// [EXT: the document layout is json4s' for those case classes; the Redis keys
// and the ElasticSink / JdbcSink field names live in unvendored code.]
//
// Queries (row 4).  FSMQuestor's get:antecedent / get:consequent
// (FSMQuestor.scala:46-98) answer with RedisDB.rulesByAntecedent /
// rulesByConsequent(items) [EXT, unvendored]; restated as: the rules whose
// antecedent (consequent) items all occur in the query items.
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <string>

#include "fsm_internal.h"

namespace fsm {
namespace {

// java.lang.Double.toString for finite doubles: the shortest digits that round
// trip; plain notation with at least one fraction digit for 1e-3 <= |d| < 1e7,
// else d.dddE[-]n.  (Java 8's FloatingDecimal is not always shortest; the
// values mined here - confidences in (0, 1] - print the same.)
void java_double(std::string& out, double d) {
    if (d == 0.0) {
        out += std::signbit(d) ? "-0.0" : "0.0";
        return;
    }
    char buf[64];
    const auto res = std::to_chars(buf, buf + sizeof buf, d, std::chars_format::scientific);
    std::string sci(buf, res.ptr);  // e.g. "-6.666666666666666e-01"
    bool neg = false;
    if (sci[0] == '-') {
        neg = true;
        sci.erase(0, 1);
    }
    const size_t e = sci.find('e');
    std::string digits = sci.substr(0, e);
    digits.erase(std::remove(digits.begin(), digits.end(), '.'), digits.end());
    const int exp10 = std::stoi(sci.substr(e + 1));
    if (neg) out += '-';
    const double a = std::fabs(d);
    if (a >= 1e-3 && a < 1e7) {
        if (exp10 >= 0) {
            const size_t ip = size_t(exp10) + 1;
            std::string intpart = digits.substr(0, std::min(ip, digits.size()));
            while (intpart.size() < ip) intpart += '0';
            std::string frac = ip < digits.size() ? digits.substr(ip) : "0";
            out += intpart + "." + frac;
        } else {
            out += "0.";
            out.append(size_t(-exp10 - 1), '0');
            out += digits;
        }
    } else {
        out += digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(exp10);
    }
}

char* hand_out(const std::string& s, int64_t* len) {
    char* p = static_cast<char*>(std::malloc(s.size() + 1));
    if (!p) throw std::bad_alloc();
    std::memcpy(p, s.data(), s.size());
    p[s.size()] = 0;
    *len = int64_t(s.size());
    return p;
}

void int_list(std::string& o, const int32_t* a, int64_t b, int64_t e) {
    o += '[';
    for (int64_t q = b; q < e; ++q) {
        if (q > b) o += ',';
        o += std::to_string(a[q]);
    }
    o += ']';
}

template <class F> int guarded(F&& f) {
    try {
        f();
        return FSM_OK;
    } catch (const Error& e) {
        set_thread_error(e.what());
        return e.code;
    } catch (const std::bad_alloc&) {
        set_thread_error("host allocation failed");
        return FSM_ENOMEM;
    }
}

}  // namespace
}  // namespace fsm

extern "C" {

int fsm_patterns_serialize(const fsm_patterns* p, char** out, int64_t* len) {
    if (!p || !out || !len) return FSM_EINVAL;
    return fsm::guarded([&] {
        std::string s;
        s.reserve(size_t(p->n_items) * 4 + size_t(p->n_sets) * 4 + size_t(p->n) * 8);
        for (int64_t k = 0; k < p->n; ++k) {
            for (int64_t q = p->pat_off[k]; q < p->pat_off[k + 1]; ++q) {
                for (int64_t i = p->set_off[q]; i < p->set_off[q + 1]; ++i) {
                    if (i > p->set_off[q]) s += ' ';
                    s += std::to_string(p->items[i]);
                }
                s += " -1 ";
            }
            s += "| " + std::to_string(p->support[k]) + "\n";
        }
        *out = fsm::hand_out(s, len);
    });
}

int fsm_patterns_json(const fsm_patterns* p, char** out, int64_t* len) {
    if (!p || !out || !len) return FSM_EINVAL;
    return fsm::guarded([&] {
        std::string s = "{\"items\":[";
        for (int64_t k = 0; k < p->n; ++k) {
            if (k) s += ',';
            s += "{\"support\":" + std::to_string(p->support[k]) + ",\"itemsets\":[";
            for (int64_t q = p->pat_off[k]; q < p->pat_off[k + 1]; ++q) {
                if (q > p->pat_off[k]) s += ',';
                fsm::int_list(s, p->items, p->set_off[q], p->set_off[q + 1]);
            }
            s += "]}";
        }
        s += "]}";
        *out = fsm::hand_out(s, len);
    });
}

int fsm_rules_json(const fsm_rules* r, char** out, int64_t* len) {
    if (!r || !out || !len) return FSM_EINVAL;
    return fsm::guarded([&] {
        std::string s = "{\"items\":[";
        for (int64_t k = 0; k < r->n; ++k) {
            if (k) s += ',';
            s += "{\"antecedent\":";
            fsm::int_list(s, r->ante, r->ante_off[k], r->ante_off[k + 1]);
            s += ",\"consequent\":";
            fsm::int_list(s, r->cons, r->cons_off[k], r->cons_off[k + 1]);
            s += ",\"support\":" + std::to_string(r->support[k]) + ",\"total\":" + std::to_string(r->total) +
                 ",\"confidence\":";
            fsm::java_double(s, r->confidence[k]);
            s += '}';
        }
        s += "]}";
        *out = fsm::hand_out(s, len);
    });
}

void fsm_buffer_free(char* p) { std::free(p); }

int fsm_rules_query(const fsm_rules* r, int32_t side, const int32_t* items, int64_t n, int64_t* out_idx,
                    int64_t* n_out) {
    if (!r || !n_out || (n > 0 && !items) || (r->n > 0 && !out_idx) || (side != 0 && side != 1))
        return FSM_EINVAL;
    return fsm::guarded([&] {
        std::vector<int32_t> q(items, items + std::max<int64_t>(n, 0));
        std::sort(q.begin(), q.end());
        const int64_t* off = side == 0 ? r->ante_off : r->cons_off;
        const int32_t* it = side == 0 ? r->ante : r->cons;
        int64_t m = 0;
        for (int64_t k = 0; k < r->n; ++k) {
            bool all = true;
            for (int64_t i = off[k]; i < off[k + 1] && all; ++i) all = std::binary_search(q.begin(), q.end(), it[i]);
            if (all) out_idx[m++] = k;
        }
        *n_out = m;
    });
}

}  // extern "C"
