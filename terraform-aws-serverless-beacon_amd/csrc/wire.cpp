// wire.cpp — the performQuery Lambda at the wire: event JSON in, response
// JSON out, for a whole batch of events in one call.
//
// Reference: lambda/performQuery/lambda_function.py:23-49 — the event (a
// PerformQueryPayload, or its SNS envelope whose Records[0].Sns.Message is
// the payload's JSON text) is loaded with jsons.load into a
// PerformQueryPayload (shared_resources/payloads/lambda_payloads.py:46-77),
// answered by search_variants(.._in_samples).perform_query, and the handler
// returns response.dump() (lambda_responses.py:14-23), which the Lambda
// runtime serialises with json.dumps.  Here the events are parsed in C++,
// every event of the batch is answered by ONE sb_query_batch per store, and
// each response is written as the text json.dumps(response.dump()) gives
// (ensure_ascii escapes, ", " / ": " separators, the dataclass field order).
// An event outside the typed fast path (a field of an unexpected JSON type,
// a key PerformQueryPayload does not take, a vcf_location no store holds,
// invalid UTF-8 or a lone surrogate) is returned with status 1 and no text:
// the caller answers it through the Python handler, which reproduces the
// reference's behaviour (including the exception it raises).
//
// Only the public C ABI (include/sbeacon.h) is used below the parser.
#include <array>
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <sys/mman.h>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "config.hpp"
#include "common.hpp"
#include "jsonesc.hpp"
#include "jsonout.hpp"

namespace sb {
namespace {
// the formatting threads' buffers, kept across calls (capacity already
// faulted in); a concurrent call formats into buffers of its own
std::mutex g_tbuf_mu;
std::vector<std::string> g_tbuf;
}  // namespace
}  // namespace sb

namespace sb {
namespace {

// ------------------------------------------------------------------ JSON DOM
// What Python's json.loads accepts (strict mode: no raw control characters in
// strings; NaN / Infinity literals are accepted and typed as floats).
struct JVal {
    enum Kind : uint8_t { NUL, BOOL, INT, FLOAT, STR, ARR, OBJ } kind = NUL;
    bool b = false;
    bool big = false;  // an integer beyond int64 (Python keeps it exactly; never a fast-path value)
    int64_t i = 0;
    std::string s;     // STR: UTF-8
    std::vector<JVal> a;
    std::vector<std::pair<std::string, JVal>> o;  // insertion order; duplicate keys: the last wins (dict semantics)

    const JVal *get(const char *key) const {
        const JVal *r = nullptr;
        for (const auto &kv : o)
            if (kv.first == key) r = &kv.second;
        return r;
    }
};

struct Parser {
    const char *p, *e;
    bool bad = false;  // not valid JSON, or outside what the fast path carries (lone surrogate, bad UTF-8)

    void ws() {
        while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) ++p;
    }
    bool lit(const char *w) {
        const size_t n = strlen(w);
        if (static_cast<size_t>(e - p) < n || memcmp(p, w, n) != 0) return false;
        p += n;
        return true;
    }
    static void put_utf8(std::string &o, uint32_t cp) {
        if (cp < 0x80) {
            o.push_back(static_cast<char>(cp));
        } else if (cp < 0x800) {
            o.push_back(static_cast<char>(0xc0 | (cp >> 6)));
            o.push_back(static_cast<char>(0x80 | (cp & 0x3f)));
        } else if (cp < 0x10000) {
            o.push_back(static_cast<char>(0xe0 | (cp >> 12)));
            o.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3f)));
            o.push_back(static_cast<char>(0x80 | (cp & 0x3f)));
        } else {
            o.push_back(static_cast<char>(0xf0 | (cp >> 18)));
            o.push_back(static_cast<char>(0x80 | ((cp >> 12) & 0x3f)));
            o.push_back(static_cast<char>(0x80 | ((cp >> 6) & 0x3f)));
            o.push_back(static_cast<char>(0x80 | (cp & 0x3f)));
        }
    }
    int hex4() {
        if (e - p < 4) return -1;
        int v = 0;
        for (int k = 0; k < 4; ++k) {
            const char c = p[k];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= c - '0';
            else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
            else return -1;
        }
        p += 4;
        return v;
    }
    bool str(std::string &o) {  // at the opening quote
        ++p;
        while (true) {
            if (p >= e) return false;
            const unsigned char c = static_cast<unsigned char>(*p);
            if (c == '"') {
                ++p;
                return true;
            }
            if (c < 0x20) return false;  // strict json.loads
            if (c == '\\') {
                if (++p >= e) return false;
                const char x = *p++;
                switch (x) {
                    case '"': o.push_back('"'); break;
                    case '\\': o.push_back('\\'); break;
                    case '/': o.push_back('/'); break;
                    case 'b': o.push_back('\b'); break;
                    case 'f': o.push_back('\f'); break;
                    case 'n': o.push_back('\n'); break;
                    case 'r': o.push_back('\r'); break;
                    case 't': o.push_back('\t'); break;
                    case 'u': {
                        int u = hex4();
                        if (u < 0) return false;
                        uint32_t cp = static_cast<uint32_t>(u);
                        if (cp >= 0xd800 && cp < 0xdc00) {  // a high surrogate needs its low half
                            if (e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                                p += 2;
                                const int lo = hex4();
                                if (lo < 0) return false;
                                if (lo < 0xdc00 || lo >= 0xe000) {
                                    bad = true;
                                    return true;
                                }
                                cp = 0x10000 + ((cp - 0xd800) << 10) + (static_cast<uint32_t>(lo) - 0xdc00);
                            } else {
                                bad = true;  // lone surrogate: Python keeps it; not UTF-8 representable
                                return true;
                            }
                        } else if (cp >= 0xdc00 && cp < 0xe000) {
                            bad = true;
                            return true;
                        }
                        put_utf8(o, cp);
                        break;
                    }
                    default: return false;
                }
                continue;
            }
            // raw bytes: must be valid UTF-8 (the event text is decoded as UTF-8);
            // a run of plain ASCII is appended at once
            if (c < 0x80) {
                const char *q = p + 1;
                while (q < e) {
                    const unsigned char d = static_cast<unsigned char>(*q);
                    if (d < 0x20 || d >= 0x80 || d == '"' || d == '\\') break;
                    ++q;
                }
                o.append(p, static_cast<size_t>(q - p));
                p = q;
                continue;
            }
            const int n = (c & 0xe0) == 0xc0 ? 2 : (c & 0xf0) == 0xe0 ? 3 : (c & 0xf8) == 0xf0 ? 4 : 0;
            if (!n || e - p < n) {
                bad = true;
                return true;
            }
            uint32_t cp = c & (0x7f >> n);
            for (int k = 1; k < n; ++k) {
                const unsigned char cc = static_cast<unsigned char>(p[k]);
                if ((cc & 0xc0) != 0x80) {
                    bad = true;
                    return true;
                }
                cp = (cp << 6) | (cc & 0x3f);
            }
            if ((n == 2 && cp < 0x80) || (n == 3 && cp < 0x800) || (n == 4 && (cp < 0x10000 || cp > 0x10ffff)) ||
                (cp >= 0xd800 && cp < 0xe000)) {
                bad = true;
                return true;
            }
            o.append(p, static_cast<size_t>(n));
            p += n;
        }
    }
    bool num(JVal &v) {
        const char *s0 = p;
        if (p < e && *p == '-') ++p;
        if (p >= e) return false;
        if (*p == '0') {
            ++p;
        } else if (*p >= '1' && *p <= '9') {
            while (p < e && *p >= '0' && *p <= '9') ++p;
        } else {
            return false;
        }
        bool is_int = true;
        if (p < e && *p == '.') {
            is_int = false;
            ++p;
            if (p >= e || *p < '0' || *p > '9') return false;
            while (p < e && *p >= '0' && *p <= '9') ++p;
        }
        if (p < e && (*p == 'e' || *p == 'E')) {
            is_int = false;
            ++p;
            if (p < e && (*p == '+' || *p == '-')) ++p;
            if (p >= e || *p < '0' || *p > '9') return false;
            while (p < e && *p >= '0' && *p <= '9') ++p;
        }
        if (!is_int) {
            v.kind = JVal::FLOAT;
            return true;
        }
        v.kind = JVal::INT;
        const bool neg = *s0 == '-';
        uint64_t m = 0;
        for (const char *q = s0 + (neg ? 1 : 0); q < p; ++q) {
            const uint64_t d = static_cast<uint64_t>(*q - '0');
            if (m > (UINT64_MAX - d) / 10) {
                v.big = true;
                return true;
            }
            m = m * 10 + d;
        }
        if (neg ? m > (1ull << 63) : m > static_cast<uint64_t>(INT64_MAX)) {
            v.big = true;
            return true;
        }
        v.i = neg ? static_cast<int64_t>(0 - m) : static_cast<int64_t>(m);
        return true;
    }
    bool value(JVal &v, int depth) {
        if (depth > 64) return false;
        ws();
        if (p >= e) return false;
        const char c = *p;
        if (c == '{') {
            v.kind = JVal::OBJ;
            v.o.reserve(16);  // a payload's keys: no regrowth
            ++p;
            ws();
            if (p < e && *p == '}') {
                ++p;
                return true;
            }
            while (true) {
                ws();
                if (p >= e || *p != '"') return false;
                std::string k;
                if (!str(k)) return false;
                ws();
                if (p >= e || *p != ':') return false;
                ++p;
                v.o.emplace_back(std::move(k), JVal{});
                if (!value(v.o.back().second, depth + 1)) return false;
                ws();
                if (p < e && *p == ',') {
                    ++p;
                    continue;
                }
                if (p < e && *p == '}') {
                    ++p;
                    return true;
                }
                return false;
            }
        }
        if (c == '[') {
            v.kind = JVal::ARR;
            ++p;
            ws();
            if (p < e && *p == ']') {
                ++p;
                return true;
            }
            while (true) {
                v.a.emplace_back();
                if (!value(v.a.back(), depth + 1)) return false;
                ws();
                if (p < e && *p == ',') {
                    ++p;
                    continue;
                }
                if (p < e && *p == ']') {
                    ++p;
                    return true;
                }
                return false;
            }
        }
        if (c == '"') {
            v.kind = JVal::STR;
            return str(v.s);
        }
        if (lit("true")) {
            v.kind = JVal::BOOL;
            v.b = true;
            return true;
        }
        if (lit("false")) {
            v.kind = JVal::BOOL;
            return true;
        }
        if (lit("null")) {
            v.kind = JVal::NUL;
            return true;
        }
        if (lit("NaN") || lit("Infinity") || lit("-Infinity")) {
            v.kind = JVal::FLOAT;
            return true;
        }
        return num(v);
    }
};

bool parse_json(const char *p, size_t n, JVal &out, bool &bad) {
    Parser P{p, p + n};
    if (!P.value(out, 0)) return false;
    P.ws();
    bad = P.bad;
    return P.p == P.e;
}

// ------------------------------------------------------------------ events
// One event on the typed fast path: the sb_query fields plus the strings the
// response echoes.  Strings are owned here (sb_query points into them).
struct Event {
    bool ok = false;
    uint32_t store = 0;
    sb_query q{};
    std::string region, ref, alt, vt, names, location, dataset;
    bool has_ref = false, has_alt = false, has_vt = false, has_names = false, dataset_null = true;
};
std::vector<Event> g_ev;  // kept across calls, under g_tbuf_mu

// PerformQueryPayload.__init__ keyword arguments (lambda_payloads.py:46-77)
const char *const kPayloadKeys[] = {"passthrough",   "dataset_id",      "query_id",     "region",
                                    "reference_bases", "end_min",       "end_max",      "alternate_bases",
                                    "variant_type",  "include_details", "requested_granularity",
                                    "variant_min_length", "variant_max_length", "vcf_location"};

// Python truthiness of a JSON value limited to the kinds the fast path takes
bool truthy(const JVal *v, bool &ok) {
    if (!v || v->kind == JVal::NUL) return false;
    if (v->kind == JVal::BOOL) return v->b;
    if (v->kind == JVal::INT && !v->big) return v->i != 0;
    ok = false;
    return false;
}

bool opt_str(const JVal *v, std::string &out, bool &has) {
    if (!v || v->kind == JVal::NUL) {
        has = false;
        return true;
    }
    if (v->kind != JVal::STR) return false;
    out = v->s;
    has = true;
    return true;
}

bool req_int(const JVal *v, int64_t &out) {
    if (!v || v->kind != JVal::INT || v->big) return false;
    out = v->i;
    return true;
}

// event text -> Event (ok = false: answer through the Python handler)
void load_event(const char *text, size_t len, sb_store *const *stores, size_t n_stores, bool strict_vt, Event &E) {
    E.ok = false;  // an Event kept from an earlier call: its flags reset, its strings overwritten where used
    E.store = 0;
    E.q = sb_query{};
    E.has_ref = E.has_alt = E.has_vt = E.has_names = false;
    E.dataset_null = true;
    E.names.clear();
    JVal root;
    bool bad = false;
    if (!parse_json(text, len, root, bad) || bad) return;
    // lambda_function.py:33-39: the SNS envelope, when Records[0].Sns.Message parses
    const JVal *ev = &root;
    JVal inner;
    if (root.kind == JVal::OBJ) {
        const JVal *rec = root.get("Records");
        if (rec && (rec->kind == JVal::ARR || rec->kind == JVal::OBJ)) {
            // Python: event['Records'][0] works on a list (and raises on a dict without key 0)
            if (rec->kind == JVal::ARR && !rec->a.empty() && rec->a[0].kind == JVal::OBJ) {
                const JVal *sns = rec->a[0].get("Sns");
                const JVal *msg = sns && sns->kind == JVal::OBJ ? sns->get("Message") : nullptr;
                if (msg && msg->kind == JVal::STR) {
                    bool bad2 = false;
                    if (parse_json(msg->s.data(), msg->s.size(), inner, bad2)) {
                        if (bad2) return;
                        ev = &inner;
                    }
                } else if (msg) {
                    return;  // json.loads of a non-string raises TypeError: caught; keep it simple, use Python
                }
            } else if (rec->kind == JVal::OBJ || (rec->kind == JVal::ARR && !rec->a.empty())) {
                return;  // indexing behaviour of odd envelopes: Python decides
            }
        }
    }
    if (ev->kind != JVal::OBJ) return;
    // one pass over the members: each to its keyword's slot (the last of a
    // duplicated key wins, as in a dict); an unknown keyword -> TypeError in
    // PerformQueryPayload(**event).  (A lookup per field scanned every
    // member with a string compare: ~200 compares per event.)
    constexpr size_t kNK = sizeof kPayloadKeys / sizeof kPayloadKeys[0];
    static const auto klen = [] {
        std::array<size_t, kNK> l{};
        for (size_t k = 0; k < kNK; ++k) l[k] = strlen(kPayloadKeys[k]);
        return l;
    }();
    const JVal *f[kNK] = {};
    for (const auto &kv : ev->o) {
        size_t k = 0;
        while (k < kNK && !(kv.first.size() == klen[k] && memcmp(kv.first.data(), kPayloadKeys[k], klen[k]) == 0)) ++k;
        if (k == kNK) return;
        f[k] = &kv.second;
    }
    // slots in kPayloadKeys order: 0 passthrough, 1 dataset_id, 3 region,
    // 4 reference_bases, 5 end_min, 6 end_max, 7 alternate_bases,
    // 8 variant_type, 9 include_details, 10 requested_granularity,
    // 11 variant_min_length, 12 variant_max_length, 13 vcf_location
    const JVal *loc = f[13];
    if (!loc || loc->kind != JVal::STR) return;
    E.location = loc->s;
    bool found = false;
    for (size_t k = 0; k < n_stores && !found; ++k) {
        uint32_t vid = 0;
        if (sb_store_find_vcf(stores[k], E.location.data(), E.location.size(), &vid) == SB_OK) {
            E.store = static_cast<uint32_t>(k);
            E.q.vcf_id = vid;
            found = true;
        }
    }
    if (!found) return;
    const JVal *region = f[3];
    if (!region || region->kind != JVal::STR) return;
    E.region = region->s;
    bool ok = true;
    int64_t emin = 0, emax = 0, vmin = 0, vmax = 0;
    if (!req_int(f[5], emin) || !req_int(f[6], emax) || !req_int(f[11], vmin) || !req_int(f[12], vmax))
        return;  // end_min, end_max, variant_min_length, variant_max_length
    if (!opt_str(f[4], E.ref, E.has_ref) || !opt_str(f[7], E.alt, E.has_alt) || !opt_str(f[8], E.vt, E.has_vt))
        return;  // reference_bases, alternate_bases, variant_type
    const JVal *ds = f[1];  // dataset_id
    if (ds && ds->kind == JVal::STR) {
        E.dataset = ds->s;
        E.dataset_null = false;
    } else if (ds && ds->kind != JVal::NUL) {
        return;
    }
    const bool details = truthy(f[9], ok);  // include_details
    uint8_t gran = 255;
    if (const JVal *g = f[10]) {  // requested_granularity
        if (g->kind == JVal::STR) {
            gran = g->s == "boolean" ? SB_GRAN_BOOLEAN : g->s == "count" ? SB_GRAN_COUNT
                 : g->s == "aggregated" ? SB_GRAN_AGGREGATED : g->s == "record" ? SB_GRAN_RECORD : 255;
        } else if (g->kind != JVal::NUL) {
            return;
        }
    }
    bool inc = false, sel = false;
    // passthrough: an object, or absent (the payload default {}); anything
    // else makes lambda_function.py:43 raise AttributeError -- the Python
    // handler answers it
    if (const JVal *pt = f[0]) {  // passthrough
        if (pt->kind == JVal::OBJ) {
            inc = truthy(pt->get("includeSamples"), ok);
            sel = truthy(pt->get("selectedSamplesOnly"), ok);
            if (const JVal *sn = pt->get("sampleNames")) {
                if (sn->kind == JVal::ARR) {
                    for (size_t k = 0; k < sn->a.size(); ++k) {
                        if (sn->a[k].kind != JVal::STR) return;
                        if (k) E.names.push_back(',');
                        E.names += sn->a[k].s;
                    }
                    E.has_names = true;
                } else if (sn->kind != JVal::NUL) {
                    return;
                }
            }
        } else {
            return;
        }
    }
    if (!ok) return;
    sb_query &q = E.q;
    q.end_min = emin;
    q.end_max = emax;
    q.variant_min_length = vmin;
    q.variant_max_length = vmax;
    q.granularity = gran;
    q.include_details = details ? 1 : 0;
    q.include_samples = inc ? 1 : 0;
    q.selected_samples_only = sel ? 1 : 0;
    q.strict_variant_type = strict_vt ? 1 : 0;
    E.ok = true;
}

void bind_strings(Event &E) {  // after E is in its final place
    sb_query &q = E.q;
    q.region = E.region.c_str();
    q.region_len = E.region.size();
    q.reference_bases = E.has_ref ? E.ref.c_str() : nullptr;
    q.reference_len = E.has_ref ? E.ref.size() : 0;
    q.alternate_bases = E.has_alt ? E.alt.c_str() : nullptr;
    q.alternate_len = E.has_alt ? E.alt.size() : 0;
    q.variant_type = E.has_vt ? E.vt.c_str() : nullptr;
    q.variant_type_len = E.has_vt ? E.vt.size() : 0;
    q.sample_names = E.has_names ? E.names.c_str() : nullptr;
    q.sample_names_len = E.has_names ? E.names.size() : 0;
}

// ------------------------------------------------------------------ output
// json.dumps (ensure_ascii=True) of a Python str holding these UTF-8 bytes
// (jsonesc.hpp); false on invalid UTF-8 (the Python path's .decode() raises)
bool put_jstr(std::string &o, const char *s, size_t n) {
    o.push_back('"');
    if (!json_escape_append(o, s, n)) return false;
    o.push_back('"');
    return true;
}

// decimal int64 (no snprintf: sample index lists run to tens of millions of
// numbers per batch); two digits per step from a table
void put_i64(std::string &o, int64_t v) {
    static const char kPairs[] =
        "00010203040506070809101112131415161718192021222324252627282930313233343536373839"
        "40414243444546474849505152535455565758596061626364656667686970717273747576777879"
        "8081828384858687888990919293949596979899";
    char b[24];
    char *e = b + sizeof b, *q = e;
    uint64_t u = v < 0 ? 0ull - static_cast<uint64_t>(v) : static_cast<uint64_t>(v);
    while (u >= 100) {
        const uint32_t r = static_cast<uint32_t>(u % 100);
        u /= 100;
        q -= 2;
        q[0] = kPairs[2 * r];
        q[1] = kPairs[2 * r + 1];
    }
    if (u >= 10) {
        q -= 2;
        q[0] = kPairs[2 * u];
        q[1] = kPairs[2 * u + 1];
    } else {
        *--q = static_cast<char>('0' + u);
    }
    if (v < 0) *--q = '-';
    o.append(q, static_cast<size_t>(e - q));
}

// decimal of a two's-complement little-endian 32-bit-limb integer; false
// when it has more digits than CPython converts (json.dumps raises ValueError)
bool put_limbs(std::string &o, const uint32_t *l, uint32_t n) {
    std::vector<uint32_t> m(l, l + n);
    const bool neg = n && (m[n - 1] >> 31);
    if (neg) {  // magnitude = ~x + 1
        uint64_t carry = 1;
        for (auto &x : m) {
            const uint64_t t = static_cast<uint64_t>(~x) + carry;
            x = static_cast<uint32_t>(t);
            carry = t >> 32;
        }
    }
    std::string digits;
    while (true) {
        bool zero = true;
        uint64_t rem = 0;
        for (size_t k = m.size(); k-- > 0;) {
            const uint64_t cur = (rem << 32) | m[k];
            m[k] = static_cast<uint32_t>(cur / 1000000000u);
            rem = cur % 1000000000u;
            zero = zero && m[k] == 0;
        }
        char b[16];
        if (zero) {
            const int w = snprintf(b, sizeof b, "%llu", static_cast<unsigned long long>(rem));
            digits.insert(0, b, static_cast<size_t>(w));
            break;
        }
        snprintf(b, sizeof b, "%09llu", static_cast<unsigned long long>(rem));
        digits.insert(0, b, 9);
    }
    if (digits.size() > kPyMaxStrDigits) return false;
    if (neg) o.push_back('-');
    o += digits;
    return true;
}

// what json.dumps raises for an int past CPython's digit limit
void put_digits_error(std::string &o, size_t start) {
    static const char kMsg[] =
        "Exceeds the limit (4300) for integer string conversion; use sys.set_int_max_str_digits() to increase the limit";
    o.resize(start);  // drop the response written so far
    o += "{\"errorMessage\": ";
    put_jstr(o, kMsg, sizeof kMsg - 1);
    o += ", \"errorType\": \"ValueError\"}";
}

// QERR -> the exception the reference raises (sbeacon/engine.py QERR / QERR_MSG)
void put_error(std::string &o, int32_t err) {
    const char *type = "RuntimeError", *msg = "error";
    switch (err) {
        case 1: type = "UnboundLocalError"; msg = "local variable 'variant_type' referenced before assignment"; break;
        case 2: type = "IndexError"; msg = "list index out of range"; break;
        case 3: type = "ValueError"; msg = "invalid literal for int() with base 10"; break;
        case 4: type = "AttributeError"; msg = "'NoneType' object has no attribute 'replace'"; break;
        case 9: type = "NotImplementedError"; msg = "referenceBases contains regex metacharacters (outside the restated contract)"; break;
        default: break;
    }
    o += "{\"errorMessage\": ";
    put_jstr(o, msg, strlen(msg));
    o += ", \"errorType\": ";
    put_jstr(o, type, strlen(type));
    o += "}";
}

// json.dumps(PerformQueryResponse.dump()) for query i of rs (engine.py
// ResultSet.responses); false = text the Python path could not decode
// SBEACON_WIRE_TRACE: time in the variant / sample-name writers, per thread
thread_local double tl_var_ms = 0, tl_samp_ms = 0;
thread_local uint64_t tl_var_n = 0, tl_samp_n = 0, tl_var_b = 0, tl_samp_b = 0;
const bool g_wire_trace = config().wire_trace;  // read once at load

// d != null: the variant list and the sample-name list are not written --
// their positions in o and exact lengths go to *d (the caller writes them in
// place in the output)
struct Defer {
    bool v = false, n = false;
    size_t vpos = 0, vlen = 0, npos = 0, nlen = 0;
};

bool put_response(std::string &o, sb_result_set *rs, size_t i, const Event &E, Defer *d = nullptr) {
    const size_t start = o.size();  // o may already hold earlier responses
    if (d) *d = Defer{};
    sb_result_view v;
    if (result_view(rs, i, &v) != SB_OK) return false;
    if (v.error) {
        put_error(o, v.error);
        return true;
    }
    o += "{\"exists\": ";
    o += v.exists ? "true" : "false";
    o += ", \"vcf_location\": ";
    if (!put_jstr(o, E.location.data(), E.location.size())) return false;
    o += ", \"dataset_id\": ";
    if (E.dataset_null) o += "null";
    else if (!put_jstr(o, E.dataset.data(), E.dataset.size())) return false;
    o += ", \"all_alleles_count\": ";
    if (v.big_limbs) {
        if (!put_limbs(o, v.big_all_alleles_count, v.big_limbs)) {
            put_digits_error(o, start);
            return true;
        }
    } else {
        put_i64(o, v.all_alleles_count);
    }
    o += ", \"variants\": [";
    if (v.n_variants && d) {
        if (!result_variants_len(rs, i, &d->vlen)) return false;
        d->v = true;
        d->vpos = o.size();
        if (g_wire_trace) {
            tl_var_n += v.n_variants;
            tl_var_b += d->vlen;
        }
    } else if (v.n_variants) {
        const auto t0 = g_wire_trace ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
        const size_t b0 = o.size();
        if (!result_variants_json(rs, i, o)) return false;
        if (g_wire_trace) {
            tl_var_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            tl_var_n += v.n_variants;
            tl_var_b += o.size() - b0;
        }
    }
    o += "], \"call_count\": ";
    if (v.big_limbs) {
        if (!put_limbs(o, v.big_call_count, v.big_limbs)) {
            put_digits_error(o, start);
            if (d) *d = Defer{};  // the error text replaces the response
            return true;
        }
    } else {
        put_i64(o, v.call_count);
    }
    // sample_indices / sample_names (engine.py ResultSet.responses)
    const bool sel = E.q.selected_samples_only, inc = E.q.include_samples;
    o += ", \"sample_indices\": [";
    if (sel)
        for (uint64_t k = 0; k < v.n_sample_indices; ++k) {
            if (k) o += ", ";
            put_i64(o, v.sample_indices[k]);
        }
    o += "], \"sample_names\": [";
    if ((sel || inc) && v.n_sample_indices && d) {
        if (!result_sample_names_len(rs, i, &d->nlen)) return false;
        d->n = true;
        d->npos = o.size();
    } else if ((sel || inc) && v.n_sample_indices) {
        const auto t0 = g_wire_trace ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
        const size_t b0 = o.size();
        if (!result_sample_names_json(rs, i, o)) return false;
        if (g_wire_trace) {
            tl_samp_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            tl_samp_n += v.n_sample_indices;
            tl_samp_b += o.size() - b0;
        }
    }
    o += "]}";
    return true;
}

template <class F>
void par(size_t n, unsigned threads, F fn) {
    const unsigned t = static_cast<unsigned>(std::min<size_t>(threads, std::max<size_t>(1, n / 256)));
    if (t <= 1) {
        for (size_t i = 0; i < n; ++i) fn(i, 0u);
        return;
    }
    run_tasks(t, [&](size_t k) {  // the host worker pool: no thread spawns per phase
        for (size_t i = n * k / t, e = n * (k + 1) / t; i < e; ++i) fn(i, static_cast<unsigned>(k));
    });
}

}  // namespace
}  // namespace sb

extern "C" {

int sb_perform_query_events(sb_store *const *stores, size_t n_stores, const char *text, const uint64_t *offsets,
                            size_t n, uint32_t flags, sb_json_out **out) {
    using namespace sb;
    try {
        if ((!stores && n_stores) || (!offsets && n) || (!text && n) || !out) throw Error(SB_EINVAL, "NULL argument");
        for (size_t i = 0; i < n; ++i)
            if (offsets[i + 1] < offsets[i]) throw Error(SB_EINVAL, "offsets not non-decreasing");
        // phases cut into more pieces than the pool has threads: the pool
        // drains them dynamically (events differ a lot in response size)
        const unsigned chunks = 64;
        const bool strict_vt = (flags & 1u) != 0;
        // SBEACON_WIRE_TRACE=1: phase times to stderr (bench diagnostics)
        const bool trace = config().wire_trace;
        auto t_last = std::chrono::steady_clock::now();
        auto tick = [&](const char *what) {
            if (!trace) return;
            const auto t = std::chrono::steady_clock::now();
            std::fprintf(stderr, "[wire] %-8s %8.2f ms\n", what,
                         std::chrono::duration<double, std::milli>(t - t_last).count());
            t_last = t;
        };
        // the event and formatting buffers persist across calls (their strings'
        // capacity kept); a concurrent call uses buffers of its own
        std::unique_lock<std::mutex> tb_lk(g_tbuf_mu, std::try_to_lock);
        std::vector<Event> own_ev;
        std::vector<Event> &ev = tb_lk.owns_lock() ? g_ev : own_ev;
        if (ev.size() < n) ev.resize(n);
        tick("events");
        par(n, chunks, [&](size_t i, unsigned) {
            load_event(text + offsets[i], offsets[i + 1] - offsets[i], stores, n_stores, strict_vt, ev[i]);
            if (ev[i].ok) bind_strings(ev[i]);
        });
        tick("parse");
        auto R = std::make_unique<sb_json_out>();
        R->status.assign(n, 1);
        // Two passes.  Format: each event's response goes to the buffer of
        // the task that formats it (a contiguous range of its store's
        // events) EXCEPT its variant and sample-name lists -- ~97 % of the
        // bytes -- whose exact lengths are recorded instead.  Write: with
        // every length known, each response is assembled in place in the
        // output: its pieces copied, its lists written straight from the
        // store's text cache (no second copy of the lists, no zero-filled
        // growth of a thread buffer)
        std::vector<uint32_t> where(n, 0), jidx(n, 0);  // formatting task; index in its store's batch
        std::vector<uint64_t> pos(n, 0), plen(n, 0), len(n, 0);
        std::vector<Defer> dfr(n);
        std::vector<std::string> own;
        std::vector<std::string> &tbuf = tb_lk.owns_lock() ? g_tbuf : own;
        tbuf.resize(chunks);
        for (auto &b : tbuf) b.clear();  // capacity kept
        std::vector<std::unique_ptr<sb_result_set, void (*)(sb_result_set *)>> sets;
        sets.reserve(n_stores);
        for (size_t k = 0; k < n_stores; ++k) sets.emplace_back(nullptr, sb_result_free);
        for (size_t k = 0; k < n_stores; ++k) {
            std::vector<uint32_t> idx;
            for (size_t i = 0; i < n; ++i)
                if (ev[i].ok && ev[i].store == k) idx.push_back(static_cast<uint32_t>(i));
            if (idx.empty()) continue;
            std::vector<sb_query> qs(idx.size());
            for (size_t j = 0; j < idx.size(); ++j) qs[j] = ev[idx[j]].q;
            sb_result_set *rs = nullptr;
            const int rc = sb_query_batch(stores[k], qs.data(), qs.size(), 0, &rs);
            if (rc != SB_OK) return rc;  // sb_last_error holds the message
            sets[k].reset(rs);
            result_prepare_json(rs);
            tick("query");
            std::vector<double> t_ms(chunks, 0.0);
            std::mutex tot_mu;
            double tot[6] = {0, 0, 0, 0, 0, 0};
            {
                const size_t m = idx.size();
                const unsigned tt = static_cast<unsigned>(std::min<size_t>(chunks, std::max<size_t>(1, m / 64)));
                // task t formats events [m t / tt, m (t + 1) / tt) into its buffer
                run_tasks(tt, [&](size_t t) {
                    const auto t0 = trace ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point{};
                    std::string &o = tbuf[t];
                    for (size_t j = m * t / tt, e = m * (t + 1) / tt; j < e; ++j) {
                        const uint32_t i = idx[j];
                        const size_t at = o.size();
                        Defer &D = dfr[i];
                        if (put_response(o, rs, j, ev[i], &D)) {
                            o.push_back('\n');
                            where[i] = static_cast<uint32_t>(t);
                            jidx[i] = static_cast<uint32_t>(j);
                            pos[i] = at;
                            plen[i] = o.size() - at;
                            len[i] = plen[i] + (D.v ? D.vlen : 0) + (D.n ? D.nlen : 0);
                            R->status[i] = 0;
                        } else {
                            o.resize(at);
                        }
                    }
                    if (trace) {  // this task's writer times into the call's totals
                        t_ms[t] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
                        std::lock_guard<std::mutex> lk(tot_mu);
                        tot[0] += tl_var_ms;
                        tot[1] += tl_samp_ms;
                        tot[2] += static_cast<double>(tl_var_n);
                        tot[3] += static_cast<double>(tl_samp_n);
                        tot[4] += static_cast<double>(tl_var_b);
                        tot[5] += static_cast<double>(tl_samp_b);
                        tl_var_ms = tl_samp_ms = 0;
                        tl_var_n = tl_samp_n = tl_var_b = tl_samp_b = 0;
                    }
                });
            }
            if (trace) {
                double mx = 0, sum = 0;
                size_t bytes = 0;
                for (unsigned t = 0; t < chunks; ++t) {
                    mx = std::max(mx, t_ms[t]);
                    sum += t_ms[t];
                    bytes += tbuf[t].size();
                }
                std::fprintf(stderr, "[wire] format tasks: max %.2f ms, sum %.2f ms, %zu bytes of pieces\n", mx, sum, bytes);
                std::fprintf(stderr,
                             "[wire] format parts: variants %.0f strings, %.0f bytes (deferred); sample names %.2f ms "
                             "(%.0f names, %.0f bytes)\n",
                             tot[2], tot[4], tot[1], tot[3], tot[5]);
            }
            tick("format");
        }
        // JSON lines: every response ends with '\n' (none for status 1)
        R->off.resize(n + 1);
        R->off[0] = 0;
        for (size_t i = 0; i < n; ++i) R->off[i + 1] = R->off[i] + len[i];
        R->n = R->off[n];
        R->buf = big_alloc(R->n, &R->cap);
        char *out_buf = R->buf.get();
        par(n, chunks, [&](size_t i, unsigned) {
            if (!len[i]) return;
            char *dst = out_buf + R->off[i];
            const char *src = tbuf[where[i]].data() + pos[i];
            const Defer &D = dfr[i];
            const sb_result_set *rs = sets[ev[i].store].get();
            size_t a = 0;  // piece bytes copied so far
            auto piece_to = [&](size_t upto) {
                std::memcpy(dst, src + a, upto - a);
                dst += upto - a;
                a = upto;
            };
            if (D.v) {
                piece_to(D.vpos - pos[i]);
                result_variants_write(rs, jidx[i], dst);
                dst += D.vlen;
            }
            if (D.n) {
                piece_to(D.npos - pos[i]);
                result_sample_names_write(rs, jidx[i], dst);
                dst += D.nlen;
            }
            piece_to(plen[i]);
        });
        tick("write");
        tick("cleanup");
        *out = R.release();
        return SB_OK;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return SB_ENOMEM;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return SB_EINVAL;
    }
}

int sb_json_out_get(const sb_json_out *o, const char **buf, size_t *len, const uint64_t **offsets,
                    const uint8_t **status) {
    if (!o || !buf || !len || !offsets || !status) return SB_EINVAL;
    *buf = o->buf.get();
    *len = o->n;
    *offsets = o->off.data();
    *status = o->status.data();
    return SB_OK;
}

void sb_json_out_free(sb_json_out *o) {
    if (o) sb::big_release(o->buf, o->cap);
    delete o;
}

}  // extern "C"
