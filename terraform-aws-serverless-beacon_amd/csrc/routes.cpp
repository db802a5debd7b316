// routes.cpp — GET / POST /g_variants bodies for a batch of route events
// from the rows and hit lists of a request pass (sb_route_bodies).
//
// Reference: lambda/getGenomicVariants/route_g_variants.py:49-208.  Per
// event the route fans out one SplitQueryPayload per dataset
// (shared_resources/variantutils/search_variants.py:158-244), splitQuery
// cuts each into performQuery slices per VCF, and the route folds the
// responses (:153-171): exists = OR; with check_all, variants |= the
// response's variant strings f'{chrom}\t{POS}\t{REF}\t{ALT}\t{VT}'
// (lambda/performQuery/search_variants.py:210) and one get_variant_entry
// (shared_resources/apiutils/entries.py:1-24) per distinct
// f'{assemblyId}\t{chrom}\t{pos}\t{ref}\t{alt}'.  Here the fan-out is the
// request rows of ONE pass (one row per (dataset, VCF): its slices' exists
// count and its hit list, sb_requests_run), and the fold runs in C++ over
// the hits, in parallel over events: hits grouped by (chrom, POS), strings
// compared byte for byte inside a group, the body written as json.dumps
// writes the response dict (responses.py:160-254, bundle_response's body).
//
// Order: the reference folds responses in thread-completion order, so its
// `results` order is not defined; here it is the rows' order (dataset, VCF)
// and each row's hit order.  The set and the count are the reference's: a
// response with variants always has exists = True (a variant needs AC != 0
// and the VCF's ACs are non-negative, so its cumulative call_count is
// positive, search_variants.py:205-232), so the route's "add only once
// exists" gate drops nothing.  A VCF with a negative AC breaks that
// argument (the gate then depends on completion order): its events go
// through the Python route (status 1).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "internal.hpp"
#include "jsonesc.hpp"
#include "jsonout.hpp"

namespace sb {
namespace {

constexpr char kB64[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";

size_t b64_len(size_t n) { return (n + 2) / 3 * 4; }

// base64.b64encode of the bytes of `parts` concatenated (standard alphabet, '=' padding)
char *b64_write(char *o, const std::pair<const char *, size_t> *parts, int np) {
    uint32_t acc = 0;
    int have = 0;
    for (int k = 0; k < np; ++k)
        for (size_t i = 0; i < parts[k].second; ++i) {
            acc = acc << 8 | static_cast<uint8_t>(parts[k].first[i]);
            if (++have == 3) {
                *o++ = kB64[(acc >> 18) & 63];
                *o++ = kB64[(acc >> 12) & 63];
                *o++ = kB64[(acc >> 6) & 63];
                *o++ = kB64[acc & 63];
                acc = 0;
                have = 0;
            }
        }
    if (have == 1) {
        acc <<= 16;
        *o++ = kB64[(acc >> 18) & 63];
        *o++ = kB64[(acc >> 12) & 63];
        *o++ = '=';
        *o++ = '=';
    } else if (have == 2) {
        acc <<= 8;
        *o++ = kB64[(acc >> 18) & 63];
        *o++ = kB64[(acc >> 12) & 63];
        *o++ = kB64[(acc >> 6) & 63];
        *o++ = '=';
    }
    return o;
}

int dec_len(uint64_t v) {
    int d = 1;
    while (v >= 10) {
        v /= 10;
        ++d;
    }
    return d;
}

char *dec_write(char *o, uint64_t v) {
    char t[24];
    int n = 0;
    do {
        t[n++] = static_cast<char>('0' + v % 10);
        v /= 10;
    } while (v);
    while (n) *o++ = t[--n];
    return o;
}

char *put(char *o, const std::string &x) {
    std::memcpy(o, x.data(), x.size());
    return o + x.size();
}
char *put(char *o, const char *x, size_t n) {
    std::memcpy(o, x, n);
    return o + n;
}
template <size_t N>
char *lit(char *o, const char (&x)[N]) {
    std::memcpy(o, x, N - 1);
    return o + N - 1;
}

// escaped length of UTF-8 text as json.dumps writes it; SIZE_MAX: not UTF-8
// (printable ASCII without '"' / '\\' -- every allele in practice -- is its own length)
bool plain(const char *p, size_t n) {
    for (size_t i = 0; i < n; ++i) {
        const unsigned char c = static_cast<unsigned char>(p[i]);
        if (c < 0x20 || c >= 0x7f || c == '"' || c == '\\') return false;
    }
    return true;
}
size_t esc_len(const char *p, size_t n) {
    if (plain(p, n)) return n;
    thread_local std::string tmp;
    tmp.clear();
    if (!json_escape_append(tmp, p, n)) return SIZE_MAX;
    return tmp.size();
}

// len(str) of valid UTF-8 text: its code points
uint64_t code_points(const char *p, size_t n) {
    uint64_t c = 0;
    for (size_t i = 0; i < n; ++i) c += (static_cast<uint8_t>(p[i]) & 0xc0) != 0x80;
    return c;
}

// one hit of an event: its (chrom, POS) group key, record, ALT and position
struct EvHit {
    uint32_t cid, pos, rec, alt, ord;
};

struct Ctx {
    const sb_store &s;
    const sb_route_input &in;
    bool compact;
    std::vector<std::vector<uint32_t>> cid;  // [vcf][contig] -> chrom id (equal strings, equal ids)
    std::vector<std::string> chrom;          // chrom id -> raw text
    std::vector<std::string> vt_json;        // VT dictionary id -> escaped ("\x01": not UTF-8)
    std::vector<std::string> asm_json;       // assembly -> "..." or null ("\x01": not UTF-8)
    std::vector<std::string> asm_raw;        // assembly -> f'{assemblyId}' bytes
    std::string head_pre, head_mid;          // envelope pieces around the granularity names

    uint32_t row_vcf(uint32_t r) const { return in.row_vcf ? in.row_vcf[r] : in.vcf_all; }
    uint32_t row_contig(uint32_t r) const { return in.row_contig ? in.row_contig[r] : in.contig_all; }
    uint64_t off(size_t r) const {
        return compact ? static_cast<const uint32_t *>(in.row_off)[r] : static_cast<const uint64_t *>(in.row_off)[r];
    }
    // (exists, errors, escaped) of row r
    void row(uint32_t r, uint64_t &ex, bool &bad) const {
        if (compact) {
            const sb_request_row32 &x = static_cast<const sb_request_row32 *>(in.rows)[r];
            ex = x.exists;
            bad = x.exists == UINT32_MAX;  // an escaped compact row: the wide sums are the batch's
        } else {
            const sb_request_partial &x = static_cast<const sb_request_partial *>(in.rows)[r];
            ex = x.exists > 0 ? 1 : 0;
            bad = x.errors != 0;  // a slice raised: the route re-raises (Python)
        }
    }
    // hit h as (record, ALT); false: an escaped compact label
    bool hit(uint64_t h, uint32_t &rec, uint32_t &alt) const {
        uint64_t r;
        if (compact) {
            const uint32_t v = static_cast<const uint32_t *>(in.hits)[h];
            alt = v >> kStageAltShift;
            if (alt == 7) return false;  // label 7: the exact ALT index is the batch's (escape)
            r = v & kStageCandMask;
        } else {
            const uint64_t v = static_cast<const uint64_t *>(in.hits)[h];
            alt = static_cast<uint32_t>(v >> kHitAltShift);
            r = v & 0xffffffffull;
        }
        if (r < in.rec_base || r - in.rec_base >= s.n_records) throw Error(SB_EINVAL, "a hit names a record outside the store");
        rec = static_cast<uint32_t>(r - in.rec_base);
        return true;
    }
    uint32_t n_alts(uint32_t rec) const {
        const uint32_t nx = (rec + 1 < s.n_records ? s.h_x_lo[rec + 1] : static_cast<uint32_t>(s.n_extra)) - s.h_x_lo[rec];
        return 1 + nx;
    }
    const char *ref(uint32_t rec, size_t &n) const {
        n = s.h_end[rec] - s.h_pos[rec] + 1;
        return reinterpret_cast<const char *>(s.h_blob.data() + s.h_ref_off[rec]);
    }
    const char *alt(uint32_t rec, uint32_t k, size_t &n) const {
        if (k == 0) {
            n = s.h_a0_len[rec];
            return reinterpret_cast<const char *>(s.h_blob.data() + s.h_a0_off[rec]);
        }
        const uint32_t x = s.h_x_lo[rec] + k - 1;
        n = s.h_x_len[x];
        return reinterpret_cast<const char *>(s.h_blob.data() + s.h_x_off[x]);
    }
    // the record columns a hit's fold reads, and (once those have arrived)
    // its allele text: each hit's record is a random line in every column,
    // so an event's hits are prefetched two and one events ahead of its fold
    void prefetch_cols(uint64_t h0, uint64_t h1) const {
        for (uint64_t h = h0; h < h1; ++h) {
            const uint64_t v = compact ? static_cast<const uint32_t *>(in.hits)[h] & kStageCandMask
                                       : static_cast<const uint64_t *>(in.hits)[h] & 0xffffffffull;
            if (v < in.rec_base || v - in.rec_base >= s.n_records) continue;
            const uint32_t r = static_cast<uint32_t>(v - in.rec_base);
            __builtin_prefetch(&s.h_pos[r]);
            __builtin_prefetch(&s.h_end[r]);
            __builtin_prefetch(&s.h_x_lo[r]);
            __builtin_prefetch(&s.h_vt[r]);
            __builtin_prefetch(&s.h_ref_off[r]);
            __builtin_prefetch(&s.h_a0_off[r]);
            __builtin_prefetch(&s.h_a0_len[r]);
        }
    }
    void prefetch_text(uint64_t h0, uint64_t h1) const {
        for (uint64_t h = h0; h < h1; ++h) {
            const uint64_t v = compact ? static_cast<const uint32_t *>(in.hits)[h] & kStageCandMask
                                       : static_cast<const uint64_t *>(in.hits)[h] & 0xffffffffull;
            if (v < in.rec_base || v - in.rec_base >= s.n_records) continue;
            const uint32_t r = static_cast<uint32_t>(v - in.rec_base);
            __builtin_prefetch(s.h_blob.data() + s.h_ref_off[r]);
            __builtin_prefetch(s.h_blob.data() + s.h_a0_off[r]);
        }
    }
    bool same_ref_alt(const EvHit &a, const EvHit &b) const {
        if (a.rec == b.rec && a.alt == b.alt) return true;
        size_t na, nb;
        const char *pa = ref(a.rec, na), *pb = ref(b.rec, nb);
        if (na != nb || std::memcmp(pa, pb, na)) return false;
        pa = alt(a.rec, a.alt, na);
        pb = alt(b.rec, b.alt, nb);
        return na == nb && !std::memcmp(pa, pb, na);
    }
};

// the body pieces (responses.py:160-254) around their values
constexpr char kB_gran2[] = ", \"requestedGranularity\": \"";
constexpr char kB_head_end[] = "\"}}, ";
constexpr char kB_sum[] = "\"responseSummary\": {\"exists\": ";
constexpr char kB_total[] = ", \"numTotalResults\": ";
constexpr char kB_close[] = "}}";
constexpr char kB_rs0[] = "\"response\": {\"resultSets\": [{\"exists\": ";
constexpr char kB_rs1[] = ", \"id\": \"redacted\", \"results\": [";
constexpr char kB_rs2[] = "], \"resultsCount\": ";
constexpr char kB_rs3[] = ", \"resultsHandovers\": [], \"setType\": \"genomicVariant\"}]}, ";
template <size_t N>
constexpr size_t L(const char (&)[N]) {
    return N - 1;
}

const char *gran_name(uint8_t g) {
    return g == SB_GRAN_BOOLEAN ? "boolean" : g == SB_GRAN_COUNT ? "count" : "record";
}

// Per event after the fold: what its body needs
struct EvOut {
    uint8_t status = 0;
    bool exists = false;
    uint64_t total = 0;    // len(variants)
    uint64_t results = 0;  // entries (first-seen internal ids)
    uint64_t len = 0;      // body bytes + '\n'
};

// entries.py:1-24 as json.dumps writes it, between its values
constexpr char kE0[] = "{\"variantInternalId\": \"";
constexpr char kE1[] = "\", \"variation\": {\"referenceBases\": \"";
constexpr char kE2[] = "\", \"alternateBases\": \"";
constexpr char kE3[] = "\", \"location\": {\"interval\": {\"start\": {\"type\": \"Number\", \"value\": ";
constexpr char kE4[] = "}, \"end\": {\"type\": \"Number\", \"value\": ";
constexpr char kE5[] = "}, \"type\": \"SequenceInterval\"}, \"sequence_id\": ";
constexpr char kE6[] = ", \"type\": \"SequenceLocation\"}, \"variantType\": \"";
constexpr char kE7[] = "\"}}";

// length of the entry of hit (rec, alt) for assembly a; 0: text Python could not decode
uint64_t entry_len(const Ctx &C, uint32_t a, uint32_t cid, uint32_t rec, uint32_t k) {
    size_t rn, an;
    const char *rp = C.ref(rec, rn), *ap = C.alt(rec, k, an);
    const size_t re = esc_len(rp, rn), ae = esc_len(ap, an);
    const std::string &vt = C.vt_json[C.s.h_vt[rec]];
    if (re == SIZE_MAX || ae == SIZE_MAX || (vt.size() == 1 && vt[0] == '\x01')) return 0;
    const uint32_t pos = C.s.h_pos[rec];
    const size_t idn = C.asm_raw[a].size() + 1 + C.chrom[cid].size() + 1 + dec_len(pos) + 1 + rn + 1 + an;
    constexpr size_t kFixed = sizeof(kE0) + sizeof(kE1) + sizeof(kE2) + sizeof(kE3) + sizeof(kE4) + sizeof(kE5) +
                              sizeof(kE6) + sizeof(kE7) - 8;
    return kFixed + b64_len(idn) + re + ae + dec_len(pos) + dec_len(pos + code_points(ap, an)) + C.asm_json[a].size() +
           vt.size();
}

char *entry_write(const Ctx &C, char *o, uint32_t a, uint32_t cid, uint32_t rec, uint32_t k) {
    size_t rn, an;
    const char *rp = C.ref(rec, rn), *ap = C.alt(rec, k, an);
    const uint32_t pos = C.s.h_pos[rec];
    char num[24];
    char *ne = dec_write(num, pos);
    o = lit(o, kE0);
    const std::pair<const char *, size_t> parts[9] = {
        {C.asm_raw[a].data(), C.asm_raw[a].size()}, {"\t", 1}, {C.chrom[cid].data(), C.chrom[cid].size()}, {"\t", 1},
        {num, static_cast<size_t>(ne - num)}, {"\t", 1}, {rp, rn}, {"\t", 1}, {ap, an}};
    o = b64_write(o, parts, 9);
    o = lit(o, kE1);
    o = plain(rp, rn) ? put(o, rp, rn) : json_escape_to(o, rp, rn);
    o = lit(o, kE2);
    o = plain(ap, an) ? put(o, ap, an) : json_escape_to(o, ap, an);
    o = lit(o, kE3);
    o = dec_write(o, pos);
    o = lit(o, kE4);
    o = dec_write(o, pos + code_points(ap, an));
    o = lit(o, kE5);
    o = put(o, C.asm_json[a]);
    o = lit(o, kE6);
    o = put(o, C.vt_json[C.s.h_vt[rec]]);
    return lit(o, kE7);
}

// the first exception of a parallel_for body, rethrown on the calling thread
// (an exception must not leave a pool worker)
struct FirstError {
    std::mutex mu;
    bool set = false;
    int code = SB_OK;
    std::string msg;
    template <class F>
    auto wrap(F fn) {
        return [this, fn](size_t i) {
            try {
                fn(i);
            } catch (const Error &x) {
                keep(x.code, x.what());
            } catch (const std::exception &x) {
                keep(SB_EINVAL, x.what());
            }
        };
    }
    void keep(int c, const char *m) {
        std::lock_guard<std::mutex> lk(mu);
        if (set) return;
        set = true;
        code = c;
        msg = m;
    }
    void rethrow() {
        if (set) throw Error(code, msg);
    }
};

}  // namespace
}  // namespace sb

extern "C" int sb_route_bodies(sb_store *s, const sb_route_input *in, sb_json_out **out) {
    using namespace sb;
    return guard([&] {
        if (!s || !in || !out || (in->n_events && !in->events)) throw Error(SB_EINVAL, "NULL argument");
        if (in->compact != 0 && in->compact != SB_COMPACT_ALL)
            throw Error(SB_EINVAL, "sb_route_bodies: compact is 0 (wide) or SB_COMPACT_ALL");
        const size_t ne = in->n_events;
        Ctx C{*s, *in, in->compact == SB_COMPACT_ALL, {}, {}, {}, {}, {}, {}, {}};
        uint32_t n_rows = 0;
        for (size_t e = 0; e < ne; ++e) {
            const sb_route_event &E = in->events[e];
            if (E.row_hi < E.row_lo || (e && E.row_lo < in->events[e - 1].row_hi))
                throw Error(SB_EINVAL, "sb_route_bodies: event rows must be ascending, non-overlapping ranges");
            if (E.assembly >= in->n_assembly || (E.granularity >= SB_GRAN_AGGREGATED && E.granularity != 255 &&
                                                 E.pagination >= in->n_pagination))
                throw Error(SB_EINVAL, "sb_route_bodies: event " + std::to_string(e) + ": dictionary index out of range");
            if (E.granularity > SB_GRAN_RECORD && E.granularity != 255)
                throw Error(SB_EINVAL, "sb_route_bodies: granularity must be SB_GRAN_* or 255");
            n_rows = std::max(n_rows, E.row_hi);
        }
        if (n_rows && (!in->rows || !in->row_off)) throw Error(SB_EINVAL, "NULL rows / row offsets");
        // chrom ids: equal contig strings across VCFs share an id (the variant
        // string holds the chrom text, not the VCF)
        std::unordered_map<std::string, uint32_t> by_name;
        C.cid.resize(s->vcfs.size());
        for (size_t v = 0; v < s->vcfs.size(); ++v)
            for (const Segment &g : s->vcfs[v].segments) {
                auto it = by_name.emplace(g.contig, static_cast<uint32_t>(C.chrom.size()));
                if (it.second) C.chrom.push_back(g.contig);
                C.cid[v].push_back(it.first->second);
            }
        C.vt_json.resize(s->vt.items.size());
        for (size_t k = 0; k < s->vt.items.size(); ++k)
            if (!json_escape_append(C.vt_json[k], s->vt.items[k].data(), s->vt.items[k].size())) C.vt_json[k] = "\x01";
        for (uint32_t a = 0; a < in->n_assembly; ++a) {
            const sb_str &x = in->assembly_dict[a];
            std::string j;
            if (!x.p) {
                C.asm_json.push_back("null");
                C.asm_raw.push_back("None");
                continue;
            }
            if (!json_escape_append(j, x.p, x.len)) j = "\x01";
            else j = "\"" + j + "\"";
            C.asm_json.push_back(j);
            C.asm_raw.emplace_back(x.p, x.len);
        }
        std::vector<std::string> pag(in->n_pagination);
        for (uint32_t k = 0; k < in->n_pagination; ++k)
            if (in->pagination_dict[k].p) pag[k].assign(in->pagination_dict[k].p, in->pagination_dict[k].len);
        auto esc = [](const sb_str &x, const char *what) {
            std::string o;
            if (!x.p || !json_escape_append(o, x.p, x.len)) throw Error(SB_EINVAL, std::string("sb_route_bodies: ") + what);
            return o;
        };
        const std::string bid = esc(in->beacon_id, "beacon_id is not UTF-8 text"),
                          api = esc(in->api_version, "api_version is not UTF-8 text");
        // responses.py:22-34 (_meta) around the granularity and the pagination
        C.head_pre = "{\"$schema\": \"https://json-schema.org/draft/2020-12/schema\", \"info\": {}, \"meta\": "
                     "{\"beaconId\": \"" + bid + "\", \"apiVersion\": \"" + api +
                     "\", \"returnedSchemas\": [{\"entityType\": \"info\", \"schema\": \"beacon-map-v2.0.0\"}], "
                     "\"returnedGranularity\": \"";
        C.head_mid = "\", \"receivedRequestSummary\": {\"apiVersion\": \"" + api +
                     "\", \"requestedSchemas\": [], \"pagination\": ";
        const uint64_t n_hits = n_rows ? C.off(n_rows) : 0;
        if (n_hits && !in->hits) throw Error(SB_EINVAL, "NULL hits");
        // SBEACON_WIRE_TRACE=1: the fold's phase times (stderr)
        const bool trace = config().wire_trace;
        auto t_last = std::chrono::steady_clock::now();
        auto tick = [&](const char *what) {
            if (!trace) return;
            const auto t = std::chrono::steady_clock::now();
            std::fprintf(stderr, "[route] %-8s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
            t_last = t;
        };
        tick("setup");
        std::vector<uint8_t> first_id(n_hits, 0);  // hit h opens its internal id's entry
        std::vector<EvOut> eo(ne);
        // pass 1: fold each event, size its body
        FirstError fe;
        // an event's hit range (prefetching: the events ahead of the fold)
        auto ev_hits = [&](size_t e, uint64_t &h0, uint64_t &h1) {
            const sb_route_event &E = in->events[e];
            h0 = h1 = 0;
            if (!n_hits || E.row_hi <= E.row_lo) return;
            h0 = C.off(E.row_lo);
            h1 = std::min<uint64_t>(C.off(E.row_hi), n_hits);
            h0 = std::min(h0, h1);
        };
        auto prefetch_ahead = [&](size_t e) {
            uint64_t a, b;
            if (e + 4 < ne) {
                ev_hits(e + 4, a, b);
                C.prefetch_cols(a, b);
            }
            if (e + 2 < ne) {
                ev_hits(e + 2, a, b);
                C.prefetch_text(a, b);
            }
        };
        parallel_for(ne, fe.wrap([&](size_t e) {
            prefetch_ahead(e);
            const sb_route_event &E = in->events[e];
            EvOut &O = eo[e];
            const uint8_t g = E.granularity;
            if (g == 255) {
                O.status = 2;  // route_g_variants.py:179-198: no branch returns
                return;
            }
            for (uint32_t r = E.row_lo; r < E.row_hi; ++r) {
                uint64_t ex;
                bool bad;
                C.row(r, ex, bad);
                if (bad) {
                    O.status = 1;
                    return;
                }
                O.exists |= ex != 0;
            }
            const bool fold = E.check_all && g != SB_GRAN_BOOLEAN && O.exists;
            if (fold) {
                thread_local std::vector<EvHit> hv;
                hv.clear();
                const uint64_t h0 = C.off(E.row_lo);
                for (uint32_t r = E.row_lo; r < E.row_hi; ++r) {
                    const uint64_t a = C.off(r), b = C.off(r + 1);
                    if (b == a) continue;
                    const uint32_t v = C.row_vcf(r), c = C.row_contig(r);
                    if (v >= s->vcfs.size() || c >= C.cid[v].size())
                        throw Error(SB_EINVAL, "sb_route_bodies: row " + std::to_string(r) + ": VCF / contig out of range");
                    if (!s->vcfs[v].nonneg) {
                        O.status = 1;
                        return;
                    }
                    const Segment &sg = s->vcfs[v].segments[c];
                    for (uint64_t h = a; h < b; ++h) {
                        uint32_t rec, k;
                        if (!C.hit(h, rec, k)) {
                            O.status = 1;
                            return;
                        }
                        if (rec < sg.lo || rec >= sg.hi || k >= C.n_alts(rec))
                            throw Error(SB_EINVAL, "sb_route_bodies: a hit outside its row's VCF contig");
                        hv.push_back(EvHit{C.cid[v][c], s->h_pos[rec], rec, k, static_cast<uint32_t>(h - h0)});
                    }
                }
                std::sort(hv.begin(), hv.end(), [](const EvHit &x, const EvHit &y) {
                    return x.cid != y.cid ? x.cid < y.cid : x.pos != y.pos ? x.pos < y.pos : x.ord < y.ord;
                });
                uint64_t total = 0;
                for (size_t i = 0; i < hv.size();) {
                    size_t j = i + 1;
                    while (j < hv.size() && hv[j].cid == hv[i].cid && hv[j].pos == hv[i].pos) ++j;
                    for (size_t x = i; x < j; ++x) {  // a (chrom, POS) group, in first-seen order
                        bool new_str = true, new_id = true;
                        for (size_t y = i; y < x && (new_str || new_id); ++y) {
                            if (!C.same_ref_alt(hv[x], hv[y])) continue;
                            new_id = false;
                            if (s->h_vt[hv[x].rec] == s->h_vt[hv[y].rec]) new_str = false;
                        }
                        total += new_str;
                        if (new_id) first_id[h0 + hv[x].ord] = 1;
                    }
                    i = j;
                }
                O.total = total;
            }
            // the body's length
            const size_t gl = std::strlen(gran_name(g));
            uint64_t n = C.head_pre.size() + gl + C.head_mid.size() + L(kB_gran2) + gl + L(kB_head_end) + 1;  // + '\n'
            const uint64_t tf = O.exists ? 4 : 5;
            if (g == SB_GRAN_BOOLEAN) {
                n += 2 + L(kB_sum) + tf + L(kB_close);
            } else if (g == SB_GRAN_COUNT) {
                n += 2 + L(kB_sum) + tf + L(kB_total) + dec_len(O.total) + L(kB_close);
            } else {
                if (C.asm_json[E.assembly].size() == 1 && C.asm_json[E.assembly][0] == '\x01') {
                    O.status = 1;
                    return;
                }
                n += pag[E.pagination].size() + L(kB_rs0) + L(kB_rs1) + L(kB_rs2) + L(kB_rs3) + L(kB_sum) + tf +
                     L(kB_total) + dec_len(O.total) + L(kB_close);
                uint64_t nres = 0;
                if (fold) {
                    const uint64_t h0 = C.off(E.row_lo);
                    for (uint32_t r = E.row_lo; r < E.row_hi; ++r) {
                        if (C.off(r + 1) == C.off(r)) continue;
                        const uint32_t cid = C.cid[C.row_vcf(r)][C.row_contig(r)];
                        for (uint64_t h = C.off(r), b = C.off(r + 1); h < b; ++h) {
                            if (!first_id[h]) continue;
                            uint32_t rec, k;
                            C.hit(h, rec, k);
                            const uint64_t el = entry_len(C, E.assembly, cid, rec, k);
                            if (!el) {
                                O.status = 1;
                                return;
                            }
                            n += el + (nres ? 2 : 0);
                            ++nres;
                        }
                    }
                    (void)h0;
                }
                O.results = nres;
                n += (nres > 0 ? 4 : 5) + dec_len(nres);
            }
            O.len = n;
        }), 16, 256);
        fe.rethrow();
        tick("fold");
        auto R = std::make_unique<sb_json_out>();
        R->status.resize(ne);
        R->off.assign(ne + 1, 0);
        for (size_t e = 0; e < ne; ++e) {
            R->status[e] = eo[e].status;
            R->off[e + 1] = R->off[e] + (eo[e].status ? 0 : eo[e].len);
        }
        R->n = R->off[ne];
        R->buf = big_alloc(R->n, &R->cap);
        char *const base = R->buf.get();
        tick("alloc");
        // pass 2: write each body in place
        parallel_for(ne, fe.wrap([&](size_t e) {
            prefetch_ahead(e);
            const EvOut &O = eo[e];
            if (O.status) return;
            const sb_route_event &E = in->events[e];
            const uint8_t g = E.granularity;
            const char *gn = gran_name(g);
            char *o = base + R->off[e];
            o = put(o, C.head_pre);
            o = put(o, gn, std::strlen(gn));
            o = put(o, C.head_mid);
            if (g == SB_GRAN_BOOLEAN || g == SB_GRAN_COUNT) o = lit(o, "{}");
            else o = put(o, pag[E.pagination]);
            o = lit(o, kB_gran2);
            o = put(o, gn, std::strlen(gn));
            o = lit(o, kB_head_end);
            auto tf = [](char *p, bool b) { return b ? lit(p, "true") : lit(p, "false"); };
            if (g == SB_GRAN_BOOLEAN) {
                o = lit(o, kB_sum);
                o = tf(o, O.exists);
                o = lit(o, kB_close);
            } else if (g == SB_GRAN_COUNT) {
                o = lit(o, kB_sum);
                o = tf(o, O.exists);
                o = lit(o, kB_total);
                o = dec_write(o, O.total);
                o = lit(o, kB_close);
            } else {
                o = lit(o, kB_rs0);
                o = tf(o, O.results > 0);
                o = lit(o, kB_rs1);
                if (O.results) {
                    bool any = false;
                    for (uint32_t r = E.row_lo; r < E.row_hi; ++r) {
                        if (C.off(r + 1) == C.off(r)) continue;
                        const uint32_t cid = C.cid[C.row_vcf(r)][C.row_contig(r)];
                        for (uint64_t h = C.off(r), b = C.off(r + 1); h < b; ++h) {
                            if (!first_id[h]) continue;
                            uint32_t rec, k;
                            C.hit(h, rec, k);
                            if (any) o = lit(o, ", ");
                            any = true;
                            o = entry_write(C, o, E.assembly, cid, rec, k);
                        }
                    }
                }
                o = lit(o, kB_rs2);
                o = dec_write(o, O.results);
                o = lit(o, kB_rs3);
                o = lit(o, kB_sum);
                o = tf(o, O.exists);
                o = lit(o, kB_total);
                o = dec_write(o, O.total);
                o = lit(o, kB_close);
            }
            *o++ = '\n';
            if (static_cast<uint64_t>(o - (base + R->off[e])) != O.len)
                throw Error(SB_EINTERNAL, "sb_route_bodies: body length mismatch at event " + std::to_string(e));
        }), 16, 256);
        fe.rethrow();
        tick("write");
        *out = R.release();
    });
}
