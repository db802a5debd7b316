// ingest.cpp — VCF text -> columnar store (host, multi-threaded).
//
// This replaces what the reference gets from htslib/bcftools per query
// (lambda/performQuery/search_variants.py:42-50): it decodes each record
// ONCE and precomputes, per record and per ALT, every quantity the query
// loop at :84-250 derives from the record text, so the device scan never
// parses text:
//   * end = POS + len(REF) - 1                        (:87-91)
//   * key(REF.upper()), key(ALT.upper())              (:94, :173, :180)
//   * ALT classes: single base, symbolic, '.', REF-repeat count (:101-166)
//   * last AC= / AN= / VT= of INFO with the int() failure modes (:195-206)
//   * genotype fallbacks: count of each allele number and of all calls in
//     the GT text (re '[0-9]+', :28, :219, :249) for records without AC/AN
//   * per-ALT carrier bitplanes: sample whose GT has a token equal to the
//     1-based allele number (the regex at :233-236)
#include <algorithm>
#include <atomic>
#include <cstring>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <zlib.h>

#include "store.hpp"

namespace sb {
namespace {

struct Local {  // one thread's parse of a run of lines
    VcfCols c;
    std::vector<uint32_t> contig_of;  // per record: index into contigs
    std::vector<std::string> contigs;
    std::string vtbuf;
    std::vector<int64_t> vt_off;  // -1 = no VT tag
    std::vector<uint32_t> vt_len;
    int err = 0;
    std::string msg;
    size_t err_line = 0;
    // per-record scratch, reused record to record
    std::vector<const char *> alt_p, ac_p;
    std::vector<size_t> alt_n, ac_n;
    std::vector<int64_t> acv, gtcount;
    std::vector<uint32_t> limbs;
    std::unordered_map<std::string_view, uint32_t> val_id;
};

inline bool is_digit(char c) { return c >= '0' && c <= '9'; }

// ---- summariseSlice per-record restatement --------------------------------
// The reference reader walks one record as recordHeader (write_data_to_s3.h:
// 150-228) then addCounts (main.cpp:52-109).  Both are simulated here on the
// record's own line; a read that would run off the line (into the next
// record) marks the record unsupported.
struct LineRd {
    const char *s;
    size_t n, pos;
    bool off_end;
};

char lr_read_past(LineRd &r, char a, char b, size_t *fs, size_t *fl) {  // readPastChars<a, b>
    const size_t st = r.pos;
    while (r.pos < r.n) {
        const char c = r.s[r.pos];
        if (c == a || c == b) {
            *fs = st;
            *fl = r.pos - st;
            ++r.pos;
            return c;
        }
        ++r.pos;
    }
    r.off_end = true;
    return '\0';
}

bool lr_skip_past(LineRd &r, char d, int N) {  // skipPast<N, d>
    int num = N;
    while (r.pos < r.n)
        if (r.s[r.pos++] == d && (N == 1 || --num == 0)) return true;
    r.off_end = true;
    return false;
}

// fast_atoi.h:73-99 atoui64(str, len); false where the reference is UB (len > 20)
bool atoui64_len(const char *str, uint8_t len, uint64_t *out) {
    if (len > 20) return false;
    static const uint64_t ones[21] = {0, 1ull, 11ull, 111ull, 1111ull, 11111ull, 111111ull, 1111111ull, 11111111ull,
                                      111111111ull, 1111111111ull, 11111111111ull, 111111111111ull,
                                      1111111111111ull, 11111111111111ull, 111111111111111ull,
                                      1111111111111111ull, 11111111111111111ull, 111111111111111111ull,
                                      1111111111111111111ull, 11111111111111111111ull};
    uint64_t v = 0, p10 = 1;
    for (int k = 1; k <= len; ++k) {
        v += static_cast<uint64_t>(static_cast<int64_t>(static_cast<signed char>(str[len - k]))) * p10;
        p10 *= 10ull;
    }
    *out = v - static_cast<uint64_t>('0') * ones[len];
    return true;
}

// generalutils.hpp:19-36 sequenceToBinary; -1 where std::map::at throws
inline int seq_code(char c) {
    switch (c) {
        case 'A': case 'a': return 1;
        case 'C': case 'c': return 2;
        case 'G': case 'g': return 3;
        case 'T': case 't': return 4;
        case 'N': case 'n': return 5;
        case '*': return 6;
        case '.': return 7;
        default: return -1;
    }
}

// write_data_to_s3.h:103-134 compressSeq; false where the reference throws.
// The reference appends each packed byte with append((char *)&contigBin),
// i.e. as a C string running past the byte (UB); the intended single byte is
// appended here.
bool compress_seq(const char *s, size_t n, std::string &out) {
    if (n == 1) {
        const int v = seq_code(s[0]);
        if (v < 0) return false;
        out.push_back(static_cast<char>(v));
        return true;
    }
    if (s[0] == '<' && s[n - 1] == '>') {
        out.append(s + 1, n - 2);
        return true;
    }
    for (size_t i = 0; i < n; i += 2) {
        int v = seq_code(s[i]);
        if (v < 0) return false;
        if (i + 1 < n) {
            const int w = seq_code(s[i + 1]);
            if (w < 0) return false;
            v = (v << 4) | w;
        }
        out.push_back(static_cast<char>(v));
    }
    return true;
}

// hash of a duplicateVariantSearch key string (FNV-1a + splitmix finaliser)
uint64_t key_hash(const char *p, size_t n, uint64_t h = 0xcbf29ce484222325ull) {
    for (size_t i = 0; i < n; ++i) {
        h ^= static_cast<uint8_t>(p[i]);
        h *= 0x100000001b3ull;
    }
    return h;
}
uint64_t key_finish(uint64_t h) {
    h ^= h >> 30;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 27;
    h *= 0x94d049bb133111ebull;
    return h ^ (h >> 31);
}

// one region-file entry {pos, ref', alt'} -> key columns
void push_key(VcfCols &c, uint64_t pos, const std::string &ref, const std::string &alt) {
    char digits[24];
    const int nd = snprintf(digits, sizeof digits, "%llu", static_cast<unsigned long long>(pos));
    uint64_t h = key_hash(digits, static_cast<size_t>(nd));
    h = key_hash(ref.data(), ref.size(), h);
    h = key_hash("_", 1, h);
    h = key_hash(alt.data(), alt.size(), h);
    const size_t tl = ref.size() + 1 + alt.size();
    uint64_t tail;
    if (tl <= static_cast<size_t>(kTailInlineMax)) {
        tail = static_cast<uint64_t>(tl) << 56;
        size_t k = 0;
        for (char ch : ref) tail |= static_cast<uint64_t>(static_cast<uint8_t>(ch)) << (8 * k++);
        tail |= static_cast<uint64_t>('_') << (8 * k++);
        for (char ch : alt) tail |= static_cast<uint64_t>(static_cast<uint8_t>(ch)) << (8 * k++);
    } else {
        tail = kTailBlob | (static_cast<uint64_t>(tl) << 40) | c.dk_blob.size();
        c.dk_blob.insert(c.dk_blob.end(), ref.begin(), ref.end());
        c.dk_blob.push_back('_');
        c.dk_blob.insert(c.dk_blob.end(), alt.begin(), alt.end());
    }
    c.dk_pos.push_back(static_cast<uint32_t>(pos));
    c.dk_hash.push_back(key_finish(h));
    c.dk_tail.push_back(tail);
}

// line = record bytes incl. its '\n' (if any); fills the summary columns and
// the record's region-file keys (c.dk_*)
void summarise_line(const char *line, size_t len, uint32_t rec, VcfCols &cols, SumHot *sum, uint32_t *cur,
                    uint32_t *dcount) {
    LineRd r{line, len, 0, false};
    bool bad = false, key_bad = false;
    uint64_t kpos = 0;
    std::string ref, alt;
    std::vector<std::string> alts;
    // recordHeader with the contig already known: skip CHROM, POS field,
    // skip ID, REF, ALT (',' continues ALT), then skip QUAL and FILTER.
    // A first record reads CHROM as a field instead: identical unless CHROM
    // is empty or holds ',' (flagged).
    {
        size_t fs, fl;
        const char c0 = lr_read_past(r, '\t', ',', &fs, &fl);
        if (c0 != '\t' || fl == 0) bad = true;
    }
    int loop_pos = 1;
    do {
        size_t fs, fl;
        const char last = lr_read_past(r, '\t', ',', &fs, &fl);
        if (last == '\0') break;
        if (fl >= 1) {  // empty parts are skipped, as the reference does
            switch (++loop_pos) {
                case 2:  // fast_atoi<uint64_t> (generalutils.hpp:38-45)
                    kpos = 0;
                    for (size_t i = 0; i < fl; ++i)
                        kpos = kpos * 10 + static_cast<uint64_t>(static_cast<int64_t>(line[fs + i] - '0'));
                    lr_skip_past(r, '\t', 1);
                    ++loop_pos;
                    break;
                case 4:
                    ref.clear();
                    if (!compress_seq(line + fs, fl, ref)) key_bad = true;
                    break;
                case 5:
                    alt.clear();
                    if (!compress_seq(line + fs, fl, alt)) key_bad = true;
                    alts.push_back(alt);
                    if (last == ',') --loop_pos;
                    break;
                default:
                    break;
            }
        }
    } while (loop_pos <= 4);
    if (r.off_end || kpos > 0xffffffffull) key_bad = true;
    for (const auto &a : alts)
        if (ref.size() + 1 + a.size() > 0xffff) key_bad = true;  // beyond the region file's u16 length
    if (key_bad) {
        cols.dk_bad.push_back(rec);  // the reference's summariseSlice throws here
        bad = true;
    } else {
        for (const auto &a : alts) push_key(cols, kpos, ref, a);
    }
    cols.dk_lo.push_back(static_cast<uint32_t>(cols.dk_hash.size()));
    lr_skip_past(r, '\t', 2);
    // addCounts
    uint64_t nv = 0, nc = 0;
    bool found_ac = false, found_an = false;
    do {
        size_t fs, fl;
        const char last = lr_read_past(r, ';', '\t', &fs, &fl);
        if (last == '\0') break;
        if (fl >= 4) {
            const char *f = line + fs;
            if (!memcmp(f, "AC=", 3)) {
                found_ac = true;
                nv += 1;
                for (size_t j = 3; j < fl; ++j) nv += f[j] == ',';
            } else if (!memcmp(f, "AN=", 3)) {
                found_an = true;
                uint64_t v;
                if (!atoui64_len(f + 3, static_cast<uint8_t>(static_cast<uint8_t>(fl) - 3), &v)) bad = true;
                else nc += v;
            }
        }
        if (last == '\t' && !(found_ac && found_an)) break;
    } while (!(found_ac && found_an));
    if (r.off_end) bad = true;  // the reference would continue into the next line
    const size_t c = r.pos;
    uint32_t d = 0;
    for (size_t i = c; i < len && line[i] != '\n'; ++i) {
        const char ch = line[i];
        d += (ch == '\t') | (ch == '/') | (ch == '|') | (ch == ';') | (ch == ':');
    }
    if (nv >= kSumUnsupported || len > 0xffffffffull) bad = true;
    sum->rem = static_cast<uint32_t>(len - c);
    sum->nvf = static_cast<uint32_t>(nv & 0x7fffffffu) | (bad ? kSumUnsupported : 0u);
    sum->nc = nc;
    *cur = static_cast<uint32_t>(c);
    *dcount = d;
}

struct Parser {
    uint32_t n_samples;
    uint32_t words;
    bool keep_gt;

    // [p, e) = the record without its line terminator; [p, full_end) with it;
    // abs = offset of p in the VCF text stream.  Returns false and sets L.err
    // on failure.
    bool line(const char *p, const char *e, const char *full_end, uint64_t abs, Local &L) {
        {
            VcfCols &c = L.c;
            SumHot sh;
            uint32_t cu, dc;
            summarise_line(p, static_cast<size_t>(full_end - p), static_cast<uint32_t>(c.start.size()), c, &sh, &cu,
                           &dc);
            c.start.push_back(abs);
            c.sum.push_back(sh);
            c.cur.push_back(cu);
            c.dcount.push_back(dc);
        }
        // ---- fixed columns
        const char *f[9];
        size_t n[9];
        const char *q = p;
        int col = 0;
        while (col < 9 && q <= e) {
            const char *t = static_cast<const char *>(memchr(q, '\t', static_cast<size_t>(e - q)));
            if (!t) t = e;
            f[col] = q;
            n[col] = static_cast<size_t>(t - q);
            ++col;
            q = t + 1;
        }
        if (col < 8) return fail(L, "record with fewer than 8 columns");
        // CHROM
        const std::string chrom(f[0], n[0]);
        if (L.contigs.empty() || L.contigs.back() != chrom) L.contigs.push_back(chrom);
        L.contig_of.push_back(static_cast<uint32_t>(L.contigs.size() - 1));
        // POS: canonical decimal (bcftools prints it back canonically)
        if (n[1] == 0 || n[1] > 10 || (n[1] > 1 && f[1][0] == '0')) return fail(L, "non-canonical POS");
        uint64_t pos = 0;
        for (size_t i = 0; i < n[1]; ++i) {
            if (!is_digit(f[1][i])) return fail(L, "non-numeric POS");
            pos = pos * 10 + static_cast<uint64_t>(f[1][i] - '0');
        }
        if (pos > 0xffffffffull) return fail(L, "POS beyond 32 bits");
        // REF
        const uint8_t *ref = reinterpret_cast<const uint8_t *>(f[3]);
        const size_t ref_len = n[3];
        if (ref_len == 0) return fail(L, "empty REF");
        const uint64_t end = pos + ref_len - 1;
        if (end > 0xffffffffull) return fail(L, "POS+len(REF) beyond 32 bits");
        bool ref_hashed;
        const uint64_t ref_key = allele_key(ref, ref_len, true, &ref_hashed);
        VcfCols &c = L.c;
        c.pos.push_back(static_cast<uint32_t>(pos));
        c.ref_key.push_back(ref_key);
        c.ref_off.push_back(c.blob.size());
        c.blob.insert(c.blob.end(), ref, ref + ref_len);
        // ALT split on ',' (:97): any number of ALTs
        auto &alt_p = L.alt_p;
        auto &alt_n = L.alt_n;
        alt_p.clear();
        alt_n.clear();
        {
            const char *a = f[4], *ae = f[4] + n[4];
            for (;;) {
                const char *cm = static_cast<const char *>(memchr(a, ',', static_cast<size_t>(ae - a)));
                if (!cm) cm = ae;
                alt_p.push_back(a);
                alt_n.push_back(static_cast<size_t>(cm - a));
                if (cm == ae) break;
                a = cm + 1;
            }
        }
        if (alt_p.size() > 0xfffffffull) return fail(L, "more than 2^28 ALTs in one record");
        uint32_t na = static_cast<uint32_t>(alt_p.size());
        // general: the packed words cannot hold this record (devtypes.hpp GenRec)
        bool general = na > 64;
        // ---- INFO (:195-201): last AC= string, every AN= parsed, last VT=
        const char *ac_s = nullptr;
        size_t ac_sn = 0;
        const char *an_s = nullptr;  // text of the last AN= (general records re-parse it)
        size_t an_sn = 0;
        bool has_ac = false, has_an = false, an_bad = false, an_big = false;
        int64_t an_val = 0;
        int64_t vt_off = -1;
        uint32_t vt_len = 0;
        {
            const char *a = f[7], *ae = f[7] + n[7];
            for (;;) {
                const char *sc = static_cast<const char *>(memchr(a, ';', static_cast<size_t>(ae - a)));
                if (!sc) sc = ae;
                const size_t fl = static_cast<size_t>(sc - a);
                if (fl >= 3 && a[2] == '=') {
                    if (a[0] == 'A' && a[1] == 'C') {
                        has_ac = true;
                        ac_s = a + 3;
                        ac_sn = fl - 3;
                    } else if (a[0] == 'A' && a[1] == 'N') {
                        int64_t v = 0;
                        if (!an_bad) {
                            const int st = py_int_ex(a + 3, fl - 3, &v);
                            if (st < 0) {
                                an_bad = true;
                            } else {
                                an_val = v;
                                an_big = st == 1;
                                an_s = a + 3;
                                an_sn = fl - 3;
                                has_an = true;
                            }
                        }
                    } else if (a[0] == 'V' && a[1] == 'T') {
                        vt_off = static_cast<int64_t>(L.vtbuf.size());
                        vt_len = static_cast<uint32_t>(fl - 3);
                        L.vtbuf.append(a + 3, fl - 3);
                    }
                }
                if (sc == ae) break;
                a = sc + 1;
            }
        }
        L.vt_off.push_back(vt_off);
        L.vt_len.push_back(vt_len);
        if (has_an && (an_big || an_val > INT32_MAX || an_val < INT32_MIN)) general = true;
        // AC values (:206)
        auto &acv = L.acv;
        acv.clear();
        L.ac_p.clear();
        L.ac_n.clear();
        bool ac_bad = false;
        if (has_ac) {
            const char *a = ac_s, *ae = ac_s + ac_sn;
            for (;;) {
                const char *cm = static_cast<const char *>(memchr(a, ',', static_cast<size_t>(ae - a)));
                if (!cm) cm = ae;
                int64_t v = 0;
                const int st = py_int_ex(a, static_cast<size_t>(cm - a), &v);
                if (st < 0) {
                    ac_bad = true;
                } else {
                    if (st == 1 || v > INT32_MAX || v < INT32_MIN) general = true;
                    acv.push_back(st == 1 ? 0 : v);
                    L.ac_p.push_back(a);
                    L.ac_n.push_back(static_cast<size_t>(cm - a));
                }
                if (cm == ae) break;
                a = cm + 1;
            }
        }
        const uint32_t n_ac = static_cast<uint32_t>(acv.size());
        // a GT fallback over >= 8 ALTs emits variants in CPython set order (:223)
        if (!has_ac && n_samples > 0 && na >= 8) general = true;
        // ---- genotypes
        auto &gtcount = L.gtcount;
        gtcount.assign(na, 0);
        int64_t gt_an = 0;
        const bool need_fb = (!has_ac || !has_an || an_bad) && n_samples > 0;
        const size_t plane0 = c.planes0.size(), planex = c.planesx.size();
        if (keep_gt && n_samples) {
            c.planes0.resize(plane0 + words, 0ull);
            c.planesx.resize(planex + static_cast<size_t>(na - 1) * words, 0ull);
        }
        const size_t fb0 = c.fb.size();
        int64_t fb_row = -1;
        if (need_fb && !general) {
            fb_row = static_cast<int64_t>(c.fb.size());
            c.fb.resize(c.fb.size() + n_samples, 0u);
        }
        int gt_idx = -1;
        if (n_samples) {
            if (col < 9) return fail(L, "missing FORMAT/sample columns");
            // FORMAT: index of GT
            {
                int k = 0;
                const char *a = f[8], *ae = f[8] + n[8];
                for (;;) {
                    const char *cl = static_cast<const char *>(memchr(a, ':', static_cast<size_t>(ae - a)));
                    if (!cl) cl = ae;
                    if (cl - a == 2 && a[0] == 'G' && a[1] == 'T') gt_idx = k;
                    ++k;
                    if (cl == ae) break;
                    a = cl + 1;
                }
            }
            uint32_t s = 0;
            const char *a = q;
            while (s < n_samples) {
                if (a > e) return fail(L, "fewer sample columns than header samples");
                const char *t = static_cast<const char *>(memchr(a, '\t', static_cast<size_t>(e - a)));
                if (!t) t = e;
                const char *g, *ge;
                gt_field(a, t, gt_idx, &g, &ge);
                const size_t gl = static_cast<size_t>(ge - g);
                if (gl == 3 && g[0] == '0' && g[2] == '0' && (g[1] == '|' || g[1] == '/')) {
                    gt_an += 2;  // hot path: homozygous REF
                    if (fb_row >= 0) c.fb[static_cast<size_t>(fb_row) + s] = 2u;
                } else {
                    // digit runs (re '[0-9]+'): calls for counts / AN fallback
                    uint32_t nrun = 0, vals[3] = {0, 0, 0};
                    for (size_t i = 0; i < gl;) {
                        if (is_digit(g[i])) {
                            uint64_t v = 0;
                            size_t j = i;
                            while (j < gl && is_digit(g[j])) {
                                if (v < (1ull << 40)) v = v * 10 + static_cast<uint64_t>(g[j] - '0');
                                ++j;
                            }
                            ++gt_an;
                            if (v >= 1 && v <= na) gtcount[v - 1]++;
                            if (need_fb) {
                                if (nrun >= 3 || v > 254)
                                    general = true;  // beyond the packed fallback row
                                else
                                    vals[nrun] = static_cast<uint32_t>(v);
                            }
                            ++nrun;
                            i = j;
                        } else {
                            ++i;
                        }
                    }
                    if (fb_row >= 0) c.fb[static_cast<size_t>(fb_row) + s] = nrun | (vals[0] << 8) | (vals[1] << 16) | (vals[2] << 24);
                    // carrier: a token (split on | and /) equal to str(allele number)
                    // (the regex at :233-236: canonical decimal, no leading zero)
                    if (keep_gt) {
                        size_t i = 0;
                        while (i <= gl) {
                            size_t j = i;
                            while (j < gl && g[j] != '|' && g[j] != '/') ++j;
                            const size_t tl = j - i;
                            if (tl >= 1 && tl <= 10 && g[i] != '0') {
                                uint64_t v = 0;
                                size_t k = i;
                                while (k < j && is_digit(g[k])) v = v * 10 + static_cast<uint64_t>(g[k++] - '0');
                                if (k == j) {
                                    if (v == 1)
                                        c.planes0[plane0 + (s >> 6)] |= 1ull << (s & 63);
                                    else if (v >= 2 && v <= na)
                                        c.planesx[planex + static_cast<size_t>(v - 2) * words + (s >> 6)] |= 1ull << (s & 63);
                                }
                            }
                            i = j + 1;
                        }
                    }
                }
                ++s;
                a = t + 1;
            }
        }
        const int64_t anv = has_an ? an_val : gt_an;
        if (!an_big && (anv > INT32_MAX || anv < INT32_MIN)) general = true;
        // ---- per-ALT class words (symbolic ids are resolved at merge)
        uint32_t hot = 0;
        if (has_ac) hot |= H_HAS_AC;
        if (has_an) hot |= H_HAS_AN;
        if (ac_bad) hot |= H_AC_BAD;
        if (an_bad) hot |= H_AN_BAD;
        if (need_fb) hot |= H_HAS_FB;
        if (na > 1) hot |= H_MULTI;
        uint32_t gen_idx = 0;
        if (general) {
            // the GenRec side table answers it (general_slice_kernel); the
            // packed words mark it (H_AN_BAD + kAnUnrepresentable, ac0 = index)
            hot = H_HAS_AN | H_AN_BAD | (na > 1 ? H_MULTI : 0u);
            if (fb_row >= 0) c.fb.resize(fb0);
            fb_row = -1;
            gen_idx = static_cast<uint32_t>(c.gen.size());
            GenRec gr{};
            gr.rec = static_cast<uint32_t>(c.pos.size() - 1);
            gr.flags = (has_ac ? GR_HAS_AC : 0u) | (has_an ? GR_HAS_AN : 0u) | (ac_bad ? GR_AC_BAD : 0u) |
                       (an_bad ? GR_AN_BAD : 0u);
            gr.n_alt = na;
            gr.n_ac = ac_bad ? 0u : n_ac;
            auto put_num = [&](const char *p, size_t len, int64_t small, bool big) {
                if (big) py_int_limbs(p, len, L.limbs);
                else i64_limbs(small, L.limbs);
                c.gnum.insert(c.gnum.end(), L.limbs.begin(), L.limbs.end());
                c.gnum_off.push_back(c.gnum.size());
            };
            gr.ac_num = c.gnum_off.size() - 1;
            if (has_ac && !ac_bad)
                for (uint32_t k = 0; k < n_ac; ++k) {
                    int64_t v = 0;
                    const bool big = py_int_ex(L.ac_p[k], L.ac_n[k], &v) == 1;
                    put_num(L.ac_p[k], L.ac_n[k], acv[k], big);
                }
            gr.an_num = c.gnum_off.size() - 1;
            if (has_an && !an_bad) put_num(an_s, an_sn, an_val, an_big);
            if ((!has_ac || !has_an) && n_samples > 0) {
                // every GT digit run of every sample, as value ids numbered in
                // first-occurrence order (:218 int(g), :249 len(all_calls))
                gr.flags |= GR_FB;
                gr.tok_off = c.gtok_off.size();
                gr.val_off = static_cast<uint32_t>(c.gval.size());
                L.val_id.clear();
                const char *a = q;
                for (uint32_t s = 0; s < n_samples; ++s) {
                    const char *t = static_cast<const char *>(memchr(a, '\t', static_cast<size_t>(e - a)));
                    if (!t) t = e;
                    const char *g, *ge;
                    gt_field(a, t, gt_idx, &g, &ge);
                    c.gtok_off.push_back(c.gtok.size());
                    for (const char *x = g; x < ge;) {
                        if (!is_digit(*x)) {
                            ++x;
                            continue;
                        }
                        const char *x0 = x;
                        while (x < ge && is_digit(*x)) ++x;
                        const size_t raw = static_cast<size_t>(x - x0);
                        const char *d = x0;
                        while (d < x - 1 && *d == '0') ++d;  // the value's significant digits
                        const std::string_view key(d, static_cast<size_t>(x - d));
                        auto it = L.val_id.find(key);
                        uint32_t id;
                        if (it == L.val_id.end()) {
                            id = static_cast<uint32_t>(L.val_id.size());
                            L.val_id.emplace(key, id);
                            GenVal gv{0, 0, 0};
                            unsigned __int128 h = 0;
                            for (const char *y = d; y < x; ++y)
                                h = (h * 10u + static_cast<unsigned>(*y - '0')) % 2305843009213693951ull;
                            gv.hash = static_cast<uint64_t>(h);
                            if (key.size() <= 10) {
                                uint64_t v = 0;
                                for (char ch : key) v = v * 10 + static_cast<uint64_t>(ch - '0');
                                if (v >= 1 && v <= na) gv.allele = static_cast<uint32_t>(v);
                            }
                            gv.huge = raw > kPyMaxStrDigits ? 1u : 0u;
                            c.gval.push_back(gv);
                        } else {
                            id = it->second;
                            if (raw > kPyMaxStrDigits) c.gval[gr.val_off + id].huge = 1u;
                        }
                        c.gtok.push_back(id);
                    }
                    a = t + 1;
                }
                c.gtok_off.push_back(c.gtok.size());
                gr.n_vals = static_cast<uint32_t>(L.val_id.size());
            }
            c.gen.push_back(gr);
        }
        int32_t ac0 = 0;
        uint32_t rh_info = 0;  // RangeHot (MODE_RANGE_N) view
        int64_t rh_c = 0;
        for (uint32_t i = 0; i < na; ++i) {
            const uint8_t *ap = reinterpret_cast<const uint8_t *>(alt_p[i]);
            const size_t al = alt_n[i];
            bool hashed;
            const uint64_t key = allele_key(ap, al, true, &hashed);
            uint32_t cls = 0;
            if (al == 1) {
                const uint8_t u = upc(ap[0]);
                if (u == 'A' || u == 'C' || u == 'G' || u == 'T' || u == 'N') cls |= C_SINGLE_BASE;
            }
            if (al >= 1 && ap[0] == '<') cls |= C_SYMBOLIC;
            if (al == 1 && ap[0] == '.') cls |= C_DOT;
            // alt == REF * k (raw bytes): fullmatch of '(REF){2,}' / '(REF)*' (:124,:146)
            uint32_t rep = C_REP_NONE;
            if (al % ref_len == 0) {
                const size_t k = al / ref_len;
                bool ok = true;
                for (size_t j = 0; j < k && ok; ++j) ok = memcmp(ap + j * ref_len, ref, ref_len) == 0;
                if (ok) rep = k >= 62 ? 62u : static_cast<uint32_t>(k);
            }
            cls |= rep << C_REP_SHIFT;
            int64_t acval = 0;
            if (general) {
                if (i == 0) c.gen.back().a0_cls = cls;
            } else if (has_ac) {
                if (i >= n_ac) cls |= C_AC_MISSING;
                acval = (!ac_bad && i < n_ac) ? acv[i] : 0;
                if (acval < 0) c.any_negative = true;
            } else {
                acval = gtcount[i];
            }
            if (!general && (cls & C_SINGLE_BASE)) {
                rh_info |= RH_HIT;
                if (!has_ac || (cls & C_AC_MISSING)) rh_info |= RH_SLOW;
                rh_c += acval;
                if (acval != 0) rh_info |= i < 8 ? (1u << i) : RH_SLOW;
            }
            if (i == 0) {
                if (!general) hot |= cls;
                ac0 = static_cast<int32_t>(acval);
                c.a0_key.push_back(key);
                c.a0_len.push_back(static_cast<uint32_t>(al));
                c.a0_off.push_back(c.blob.size());
            } else {
                c.x_key.push_back(key);
                c.x_len.push_back(static_cast<uint32_t>(al));
                c.x_cls.push_back(cls);
                c.x_ac.push_back(static_cast<int32_t>(acval));
                c.x_off.push_back(c.blob.size());
            }
            c.blob.insert(c.blob.end(), ap, ap + al);
        }
        if (general) {
            ac0 = static_cast<int32_t>(gen_idx);  // GenRec index (vcf-local until merge)
            rh_info = RH_HIT | RH_SLOW;           // every range query evaluates it
        }
        const int32_t an32 = general ? kAnUnrepresentable : static_cast<int32_t>(anv);
        c.rec.push_back(RecHot{static_cast<uint32_t>(end), hot, an32, ac0});
        if (an_bad || ac_bad || rh_c > INT32_MAX || rh_c < INT32_MIN) rh_info |= RH_SLOW;
        c.rng.push_back(RangeHot{static_cast<uint32_t>(end), rh_info, an32,
                                 static_cast<int32_t>((rh_info & RH_SLOW) ? 0 : rh_c)});
        c.fb_off.push_back(fb_row);
        c.x_lo.push_back(static_cast<uint32_t>(c.x_key.size()));
        return true;
    }

    // the GT subfield of one sample column [a, t) (FORMAT index gt_idx; none: '.')
    static void gt_field(const char *a, const char *t, int gt_idx, const char **g, const char **ge) {
        if (gt_idx < 0) {
            *g = ".";
            *ge = *g + 1;  // no GT key: bcftools prints '.'  (unpinned)
            return;
        }
        const char *x = a, *xe = t;
        for (int k = 0; k < gt_idx && x < xe; ++k) {
            const char *cl = static_cast<const char *>(memchr(x, ':', static_cast<size_t>(xe - x)));
            x = cl ? cl + 1 : xe;
        }
        const char *cl = static_cast<const char *>(memchr(x, ':', static_cast<size_t>(xe - x)));
        if (cl) xe = cl;
        *g = x;
        *ge = xe;
    }

    static bool fail(Local &L, const char *m) {
        L.err = SB_EPARSE;
        L.msg = m;
        return false;
    }
};

void parse_header_line(VcfData &v, const char *p, const char *e) {
    if (e - p >= 2 && p[1] == '#') return;
    // #CHROM POS ID REF ALT QUAL FILTER INFO [FORMAT samples...]
    std::vector<std::string> cols;
    const char *q = p;
    for (;;) {
        const char *t = static_cast<const char *>(memchr(q, '\t', static_cast<size_t>(e - q)));
        if (!t) t = e;
        cols.emplace_back(q, static_cast<size_t>(t - q));
        if (t == e) break;
        q = t + 1;
    }
    v.samples.clear();
    for (size_t i = 9; i < cols.size(); ++i) v.samples.push_back(cols[i]);
    v.words = static_cast<uint32_t>((v.samples.size() + 63) / 64);
    v.header_seen = true;
}

uint32_t sym_id(sb_builder &b, const uint8_t *p, uint32_t n) {
    const uint32_t id = b.sym.get(std::string(reinterpret_cast<const char *>(p), n));
    if (id > 0xffff) throw Error(SB_EPARSE, "more than 65535 distinct symbolic ALT strings");
    return id;
}

// reserve room for `extra` more elements with geometric growth (an exact
// reserve per merged chunk would copy the whole column every chunk)
template <class V>
void grow(V &v, size_t extra) {
    const size_t need = v.size() + extra;
    if (need > v.capacity()) v.reserve(std::max(need, 2 * v.capacity()));
}

void merge(sb_builder &b, VcfData &v, Local &L) {
    VcfCols &d = v.c;
    const VcfCols &s = L.c;
    const uint32_t rec0 = static_cast<uint32_t>(d.pos.size());
    const uint32_t x0 = static_cast<uint32_t>(d.x_key.size());
    const uint64_t blob0 = d.blob.size();
    const int64_t fb0 = static_cast<int64_t>(d.fb.size());
    const size_t nr = s.pos.size();
    // segments + sortedness (bcftools needs a sorted, indexed VCF)
    for (size_t i = 0; i < nr; ++i) {
        const std::string &ctg = L.contigs[L.contig_of[i]];
        const uint32_t r = rec0 + static_cast<uint32_t>(i);
        if (v.segments.empty() || v.segments.back().contig != ctg) {
            if (v.seg_index.count(ctg)) throw Error(SB_EPARSE, "contig " + ctg + " is not contiguous (unsorted VCF)");
            v.seg_index.emplace(ctg, static_cast<uint32_t>(v.segments.size()));
            v.segments.push_back(Segment{ctg, r, r + 1});
        } else {
            const uint32_t prev = i > 0 ? s.pos[i - 1] : d.pos.back();
            if (s.pos[i] < prev) throw Error(SB_EPARSE, "unsorted file: POS decreases on contig " + ctg);
            v.segments.back().hi = r + 1;
        }
    }
    auto app = [](auto &dst, const auto &src) { dst.insert(dst.end(), src.begin(), src.end()); };
    app(d.pos, s.pos);
    app(d.ref_key, s.ref_key);
    app(d.a0_key, s.a0_key);
    app(d.a0_len, s.a0_len);
    grow(d.rec, nr);
    app(d.rng, s.rng);
    grow(d.vt, nr);
    std::string last_vt;
    uint32_t last_id = 0;
    bool have_last = false;
    for (size_t i = 0; i < nr; ++i) {
        uint32_t id = 0;
        if (L.vt_off[i] >= 0) {
            if (have_last && last_vt.size() == L.vt_len[i] &&
                !memcmp(last_vt.data(), L.vtbuf.data() + L.vt_off[i], L.vt_len[i])) {
                id = last_id;
            } else {
                last_vt.assign(L.vtbuf.data() + L.vt_off[i], L.vt_len[i]);
                id = b.vt.get(last_vt);
                last_id = id;
                have_last = true;
            }
            if (id > 0xffff) throw Error(SB_EPARSE, "more than 65535 distinct VT values");
        }
        d.vt.push_back(static_cast<uint16_t>(id));
        RecHot h = s.rec[i];
        if (h.hot & C_SYMBOLIC) h.hot |= sym_id(b, s.blob.data() + s.a0_off[i], s.a0_len[i]) << C_SYM_SHIFT;
        if ((h.hot & H_AN_BAD) && h.an == kAnUnrepresentable) h.ac0 += static_cast<int32_t>(d.gen.size());
        d.rec.push_back(h);
    }
    {  // general records: indices into the merged side table
        const uint64_t num0 = d.gnum_off.size() - 1, tok0 = d.gtok_off.size(), gt0 = d.gtok.size();
        const uint32_t val0 = static_cast<uint32_t>(d.gval.size());
        const uint64_t limb0 = d.gnum.size();
        for (GenRec g : s.gen) {
            if (g.a0_cls & C_SYMBOLIC)
                g.a0_cls |= sym_id(b, s.blob.data() + s.a0_off[g.rec], s.a0_len[g.rec]) << C_SYM_SHIFT;
            g.rec += rec0;
            g.ac_num += num0;
            g.an_num += num0;
            if (g.flags & GR_FB) {
                g.tok_off += tok0;
                g.val_off += val0;
            }
            d.gen.push_back(g);
        }
        for (size_t k = 1; k < s.gnum_off.size(); ++k) d.gnum_off.push_back(s.gnum_off[k] + limb0);
        app(d.gnum, s.gnum);
        for (uint64_t o : s.gtok_off) d.gtok_off.push_back(o + gt0);
        app(d.gtok, s.gtok);
        app(d.gval, s.gval);
    }
    for (size_t i = 0; i < nr; ++i) d.ref_off.push_back(s.ref_off[i] + blob0);
    for (size_t i = 0; i < nr; ++i) d.a0_off.push_back(s.a0_off[i] + blob0);
    for (size_t i = 0; i < nr; ++i) d.fb_off.push_back(s.fb_off[i] < 0 ? -1 : s.fb_off[i] + fb0);
    for (size_t i = 1; i < s.x_lo.size(); ++i) d.x_lo.push_back(s.x_lo[i] + x0);
    app(d.x_key, s.x_key);
    app(d.x_len, s.x_len);
    app(d.x_ac, s.x_ac);
    for (size_t i = 0; i < s.x_off.size(); ++i) d.x_off.push_back(s.x_off[i] + blob0);
    grow(d.x_cls, s.x_cls.size());
    for (size_t i = 0; i < s.x_cls.size(); ++i) {
        uint32_t cls = s.x_cls[i];
        if (cls & C_SYMBOLIC) cls |= sym_id(b, s.blob.data() + s.x_off[i], s.x_len[i]) << C_SYM_SHIFT;
        d.x_cls.push_back(cls);
    }
    app(d.blob, s.blob);
    app(d.planes0, s.planes0);
    app(d.planesx, s.planesx);
    app(d.fb, s.fb);
    app(d.start, s.start);
    app(d.sum, s.sum);
    app(d.cur, s.cur);
    app(d.dcount, s.dcount);
    {
        const uint32_t k0 = static_cast<uint32_t>(d.dk_hash.size());
        const uint64_t kb0 = d.dk_blob.size();
        for (size_t i = 1; i < s.dk_lo.size(); ++i) d.dk_lo.push_back(s.dk_lo[i] + k0);
        app(d.dk_pos, s.dk_pos);
        app(d.dk_hash, s.dk_hash);
        grow(d.dk_tail, s.dk_tail.size());
        for (uint64_t t : s.dk_tail) d.dk_tail.push_back((t & kTailBlob) ? t + kb0 : t);
        app(d.dk_blob, s.dk_blob);
        for (uint32_t r : s.dk_bad) d.dk_bad.push_back(r + rec0);
    }
    d.any_negative = d.any_negative || s.any_negative;
}

// [p, p + len): whole lines; base = offset of p in the VCF text stream
void parse_records(sb_builder &b, VcfData &v, const char *p, size_t len, uint64_t base) {
    // line starts
    std::vector<const char *> starts;
    const char *e = p + len;
    for (const char *q = p; q < e;) {
        const char *nl = static_cast<const char *>(memchr(q, '\n', static_cast<size_t>(e - q)));
        if (!nl) nl = e;
        if (nl > q && !(nl - q == 1 && *q == '\r')) starts.push_back(q);
        q = nl + 1;
    }
    if (starts.empty()) return;
    for (const char *s : starts)
        if (*s == '#') throw Error(SB_EPARSE, "header line after records");
    if (!v.header_seen) throw Error(SB_EPARSE, "records before the #CHROM header line");
    {  // a shard build keeps the records [rec_lo, rec_hi) of the file
        const uint64_t o0 = v.lines_seen;
        v.lines_seen += starts.size();
        if (v.rec_lo > o0 || v.rec_hi < v.lines_seen) {
            const uint64_t a = std::min<uint64_t>(std::max(v.rec_lo, o0) - o0, starts.size());
            const uint64_t b = std::max<uint64_t>(std::min(v.rec_hi, v.lines_seen), o0 + a) - o0;
            starts = std::vector<const char *>(starts.begin() + static_cast<std::ptrdiff_t>(a),
                                               starts.begin() + static_cast<std::ptrdiff_t>(std::min<uint64_t>(b, starts.size())));
            if (starts.empty()) return;
        }
    }
    const size_t nl = starts.size();
    unsigned nt = b.opts.n_threads > 0 ? static_cast<unsigned>(b.opts.n_threads) : std::thread::hardware_concurrency();
    nt = std::max(1u, std::min<unsigned>(nt, static_cast<unsigned>((nl + 4095) / 4096)));
    nt = std::min(nt, 64u);
    std::vector<Local> locals(nt);
    Parser proto{static_cast<uint32_t>(v.samples.size()), v.words, b.opts.keep_genotypes != 0};
    auto work = [&](unsigned t) {
        const size_t lo = nl * t / nt, hi = nl * (t + 1) / nt;
        Parser P = proto;
        Local &L = locals[t];
        for (size_t i = lo; i < hi; ++i) {
            const char *s = starts[i];
            const char *le = static_cast<const char *>(memchr(s, '\n', static_cast<size_t>(e - s)));
            const char *full = le ? le + 1 : e;
            if (!le) le = e;
            if (le > s && le[-1] == '\r') --le;
            if (!P.line(s, le, full, base + static_cast<uint64_t>(s - p), L)) {
                L.err_line = i;
                return;
            }
        }
    };
    if (nt == 1) {
        work(0);
    } else {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t) th.emplace_back(work, t);
        for (auto &t : th) t.join();
    }
    for (auto &L : locals)
        if (L.err) throw Error(L.err, L.msg);
    for (auto &L : locals) merge(b, v, L);
}

void add_text(sb_builder &b, VcfData &v, const char *text, size_t len) {
    std::string joined;
    if (!v.carry.empty()) {
        joined = v.carry;
        joined.append(text, len);
        v.carry.clear();
        text = joined.data();
        len = joined.size();
    }
    const uint64_t base = v.stream_off;  // stream offset of text[0]
    // keep an unterminated tail for the next call
    size_t upto = len;
    while (upto > 0 && text[upto - 1] != '\n') --upto;
    if (upto < len) v.carry.assign(text + upto, len - upto);
    v.stream_off = base + upto;
    const char *p = text, *e = text + upto;
    // header lines first (sequential)
    while (p < e && *p == '#') {
        const char *nl = static_cast<const char *>(memchr(p, '\n', static_cast<size_t>(e - p)));
        if (!nl) nl = e;
        const char *le = nl;
        if (le > p && le[-1] == '\r') --le;
        parse_header_line(v, p, le);
        p = nl + 1;
    }
    if (p < e) parse_records(b, v, p, static_cast<size_t>(e - p), base + static_cast<uint64_t>(p - text));
}

// BGZF (SAMv1 §4.1): gzip members with a 'BC' extra subfield holding BSIZE-1
bool bgzf_block_size(const uint8_t *c, size_t avail, size_t *bsize) {
    if (avail < 18 || c[0] != 0x1f || c[1] != 0x8b || c[2] != 8 || !(c[3] & 4)) return false;
    const size_t xlen = c[10] | (c[11] << 8);
    for (size_t x = 12; x + 4 <= 12 + xlen && x + 4 <= avail;) {
        const size_t slen = c[x + 2] | (c[x + 3] << 8);
        if (c[x] == 'B' && c[x + 1] == 'C' && slen == 2 && x + 6 <= avail) {
            *bsize = (c[x + 4] | (c[x + 5] << 8)) + 1u;
            return *bsize >= 26;
        }
        x += 4 + slen;
    }
    return false;
}

}  // namespace

void builder_add_text(sb_builder &b, uint32_t vcf_id, const char *text, size_t len) {
    if (vcf_id >= b.vcfs.size()) throw Error(SB_ENOSTORE, "unknown vcf id");
    add_text(b, b.vcfs[vcf_id], text, len);
}

void builder_flush(sb_builder &b, uint32_t vcf_id) {
    VcfData &v = b.vcfs[vcf_id];
    if (!v.carry.empty()) {
        std::string tail = v.carry + "\n";
        v.carry.clear();
        add_text(b, v, tail.data(), tail.size());
    }
}

// BGZF blocks of a file image: (compressed offset, size, uncompressed size, uncompressed start)
struct Blk {
    size_t coff, bsize;
    uint32_t isize;
    uint64_t ustart;
};

std::vector<Blk> bgzf_blocks(const std::vector<uint8_t> &c, const char *path) {
    std::vector<Blk> blks;
    uint64_t u = 0;
    for (size_t p = 0; p < c.size();) {
        size_t bs;
        if (!bgzf_block_size(c.data() + p, c.size() - p, &bs) || p + bs > c.size())
            throw Error(SB_EIO, std::string("corrupt BGZF block in ") + path);
        const uint8_t *t = c.data() + p + bs - 4;
        const uint32_t is = t[0] | (t[1] << 8) | (t[2] << 16) | (static_cast<uint32_t>(t[3]) << 24);
        blks.push_back(Blk{p, bs, is, u});
        u += is;
        p += bs;
    }
    return blks;
}

// blocks inflated in parallel (nt threads) in ~64 MiB batches, handed to
// `feed` in file order
template <class F>
void bgzf_inflate(const std::vector<uint8_t> &c, const std::vector<Blk> &blks, const char *path, unsigned nt, F feed) {
    std::vector<char> buf;
    for (size_t i = 0; i < blks.size();) {
        size_t j = i;
        uint64_t bu = 0;
        while (j < blks.size() && (bu < (uint64_t(64) << 20) || j == i)) bu += blks[j++].isize;
        buf.resize(bu);
        std::atomic<size_t> next{i};
        std::atomic<int> bad{0};
        auto work = [&] {
            for (size_t k; (k = next.fetch_add(1)) < j;) {
                const Blk &bk = blks[k];
                const size_t xlen = c[bk.coff + 10] | (c[bk.coff + 11] << 8);
                z_stream z;
                memset(&z, 0, sizeof z);
                if (inflateInit2(&z, -15) != Z_OK) {
                    bad = 1;
                    continue;
                }
                z.next_in = const_cast<uint8_t *>(c.data() + bk.coff + 12 + xlen);
                z.avail_in = static_cast<uInt>(bk.bsize - 12 - xlen - 8);
                z.next_out = reinterpret_cast<Bytef *>(buf.data() + (bk.ustart - blks[i].ustart));
                z.avail_out = bk.isize;
                const int rc = inflate(&z, Z_FINISH);
                if (bk.isize && rc != Z_STREAM_END) bad = 1;
                inflateEnd(&z);
            }
        };
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t) th.emplace_back(work);
        for (auto &t : th) t.join();
        if (bad) throw Error(SB_EIO, std::string("BGZF inflate failed in ") + path);
        feed(buf.data(), buf.size());
        i = j;
    }
}

// BGZF ingest: block table for virtual offsets, blocks inflated in parallel
// in ~64 MiB batches that are fed to the text parser in order.
void add_bgzf(sb_builder &b, VcfData &v, const std::vector<uint8_t> &c, const char *path) {
    if (v.stream_off != 0 || !v.carry.empty()) throw Error(SB_EINVAL, "a BGZF file must be the only text source of its VCF");
    const std::vector<Blk> blks = bgzf_blocks(c, path);
    for (const Blk &bk : blks) {
        v.blk_coff.push_back(bk.coff);
        v.blk_ustart.push_back(bk.ustart);
    }
    v.stream_len = blks.empty() ? 0 : blks.back().ustart + blks.back().isize;
    const unsigned nt = std::max(1u, std::min(16u, b.opts.n_threads > 0 ? static_cast<unsigned>(b.opts.n_threads)
                                                                          : std::thread::hardware_concurrency()));
    bgzf_inflate(c, blks, path, nt, [&](const char *t, size_t n) { add_text(b, v, t, n); });
}

// the text of a plain, gzip or BGZF file, in order, in chunks
template <class F>
void read_vcf_file(const char *path, unsigned nt, F feed) {
    FILE *fp = fopen(path, "rb");
    if (!fp) throw Error(SB_EIO, std::string("cannot open ") + path);
    uint8_t hdr[18];
    const size_t got = fread(hdr, 1, sizeof hdr, fp);
    size_t bs;
    if (got == sizeof hdr && bgzf_block_size(hdr, got, &bs)) {
        fseek(fp, 0, SEEK_END);
        const long n = ftell(fp);
        fseek(fp, 0, SEEK_SET);
        std::vector<uint8_t> c(static_cast<size_t>(n));
        const size_t rd = fread(c.data(), 1, c.size(), fp);
        fclose(fp);
        if (rd != c.size()) throw Error(SB_EIO, std::string("short read: ") + path);
        bgzf_inflate(c, bgzf_blocks(c, path), path, nt, feed);
        return;
    }
    fclose(fp);
    gzFile f = gzopen(path, "rb");
    if (!f) throw Error(SB_EIO, std::string("cannot open ") + path);
    gzbuffer(f, 1 << 20);
    const size_t chunk = size_t(64) << 20;
    std::vector<char> buf(chunk);
    for (;;) {
        const int r = gzread(f, buf.data(), static_cast<unsigned>(chunk));
        if (r < 0) {
            gzclose(f);
            throw Error(SB_EIO, std::string("decompression failed: ") + path);
        }
        if (r == 0) break;
        feed(buf.data(), static_cast<size_t>(r));
    }
    gzclose(f);
}

// CHROM / POS of every record of a VCF file (shard planning): contigs in
// file order with their record ranges, POS per record.  Text from the same
// readers as the builder (BGZF in parallel, gzip, plain).
struct ScanState {
    std::string carry;
    VcfScan *out;
    void feed(const char *t, size_t n) {
        std::string joined;
        if (!carry.empty()) {
            joined = carry;
            joined.append(t, n);
            carry.clear();
            t = joined.data();
            n = joined.size();
        }
        size_t upto = n;
        while (upto > 0 && t[upto - 1] != '\n') --upto;
        if (upto < n) carry.assign(t + upto, n - upto);
        line_loop(t, upto);
    }
    void line_loop(const char *p, size_t n) {
        const char *e = p + n;
        while (p < e) {
            const char *nl = static_cast<const char *>(memchr(p, '\n', static_cast<size_t>(e - p)));
            if (!nl) nl = e;
            if (nl > p && *p != '#' && !(nl - p == 1 && *p == '\r')) {
                const char *t = static_cast<const char *>(memchr(p, '\t', static_cast<size_t>(nl - p)));
                if (!t) throw Error(SB_EPARSE, "record without a tab");
                const std::string chrom(p, static_cast<size_t>(t - p));
                uint64_t pos = 0;
                for (const char *q = t + 1; q < nl && is_digit(*q); ++q) pos = pos * 10 + static_cast<uint64_t>(*q - '0');
                if (pos > 0xffffffffull) throw Error(SB_EPARSE, "POS beyond 32 bits");
                const uint64_t r = out->pos.size();
                if (out->contigs.empty() || out->contigs.back().name != chrom)
                    out->contigs.push_back(VcfScan::Contig{chrom, r, r});
                out->pos.push_back(static_cast<uint32_t>(pos));
                out->contigs.back().hi = r + 1;
            }
            p = nl + 1;
        }
    }
};

void vcf_scan_file(const char *path, VcfScan &out) {
    ScanState st{{}, &out};
    read_vcf_file(path, 16, [&](const char *t, size_t n) { st.feed(t, n); });
    if (!st.carry.empty()) {
        st.carry.push_back('\n');
        st.line_loop(st.carry.data(), st.carry.size());
    }
}

void builder_add_file(sb_builder &b, uint32_t vcf_id, const char *path) {
    if (vcf_id >= b.vcfs.size()) throw Error(SB_ENOSTORE, "unknown vcf id");
    b.vcfs[vcf_id].sources.push_back(fingerprint(path));  // sb_store_save / sb_store_open
    {
        FILE *fp = fopen(path, "rb");
        if (!fp) throw Error(SB_EIO, std::string("cannot open ") + path);
        uint8_t hdr[18];
        const size_t got = fread(hdr, 1, sizeof hdr, fp);
        size_t bs;
        if (got == sizeof hdr && bgzf_block_size(hdr, got, &bs)) {
            fseek(fp, 0, SEEK_END);
            const long n = ftell(fp);
            fseek(fp, 0, SEEK_SET);
            std::vector<uint8_t> c(static_cast<size_t>(n));
            const size_t rd = fread(c.data(), 1, c.size(), fp);
            fclose(fp);
            if (rd != c.size()) throw Error(SB_EIO, std::string("short read: ") + path);
            add_bgzf(b, b.vcfs[vcf_id], c, path);
            builder_flush(b, vcf_id);
            return;
        }
        fclose(fp);
    }
    gzFile f = gzopen(path, "rb");
    if (!f) throw Error(SB_EIO, std::string("cannot open ") + path);
    gzbuffer(f, 1 << 20);
    const size_t chunk = size_t(64) << 20;
    std::vector<char> buf(chunk);
    for (;;) {
        const int r = gzread(f, buf.data(), static_cast<unsigned>(chunk));
        if (r < 0) {
            gzclose(f);
            throw Error(SB_EIO, std::string("decompression failed: ") + path);
        }
        if (r == 0) break;
        add_text(b, b.vcfs[vcf_id], buf.data(), static_cast<size_t>(r));
    }
    gzclose(f);
    builder_flush(b, vcf_id);
}

// Carrier matrix for a sites-only VCF (config 5: gnomAD-shape sites with a
// separately held 2,504-sample genotype bit-matrix).  `planes` holds one row
// of ceil(n_samples/64) words per ALT, in record-then-ALT order: bit s of
// ALT k's row = sample s has a GT token equal to str(k + 1) -- exactly the
// set the reference's regex at search_variants.py:233-236 collects, and what
// the text path builds from GT columns above.  Every record must carry AC and
// a valid AN: without them the reference counts GT tokens (:215-226,
// :244-250), which a carrier matrix does not determine.
void builder_attach_carriers(sb_builder &b, uint32_t vcf_id, const char *const *names, const uint32_t *name_len,
                             uint32_t n_samples, const uint64_t *planes, uint64_t n_rows) {
    if (vcf_id >= b.vcfs.size()) throw Error(SB_ENOSTORE, "unknown vcf id");
    builder_flush(b, vcf_id);
    VcfData &v = b.vcfs[vcf_id];
    VcfCols &c = v.c;
    if (!v.samples.empty()) throw Error(SB_EINVAL, "VCF already has sample columns");
    if (n_samples == 0 || !planes || !names || !name_len) throw Error(SB_EINVAL, "empty carrier matrix");
    const size_t nr = c.pos.size(), nx = c.x_key.size();
    if (n_rows != nr + nx) throw Error(SB_EINVAL, "carrier matrix rows != ALT rows of the VCF");
    for (size_t i = 0; i < nr; ++i) {
        const RecHot &r = c.rec[i];
        const uint32_t h = r.hot;
        bool ok = (h & (H_HAS_AC | H_HAS_AN)) == (H_HAS_AC | H_HAS_AN) && !(h & H_AN_BAD);
        if ((h & H_AN_BAD) && r.an == kAnUnrepresentable) {  // a general record: its own flags
            const uint32_t gf = c.gen[static_cast<size_t>(r.ac0)].flags;
            ok = (gf & (GR_HAS_AC | GR_HAS_AN)) == (GR_HAS_AC | GR_HAS_AN) && !(gf & GR_AN_BAD);
        }
        if (!ok) throw Error(SB_EINVAL, "carrier matrix needs AC and AN on every record");
    }
    v.samples.resize(n_samples);
    for (uint32_t s = 0; s < n_samples; ++s) v.samples[s].assign(names[s], name_len[s]);
    const uint32_t words = static_cast<uint32_t>((n_samples + 63) / 64);
    v.words = words;
    c.planes0.resize(nr * words);
    c.planesx.resize(nx * words);
    unsigned nt = b.opts.n_threads > 0 ? static_cast<unsigned>(b.opts.n_threads) : std::thread::hardware_concurrency();
    nt = std::max(1u, std::min<unsigned>(nt, static_cast<unsigned>(nr / 4096 + 1)));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            const size_t a = nr * t / nt, e = nr * (t + 1) / nt;
            for (size_t i = a; i < e; ++i) {
                const size_t row = i + c.x_lo[i];  // rows before record i
                const size_t nalt = 1 + c.x_lo[i + 1] - c.x_lo[i];
                memcpy(&c.planes0[i * words], planes + row * words, words * 8);
                if (nalt > 1)
                    memcpy(&c.planesx[static_cast<size_t>(c.x_lo[i]) * words], planes + (row + 1) * words,
                           (nalt - 1) * words * 8);
            }
        });
    for (auto &x : th) x.join();
}

}  // namespace sb
