// synth.cpp — seeded 1000 Genomes-shape VCF text generator (libsbeacon_synth.so).
//
// Synthetic-data source for the BASELINE.json configs; the
// reference ships no VCF.  Shape of config 2 (chr22): geometric POS gaps,
// 96.8 % SNV / 3.0 % indel (len 1-50) / 0.2 % symbolic, 1.5 % multiallelic,
// P(AC = k) ~ 1/k, AN = 2 x samples, INFO
// AC;AF;AN;NS;DP;EAS_AF;AMR_AF;AFR_AF;EUR_AF;SAS_AF;AA=.|||;VT, phased GTs
// consistent with AC.  Every record is a pure function of (seed, index), so
// chunks are generated in parallel and any record range is reproducible
// (also "sites-only": the same records without FORMAT/sample columns, for
// the CPU oracle).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

inline uint64_t splitmix(uint64_t &x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Rng {
    uint64_t s;
    Rng(uint64_t seed, uint64_t idx, uint64_t stream) : s(seed * 0x9E3779B97F4A7C15ull ^ (idx + 1) * 0xD1B54A32D192ED03ull ^ stream) {
        splitmix(s);
    }
    uint64_t next() { return splitmix(s); }
    double uni() { return static_cast<double>(next() >> 11) * (1.0 / 9007199254740992.0); }
    uint32_t below(uint32_t n) { return static_cast<uint32_t>((next() >> 32) * n >> 32); }
};

const char *kBase = "ACGT";
const char *kSym[] = {"<DEL>", "<DUP>", "<CN0>", "<INS>", "<INV>", "<CN2>", "<DUP:TANDEM>", "<DEL:ME:ALU>"};

struct Gen {
    uint64_t seed;
    uint64_t n;
    uint32_t n_samples;
    uint32_t start;
    double mean_gap;
    std::string contig;
    std::vector<uint32_t> pos;
    // cohort member (config 4): record i comes from the pool's seed with
    // probability `share`, otherwise from this member's own seed
    uint64_t own_seed = 0;
    double share = 1.0;
    // config 5 (gnomAD-shape sites): INFO AC/AN over a cohort of an_sites
    // alleles (0 = 2 x n_samples), genotypes over n_samples with carriers
    // scaled by 2 n_samples / an_sites
    uint32_t an_sites = 0;
    double multi_frac = 0.015;  // multiallelic share of all records (SBS_MULTI_FRAC overrides; experiments)
    uint64_t rec_seed(uint64_t i) const {
        if (share >= 1.0) return seed;
        Rng r(own_seed, i, 7);
        return r.uni() < share ? seed : own_seed;
    }
};

struct Rec {
    std::string ref;
    std::vector<std::string> alts;
    std::vector<uint32_t> ac;
    const char *vt;
    bool sym;
};

void make_record(const Gen &g, uint64_t i, Rec &r) {
    Rng rng(g.rec_seed(i), i, 1);
    const double u = rng.uni();
    r.alts.clear();
    r.ac.clear();
    r.sym = false;
    const uint32_t hap = 2 * g.n_samples;
    const uint32_t N = g.an_sites ? g.an_sites : (hap ? hap : 5008);
    auto draw_ac = [&](uint32_t cap) {
        // P(k) ~ 1/k on [1, cap]: k = floor((cap+1)^u)
        const double x = std::pow(static_cast<double>(cap) + 1.0, rng.uni());
        uint32_t k = static_cast<uint32_t>(x);
        return std::max(1u, std::min(k, cap));
    };
    if (u < 0.002) {  // symbolic SV
        r.ref.assign(1, kBase[rng.below(4)]);
        r.alts.push_back(kSym[rng.below(8)]);
        r.vt = "SV";
        r.sym = true;
    } else if (u < 0.032) {  // indel, len 1..50
        const uint32_t len = 1 + rng.below(50);
        std::string s(len + 1, 'A');
        for (auto &c : s) c = kBase[rng.below(4)];
        if (rng.uni() < 0.5) {
            r.ref = s;
            r.alts.push_back(s.substr(0, 1));
        } else {
            r.ref = s.substr(0, 1);
            r.alts.push_back(s);
        }
        r.vt = "INDEL";
    } else {  // SNV (1.5 % of all records multiallelic)
        const uint32_t b = rng.below(4);
        r.ref.assign(1, kBase[b]);
        uint32_t na = 1;
        if (rng.uni() < g.multi_frac / 0.968) na = 2 + rng.below(2);
        uint32_t used = 1u << b;
        for (uint32_t k = 0; k < na; ++k) {
            uint32_t a;
            do a = rng.below(4);
            while (used & (1u << a));
            used |= 1u << a;
            r.alts.emplace_back(1, kBase[a]);
        }
        r.vt = "SNP";
    }
    uint32_t left = N;
    for (size_t k = 0; k < r.alts.size(); ++k) {
        const uint32_t cap = std::max(1u, left / static_cast<uint32_t>(r.alts.size() - k + 1));
        const uint32_t c = std::min(draw_ac(cap), left);
        r.ac.push_back(c);
        left -= c;
    }
}

size_t write_u(char *p, uint64_t v) {
    char t[24];
    int n = 0;
    do {
        t[n++] = static_cast<char>('0' + v % 10);
        v /= 10;
    } while (v);
    for (int i = 0; i < n; ++i) p[i] = t[n - 1 - i];
    return static_cast<size_t>(n);
}

// Carrier haplotypes of record i, drawn from rng stream 2 after the INFO
// draws render() makes (DP, five population AFs per ALT, END of a symbolic
// record): f(k, h) for each haplotype h carrying ALT k (0-based).  Distinct
// haplotypes per record; AC carriers per ALT, or AC scaled to the sample
// cohort for an_sites VCFs.
template <typename F>
void draw_carriers(const Gen &g, const Rec &r, Rng &rng, std::vector<uint8_t> &taken, F f) {
    const uint32_t hap = 2 * g.n_samples;
    std::fill(taken.begin(), taken.end(), 0);
    uint32_t free_h = hap;
    for (size_t k = 0; k < r.ac.size(); ++k) {
        uint32_t n = r.ac[k];
        if (g.an_sites) n = static_cast<uint32_t>((static_cast<uint64_t>(n) * hap + g.an_sites - 1) / g.an_sites);
        n = std::min(n, free_h);
        free_h -= n;
        for (uint32_t c = 0; c < n; ++c) {
            uint32_t h;
            do h = rng.below(hap);
            while (taken[h]);
            taken[h] = 1;
            f(k, h);
        }
    }
}

// The stream-2 draws render() makes before the genotypes.
void skip_site_draws(const Rec &r, Rng &rng) {
    rng.below(30000);
    for (int p = 0; p < 5; ++p)
        for (size_t k = 0; k < r.ac.size(); ++k) rng.uni();
    if (r.sym) rng.below(5000);
}

// Render records [lo, hi) into out (appends).
void render(const Gen &g, uint64_t lo, uint64_t hi, bool sites_only, std::string &out) {
    Rec r;
    const uint32_t ns = sites_only ? 0 : g.n_samples;
    const uint32_t hap = 2 * g.n_samples;
    std::string gt;
    if (ns) {
        gt.resize(static_cast<size_t>(ns) * 4);
        for (uint32_t s = 0; s < ns; ++s) memcpy(&gt[4 * s], "0|0\t", 4);
        gt[4 * ns - 1] = '\n';
    }
    std::vector<uint8_t> taken(hap ? hap : 1);
    char buf[4096];
    for (uint64_t i = lo; i < hi; ++i) {
        make_record(g, i, r);
        Rng rng(g.rec_seed(i), i, 2);
        size_t n = 0;
        auto put = [&](const char *s, size_t l) {
            if (n + l > sizeof buf) {
                out.append(buf, n);
                n = 0;
            }
            memcpy(buf + n, s, l);
            n += l;
        };
        auto puts_ = [&](const std::string &s) { put(s.data(), s.size()); };
        auto putc_ = [&](char c) { put(&c, 1); };
        auto putu = [&](uint64_t v) {
            char t[24];
            put(t, write_u(t, v));
        };
        puts_(g.contig);
        putc_('\t');
        putu(g.pos[i]);
        put("\t.\t", 3);
        puts_(r.ref);
        putc_('\t');
        for (size_t k = 0; k < r.alts.size(); ++k) {
            if (k) putc_(',');
            puts_(r.alts[k]);
        }
        put("\t100\tPASS\tAC=", 13);
        for (size_t k = 0; k < r.ac.size(); ++k) {
            if (k) putc_(',');
            putu(r.ac[k]);
        }
        const uint32_t an = g.an_sites ? g.an_sites : (hap ? hap : 5008);
        put(";AF=", 4);
        for (size_t k = 0; k < r.ac.size(); ++k) {
            if (k) putc_(',');
            char t[32];
            const int l = snprintf(t, sizeof t, "%.4g", static_cast<double>(r.ac[k]) / an);
            put(t, static_cast<size_t>(l));
        }
        put(";AN=", 4);
        putu(an);
        put(";NS=", 4);
        putu(g.n_samples ? g.n_samples : 2504);
        put(";DP=", 4);
        putu(5000 + rng.below(30000));
        static const char *pops[] = {";EAS_AF=", ";AMR_AF=", ";AFR_AF=", ";EUR_AF=", ";SAS_AF="};
        for (const char *pp : pops) {
            put(pp, 8);
            for (size_t k = 0; k < r.ac.size(); ++k) {
                if (k) putc_(',');
                char t[16];
                const int l = snprintf(t, sizeof t, "%.2f", rng.uni() * 0.1);
                put(t, static_cast<size_t>(l));
            }
        }
        if (r.sym) {
            put(";END=", 5);
            putu(g.pos[i] + 50 + rng.below(5000));
        }
        put(";AA=.|||;VT=", 12);
        put(r.vt, strlen(r.vt));
        if (!ns) {
            putc_('\n');
            out.append(buf, n);
            continue;
        }
        put("\tGT\t", 4);
        out.append(buf, n);
        // genotypes consistent with AC: distinct carrier haplotypes per allele
        const size_t g0 = out.size();
        out.append(gt);
        draw_carriers(g, r, rng, taken,
                      [&](size_t k, uint32_t h) { out[g0 + 4 * (h >> 1) + 2 * (h & 1)] = static_cast<char>('1' + k); });
    }
}

}  // namespace

extern "C" {

// contig: NUL-terminated; mean_gap: geometric mean gap between POS values.
void *sbs_new(uint64_t seed, uint64_t n_records, uint32_t n_samples, uint32_t start_pos, double mean_gap,
              const char *contig) {
    auto *g = new Gen;
    g->seed = seed;
    g->n = n_records;
    g->n_samples = n_samples;
    g->start = start_pos;
    g->mean_gap = mean_gap;
    g->contig = contig;
    if (const char *e = getenv("SBS_MULTI_FRAC")) g->multi_frac = atof(e);
    g->pos.resize(n_records);
    uint64_t p = start_pos;
    const double lq = std::log(1.0 - 1.0 / mean_gap);
    for (uint64_t i = 0; i < n_records; ++i) {
        if (i) {
            Rng rng(seed, i, 0);
            // geometric on {0,1,...} with mean ~ mean_gap - 1, plus 1 (same-POS records stay rare)
            const double x = std::floor(std::log(1.0 - rng.uni()) / lq);
            p += 1 + static_cast<uint64_t>(x);
        }
        g->pos[i] = static_cast<uint32_t>(std::min<uint64_t>(p, 0xfffffff0ull));
    }
    return g;
}

// A cohort member of `pool`: same positions, record i shared with the pool
// with probability share (else drawn from own_seed), n_samples of its own.
void *sbs_new_member(void *pool, uint64_t own_seed, double share, uint32_t n_samples) {
    auto *g = new Gen(*static_cast<Gen *>(pool));
    g->own_seed = own_seed;
    g->share = share;
    g->n_samples = n_samples;
    return g;
}

void sbs_free(void *h) { delete static_cast<Gen *>(h); }

uint32_t sbs_pos(void *h, uint64_t i) { return static_cast<Gen *>(h)->pos[i]; }

// copy POS array (n_records u32)
void sbs_positions(void *h, uint32_t *out) {
    auto *g = static_cast<Gen *>(h);
    memcpy(out, g->pos.data(), g->pos.size() * 4);
}

// REF / first ALT of record i into caller buffers (for point-query generation)
int sbs_alleles(void *h, uint64_t i, char *ref, size_t ref_cap, char *alt, size_t alt_cap) {
    auto *g = static_cast<Gen *>(h);
    Rec r;
    make_record(*g, i, r);
    if (r.ref.size() + 1 > ref_cap || r.alts[0].size() + 1 > alt_cap) return -1;
    memcpy(ref, r.ref.c_str(), r.ref.size() + 1);
    memcpy(alt, r.alts[0].c_str(), r.alts[0].size() + 1);
    return static_cast<int>(r.alts.size());
}

// Header text (caller frees with sbs_free_text).
char *sbs_header(void *h, int sites_only, size_t *len) {
    auto *g = static_cast<Gen *>(h);
    std::string s = "##fileformat=VCFv4.2\n##contig=<ID=" + g->contig + ">\n";
    s += "##INFO=<ID=AC,Number=A,Type=Integer,Description=\"Allele count\">\n";
    s += "##INFO=<ID=AN,Number=1,Type=Integer,Description=\"Total alleles\">\n";
    s += "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO";
    if (!sites_only && g->n_samples) {
        s += "\tFORMAT";
        char t[32];
        for (uint32_t i = 0; i < g->n_samples; ++i) {
            snprintf(t, sizeof t, "\tHG%05u", i + 96);
            s += t;
        }
    }
    s += "\n";
    char *o = static_cast<char *>(malloc(s.size()));
    memcpy(o, s.data(), s.size());
    *len = s.size();
    return o;
}

// Records [lo, hi) as VCF text, rendered by n_threads threads.
char *sbs_records(void *h, uint64_t lo, uint64_t hi, int sites_only, int n_threads, size_t *len) {
    auto *g = static_cast<Gen *>(h);
    hi = std::min<uint64_t>(hi, g->n);
    if (lo >= hi) {
        *len = 0;
        return static_cast<char *>(malloc(1));
    }
    unsigned nt = n_threads > 0 ? static_cast<unsigned>(n_threads) : std::thread::hardware_concurrency();
    nt = std::max(1u, std::min<unsigned>(nt, static_cast<unsigned>((hi - lo + 1023) / 1024)));
    std::vector<std::string> parts(nt);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            const uint64_t a = lo + (hi - lo) * t / nt, b = lo + (hi - lo) * (t + 1) / nt;
            render(*g, a, b, sites_only != 0, parts[t]);
        });
    for (auto &x : th) x.join();
    size_t total = 0;
    for (auto &p : parts) total += p.size();
    char *o = static_cast<char *>(malloc(total ? total : 1));
    size_t off = 0;
    for (auto &p : parts) {
        memcpy(o + off, p.data(), p.size());
        off += p.size();
    }
    *len = total;
    return o;
}

// config 5: INFO AN of every record (and the AC scale); 0 = 2 x n_samples
void sbs_set_an_sites(void *h, uint32_t an) { static_cast<Gen *>(h)->an_sites = an; }

// ALT rows (records + extra ALTs) of records [lo, hi)
uint64_t sbs_alt_rows(void *h, uint64_t lo, uint64_t hi, int n_threads) {
    auto *g = static_cast<Gen *>(h);
    hi = std::min<uint64_t>(hi, g->n);
    if (lo >= hi) return 0;
    unsigned nt = n_threads > 0 ? static_cast<unsigned>(n_threads) : std::thread::hardware_concurrency();
    nt = std::max(1u, std::min<unsigned>(nt, static_cast<unsigned>((hi - lo + 1023) / 1024)));
    std::vector<uint64_t> cnt(nt, 0);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            Rec r;
            const uint64_t a = lo + (hi - lo) * t / nt, b = lo + (hi - lo) * (t + 1) / nt;
            for (uint64_t i = a; i < b; ++i) {
                make_record(*g, i, r);
                cnt[t] += r.alts.size();
            }
        });
    for (auto &x : th) x.join();
    uint64_t n = 0;
    for (auto c : cnt) n += c;
    return n;
}

// Carrier bit-matrix of records [lo, hi): one row of ceil(n_samples/64)
// words per ALT, record-then-ALT order (sb_builder_attach_carriers), the
// same genotypes sbs_records renders as GT text.  out: n_rows x words u64.
int sbs_carrier_planes(void *h, uint64_t lo, uint64_t hi, int n_threads, uint64_t *out, uint64_t n_rows) {
    auto *g = static_cast<Gen *>(h);
    hi = std::min<uint64_t>(hi, g->n);
    if (lo >= hi) return n_rows == 0 ? 0 : -1;
    const uint32_t words = (g->n_samples + 63) / 64;
    unsigned nt = n_threads > 0 ? static_cast<unsigned>(n_threads) : std::thread::hardware_concurrency();
    nt = std::max(1u, std::min<unsigned>(nt, static_cast<unsigned>((hi - lo + 1023) / 1024)));
    std::vector<uint64_t> cnt(nt + 1, 0);
    auto run = [&](bool fill) {
        std::vector<std::thread> th;
        for (unsigned t = 0; t < nt; ++t)
            th.emplace_back([&, t, fill] {
                Rec r;
                std::vector<uint8_t> taken(2 * g->n_samples + 1);
                const uint64_t a = lo + (hi - lo) * t / nt, b = lo + (hi - lo) * (t + 1) / nt;
                uint64_t row = fill ? cnt[t] : 0;
                for (uint64_t i = a; i < b; ++i) {
                    make_record(*g, i, r);
                    if (!fill) {
                        row += r.alts.size();
                        continue;
                    }
                    uint64_t *base = out + row * words;
                    memset(base, 0, r.alts.size() * words * 8);
                    Rng rng(g->rec_seed(i), i, 2);
                    skip_site_draws(r, rng);
                    draw_carriers(*g, r, rng, taken, [&](size_t k, uint32_t hp) {
                        const uint32_t s = hp >> 1;
                        base[k * words + (s >> 6)] |= 1ull << (s & 63);
                    });
                    row += r.alts.size();
                }
                if (!fill) cnt[t + 1] = row;
            });
        for (auto &x : th) x.join();
    };
    run(false);
    for (unsigned t = 0; t < nt; ++t) cnt[t + 1] += cnt[t];
    if (cnt[nt] != n_rows) return -1;
    run(true);
    return 0;
}

void sbs_free_text(char *p) { free(p); }

}  // extern "C"

// ---------------------------------------------------------------- BGZF writer
// bgzip-compatible output: blocks of <= 0xff00 input bytes, each a gzip
// member with the BC extra subfield (SAMv1 §4.1), then the 28-byte EOF block.
#include <zlib.h>

namespace {
size_t bgzf_block(const uint8_t *in, size_t n, int level, uint8_t *out) {
    z_stream z;
    memset(&z, 0, sizeof z);
    deflateInit2(&z, level, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
    z.next_in = const_cast<uint8_t *>(in);
    z.avail_in = static_cast<uInt>(n);
    z.next_out = out + 18;
    z.avail_out = 65536 - 18 - 8;
    int rc = deflate(&z, Z_FINISH);
    size_t clen = z.total_out;
    deflateEnd(&z);
    if (rc != Z_STREAM_END) {  // incompressible: stored block
        memset(&z, 0, sizeof z);
        deflateInit2(&z, 0, Z_DEFLATED, -15, 8, Z_DEFAULT_STRATEGY);
        z.next_in = const_cast<uint8_t *>(in);
        z.avail_in = static_cast<uInt>(n);
        z.next_out = out + 18;
        z.avail_out = 65536 - 18 - 8;
        deflate(&z, Z_FINISH);
        clen = z.total_out;
        deflateEnd(&z);
    }
    const size_t bsize = 18 + clen + 8;
    static const uint8_t hdr[12] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0};
    memcpy(out, hdr, 12);
    out[12] = 'B';
    out[13] = 'C';
    out[14] = 2;
    out[15] = 0;
    out[16] = static_cast<uint8_t>((bsize - 1) & 0xff);
    out[17] = static_cast<uint8_t>((bsize - 1) >> 8);
    const uint32_t crc = static_cast<uint32_t>(crc32(crc32(0L, Z_NULL, 0), in, static_cast<uInt>(n)));
    uint8_t *t = out + 18 + clen;
    for (int i = 0; i < 4; ++i) t[i] = static_cast<uint8_t>(crc >> (8 * i));
    for (int i = 0; i < 4; ++i) t[4 + i] = static_cast<uint8_t>(static_cast<uint32_t>(n) >> (8 * i));
    return bsize;
}
}  // namespace

extern "C" {

// Compress `n` bytes into BGZF (appending the EOF block when eof != 0).
char *sbs_bgzf_compress(const char *in, size_t n, int level, int eof, int n_threads, size_t *out_len) {
    const size_t B = 0xff00;
    const size_t nb = (n + B - 1) / B;
    std::vector<std::vector<uint8_t>> blocks(nb);
    unsigned nt = n_threads > 0 ? static_cast<unsigned>(n_threads) : std::thread::hardware_concurrency();
    nt = std::max(1u, std::min<unsigned>(nt, static_cast<unsigned>(nb ? nb : 1)));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            for (size_t i = t; i < nb; i += nt) {
                blocks[i].resize(65536);
                const size_t off = i * B, len = std::min(B, n - off);
                blocks[i].resize(bgzf_block(reinterpret_cast<const uint8_t *>(in) + off, len, level, blocks[i].data()));
            }
        });
    for (auto &x : th) x.join();
    static const uint8_t kEof[28] = {0x1f, 0x8b, 8, 4, 0, 0, 0, 0, 0, 0xff, 6, 0, 0x42, 0x43,
                                     2, 0, 0x1b, 0, 3, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    size_t total = eof ? 28 : 0;
    for (auto &b : blocks) total += b.size();
    char *o = static_cast<char *>(malloc(total ? total : 1));
    size_t off = 0;
    for (auto &b : blocks) {
        memcpy(o + off, b.data(), b.size());
        off += b.size();
    }
    if (eof) memcpy(o + off, kEof, 28);
    *out_len = total;
    return o;
}

}  // extern "C"
