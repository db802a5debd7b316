/*
 * sbeacon_oracle.c — CPU restatement of the reference performQuery slice loop.
 *
 * TEST INFRASTRUCTURE ONLY (see sbeacon_oracle.h).  Every block cites the
 * reference line it restates; "sv:" = lambda/performQuery/search_variants.py,
 * "svs:" = lambda/performQuery/search_variants_in_samples.py.
 *
 * Input is a plain or gzip VCF (zlib).  `bcftools query --regions chrom:a-b`
 * (sv:42-50) is restated as "records of chrom with a <= POS <= b, file order",
 * which is exactly the set the reference keeps after sv:84-85.
 */
#define _GNU_SOURCE
#include "sbeacon_oracle.h"

#include <ctype.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    const char *p;
    int64_t n;
} sv_t; /* string view */

typedef struct {
    sv_t chrom, pos_txt, ref, alt, info;
    int64_t pos;
    const char *gt; /* start of sample columns (NULL when not loaded) */
    int64_t gt_len;
} rec_t;

typedef struct {
    char *buf;
    int64_t n_rec;
    rec_t *recs;
    int32_t n_samples;
    sv_t *names;
    int load_gt;
    int32_t n_contigs;
    sv_t *contig;      /* contig blocks in file order */
    int64_t *contig_lo, *contig_hi;
} vcf_t;

/* ------------------------------------------------------------------ utils */
typedef struct {
    char *p;
    int64_t n, cap;
} dbuf;

static void db_put(dbuf *b, const char *s, int64_t n) {
    if (b->n + n + 1 > b->cap) {
        int64_t c = b->cap ? b->cap * 2 : 256;
        while (c < b->n + n + 1) c *= 2;
        b->p = (char *)realloc(b->p, (size_t)c);
        b->cap = c;
    }
    memcpy(b->p + b->n, s, (size_t)n);
    b->n += n;
    b->p[b->n] = 0;
}
static void db_putc(dbuf *b, char c) { db_put(b, &c, 1); }

static int sv_eq(sv_t a, const char *s) {
    int64_t n = (int64_t)strlen(s);
    return a.n == n && memcmp(a.p, s, (size_t)n) == 0;
}
static int sv_starts(sv_t a, const char *s) {
    int64_t n = (int64_t)strlen(s);
    return a.n >= n && memcmp(a.p, s, (size_t)n) == 0;
}

/* Python int(str) for the ASCII forms VCF carries: ws, sign, digits, '_' */
static int py_int(const char *p, int64_t n, int64_t *out) {
    int64_t i = 0, j = n;
    while (i < j && isspace((unsigned char)p[i])) i++;
    while (j > i && isspace((unsigned char)p[j - 1])) j--;
    if (i == j) return -1;
    int neg = 0;
    if (p[i] == '+' || p[i] == '-') {
        neg = p[i] == '-';
        i++;
    }
    if (i == j || !isdigit((unsigned char)p[i])) return -1;
    int64_t v = 0;
    for (int64_t k = i; k < j; k++) {
        if (p[k] == '_') {
            if (k + 1 >= j || !isdigit((unsigned char)p[k + 1]) || !isdigit((unsigned char)p[k - 1])) return -1;
            continue;
        }
        if (!isdigit((unsigned char)p[k])) return -1;
        v = v * 10 + (p[k] - '0');
    }
    *out = neg ? -v : v;
    return 0;
}

/* ------------------------------------------------------------------ load */
static char *slurp(const char *path, int64_t *len) {
    gzFile f = gzopen(path, "rb");
    if (!f) return NULL;
    int64_t cap = 1 << 20, n = 0;
    char *b = (char *)malloc((size_t)cap);
    for (;;) {
        if (n + (1 << 20) + 1 > cap) {
            cap *= 2;
            b = (char *)realloc(b, (size_t)cap);
        }
        int r = gzread(f, b + n, 1 << 20);
        if (r < 0) {
            gzclose(f);
            free(b);
            return NULL;
        }
        if (r == 0) break;
        n += r;
    }
    gzclose(f);
    b[n] = 0;
    *len = n;
    return b;
}

void *orc_load_vcf(const char *path, int load_gt) {
    int64_t len = 0;
    char *buf = slurp(path, &len);
    if (!buf) return NULL;
    vcf_t *v = (vcf_t *)calloc(1, sizeof(vcf_t));
    v->buf = buf;
    v->load_gt = load_gt;
    int64_t cap = 1024;
    v->recs = (rec_t *)malloc(sizeof(rec_t) * (size_t)cap);
    char *p = buf, *end = buf + len;
    while (p < end) {
        char *nl = memchr(p, '\n', (size_t)(end - p));
        if (!nl) nl = end;
        *nl = 0;
        if (p[0] == '#' && p[1] == '#') {
        } else if (p[0] == '#') {
            /* #CHROM ... FORMAT s1 s2 ... */
            int col = 0;
            char *q = p;
            int64_t ncap = 64;
            v->names = (sv_t *)malloc(sizeof(sv_t) * (size_t)ncap);
            while (q <= nl) {
                char *t = q;
                while (t < nl && *t != '\t') t++;
                if (col >= 9) {
                    if (v->n_samples == ncap) {
                        ncap *= 2;
                        v->names = (sv_t *)realloc(v->names, sizeof(sv_t) * (size_t)ncap);
                    }
                    v->names[v->n_samples].p = q;
                    v->names[v->n_samples].n = t - q;
                    v->n_samples++;
                }
                col++;
                q = t + 1;
            }
        } else if (nl > p) {
            rec_t r;
            memset(&r, 0, sizeof r);
            sv_t f[9];
            char *q = p;
            int col = 0;
            while (col < 9 && q <= nl) {
                char *t = q;
                while (t < nl && *t != '\t') t++;
                f[col].p = q;
                f[col].n = t - q;
                col++;
                q = t + 1;
            }
            if (col < 8) goto next;
            r.chrom = f[0];
            r.pos_txt = f[1];
            if (py_int(f[1].p, f[1].n, &r.pos)) goto next;
            r.ref = f[3];
            r.alt = f[4];
            r.info = f[7];
            if (load_gt && col == 9 && q <= nl) {
                r.gt = q;
                r.gt_len = nl - q;
            }
            if (v->n_rec == cap) {
                cap *= 2;
                v->recs = (rec_t *)realloc(v->recs, sizeof(rec_t) * (size_t)cap);
            }
            v->recs[v->n_rec++] = r;
        }
    next:
        p = nl + 1;
    }
    /* contig blocks (records of one contig are contiguous in a sorted VCF) */
    v->contig = (sv_t *)malloc(sizeof(sv_t) * (size_t)(v->n_rec + 1));
    v->contig_lo = (int64_t *)malloc(sizeof(int64_t) * (size_t)(v->n_rec + 1));
    v->contig_hi = (int64_t *)malloc(sizeof(int64_t) * (size_t)(v->n_rec + 1));
    for (int64_t i = 0; i < v->n_rec; i++) {
        sv_t c = v->recs[i].chrom;
        int32_t k = v->n_contigs - 1;
        if (k >= 0 && v->contig[k].n == c.n && !memcmp(v->contig[k].p, c.p, (size_t)c.n)) {
            v->contig_hi[k] = i + 1;
        } else {
            v->contig[v->n_contigs] = c;
            v->contig_lo[v->n_contigs] = i;
            v->contig_hi[v->n_contigs] = i + 1;
            v->n_contigs++;
        }
    }
    return v;
}

void orc_free(void *h) {
    vcf_t *v = (vcf_t *)h;
    if (!v) return;
    free(v->buf);
    free(v->recs);
    free(v->names);
    free(v->contig);
    free(v->contig_lo);
    free(v->contig_hi);
    free(v);
}
int64_t orc_n_records(void *h) { return ((vcf_t *)h)->n_rec; }
int32_t orc_n_samples(void *h) { return ((vcf_t *)h)->n_samples; }

void orc_result_free(orc_result *r) {
    free(r->variants);
    free(r->sample_indices);
    free(r->sample_names);
    memset(r, 0, sizeof *r);
}

/* ------------------------------------------------------------------ query */
typedef struct {
    sv_t chrom;
    int64_t first_bp, last_bp;
} region_t;

/* sv:56-58: first ':' splits chrom; first '-' ends first_bp */
static int parse_region(const char *s, region_t *r) {
    const char *c = strchr(s, ':');
    const char *d = strchr(s, '-');
    if (!c || !d || d < c) return -1;
    r->chrom.p = s;
    r->chrom.n = c - s;
    if (py_int(c + 1, d - c - 1, &r->first_bp)) return -1;
    if (py_int(d + 1, (int64_t)strlen(d + 1), &r->last_bp)) return -1;
    return 0;
}

/* first record of chrom with POS >= a (records are POS-sorted within a contig) */
static int64_t lower_bound(const vcf_t *v, sv_t chrom, int64_t a, int64_t *hi_out) {
    int64_t lo = -1, hi = -1;
    for (int32_t k = 0; k < v->n_contigs; k++)
        if (v->contig[k].n == chrom.n && !memcmp(v->contig[k].p, chrom.p, (size_t)chrom.n)) {
            lo = v->contig_lo[k];
            hi = v->contig_hi[k];
            break;
        }
    if (lo < 0) {
        *hi_out = 0;
        return 0;
    }
    int64_t L = lo, H = hi;
    while (L < H) {
        int64_t m = (L + H) / 2;
        if (v->recs[m].pos < a)
            L = m + 1;
        else
            H = m;
    }
    *hi_out = hi;
    return L;
}

/* svs:88-91 regex '^' + ref.replace('N','[ACGTN]{1}') + '$' on REF.upper() */
static int wild_ref_match(const char *pat, sv_t ref) {
    int64_t n = (int64_t)strlen(pat);
    if (n != ref.n) return 0;
    for (int64_t i = 0; i < n; i++) {
        char c = (char)toupper((unsigned char)ref.p[i]);
        if (pat[i] == 'N') {
            if (!(c == 'A' || c == 'C' || c == 'G' || c == 'T' || c == 'N')) return 0;
        } else if (pat[i] == '.') {
            if (c == '\n') return 0;
        } else if (pat[i] != c) {
            return 0;
        }
    }
    return 1;
}

static int upper_eq(sv_t a, const char *s) { /* a.upper() == s */
    int64_t n = (int64_t)strlen(s);
    if (a.n != n) return 0;
    for (int64_t i = 0; i < n; i++)
        if ((char)toupper((unsigned char)a.p[i]) != s[i]) return 0;
    return 1;
}

/* alt == ref * k for some k >= kmin (fullmatch('(ref){k,}')) */
static int is_repeat(sv_t alt, sv_t ref, int kmin) {
    if (ref.n == 0) return alt.n == 0;
    if (alt.n % ref.n) return 0;
    int64_t k = alt.n / ref.n;
    if (k < kmin) return 0;
    for (int64_t i = 0; i < k; i++)
        if (memcmp(alt.p + i * ref.n, ref.p, (size_t)ref.n)) return 0;
    return 1;
}

#define MAX_ALTS 4096

/* sv:100-183 hit_indexes for one record; returns count, fills hits[] */
static int compute_hits(const orc_query *q, sv_t ref, sv_t *alts, int n_alt, int *hits) {
    int nh = 0;
    int64_t vmax = q->variant_max_length; /* sv:67 */
    char vprefix[256];
    snprintf(vprefix, sizeof vprefix, "<%s", q->variant_type ? q->variant_type : "None"); /* sv:54 */
    const char *vt = q->variant_type;
    for (int i = 0; i < n_alt; i++) {
        sv_t a = alts[i];
        int len_ok = q->variant_min_length <= a.n && (vmax < 0 || a.n <= vmax);
        int ok = 0;
        if (q->alternate_bases == NULL) {
            int sym = a.n > 0 && a.p[0] == '<';
            if (vt && !strcmp(vt, "DEL")) { /* sv:101-111 */
                ok = sym ? (sv_starts(a, vprefix) || sv_eq(a, "<CN0>")) : a.n < ref.n;
            } else if (vt && !strcmp(vt, "INS")) { /* sv:112-122 */
                ok = sym ? sv_starts(a, vprefix) : a.n > ref.n;
            } else if (vt && !strcmp(vt, "DUP")) { /* sv:123-133 */
                ok = sym ? (sv_starts(a, vprefix) ||
                            (sv_starts(a, "<CN") && !sv_eq(a, "<CN0>") && !sv_eq(a, "<CN1>")))
                         : is_repeat(a, ref, 2);
            } else if (vt && !strcmp(vt, "DUP:TANDEM")) { /* sv:134-144 */
                ok = sym ? (sv_starts(a, vprefix) || sv_eq(a, "<CN2>"))
                         : (a.n == 2 * ref.n && is_repeat(a, ref, 2));
            } else if (vt && !strcmp(vt, "CNV")) { /* sv:145-158 */
                ok = sym ? (sv_starts(a, vprefix) || sv_starts(a, "<CN") || sv_starts(a, "<DEL") ||
                            sv_starts(a, "<DUP"))
                         : (sv_eq(a, ".") || is_repeat(a, ref, 0));
            } else { /* sv:159-166 */
                ok = sv_starts(a, vprefix);
            }
        } else if (!strcmp(q->alternate_bases, "N")) { /* sv:170-176 */
            ok = a.n == 1 && strchr("ACGTN", toupper((unsigned char)a.p[0])) && a.p[0] != 0;
        } else { /* sv:177-183 */
            ok = upper_eq(a, q->alternate_bases);
        }
        if (ok && len_ok) hits[nh++] = i;
    }
    return nh;
}

/* digits runs of the GT text of the selected samples (re '[0-9]+' at sv:28) */
typedef struct {
    const vcf_t *v;
    const int32_t *sel; /* selected sample column indices (header order) */
    int32_t n_sel;
} gtsel_t;

/* iterate sample GT strings (the GT subfield before ':') for the selected samples */
static int64_t gt_columns(const rec_t *r, sv_t *cols, int32_t n_samples) {
    int64_t k = 0;
    const char *p = r->gt, *e = r->gt + r->gt_len;
    while (p <= e && k < n_samples) {
        const char *t = p;
        while (t < e && *t != '\t') t++;
        const char *c = p;
        while (c < t && *c != ':') c++;
        cols[k].p = p;
        cols[k].n = c - p;
        k++;
        p = t + 1;
    }
    return k;
}

int orc_query_one(void *h, const orc_query *q, orc_result *res) {
    const vcf_t *v = (const vcf_t *)h;
    memset(res, 0, sizeof *res);
    region_t rg;
    if (parse_region(q->region, &rg)) return res->error = ORC_VALUE_ERROR;
    const int samples_variant = q->selected_samples_only != 0;
    const int include_samples = q->include_samples != 0;

    /* sample selection: svs:40 --samples (header order), sv:45 all samples */
    int32_t *sel = (int32_t *)malloc(sizeof(int32_t) * (size_t)(v->n_samples + 1));
    int32_t n_sel = 0;
    int bcftools_failed = 0;
    if (samples_variant) {
        const char *names = q->sample_names ? q->sample_names : "_";
        char *flag = (char *)calloc((size_t)v->n_samples + 1, 1);
        const char *p = names;
        for (;;) {
            const char *c = strchr(p, ',');
            int64_t n = c ? c - p : (int64_t)strlen(p);
            int found = 0;
            for (int32_t s = 0; s < v->n_samples; s++)
                if (v->names[s].n == n && !memcmp(v->names[s].p, p, (size_t)n)) {
                    flag[s] = 1;
                    found = 1;
                }
            if (!found) bcftools_failed = 1; /* bcftools: unknown sample -> no output */
            if (!c) break;
            p = c + 1;
        }
        for (int32_t s = 0; s < v->n_samples; s++)
            if (flag[s]) sel[n_sel++] = s;
        free(flag);
    } else {
        for (int32_t s = 0; s < v->n_samples; s++) sel[n_sel++] = s;
    }

    const int approx = q->reference_bases && !strcmp(q->reference_bases, "N"); /* sv:59 */
    int exists = 0;
    int64_t call_count = 0, all_alleles_count = 0;
    dbuf variants = {0};
    int64_t n_variants = 0;
    char *sample_hit = (char *)calloc((size_t)n_sel + 1, 1);
    int any_line = 0;
    int err = ORC_OK;
    sv_t *alts = (sv_t *)malloc(sizeof(sv_t) * MAX_ALTS);
    int *hits = (int *)malloc(sizeof(int) * MAX_ALTS);
    sv_t *cols = (sv_t *)malloc(sizeof(sv_t) * (size_t)(v->n_samples + 1));
    int64_t *ac = (int64_t *)malloc(sizeof(int64_t) * MAX_ALTS);
    int64_t *calls = NULL;
    int64_t calls_cap = 0;

    int64_t hi = 0;
    int64_t i0 = bcftools_failed ? 0 : lower_bound(v, rg.chrom, rg.first_bp, &hi);
    if (bcftools_failed) hi = 0;
    for (int64_t ri = i0; ri < hi; ri++) { /* sv:70 for line in stdout */
        const rec_t *r = &v->recs[ri];
        if (r->pos > rg.last_bp) break; /* sv:84 first_bp <= pos <= last_bp */
        any_line = 1;
        const int64_t ref_length = r->ref.n; /* sv:87 */
        const int64_t e = r->pos + ref_length - 1;
        if (!(q->end_min <= e && e <= q->end_max)) continue; /* sv:90 */
        if (!samples_variant) {
            if (!approx && (!q->reference_bases || !upper_eq(r->ref, q->reference_bases))) continue; /* sv:94 */
        } else if (!approx) {
            if (!q->reference_bases) {
                err = ORC_ATTRIBUTE_ERROR; /* svs:89 None.replace */
                break;
            }
            for (const char *c = q->reference_bases; *c; c++)
                if (strchr("*+?()[]{}|^$\\", *c)) {
                    err = ORC_UNSUPPORTED;
                    break;
                }
            if (err) break;
            if (!wild_ref_match(q->reference_bases, r->ref)) continue; /* svs:88-91 */
        }
        /* sv:97 alts = all_alts.split(',') */
        int n_alt = 0;
        {
            const char *p = r->alt.p, *end = r->alt.p + r->alt.n;
            for (;;) {
                const char *c = memchr(p, ',', (size_t)(end - p));
                if (!c) c = end;
                if (n_alt < MAX_ALTS) {
                    alts[n_alt].p = p;
                    alts[n_alt].n = c - p;
                    n_alt++;
                }
                if (c == end) break;
                p = c + 1;
            }
        }
        if (q->alternate_bases == NULL && !q->patched) {
            err = ORC_UNBOUND_LOCAL; /* sv:101 */
            break;
        }
        int nh = compute_hits(q, r->ref, alts, n_alt, hits);
        if (!nh) continue; /* sv:184 */

        /* sv:191-201 INFO scan: last AC=, last AN= (int), last VT= */
        sv_t ac_s = {0, -1};
        int have_an = 0;
        int64_t an = 0;
        sv_t vt = {"N/A", 3};
        {
            const char *p = r->info.p, *end = r->info.p + r->info.n;
            for (;;) {
                const char *c = memchr(p, ';', (size_t)(end - p));
                if (!c) c = end;
                sv_t f = {p, c - p};
                if (sv_starts(f, "AC=")) {
                    ac_s.p = p + 3;
                    ac_s.n = f.n - 3;
                } else if (sv_starts(f, "AN=")) {
                    if (py_int(p + 3, f.n - 3, &an)) {
                        err = ORC_VALUE_ERROR;
                        break;
                    }
                    have_an = 1;
                } else if (sv_starts(f, "VT=")) {
                    vt.p = p + 3;
                    vt.n = f.n - 3;
                }
                if (c == end) break;
                p = c + 1;
            }
        }
        if (err) break;

        /* genotypes of the emitted samples (needed by the GT fallbacks / sample regex) */
        int64_t ncols = 0;
        int have_calls = 0;
        int64_t n_calls = 0;
        if (r->gt) ncols = gt_columns(r, cols, v->n_samples);
#define GATHER_CALLS()                                                                          \
    do {                                                                                        \
        n_calls = 0;                                                                            \
        for (int32_t si = 0; si < n_sel; si++) {                                                \
            if (sel[si] >= ncols) continue;                                                     \
            sv_t g = cols[sel[si]];                                                             \
            for (int64_t k = 0; k < g.n;) {                                                     \
                if (isdigit((unsigned char)g.p[k])) {                                           \
                    int64_t val = 0;                                                            \
                    while (k < g.n && isdigit((unsigned char)g.p[k])) val = val * 10 + (g.p[k++] - '0'); \
                    if (n_calls == calls_cap) {                                                 \
                        calls_cap = calls_cap ? calls_cap * 2 : 1024;                          \
                        calls = (int64_t *)realloc(calls, sizeof(int64_t) * (size_t)calls_cap); \
                    }                                                                           \
                    calls[n_calls++] = val;                                                     \
                } else                                                                          \
                    k++;                                                                        \
            }                                                                                   \
        }                                                                                       \
        have_calls = 1;                                                                         \
    } while (0)

        if (ac_s.n >= 0) { /* sv:205-214 */
            int n_ac = 0;
            const char *p = ac_s.p, *end = ac_s.p + ac_s.n;
            for (;;) {
                const char *c = memchr(p, ',', (size_t)(end - p));
                if (!c) c = end;
                int64_t val;
                if (py_int(p, c - p, &val)) {
                    err = ORC_VALUE_ERROR;
                    break;
                }
                if (n_ac < MAX_ALTS) ac[n_ac++] = val;
                if (c == end) break;
                p = c + 1;
            }
            if (err) break;
            for (int k = 0; k < nh; k++)
                if (hits[k] >= n_ac) err = ORC_INDEX_ERROR; /* sv:207 */
            if (err) break;
            for (int k = 0; k < nh; k++) {
                int i = hits[k];
                if (ac[i] != 0) { /* sv:209-213 */
                    if (n_variants) db_putc(&variants, '\n');
                    db_put(&variants, rg.chrom.p, rg.chrom.n);
                    db_putc(&variants, '\t');
                    db_put(&variants, r->pos_txt.p, r->pos_txt.n);
                    db_putc(&variants, '\t');
                    db_put(&variants, r->ref.p, r->ref.n);
                    db_putc(&variants, '\t');
                    db_put(&variants, alts[i].p, alts[i].n);
                    db_putc(&variants, '\t');
                    db_put(&variants, vt.p, vt.n);
                    n_variants++;
                }
                call_count += ac[i]; /* sv:214 */
            }
        } else { /* sv:215-226 genotype fallback */
            GATHER_CALLS();
            /* set(all_calls) & {i+1}: iterated ascending (CPython small-int set order) */
            for (int k = 0; k < nh && !err; k++) {
                int64_t want = hits[k] + 1;
                int present = 0;
                for (int64_t c = 0; c < n_calls; c++)
                    if (calls[c] == want) {
                        present = 1;
                        break;
                    }
                if (!present) continue;
                if (want >= n_alt) {
                    err = ORC_INDEX_ERROR; /* sv:223 alts[i] with 1-based i */
                    break;
                }
                if (n_variants) db_putc(&variants, '\n');
                db_put(&variants, rg.chrom.p, rg.chrom.n);
                db_putc(&variants, '\t');
                db_put(&variants, r->pos_txt.p, r->pos_txt.n);
                db_putc(&variants, '\t');
                db_put(&variants, r->ref.p, r->ref.n);
                db_putc(&variants, '\t');
                db_put(&variants, alts[want].p, alts[want].n);
                db_putc(&variants, '\t');
                db_put(&variants, vt.p, vt.n);
                n_variants++;
            }
            if (err) break;
            for (int64_t c = 0; c < n_calls; c++)
                for (int k = 0; k < nh; k++)
                    if (calls[c] == hits[k] + 1) {
                        call_count++; /* sv:226 */
                        break;
                    }
        }

        if (call_count) { /* sv:229 cumulative */
            exists = 1;
            if (!q->include_details) break; /* sv:231-232 (before AN is added) */
            int collect = (q->granularity == ORC_RECORD || q->granularity == ORC_AGGREGATED) &&
                          (samples_variant || include_samples); /* sv:235, svs:231 */
            if (collect) {
                /* sv:233-236: GT token (split on | and /) equal to a hit allele number */
                for (int32_t si = 0; si < n_sel; si++) {
                    if (sample_hit[si] || sel[si] >= ncols) continue;
                    sv_t g = cols[sel[si]];
                    int64_t k = 0;
                    while (k <= g.n && !sample_hit[si]) {
                        int64_t t = k;
                        while (t < g.n && g.p[t] != '|' && g.p[t] != '/') t++;
                        /* token g[k:t] */
                        for (int x = 0; x < nh; x++) {
                            char num[32];
                            int nn = snprintf(num, sizeof num, "%d", hits[x] + 1);
                            if (t - k == nn && !memcmp(g.p + k, num, (size_t)nn)) {
                                sample_hit[si] = 1;
                                break;
                            }
                        }
                        k = t + 1;
                    }
                }
            }
        }
        /* sv:244-250 */
        if (have_an) {
            all_alleles_count += an;
        } else {
            if (!have_calls) GATHER_CALLS();
            all_alleles_count += n_calls;
        }
        if (!samples_variant && q->granularity == ORC_BOOLEAN && exists) break; /* sv:253-254 */
    }
#undef GATHER_CALLS

    free(alts);
    free(hits);
    free(cols);
    free(ac);
    free(calls);
    if (err) {
        free(sel);
        free(sample_hit);
        free(variants.p);
        res->error = err;
        return err;
    }
    res->exists = exists;
    res->call_count = call_count;
    res->all_alleles_count = all_alleles_count;
    res->variants = variants.p ? variants.p : (char *)calloc(1, 1);
    res->n_variants = n_variants;
    /* sv:257-258 / svs:248-249 sample names; all_sample_names comes from the first
     * emitted line, so an empty slice yields no names. */
    dbuf names = {0};
    int64_t n_names = 0;
    int want_names = (q->granularity == ORC_RECORD || q->granularity == ORC_AGGREGATED) &&
                     (samples_variant || include_samples);
    res->sample_indices = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n_sel + 1));
    for (int32_t si = 0; si < n_sel; si++) {
        if (!sample_hit[si]) continue;
        if (samples_variant) res->sample_indices[res->n_sample_indices++] = si;
        if (want_names && any_line) {
            if (n_names) db_putc(&names, ',');
            db_put(&names, v->names[sel[si]].p, v->names[sel[si]].n);
            n_names++;
        }
    }
    res->sample_names = names.p ? names.p : (char *)calloc(1, 1);
    res->n_sample_names = n_names;
    free(sel);
    free(sample_hit);
    return 0;
}

int orc_query_batch(void *h, const orc_query *qs, int64_t n, orc_result *rs, int threads) {
#ifdef _OPENMP
    if (threads > 0) omp_set_num_threads(threads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (int64_t i = 0; i < n; i++) orc_query_one(h, &qs[i], &rs[i]);
    (void)threads;
    return 0;
}

int64_t orc_records_in_region(void *h, const char *region) {
    const vcf_t *v = (const vcf_t *)h;
    region_t rg;
    if (parse_region(region, &rg)) return -1;
    int64_t hi = 0, n = 0;
    for (int64_t i = lower_bound(v, rg.chrom, rg.first_bp, &hi); i < hi && v->recs[i].pos <= rg.last_bp; i++) n++;
    return n;
}
