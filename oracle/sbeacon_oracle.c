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

/* ----------------------------------------------------------- Python ints
 * int(str) is unbounded in the reference (sv:199, :206, :218) up to
 * CPython's 4300-digit str->int limit (ValueError past it; Python >= 3.10.7 /
 * 3.9.14, the Lambda python3.9 runtime included).  Values are kept as int64
 * while they fit and as two's complement bignums (BN_LIMBS x 32 bits) past
 * that. */
#define PY_MAX_STR_DIGITS 4300
#define BN_LIMBS 480 /* 15360 bits: a 4300-digit value (14284 bits) + sum headroom */

typedef struct {
    uint32_t l[BN_LIMBS];
} bn_t;

static void bn_from_i64(bn_t *b, int64_t v) {
    uint64_t u = (uint64_t)v;
    b->l[0] = (uint32_t)u;
    b->l[1] = (uint32_t)(u >> 32);
    uint32_t s = v < 0 ? 0xffffffffu : 0u;
    for (int i = 2; i < BN_LIMBS; i++) b->l[i] = s;
}
static void bn_add(bn_t *a, const bn_t *b) {
    uint64_t c = 0;
    for (int i = 0; i < BN_LIMBS; i++) {
        c += (uint64_t)a->l[i] + b->l[i];
        a->l[i] = (uint32_t)c;
        c >>= 32;
    }
}
static void bn_neg(bn_t *a) {
    uint64_t c = 1;
    for (int i = 0; i < BN_LIMBS; i++) {
        c += (uint64_t)(uint32_t)~a->l[i];
        a->l[i] = (uint32_t)c;
        c >>= 32;
    }
}
static int bn_is_zero(const bn_t *a) {
    for (int i = 0; i < BN_LIMBS; i++)
        if (a->l[i]) return 0;
    return 1;
}
static int bn_fits_i64(const bn_t *a, int64_t *v) {
    uint32_t s = (a->l[1] >> 31) ? 0xffffffffu : 0u;
    for (int i = 2; i < BN_LIMBS; i++)
        if (a->l[i] != s) return 0;
    *v = (int64_t)(((uint64_t)a->l[1] << 32) | a->l[0]);
    return 1;
}
static char *bn_to_hex(const bn_t *a) { /* "0x.." / "-0x.." (malloc) */
    bn_t m = *a;
    int neg = (m.l[BN_LIMBS - 1] >> 31) != 0;
    if (neg) bn_neg(&m);
    char *s = (char *)malloc(BN_LIMBS * 8 + 4), *p = s;
    if (neg) *p++ = '-';
    *p++ = '0';
    *p++ = 'x';
    int top = BN_LIMBS - 1;
    while (top > 0 && !m.l[top]) top--;
    p += sprintf(p, "%x", m.l[top]);
    for (int i = top - 1; i >= 0; i--) p += sprintf(p, "%08x", m.l[i]);
    return s;
}

/* Python int(str) for the ASCII forms VCF text carries: strip whitespace,
 * optional sign, digits with single '_' between digits, at most 4300 digits.
 * small = |v| < 10^18; otherwise *big (caller frees). 0 ok, -1 ValueError. */
typedef struct {
    int64_t v;
    bn_t *big; /* NULL = small */
} pyint_t;

static int py_int_big(const char *p, int64_t n, pyint_t *out) {
    int64_t i = 0, j = n;
    out->v = 0;
    out->big = NULL;
    while (i < j && isspace((unsigned char)p[i])) i++;
    while (j > i && isspace((unsigned char)p[j - 1])) j--;
    if (i == j) return -1;
    int neg = 0;
    if (p[i] == '+' || p[i] == '-') {
        neg = p[i] == '-';
        i++;
    }
    if (i == j || !isdigit((unsigned char)p[i])) return -1;
    int64_t digits = 0, sig = 0; /* all digits / digits after leading zeros */
    for (int64_t k = i; k < j; k++) {
        if (p[k] == '_') {
            if (k + 1 >= j || !isdigit((unsigned char)p[k + 1]) || !isdigit((unsigned char)p[k - 1])) return -1;
            continue;
        }
        if (!isdigit((unsigned char)p[k])) return -1;
        digits++;
        if (sig || p[k] != '0') sig++;
    }
    if (digits > PY_MAX_STR_DIGITS) return -1;
    if (sig <= 18) {
        int64_t v = 0;
        for (int64_t k = i; k < j; k++)
            if (p[k] != '_') v = v * 10 + (p[k] - '0');
        out->v = neg ? -v : v;
        return 0;
    }
    bn_t *b = (bn_t *)calloc(1, sizeof(bn_t));
    for (int64_t k = i; k < j; k++) {
        if (p[k] == '_') continue;
        uint64_t c = (uint64_t)(p[k] - '0');
        for (int t = 0; t < BN_LIMBS; t++) {
            c += (uint64_t)b->l[t] * 10u;
            b->l[t] = (uint32_t)c;
            c >>= 32;
        }
    }
    if (neg) bn_neg(b);
    out->big = b;
    return 0;
}
static int py_is_zero(const pyint_t *x) { return x->big ? bn_is_zero(x->big) : x->v == 0; }

/* running Python-int sum: v + (b ? *b : 0) */
typedef struct {
    int64_t v;
    bn_t *b;
} acc_t;

static void acc_spill(acc_t *a) {
    if (!a->b) {
        a->b = (bn_t *)calloc(1, sizeof(bn_t));
    }
    bn_t t;
    bn_from_i64(&t, a->v);
    bn_add(a->b, &t);
    a->v = 0;
}
static void acc_add_i64(acc_t *a, int64_t x) {
    int64_t r;
    if (__builtin_add_overflow(a->v, x, &r)) {
        acc_spill(a);
        a->v = x;
    } else {
        a->v = r;
    }
}
static void acc_add(acc_t *a, const pyint_t *x) {
    if (!x->big) {
        acc_add_i64(a, x->v);
        return;
    }
    if (!a->b) a->b = (bn_t *)calloc(1, sizeof(bn_t));
    bn_add(a->b, x->big);
}
static int acc_nonzero(acc_t *a) {
    if (!a->b) return a->v != 0;
    acc_spill(a);
    return !bn_is_zero(a->b);
}
static void acc_out(acc_t *a, int64_t *v, char **hex) {
    *hex = NULL;
    if (!a->b) {
        *v = a->v;
        return;
    }
    acc_spill(a);
    if (!bn_fits_i64(a->b, v)) {
        *v = (int64_t)(((uint64_t)a->b->l[1] << 32) | a->b->l[0]);
        *hex = bn_to_hex(a->b);
    }
}
static void acc_free(acc_t *a) {
    free(a->b);
    a->b = NULL;
}

/* --------------------------------------------- CPython set emulation
 * sv:223 emits `alts[i] for i in set(all_calls) & hit_set`: the variant
 * order is CPython's iteration order of that set (Objects/setobject.c,
 * 3.10: set_add_entry / set_insert_clean / set_table_resize /
 * set_intersection; LINEAR_PROBES 9, PERTURB_SHIFT 5, PySet_MINSIZE 8, growth
 * at fill*5 >= mask*3 to 4*used).  An int's hash is its value mod 2**61 - 1.
 * Keys index a table of call values compared by value. */
typedef struct {
    uint64_t hash;
    int64_t v;      /* small value (sig digits <= 18) */
    const char *d;  /* big: significant digits */
    int64_t dl;     /* big: their count (0 = small) */
} pyval_t;

static int pyval_eq(const pyval_t *a, const pyval_t *b) {
    if (a->dl != b->dl) return 0;
    if (!a->dl) return a->v == b->v;
    return !memcmp(a->d, b->d, (size_t)a->dl);
}

typedef struct {
    uint64_t hash;
    int64_t key;
    int used;
} sent_t;
typedef struct {
    sent_t *t;
    uint64_t mask, fill, used;
} pset_t;

static void pset_init(pset_t *s) {
    s->mask = 7;
    s->t = (sent_t *)calloc(8, sizeof(sent_t));
    s->fill = s->used = 0;
}
static void pset_insert_clean(sent_t *t, uint64_t mask, uint64_t hash, int64_t key) {
    uint64_t perturb = hash, i = hash & mask;
    sent_t *e;
    for (;;) {
        e = &t[i];
        if (!e->used) goto found;
        if (i + 9 <= mask)
            for (int j = 0; j < 9; j++) {
                e++;
                if (!e->used) goto found;
            }
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
found:
    e->used = 1;
    e->hash = hash;
    e->key = key;
}
static void pset_add(pset_t *s, const pyval_t *vals, uint64_t hash, int64_t key) {
    uint64_t mask = s->mask, i = hash & mask, perturb = hash;
    sent_t *e;
    for (;;) {
        e = &s->t[i];
        int probes = (i + 9 <= mask) ? 9 : 0;
        do {
            if (!e->used) goto unused;
            if (e->hash == hash && pyval_eq(&vals[e->key], &vals[key])) return;
            e++;
        } while (probes--);
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
unused:
    e->used = 1;
    e->hash = hash;
    e->key = key;
    s->fill++;
    s->used++;
    if (s->fill * 5 < mask * 3) return;
    uint64_t minused = s->used > 50000 ? s->used * 2 : s->used * 4, newsize = 8;
    while (newsize <= minused) newsize <<= 1;
    sent_t *nt = (sent_t *)calloc(newsize, sizeof(sent_t));
    for (uint64_t k = 0; k <= mask; k++)
        if (s->t[k].used) pset_insert_clean(nt, newsize - 1, s->t[k].hash, s->t[k].key);
    free(s->t);
    s->t = nt;
    s->mask = newsize - 1;
    s->fill = s->used;
}
static int pset_contains(const pset_t *s, const pyval_t *vals, uint64_t hash, int64_t key) {
    uint64_t mask = s->mask, i = hash & mask, perturb = hash;
    for (;;) {
        const sent_t *e = &s->t[i];
        int probes = (i + 9 <= mask) ? 9 : 0;
        do {
            if (!e->used) return 0;
            if (e->hash == hash && pyval_eq(&vals[e->key], &vals[key])) return 1;
            e++;
        } while (probes--);
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
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
    free(r->call_count_hex);
    free(r->all_alleles_count_hex);
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
    acc_t call_count = {0, NULL}, all_alleles_count = {0, NULL};
    dbuf variants = {0};
    int64_t n_variants = 0;
    char *sample_hit = (char *)calloc((size_t)n_sel + 1, 1);
    int any_line = 0;
    int err = ORC_OK;
    sv_t *alts = (sv_t *)malloc(sizeof(sv_t) * MAX_ALTS);
    int *hits = (int *)malloc(sizeof(int) * MAX_ALTS);
    char *is_hit = (char *)malloc(MAX_ALTS + 1);
    sv_t *cols = (sv_t *)malloc(sizeof(sv_t) * (size_t)(v->n_samples + 1));
    pyint_t *ac = (pyint_t *)calloc(MAX_ALTS, sizeof(pyint_t));
    int n_ac_alloc = 0; /* entries of ac[] holding a bignum to free */
    pyval_t *calls = NULL; /* all_calls (sv:218), then the hit_set values */
    int64_t calls_cap = 0;
    int calls_huge = 0;    /* a digit run int() rejects (> 4300 digits) */

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
        pyint_t an = {0, NULL};
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
                    free(an.big);
                    if (py_int_big(p + 3, f.n - 3, &an)) {
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
        if (err) {
            free(an.big);
            break;
        }

        /* genotypes of the emitted samples (needed by the GT fallbacks / sample regex) */
        int64_t ncols = 0;
        int have_calls = 0;
        int64_t n_calls = 0;
        if (r->gt) ncols = gt_columns(r, cols, v->n_samples);
        /* all_calls = digit runs of the subset's GT text (sv:218, :249): value
         * identity and hash of int(run) (hash(int) = value mod 2**61 - 1) */
#define GATHER_CALLS()                                                                          \
    do {                                                                                        \
        n_calls = 0;                                                                            \
        calls_huge = 0;                                                                         \
        for (int32_t si = 0; si < n_sel; si++) {                                                \
            if (sel[si] >= ncols) continue;                                                     \
            sv_t g = cols[sel[si]];                                                             \
            for (int64_t k = 0; k < g.n;) {                                                     \
                if (isdigit((unsigned char)g.p[k])) {                                           \
                    int64_t k0 = k;                                                             \
                    while (k < g.n && isdigit((unsigned char)g.p[k])) k++;                      \
                    if (n_calls + nh + 1 >= calls_cap) {                                        \
                        calls_cap = calls_cap ? calls_cap * 2 : 1024;                          \
                        while (calls_cap <= n_calls + nh + 1) calls_cap *= 2;                   \
                        calls = (pyval_t *)realloc(calls, sizeof(pyval_t) * (size_t)calls_cap); \
                    }                                                                           \
                    if (k - k0 > PY_MAX_STR_DIGITS) calls_huge = 1;                             \
                    while (k0 < k - 1 && g.p[k0] == '0') k0++;                                  \
                    pyval_t *pv = &calls[n_calls++];                                            \
                    pv->v = 0;                                                                  \
                    pv->hash = 0;                                                               \
                    pv->d = g.p + k0;                                                           \
                    pv->dl = (k - k0 > 18) ? k - k0 : 0;                                        \
                    for (int64_t t = k0; t < k; t++) {                                          \
                        unsigned __int128 h = (unsigned __int128)pv->hash * 10u + (unsigned)(g.p[t] - '0'); \
                        pv->hash = (uint64_t)(h % 2305843009213693951ull);                      \
                        if (!pv->dl) pv->v = pv->v * 10 + (g.p[t] - '0');                       \
                    }                                                                           \
                } else                                                                          \
                    k++;                                                                        \
            }                                                                                   \
        }                                                                                       \
        have_calls = 1;                                                                         \
    } while (0)
#define EMIT_VARIANT(ALT)                                  \
    do {                                                   \
        if (n_variants) db_putc(&variants, '\n');          \
        db_put(&variants, rg.chrom.p, rg.chrom.n);         \
        db_putc(&variants, '\t');                          \
        db_put(&variants, r->pos_txt.p, r->pos_txt.n);     \
        db_putc(&variants, '\t');                          \
        db_put(&variants, r->ref.p, r->ref.n);             \
        db_putc(&variants, '\t');                          \
        db_put(&variants, (ALT).p, (ALT).n);               \
        db_putc(&variants, '\t');                          \
        db_put(&variants, vt.p, vt.n);                     \
        n_variants++;                                      \
    } while (0)

        if (ac_s.n >= 0) { /* sv:205-214 */
            int n_ac = 0;
            for (int k = 0; k < n_ac_alloc; k++) {
                free(ac[k].big);
                ac[k].big = NULL;
            }
            const char *p = ac_s.p, *end = ac_s.p + ac_s.n;
            for (;;) {
                const char *c = memchr(p, ',', (size_t)(end - p));
                if (!c) c = end;
                pyint_t val;
                if (py_int_big(p, c - p, &val)) {
                    err = ORC_VALUE_ERROR;
                    break;
                }
                if (n_ac < MAX_ALTS) ac[n_ac++] = val;
                else free(val.big);
                n_ac_alloc = n_ac;
                if (c == end) break;
                p = c + 1;
            }
            if (!err)
                for (int k = 0; k < nh; k++)
                    if (hits[k] >= n_ac) err = ORC_INDEX_ERROR; /* sv:207 */
            if (err) {
                free(an.big);
                break;
            }
            for (int k = 0; k < nh; k++) {
                int i = hits[k];
                if (!py_is_zero(&ac[i])) EMIT_VARIANT(alts[i]); /* sv:209-213 */
                acc_add(&call_count, &ac[i]);                   /* sv:214 */
            }
        } else { /* sv:215-226 genotype fallback */
            GATHER_CALLS();
            if (n_calls + nh + 1 >= calls_cap) { /* room for the hit_set values after the calls */
                calls_cap = n_calls + nh + 1024;
                calls = (pyval_t *)realloc(calls, sizeof(pyval_t) * (size_t)calls_cap);
            }
            if (calls_huge) { /* int(g) of a run past 4300 digits */
                err = ORC_VALUE_ERROR;
                free(an.big);
                break;
            }
            /* set(all_calls) & {i + 1 for i in hit_indexes}, iterated in CPython order */
            pset_t sc, hs, res;
            pset_init(&sc);
            pset_init(&hs);
            pset_init(&res);
            for (int64_t c = 0; c < n_calls; c++) pset_add(&sc, calls, calls[c].hash, c);
            for (int k = 0; k < nh; k++) {
                pyval_t *hv = &calls[n_calls + k];
                hv->v = hits[k] + 1;
                hv->hash = (uint64_t)hv->v;
                hv->d = NULL;
                hv->dl = 0;
                pset_add(&hs, calls, hv->hash, n_calls + k);
            }
            const pset_t *so = &sc, *other = &hs; /* set_intersection(so, other) */
            if (hs.used > sc.used) {
                so = &hs;
                other = &sc;
            }
            for (uint64_t k = 0; k <= other->mask; k++)
                if (other->t[k].used && pset_contains(so, calls, other->t[k].hash, other->t[k].key))
                    pset_add(&res, calls, other->t[k].hash, other->t[k].key);
            for (uint64_t k = 0; k <= res.mask && !err; k++)
                if (res.t[k].used && calls[res.t[k].key].v >= n_alt) err = ORC_INDEX_ERROR; /* sv:223 alts[i], 1-based i */
            if (!err)
                for (uint64_t k = 0; k <= res.mask; k++)
                    if (res.t[k].used) EMIT_VARIANT(alts[calls[res.t[k].key].v]);
            free(sc.t);
            free(hs.t);
            free(res.t);
            if (err) {
                free(an.big);
                break;
            }
            memset(is_hit, 0, (size_t)n_alt + 1);
            for (int k = 0; k < nh; k++) is_hit[hits[k] + 1] = 1;
            int64_t cnt = 0;
            for (int64_t c = 0; c < n_calls; c++)
                if (!calls[c].dl && calls[c].v >= 1 && calls[c].v <= n_alt && is_hit[calls[c].v]) cnt++; /* sv:226 */
            acc_add_i64(&call_count, cnt);
        }

        if (acc_nonzero(&call_count)) { /* sv:229 cumulative */
            exists = 1;
            if (!q->include_details) { /* sv:231-232 (before AN is added) */
                free(an.big);
                break;
            }
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
            acc_add(&all_alleles_count, &an);
        } else {
            if (!have_calls) GATHER_CALLS(); /* get_all_calls: strings, no int() */
            acc_add_i64(&all_alleles_count, n_calls);
        }
        free(an.big);
        if (!samples_variant && q->granularity == ORC_BOOLEAN && exists) break; /* sv:253-254 */
    }
#undef GATHER_CALLS
#undef EMIT_VARIANT

    free(alts);
    free(hits);
    free(is_hit);
    free(cols);
    for (int k = 0; k < n_ac_alloc; k++) free(ac[k].big);
    free(ac);
    free(calls);
    if (err) {
        acc_free(&call_count);
        acc_free(&all_alleles_count);
        free(sel);
        free(sample_hit);
        free(variants.p);
        res->error = err;
        return err;
    }
    res->exists = exists;
    acc_out(&call_count, &res->call_count, &res->call_count_hex);
    acc_out(&all_alleles_count, &res->all_alleles_count, &res->all_alleles_count_hex);
    acc_free(&call_count);
    acc_free(&all_alleles_count);
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
