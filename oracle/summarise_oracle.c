/*
 * summarise_oracle.c — CPU restatement of the reference summariseSlice counter
 * and of duplicateVariantSearch's unique count over the region entries
 * summariseSlice writes.
 *
 * TEST INFRASTRUCTURE ONLY (checker for the device summarise / dedup paths).
 *
 * Restates lambda/summariseSlice/source/main.cpp:195-245 (getRegionStats),
 * :52-109 (addCounts), write_data_to_s3.h:150-228 (recordHeader's reader
 * movement) and vcf_chunk_reader.h:24-373 (VcfChunkReader) over a BGZF file
 * held in memory.  The reader's block walk is equivalent to a character
 * stream S = uncompressed[U(vstart), U(vend)): every read stops where the
 * final block's blockChars = endUncompressed cuts it (vcf_chunk_reader.h:172,
 * :223-231), keepReading() is "cursor < |S|", and seek() may overshoot.
 *
 * The reference summariseSlice / duplicateVariantSearch programs cannot be
 * built here (AWS SDK C++ and aws-lambda-runtime are absent).
 * Their AWS-free pieces are: oracle/_ref (Makefile.ref) compiles
 * lambda/shared/gzip/gzip.cpp, lambda/shared/source/generalutils.* and
 * lambda/summariseSlice/source/fast_atoi.h where they lie, and
 * tests/test_ref_pinned.py pins this file's sequenceToBinary table
 * (seq_code), atoui64 (atoui64_len) and the region-file gzip round trip to
 * them; the reader walk and the skip heuristic remain checked against
 * hand-derived cases (tests/test_summarise_oracle.py).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

typedef struct {
    uint8_t *u;       /* whole uncompressed stream */
    int64_t ulen;
    int64_t nblk;
    uint64_t *coff;   /* compressed offset of block i */
    uint64_t *ustart; /* uncompressed offset of block i */
    uint32_t *isize;
} bgzf_t;

void orc_bgzf_close(void *h) {
    bgzf_t *b = (bgzf_t *)h;
    if (!b) return;
    free(b->u);
    free(b->coff);
    free(b->ustart);
    free(b->isize);
    free(b);
}

/* parse + inflate every BGZF block (gzip header with the BC extra subfield) */
void *orc_bgzf_open(const char *path) {
    FILE *f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t *c = (uint8_t *)malloc((size_t)n + 1);
    if (fread(c, 1, (size_t)n, f) != (size_t)n) {
        fclose(f);
        free(c);
        return NULL;
    }
    fclose(f);
    bgzf_t *b = (bgzf_t *)calloc(1, sizeof(bgzf_t));
    int64_t cap = 1024;
    b->coff = (uint64_t *)malloc(8 * (size_t)cap);
    b->ustart = (uint64_t *)malloc(8 * (size_t)cap);
    b->isize = (uint32_t *)malloc(4 * (size_t)cap);
    int64_t p = 0, u = 0;
    while (p + 18 <= n) {
        if (c[p] != 0x1f || c[p + 1] != 0x8b || c[p + 2] != 8 || !(c[p + 3] & 4)) goto bad;
        const uint32_t xlen = c[p + 10] | (c[p + 11] << 8);
        int64_t bsize = -1;
        for (int64_t x = p + 12; x + 4 <= p + 12 + xlen;) {
            const uint32_t slen = c[x + 2] | (c[x + 3] << 8);
            if (c[x] == 'B' && c[x + 1] == 'C' && slen == 2) bsize = (c[x + 4] | (c[x + 5] << 8)) + 1;
            x += 4 + slen;
        }
        if (bsize < 0 || p + bsize > n) goto bad;
        if (b->nblk == cap) {
            cap *= 2;
            b->coff = (uint64_t *)realloc(b->coff, 8 * (size_t)cap);
            b->ustart = (uint64_t *)realloc(b->ustart, 8 * (size_t)cap);
            b->isize = (uint32_t *)realloc(b->isize, 4 * (size_t)cap);
        }
        const uint32_t is = c[p + bsize - 4] | (c[p + bsize - 3] << 8) | (c[p + bsize - 2] << 16) |
                            ((uint32_t)c[p + bsize - 1] << 24);
        b->coff[b->nblk] = (uint64_t)p;
        b->ustart[b->nblk] = (uint64_t)u;
        b->isize[b->nblk] = is;
        b->nblk++;
        u += is;
        p += bsize;
    }
    b->ulen = u;
    b->u = (uint8_t *)malloc((size_t)u + 1);
    for (int64_t i = 0; i < b->nblk; ++i) {
        const int64_t s = (int64_t)b->coff[i];
        const uint32_t xlen = c[s + 10] | (c[s + 11] << 8);
        const int64_t bsize = (i + 1 < b->nblk ? (int64_t)b->coff[i + 1] : n) - s;
        z_stream z;
        memset(&z, 0, sizeof z);
        inflateInit2(&z, -15);
        z.next_in = c + s + 12 + xlen;
        z.avail_in = (uInt)(bsize - 12 - xlen - 8);
        z.next_out = b->u + b->ustart[i];
        z.avail_out = b->isize[i];
        inflate(&z, Z_FINISH);
        inflateEnd(&z);
    }
    free(c);
    return b;
bad:
    free(c);
    orc_bgzf_close(b);
    return NULL;
}

int64_t orc_bgzf_ulen(void *h) { return ((bgzf_t *)h)->ulen; }
int64_t orc_bgzf_nblocks(void *h) { return ((bgzf_t *)h)->nblk; }

/* virtual offset (coffset << 16 | uoffset) -> absolute uncompressed offset */
int orc_bgzf_voff_to_u(void *h, uint64_t voff, uint64_t *out) {
    bgzf_t *b = (bgzf_t *)h;
    const uint64_t co = voff >> 16, uo = voff & 0xffff;
    int64_t lo = 0, hi = b->nblk;
    while (lo < hi) {
        int64_t m = (lo + hi) / 2;
        if (b->coff[m] < co)
            lo = m + 1;
        else
            hi = m;
    }
    if (lo == b->nblk || b->coff[lo] != co) {
        if (co >= (b->nblk ? b->coff[b->nblk - 1] + 1 : 0)) { /* at / past the end */
            *out = (uint64_t)b->ulen;
            return 0;
        }
        return -1;
    }
    *out = b->ustart[lo] + uo;
    return 0;
}

/* ------------------------------------------------------------ reader on S */
typedef struct {
    const char *s;
    int64_t n, pos;
} rd_t;

/* readPastChars<A, B> (vcf_chunk_reader.h:262-301): '\0' at the cut */
static char read_past(rd_t *r, char a, char b, const char **f, int64_t *fl) {
    const int64_t st = r->pos;
    while (r->pos < r->n) {
        const char c = r->s[r->pos];
        if (c == a || c == b) {
            *f = r->s + st;
            *fl = r->pos - st;
            r->pos++;
            return c;
        }
        r->pos++;
    }
    *f = r->s + st;
    *fl = r->pos - st;
    return '\0';
}

/* skipPast<N, delim> (:308-328) */
static int skip_past(rd_t *r, char d, int N) {
    int num = N;
    while (r->pos < r->n)
        if (r->s[r->pos++] == d && (N == 1 || --num == 0)) return 1;
    return 0;
}

/* skipPastAndCountChars (:330-350) */
static uint64_t skip_count(rd_t *r, char d) {
    uint64_t k = 0;
    while (r->pos < r->n) {
        const char c = r->s[r->pos];
        k += (c == '\t') || (c == '/') || (c == '|') || (c == ';') || (c == ':');
        r->pos++;
        if (c == d) return k;
    }
    return k;
}

/* fast_atoi.h:73-99 atoui64(str, len) for len <= 20 (UB beyond) */
static int atoui64_len(const char *str, uint8_t len, uint64_t *out) {
    static const uint64_t off[21] = {0,
                                     (uint64_t)'0',
                                     (uint64_t)'0' * 11ull,
                                     (uint64_t)'0' * 111ull,
                                     (uint64_t)'0' * 1111ull,
                                     (uint64_t)'0' * 11111ull,
                                     (uint64_t)'0' * 111111ull,
                                     (uint64_t)'0' * 1111111ull,
                                     (uint64_t)'0' * 11111111ull,
                                     (uint64_t)'0' * 111111111ull,
                                     (uint64_t)'0' * 1111111111ull,
                                     (uint64_t)'0' * 11111111111ull,
                                     (uint64_t)'0' * 111111111111ull,
                                     (uint64_t)'0' * 1111111111111ull,
                                     (uint64_t)'0' * 11111111111111ull,
                                     (uint64_t)'0' * 111111111111111ull,
                                     (uint64_t)'0' * 1111111111111111ull,
                                     (uint64_t)'0' * 11111111111111111ull,
                                     (uint64_t)'0' * 111111111111111111ull,
                                     (uint64_t)'0' * 1111111111111111111ull,
                                     (uint64_t)'0' * 11111111111111111111ull};
    if (len > 20) return -1;
    uint64_t v = 0, p10 = 1;
    for (int k = 1; k <= len; ++k) {
        v += (uint64_t)(int64_t)(signed char)str[len - k] * p10;
        p10 *= 10ull;
    }
    *out = v - off[len];
    return 0;
}

/* generalutils.hpp:19-36 sequenceToBinary (-1: std::map::at throws) */
static int seq_code(char c) {
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

int orc_seq_code(int c) { return seq_code((char)c); }
int orc_atoui64_len(const char *s, uint8_t len, uint64_t *out) { return atoui64_len(s, len, out); }

/* write_data_to_s3.h:103-134 compressSeq into out (returns length, -1 where
 * the reference throws).  Each packed byte is appended once (the reference's
 * append((char *)&contigBin) reads a C string past the byte: UB) */
static int64_t compress_seq(const char *s, int64_t n, char *out) {
    if (n == 1) {
        const int v = seq_code(s[0]);
        if (v < 0) return -1;
        out[0] = (char)v;
        return 1;
    }
    if (s[0] == '<' && s[n - 1] == '>') {
        memcpy(out, s + 1, (size_t)(n - 2));
        return n - 2;
    }
    int64_t k = 0;
    for (int64_t i = 0; i < n; i += 2) {
        int v = seq_code(s[i]);
        if (v < 0) return -1;
        if (i + 1 < n) {
            const int w = seq_code(s[i + 1]);
            if (w < 0) return -1;
            v = (v << 4) | w;
        }
        out[k++] = (char)v;
    }
    return k;
}

/* region-file entries {pos, ref', alt'} as key strings to_string(pos) +
 * ref' + '_' + alt' (readVcfData.cpp:23) */
typedef struct {
    char **s;
    int64_t *len;
    uint64_t *pos;
    int64_t n, cap;
} keys_t;

static void keys_push(keys_t *k, uint64_t pos, const char *ref, int64_t rl, const char *alt, int64_t al) {
    if (k->n == k->cap) {
        k->cap = k->cap ? 2 * k->cap : 1024;
        k->s = (char **)realloc(k->s, sizeof(char *) * (size_t)k->cap);
        k->len = (int64_t *)realloc(k->len, sizeof(int64_t) * (size_t)k->cap);
        k->pos = (uint64_t *)realloc(k->pos, sizeof(uint64_t) * (size_t)k->cap);
    }
    char d[24];
    const int nd = snprintf(d, sizeof d, "%llu", (unsigned long long)pos);
    const int64_t L = nd + rl + 1 + al;
    char *p = (char *)malloc((size_t)L);
    memcpy(p, d, (size_t)nd);
    memcpy(p + nd, ref, (size_t)rl);
    p[nd + rl] = '_';
    memcpy(p + nd + rl + 1, alt, (size_t)al);
    k->s[k->n] = p;
    k->len[k->n] = L;
    k->pos[k->n] = pos;
    k->n++;
}

/* move entry i of src to the end of dst */
static void keys_move(keys_t *dst, keys_t *src, int64_t i) {
    if (dst->n == dst->cap) {
        dst->cap = dst->cap ? 2 * dst->cap : 1024;
        dst->s = (char **)realloc(dst->s, sizeof(char *) * (size_t)dst->cap);
        dst->len = (int64_t *)realloc(dst->len, sizeof(int64_t) * (size_t)dst->cap);
        dst->pos = (uint64_t *)realloc(dst->pos, sizeof(uint64_t) * (size_t)dst->cap);
    }
    dst->s[dst->n] = src->s[i];
    dst->len[dst->n] = src->len[i];
    dst->pos[dst->n] = src->pos[i];
    dst->n++;
    src->s[i] = NULL;
}

static void keys_free(keys_t *k) {
    for (int64_t i = 0; i < k->n; ++i) free(k->s[i]);
    free(k->s);
    free(k->len);
    free(k->pos);
}

/* write_data_to_s3.h:150-228 recordHeader: reader movement, the POS parse
 * (fast_atoi, generalutils.hpp:38-45), compressSeq of REF and each ALT part
 * and the region entries pushed (into keys when non-NULL).  Returns -1 where
 * the reference throws (compressSeq on a character outside the table).  *pos
 * receives the record's POS. */
static int record_header(rd_t *r, int *contig_set, keys_t *keys, uint64_t *pos_out) {
    int loop_pos = 0, bad = 0;
    uint64_t pos = 0;
    char ref[65536], alt[65536];
    int64_t rl = 0;
    if (*contig_set) {
        skip_past(r, '\t', 1);
        loop_pos = 1;
    }
    do {
        const char *f;
        int64_t fl;
        const char last = read_past(r, '\t', ',', &f, &fl);
        if (last == '\0') break;
        if (fl >= 1) {
            switch (++loop_pos) {
                case 1:
                    *contig_set = 1;
                    break;
                case 2:
                    pos = 0;
                    for (int64_t i = 0; i < fl; ++i) pos = pos * 10 + (uint64_t)(int64_t)(f[i] - '0');
                    skip_past(r, '\t', 1);
                    loop_pos++;
                    break;
                case 4:
                    rl = fl <= 65535 ? compress_seq(f, fl, ref) : -1;
                    if (rl < 0) bad = 1;
                    break;
                case 5: {
                    const int64_t al = fl <= 65535 ? compress_seq(f, fl, alt) : -1;
                    if (al < 0) bad = 1;
                    if (!bad && keys) keys_push(keys, pos, ref, rl, alt, al);
                    if (last == ',') loop_pos--;
                    break;
                }
                default:
                    break;
            }
        }
    } while (loop_pos <= 4);
    skip_past(r, '\t', 2);
    if (pos_out) *pos_out = pos;
    return bad ? -1 : 0;
}

/* main.cpp:52-109 addCounts */
static int add_counts(rd_t *r, uint64_t *nv, uint64_t *nc) {
    int found_ac = 0, found_an = 0;
    do {
        const char *f;
        int64_t fl;
        const char last = read_past(r, ';', '\t', &f, &fl);
        if (last == '\0') break;
        if (fl >= 4) {
            if (!memcmp(f, "AC=", 3)) {
                found_ac = 1;
                *nv += 1;
                for (int64_t j = 3; j < fl; ++j)
                    if (f[j] == ',') *nv += 1;
            } else if (!memcmp(f, "AN=", 3)) {
                uint64_t v;
                found_an = 1;
                if (atoui64_len(f + 3, (uint8_t)((uint8_t)fl - 3), &v)) return -1;
                *nc += v;
            }
        }
        if (last == '\t' && !(found_ac && found_an)) break;
    } while (!(found_ac && found_an));
    return 0;
}

/* main.cpp:195-245 getRegionStats over S = U[u_start, u_end) */
int orc_region_stats(const char *s, int64_t n, uint64_t *num_variants, uint64_t *num_calls, uint64_t *records) {
    rd_t r = {s, n, 0};
    uint64_t nv = 0, nc = 0, recs = n > 0; /* `records` is diagnostic only (main.cpp:230) */
    int contig_set = 0;
    if (record_header(&r, &contig_set, NULL, NULL)) return -1;
    if (add_counts(&r, &nv, &nc)) return -1;
    const uint64_t skip = 2 * skip_count(&r, '\n');
    while (r.pos < r.n) { /* keepReading() */
        if (record_header(&r, &contig_set, NULL, NULL)) return -1;
        if (add_counts(&r, &nv, &nc)) return -1;
        r.pos += (int64_t)skip; /* seek(skipSize) */
        skip_past(&r, '\n', 1);
        recs++;
    }
    *num_variants = nv;
    *num_calls = nc;
    *records = recs;
    return 0;
}

/* write_data_to_s3.h:150-228 (recordHeader), :93-101 (saveNewFile),
 * :39-92 (saveOutputToS3) over the records getRegionStats visits
 * (main.cpp:217-237): the slice's region files.  rows gets up to cap rows of
 * {first_pos, last_pos, bytes, entries}; data (optional, capacity data_cap)
 * the files' uncompressed bytes {pos u64, len u16, ref' '_' alt'}.  Returns
 * the number of files, -1 where the reference throws, -2 on overflow. */
#define ORC_MAX_SLICE_GAP 100000ULL       /* main.tf:215 */
#define ORC_OUTPUT_SIZE_LIMIT 50000000ULL /* main.tf:17,216 */
int64_t orc_region_files(const char *s, int64_t n, uint64_t *rows, int64_t cap, char *data, int64_t data_cap,
                         int64_t *data_len) {
    rd_t r = {s, n, 0};
    int contig_set = 0;
    int64_t nf = 0, dl = 0;
    uint64_t first = 0, last = 0, bytes = 0, entries = 0;
    uint64_t skip = 0;
    int first_rec = 1;
    while (first_rec || r.pos < r.n) {
        keys_t one = {0};
        uint64_t pos = 0, nv = 0, nc = 0;
        /* recordHeader: the POS check (gap / unsorted) happens before this
         * record's entries are pushed */
        const int bad = record_header(&r, &contig_set, &one, &pos);
        if (bad) {
            keys_free(&one);
            return -1;
        }
        if (entries) {
            if (pos < last) {
                keys_free(&one);
                return -1; /* "unsorted file" */
            }
            if (pos > last + ORC_MAX_SLICE_GAP) {
                if (nf < cap) {
                    rows[4 * nf] = first;
                    rows[4 * nf + 1] = last;
                    rows[4 * nf + 2] = bytes;
                    rows[4 * nf + 3] = entries;
                }
                nf++;
                bytes = entries = 0;
            }
        }
        for (int64_t i = 0; i < one.n; ++i) {
            char d[24];
            const int nd = snprintf(d, sizeof d, "%llu", (unsigned long long)one.pos[i]);
            const int64_t tl = one.len[i] - nd;
            if (!entries) first = one.pos[i];
            last = one.pos[i];
            bytes += 10 + (uint64_t)tl;
            entries++;
            if (data) {
                if (dl + 10 + tl > data_cap) {
                    keys_free(&one);
                    return -2;
                }
                const uint64_t p = one.pos[i];
                const uint16_t l16 = (uint16_t)tl;
                memcpy(data + dl, &p, 8);
                memcpy(data + dl + 8, &l16, 2);
                memcpy(data + dl + 10, one.s[i] + nd, (size_t)tl);
            }
            dl += 10 + tl;
        }
        keys_free(&one);
        if (add_counts(&r, &nv, &nc)) return -1;
        if (entries > ORC_OUTPUT_SIZE_LIMIT) {
            if (nf < cap) {
                rows[4 * nf] = first;
                rows[4 * nf + 1] = last;
                rows[4 * nf + 2] = bytes;
                rows[4 * nf + 3] = entries;
            }
            nf++;
            bytes = entries = 0;
        }
        if (first_rec) {
            skip = 2 * skip_count(&r, '\n');
            first_rec = 0;
        } else {
            r.pos += (int64_t)skip; /* seek(skipSize) */
            skip_past(&r, '\n', 1);
        }
        if (n == 0) break;
    }
    if (entries) {
        if (nf < cap) {
            rows[4 * nf] = first;
            rows[4 * nf + 1] = last;
            rows[4 * nf + 2] = bytes;
            rows[4 * nf + 3] = entries;
        }
        nf++;
    }
    if (data_len) *data_len = dl;
    return nf > cap ? -2 : nf;
}

int64_t orc_slice_region_files(void *h, uint64_t vstart, uint64_t vend, uint64_t *rows, int64_t cap, char *data,
                               int64_t data_cap, int64_t *data_len) {
    bgzf_t *b = (bgzf_t *)h;
    uint64_t u0, u1;
    if (orc_bgzf_voff_to_u(b, vstart, &u0) || orc_bgzf_voff_to_u(b, vend, &u1)) return -3;
    if (u1 <= u0) {
        if (data_len) *data_len = 0;
        return 0;
    }
    return orc_region_files((const char *)b->u + u0, (int64_t)(u1 - u0), rows, cap, data, data_cap, data_len);
}

int orc_summarise_slice(void *h, uint64_t vstart, uint64_t vend, uint64_t *num_variants, uint64_t *num_calls,
                        uint64_t *records) {
    bgzf_t *b = (bgzf_t *)h;
    uint64_t u0, u1;
    if (orc_bgzf_voff_to_u(b, vstart, &u0) || orc_bgzf_voff_to_u(b, vend, &u1)) return -2;
    if (u1 < u0) u1 = u0;
    return orc_region_stats((const char *)b->u + u0, (int64_t)(u1 - u0), num_variants, num_calls, records);
}

/* ------------------------------------------------ duplicateVariantSearch */
static int cmp_key(const void *a, const void *b) {
    const char *const *x = (const char *const *)a, *const *y = (const char *const *)b;
    const int64_t lx = *(const int64_t *)(*x - 8), ly = *(const int64_t *)(*y - 8);
    const int64_t m = lx < ly ? lx : ly;
    const int c = memcmp(*x, *y, (size_t)m);
    if (c) return c;
    return lx < ly ? -1 : lx > ly;
}

/* duplicateVariantSearch.cpp:31-84 + readVcfData.cpp:3-38 (intended range
 * semantics: every entry with range_start <= pos <= range_end) over the
 * region entries summariseSlice would write for the records of `contig` in
 * each VCF text (write_data_to_s3.h:150-228).  Returns -1 when a record in
 * the range makes the reference's summariseSlice throw. */
int orc_dedup_count(const char *const *texts, const int64_t *lens, int nvcf, const char *contig, int64_t clen,
                    uint64_t rs, uint64_t re, uint64_t *unique) {
    keys_t k = {0};
    int rc = 0;
    for (int v = 0; v < nvcf && !rc; ++v) {
        const char *t = texts[v];
        const int64_t n = lens[v];
        int64_t p = 0;
        while (p < n) {
            const char *nl = (const char *)memchr(t + p, '\n', (size_t)(n - p));
            const int64_t e = nl ? (int64_t)(nl - t) + 1 : n;
            if (t[p] != '#' && e - p > clen && !memcmp(t + p, contig, (size_t)clen) && t[p + clen] == '\t') {
                rd_t r = {t + p, e - p, 0};
                int contig_set = 1;
                keys_t one = {0};
                uint64_t pos = 0;
                const int bad = record_header(&r, &contig_set, &one, &pos);
                if (pos >= rs && pos <= re) {
                    if (bad) rc = -1;
                    for (int64_t i = 0; i < one.n && !bad; ++i) keys_move(&k, &one, i);
                }
                keys_free(&one);
            }
            p = e;
        }
    }
    if (!rc) {
        /* sort (length-prefixed copies) and count distinct */
        char **arr = (char **)malloc(sizeof(char *) * (size_t)(k.n ? k.n : 1));
        for (int64_t i = 0; i < k.n; ++i) {
            char *c = (char *)malloc((size_t)k.len[i] + 8);
            memcpy(c, &k.len[i], 8);
            memcpy(c + 8, k.s[i], (size_t)k.len[i]);
            arr[i] = c + 8;
        }
        qsort(arr, (size_t)k.n, sizeof(char *), cmp_key);
        uint64_t u = 0;
        for (int64_t i = 0; i < k.n; ++i)
            if (i == 0 || cmp_key(&arr[i - 1], &arr[i])) u++;
        for (int64_t i = 0; i < k.n; ++i) free(arr[i] - 8);
        free(arr);
        *unique = u;
    }
    keys_free(&k);
    return rc;
}
