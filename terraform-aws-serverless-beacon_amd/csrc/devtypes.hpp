// devtypes.hpp — POD types shared by the host orchestration (api.cpp) and the
// HIP kernels (query_kernels.hip).  Layout of the HBM-resident variant store
// and of one resolved slice query.
//
// Store = struct of arrays, records position-sorted inside each
// (vcf, contig) segment (the unit `bcftools query --regions` walks,
// lambda/performQuery/search_variants.py:42-50).  Per-record columns are read
// by the range scan; per-alt columns hang off alt_lo[] (multiallelic records
// own alt_lo[r+1]-alt_lo[r] rows).
#pragma once
#include <cstdint>

namespace sb {

// ---- record meta bits (DStore::meta) -------------------------------------
enum : uint32_t {
    M_HAS_AC = 1u << 0,   // INFO has an AC= tag (search_variants.py:196)
    M_HAS_AN = 1u << 1,   // INFO has an AN= tag (:198)
    M_AC_BAD = 1u << 2,   // last AC= has a non-int entry -> ValueError (:206)
    M_AN_BAD = 1u << 3,   // some AN= is not an int -> ValueError (:199)
    M_HAS_FB = 1u << 4,   // record has a genotype fallback row (no AC or no AN)
    M_REF_HASHED = 1u << 5,
    M_VT_SHIFT = 16,      // VT dictionary id in bits 16..31 (0 = 'N/A')
};

// ---- alt class bits (DStore::alt_cls) ------------------------------------
enum : uint32_t {
    A_SINGLE_BASE = 1u << 0, // alt.upper() in {A,C,G,T,N} (:173)
    A_SYMBOLIC = 1u << 1,    // alt.startswith('<')
    A_DOT = 1u << 2,         // alt == '.'
    A_AC_MISSING = 1u << 3,  // fewer AC entries than alts -> IndexError (:207)
    A_HASHED = 1u << 4,      // alt_key is a hash (len > 8 or non-ASCII)
    A_REP_SHIFT = 8,         // k with alt == REF*k (raw, k >= 0), 63 = none
    A_REP_NONE = 63,
    A_SYM_SHIFT = 16,        // symbolic dictionary id (bits 16..31)
};

// ---- query modes -----------------------------------------------------------
enum : uint32_t {
    REF_ANY = 0,      // reference_bases == 'N' (:59)
    REF_EXACT = 1,    // REF.upper() == reference_bases
    REF_WILD = 2,     // samples variant regex with N -> [ACGTN] (svs:88-91)
    REF_NEVER = 3,    // None in search_variants (never equal)
    REF_ERROR = 4,    // raise ref_err at the first record passing the end filter
};
enum : uint32_t { ALT_N = 0, ALT_EXACT = 1, ALT_VTYPE = 2 };
enum : uint32_t { VT_DEL = 0, VT_INS = 1, VT_DUP = 2, VT_DUPT = 3, VT_CNV = 4, VT_OTHER = 5 };
enum : uint32_t {
    F_DETAILS = 1u << 0,        // include_details
    F_BOOL_BREAK = 1u << 1,     // granularity boolean in search_variants (:253)
    F_COLLECT = 1u << 2,        // collect sample indices (:235 / svs:231)
    F_SAMPLES_VARIANT = 1u << 3,// search_variants_in_samples
    F_STRICT_UNBOUND = 1u << 4, // alt None, reproduce UnboundLocalError (:101)
    F_EMPTY = 1u << 5,          // bcftools emits nothing (unknown contig/sample)
};

struct DStore {
    // per record
    const uint32_t *pos;
    const uint32_t *end;      // POS + len(REF) - 1 (:90)
    const uint64_t *ref_key;  // key(REF.upper())
    const uint32_t *meta;
    const int32_t *an;        // INFO AN, or #called alleles over all samples
    const uint32_t *alt_lo;   // [n_records + 1]
    const uint64_t *ref_off;  // into blob (raw REF bytes)
    const int64_t *fb_off;    // genotype fallback row (u32 words) or -1
    // per alt row
    const uint64_t *alt_key;  // key(ALT.upper())
    const uint32_t *alt_len;
    const uint32_t *alt_cls;
    const int32_t *ac;        // INFO AC entry, or GT count of this allele (no AC)
    const uint64_t *alt_off;  // into blob (raw ALT bytes)
    // bulk
    const uint8_t *blob;
    const uint64_t *planes;   // carrier bitplanes, [alt row][W words] per vcf
    const uint32_t *fb;       // fallback rows: per sample [n:8][v0:8][v1:8][v2:8]
    const uint32_t *sym_lut;  // per query-distinct variantType: bitset over sym ids
};

struct QDev {
    uint32_t seg_lo, seg_hi;  // record range of the (vcf, contig) segment
    int64_t first_bp, last_bp;
    int64_t end_min, end_max;
    uint64_t ref_key;
    uint64_t alt_key;
    int64_t vmin, vmax;       // vmax = INT64_MAX when < 0 (:67)
    uint64_t plane_base;      // word offset of this vcf's first plane row
    uint32_t alt_base;        // first alt row of this vcf
    uint32_t words;           // W = ceil(n_samples / 64)
    uint32_t ref_len, alt_len;
    uint32_t ref_mode, alt_mode;
    uint32_t ref_err;         // SB_QERR_* for REF_ERROR
    uint32_t vt_kind;
    uint32_t lut_off;         // u32 word offset into sym_lut
    uint32_t flags;
    uint32_t qbytes_off;      // query REF bytes then ALT bytes
    uint32_t n_samples;
    uint64_t subset_off;      // word offset of subset mask (samples variant), ~0 = none
    uint64_t samples_out_off; // word offset of the per-query sample bitset, ~0 = none
};

struct QRes {
    int32_t error;
    int32_t exists;
    int64_t call_count;
    int64_t all_alleles_count;
    uint32_t n_hits;
    uint32_t n_scanned;
};

}  // namespace sb
