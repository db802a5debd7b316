// devtypes.hpp — POD types shared by the host orchestration (api.cpp) and the
// HIP kernels (query_kernels.hip): layout of the HBM-resident variant store
// and of one resolved slice query.
//
// Store = records position-sorted inside each (vcf, contig) *segment* (the
// unit `bcftools query --regions` walks, lambda/performQuery/
// search_variants.py:42-50).  The range scan reads ONE 16-byte word per
// record (RecHot: one global_load_dwordx4 per lane, 1 KiB per wave
// instruction); the first ALT of every record lives in that word and in
// record-indexed columns, so biallelic records (98.5 % of a 1000G VCF) need
// no dependent load.  ALTs 2..n live in "extra" rows reached through x_lo[].
#pragma once
#include <climits>
#include <cstdint>

namespace sb {

// ---- RecHot::hot bits; bits 6..31 are also the layout of x_cls ------------
enum : uint32_t {
    H_HAS_AC = 1u << 0,   // INFO has an AC= tag (search_variants.py:196)
    H_HAS_AN = 1u << 1,   // INFO has an AN= tag (:198)
    H_AC_BAD = 1u << 2,   // last AC= has a non-int entry -> ValueError (:206)
    H_AN_BAD = 1u << 3,   // some AN= is not an int -> ValueError (:199)
    H_HAS_FB = 1u << 4,   // record has a genotype fallback row (no AC or no AN)
    H_MULTI = 1u << 5,    // more than one ALT (extra rows in x_*)
    // per-ALT class (alt 0 in hot, alt k>0 in x_cls)
    C_SINGLE_BASE = 1u << 6,  // alt.upper() in {A,C,G,T,N} (:173)
    C_AC_MISSING = 1u << 7,   // fewer AC entries than alts -> IndexError (:207)
    C_SYMBOLIC = 1u << 8,     // alt.startswith('<')
    C_DOT = 1u << 9,          // alt == '.'
    C_REP_SHIFT = 10,         // k with alt == REF*k (raw bytes, k >= 0); 63 = none
    C_REP_NONE = 63,
    C_SYM_SHIFT = 16,         // symbolic-ALT dictionary id
};

// RecHot::an of a *general record* (H_AN_BAD is set too; RecHot::ac0 = its
// GenRec index): one the packed words cannot hold -- more than 64 ALTs, an
// AC / AN integer outside int32 (Python ints are unbounded below CPython's
// 4300-digit int() limit), a GT fallback with ploidy > 3 or allele numbers >=
// 255, or a GT fallback over >= 8 ALTs (the variant order is then CPython's
// set iteration order, search_variants.py:223).  Every scan kernel stops at a
// general record it reaches and hands the slice (SB_QERR_GENERAL, internal)
// to general_slice_kernel, which answers it from the GenRec side table.
constexpr int32_t kAnUnrepresentable = INT32_MIN;
constexpr int32_t SB_QERR_GENERAL = 10;  // internal: never leaves the library

enum : uint32_t {
    GR_HAS_AC = 1u << 0,    // INFO has an AC= tag
    GR_HAS_AN = 1u << 1,    // INFO has an AN= tag
    GR_AC_BAD = 1u << 2,    // an entry of the last AC= fails int() -> ValueError (:206)
    GR_AN_BAD = 1u << 3,    // an AN= fails int() -> ValueError (:199)
    GR_FB = 1u << 4,        // no AC or no AN, and samples: GT digit runs kept (tok / val)
};
struct alignas(16) GenRec {
    uint32_t rec;       // global record index
    uint32_t flags;     // GR_*
    uint32_t n_alt;     // len(ALT.split(','))
    uint32_t n_ac;      // entries of the last AC= (GR_HAS_AC, not GR_AC_BAD)
    uint64_t ac_num;    // first of its n_ac numbers (GStore::num)
    uint64_t an_num;    // its AN (GR_HAS_AN, not GR_AN_BAD)
    uint64_t tok_off;   // GR_FB: n_samples + 1 offsets into GStore::tok (per header sample)
    uint32_t n_vals;    // GR_FB: distinct digit-run values, numbered in first-occurrence order
    uint32_t val_off;   //   (over all samples) from GStore::val + val_off
    uint32_t a0_cls;    // C_* class bits of ALT 0 (+ symbolic id); ALTs >= 1 are extra rows
    uint32_t pad[3];
};
static_assert(sizeof(GenRec) == 64, "GenRec is four 16-byte words");
// one distinct GT digit-run value of a GR_FB record (int(run), :218)
struct alignas(16) GenVal {
    uint64_t hash;    // CPython hash(int): value mod 2**61 - 1
    uint32_t allele;  // the value when it is an allele number 1 .. n_alt, else 0
    uint32_t huge;    // run longer than 4300 digits: int() raises ValueError
};
struct GStore {
    const GenRec *rec;
    const uint32_t *num;      // numbers as `limbs` u32 limbs each, two's complement, little-endian
    const uint64_t *tok_off;  // per GR_FB record: n_samples + 1 offsets into tok
    const uint32_t *tok;      // digit-run value ids, sample by sample, in GT text order
    const GenVal *val;
    uint32_t n, limbs;        // records; limbs per number
    uint32_t acc_limbs;       // limbs of a running sum (limbs + 2, <= kGenAccMax)
    uint32_t max_alt, max_vals;  // over the records (scratch sizing)
};
constexpr uint32_t kGenAccGroups = 8;                 // 64-limb groups a sum may span
constexpr uint32_t kGenAccMax = 64 * kGenAccGroups;   // 16384 bits > a 4300-digit value + headroom
// a general slice whose call_count or all_alleles_count needs more than 64 bits
struct GenBig {
    uint32_t orig;  // QRes row
    uint32_t pad;
};

struct alignas(16) RecHot {
    uint32_t end;  // POS + len(REF) - 1 (:90)
    uint32_t hot;  // H_* flags + class of ALT 0
    int32_t an;    // INFO AN, or #called alleles over all samples (:244-250)
    int32_t ac0;   // INFO AC entry of ALT 0, or its GT count when AC is absent
};

// What a referenceBases='N' / alternateBases='N' query (MODE_RANGE_N) needs of
// a record, precomputed at ingest because none of it depends on the query
// (search_variants.py:170-176 with len(alt) = 1 for a single base, :205-214):
//   info bits 0..7 = ALTs emitted as variants (single base and AC != 0),
//   RH_HIT = some ALT is a single base, RH_SLOW = the record needs the general
//   evaluation (no AC tag, int() failures, AC entries missing, > 8 ALTs,
//   |sum| beyond int32);  c = sum of AC over the single-base ALTs.
struct alignas(16) RangeHot {
    uint32_t end;
    uint32_t info;
    int32_t an;
    int32_t c;
};
enum : uint32_t { RH_EMIT_MASK = 0xffu, RH_HIT = 1u << 8, RH_SLOW = 1u << 9 };
// The same in 8 bytes for a VCF whose records (almost) all carry one AN (the
// 1000 Genomes shape: AN = 2 x samples at every site): w = info bits 0..9 as
// above | c << RH8_C_SHIFT (21 bits), AN = the VCF's common value
// (QDev::an_default).  A record whose AN differs, or whose c is negative or
// >= 2^21, is RH_SLOW here.  Halves the bytes a range scan streams.
struct alignas(8) RangeHot8 {
    uint32_t end;
    uint32_t w;
};
enum : uint32_t { RH8_C_SHIFT = 11, RH8_C_MAX = (1u << 21) - 1 };

enum : uint32_t { VT_DEL = 0, VT_INS = 1, VT_DUP = 2, VT_DUPT = 3, VT_CNV = 4, VT_OTHER = 5 };
// What a referenceBases='N' / alternateBases=None variantType query
// (MODE_VTYPE) reads of a record: END and everything the predicate of
// search_variants.py:100-183 needs about the first ALT, plus AC0 and AN, in
// 16 bytes (one global_load_dwordx4 per lane): a biallelic hit needs no other
// load, which matters because vmcnt retires in order, so a dependent load in
// a chunk would drain the whole stream window behind it.  Only multiallelic
// lanes read their extra rows.  The non-symbolic predicates depend on an ALT
// only through (len(ALT) vs len(REF), the REF*k class, ALT == '.'), so that
// triple is stored as a 5-bit class index and each variantType becomes a
// 24-bit mask over it (vt_class_mask): the per-ALT test is one shift.
// ALTs 2..n of a multiallelic record (at most 7) have the same 32-bit word in
// DStore::xvt; the record's own word says, per variantType, whether any of
// them could match (VT_XK_*, length bounds aside), so a lane reads its extra
// rows only then (a typical multiallelic SNV never does).  Built at upload.  Records the packing cannot represent (AC-less,
// int() failures, a missing AC entry, more than 8 ALTs, lengths or symbolic
// ids >= 255) carry VT_SLOW and take eval_record.
struct alignas(16) VtHot {
    uint32_t end;
    uint32_t w;  // len(ALT0):8 | class:5 << 8 | VT_SYM | sym id:8 << 16 | VT_SLOW | n extra ALTs:3 << 29
    int32_t ac0;
    int32_t an;
};
enum : uint32_t {
    VT_CLASS_SHIFT = 8,  // class = cmp * 8 + rep * 2 + dot; cmp 0/1/2: len(ALT) <, ==, > len(REF);
                         // rep 0: ALT is not REF*k, 1: k in {0, 1}, 2: k == 2, 3: k > 2
    VT_SYM = 1u << 13,   // symbolic ALT (sym id in bits 16..23)
    // some extra ALT is of a class DEL / INS / DUP / DUP:TANDEM / CNV accepts, or symbolic
    VT_XK_DEL = 1u << 14,
    VT_XK_INS = 1u << 15,
    VT_XK_DUP = 1u << 24,
    VT_XK_DUPT = 1u << 25,
    VT_XK_CNV = 1u << 26,
    VT_XK_SYM = 1u << 27,
    VT_SLOW = 1u << 28,
    VT_NX_SHIFT = 29,
    VT_MAX_NX = 7,
};
// Candidate index of MODE_VTYPE (built at upload): for each variantType kind
// k in 0..5 (VT_DEL .. VT_OTHER) the records that could satisfy it for some
// length bounds / END window -- ALT0 of an accepted class, a symbolic ALT0,
// an extra ALT that might (VT_XK_*), or VT_SLOW -- in record order, with
// their VtHot words copied alongside (vc_word / vc_idx, kind k at
// vc_off[k]).  Every other record can neither hit nor raise for that kind,
// so a slice scans only its candidates: [lo, hi) maps to candidate positions
// through a per-64-record block table (prefix count + bitmask).  In a
// 1000G-shape store a kind has a few % of the records as candidates.
constexpr int kVtKinds = 6;
struct alignas(16) VcBlock {
    uint64_t mask;  // bit i: record 64 b + i is a candidate
    uint32_t pre;   // candidates of this kind before record 64 b (+ vc_off[k])
    uint32_t pad;
};
// Slice chains (MODE_VTYPE): splitQuery cuts one request into consecutive
// 10 kb slices that share every filter (lambda/splitQuery/lambda_function.py:
// 82-106).  When none of them needs the order-dependent machinery
// (include_details, no boolean break, non-negative AC, no VT_SLOW record in
// the window) a chain of up to kChainMax such slices is answered by ONE wave:
// the chain's candidate range comes from a per-(kind, segment) coarse index
// over candidate POS (vc_bucket: entry b = first candidate of the pair with
// POS >= base + (b << shift)), each candidate lane filters POS against the
// chain window and finds its slice as (POS - first) / width, and per-slice
// sums are kept in LDS.  Per-slice QRes rows are exactly what vt_slice
// writes for each slice alone; the chain's hits are written densely in slice
// order from `out` (slice j's hits start after slices 0..j-1's n_hits).  The
// descriptor carries the chain's filters already reduced to the compare
// constants vt_slice derives from its QDev (VtPred), so a wave reads nothing
// else before the index.
constexpr uint32_t kChainMax = 32;
// coarse POS index of the variantType candidates of one (segment, kind):
// vc_bucket[off + b] = first candidate with POS >= base + (b << shift), b <= n
// (host planning, and DStore::vcx for request planning on the device)
// The request path's copy of a candidate (request_eval_kernel reads one
// 16-byte word per candidate): POS, END, the VtHot word and ALT0's AC.  The
// record index (vc_idx) is read only for staged hits (request_deliver_kernel)
// and extra-ALT lookups, AN (vc_word) only by runs without a common AN.
struct alignas(16) VcQ {
    uint32_t pos, end, w;
    int32_t ac0;
};
// a staged request hit: candidate index | ALT label << kStageAltShift (labels <= VT_MAX_NX)
constexpr uint32_t kStageAltShift = 29;
constexpr uint32_t kStageCandMask = (1u << kStageAltShift) - 1u;
struct VcIndex {
    uint64_t off = 0;
    uint32_t base = 0, shift = 31, n = 1;
    uint32_t c_lo = 0, c_hi = 0;  // the pair's candidates in the kind's list
    // what request_eval_kernel may assume of the pair's candidates (VT_SLOW
    // ones aside: a chain that reaches one is answered per slice):
    // kVcNarrow = every record's AN and sum of |AC| over its ALTs in [0, 2^25)
    // (a chunk's sums fit 32 bits); below it AN + 1 when they all share one
    // AN (then a chain's AN sum is its hit records times that AN), else 0
    uint32_t xinfo = 0;
};
static_assert(sizeof(VcIndex) == 32, "VcIndex is two 16-byte words");
constexpr uint32_t kVcNarrow = 1u << 31;
constexpr uint32_t kVcAnMask = (1u << 26) - 1u;
// first candidate of the pair with POS >= x (up = 0), or the end of the
// bucket holding x - 1 (up = 1: a bound >= the exact upper bound of x - 1)
__host__ __device__ inline uint32_t vc_bound(const VcIndex &vi, const uint32_t *bucket, uint64_t x, uint32_t up) {
    if (x <= vi.base) return vi.c_lo;
    const uint64_t b = (x - vi.base) >> vi.shift;
    return b >= vi.n ? vi.c_hi : bucket[vi.off + b + up];
}
struct alignas(16) ChainDev {
    uint32_t s0;        // first slice in the chain-ordered arrays (chain_orig)
    uint32_t n;         // slices, 1 .. kChainMax
    uint32_t first;     // first_bp of slice 0
    uint32_t last;      // last_bp of slice n - 1
    uint32_t width;     // slices 0 .. n-2 span exactly `width` bp; the last at most that
    uint32_t c_lo, c_hi;  // the (kind, segment) pair's candidates; request chains: the chain's own range (host-resolved)
    uint32_t cb_base;   // coarse candidate index of the pair (vc_bucket)
    uint64_t cb_off;
    uint32_t cb_shift, cb_n;
    uint32_t e0, espan;   // END in [e0, e0 + espan]
    uint32_t vlo, vspan;  // len(ALT) in [vlo, vlo + vspan] (vlo = 256: empty)
    uint32_t kind;        // vt_kind | kChainEndVoid
    uint32_t lut_off;     // symbolic-ALT LUT of the chain's variantType
    uint64_t out;         // first hit slot of the chain
};
static_assert(sizeof(ChainDev) == 80, "ChainDev is five 16-byte words");
constexpr uint32_t kChainEndVoid = 1u << 8;  // no END can match

// Request batches (sb_requests_prepare / sb_requests_run): every request is a
// row; request_eval_kernel answers one run of consecutive rows per wave --
// the rows' chains (ReqChain, below) evaluated as
// chain_pack_kernel does, their hits appended to the run's staging region --
// and request_deliver_kernel writes the rows' offsets and hits densely in row
// order at the run's offset, from the runs' totals and a scan over tiles of
// runs (the other rows' hits, from per-slice queries answered before,
// gathered there too).
constexpr uint32_t kRunRows = 64;     // rows per run at most (one lane each)
constexpr uint32_t kRunSimple = 1u;   // RowRun::flags: no row of the run is answered per slice
constexpr uint32_t kRunNarrow = 2u;   // every chain's (segment, kind) pair is kVcNarrow
constexpr uint32_t kRunAnCommon = 4u; // ... and they share one AN: flags >> kRunAnShift
constexpr uint32_t kRunAnShift = 6u;
struct alignas(16) RowRun {
    uint32_t row_lo, row_hi;  // rows [row_lo, row_hi)
    uint32_t c_lo, c_hi;      // the run's chains, rows increasing
    uint64_t stage;           // first staging slot of the run (its chains' hit capacity follows)
    uint32_t n_slots;         // slices of its chains
    uint32_t flags;           // kRunSimple | kRunNarrow | kRunAnCommon | common AN << kRunAnShift
};
static_assert(sizeof(RowRun) == 32, "RowRun is two 16-byte words");

// A request's chain as request_eval_kernel reads it (kReqRun slots per run:
// the chains with candidates first, in row order, then those without, then
// first == 0 = an empty slot): splitQuery's slices are [first + j * kReqWidth,
// ...] up to `last`, so width and slice count follow from the window; the
// row, kind and length bounds share one word.  32 B, not ChainDev's 80.
constexpr uint32_t kReqWidth = 10000;  // lambda/splitQuery/lambda_function.py:12
constexpr uint32_t kReqRun = 64;       // ReqChain slots per run (one lane of request_eval_kernel each)
// chain starts below position 64 * kReqStartChunks of a run's candidates
// (laid end to end) are found through the wave's chain-start bitmap, later
// ones by ballot (runs are cut there when they can be)
constexpr uint32_t kReqStartChunks = 64;
// slices of one request chain at most (slice keys of request_eval_kernel are
// chain << 20 | slice)
constexpr uint32_t kReqChainSlices = (1u << 20) - 1;
// LUT offsets a chain can carry (request_eval_kernel packs the offset into
// 15 bits): a request whose variantType string's LUT lies past it is
// answered per slice (only batches with > 4 k distinct variantType strings)
constexpr uint32_t kReqLutMax = 1u << 15;
struct alignas(16) ReqChain {
    uint32_t first, last;  // the request's [start_min, start_max] (first >= 1)
    uint32_t c_lo, c_hi;   // candidate range (host-resolved from the coarse index)
    uint32_t e0, espan;    // END in [e0, e0 + espan]
    uint32_t bits;         // vlo : 9 | vspan : 8 | row - run.row_lo : 6 | vt kind : 3 | end void : 1
    uint32_t lut_off;      // symbolic-ALT LUT of the request's variantType
};
static_assert(sizeof(ReqChain) == 32, "ReqChain is two 16-byte words");
__host__ __device__ constexpr uint32_t req_bits(uint32_t vlo, uint32_t vspan, uint32_t row, uint32_t kind, bool end_void) {
    return vlo | vspan << 9 | row << 17 | kind << 23 | (end_void ? 1u << 26 : 0u);
}

// One request as the host packs it for planning on the device
// (sb_requests_prepare_columns when every varying column is numeric): the
// ReqChain fields that do not depend on the store, its store-wide segment
// and its class.  request_plan_kernel turns a run of 64 of them into the
// run's ReqChain slots and RowRun.
enum : uint32_t { REQ_CHAIN = 0, REQ_NONE = 1, REQ_SLICES = 2 };
struct alignas(16) ReqIn {
    uint32_t first, last;  // start_min, start_max (REQ_CHAIN: 1 <= first <= last <= 0xfffffffe)
    uint32_t e0, espan;    // END in [e0, e0 + espan]
    uint32_t bits;         // req_bits(vlo, vspan, 0, kind, end_void)
    uint32_t seg;          // store-wide segment (DStore::vcx row)
    uint32_t lut_off;      // symbolic-ALT LUT of the variantType
    uint32_t cls;          // REQ_* | slices << 2
};
static_assert(sizeof(ReqIn) == 32, "ReqIn is two 16-byte words");

// bit c set = an ALT of class c satisfies variantType `kind` (vtype_hit)
__host__ __device__ constexpr uint32_t vt_class_mask(uint32_t kind) {
    uint32_t m = 0;
    for (uint32_t c = 0; c < 24; ++c) {
        const uint32_t cmp = c >> 3, rep = (c >> 1) & 3u, dot = c & 1u;
        if (kind == VT_DEL ? cmp == 0 : kind == VT_INS ? cmp == 2 : kind == VT_DUP ? rep >= 2
            : kind == VT_DUPT ? rep == 2 : kind == VT_CNV ? (dot != 0 || rep != 0) : false)
            m |= 1u << c;
    }
    return m;
}
__host__ __device__ constexpr uint32_t vt_xk_bit(uint32_t kind) {
    return kind == VT_DEL ? VT_XK_DEL : kind == VT_INS ? VT_XK_INS : kind == VT_DUP ? VT_XK_DUP
         : kind == VT_DUPT ? VT_XK_DUPT : kind == VT_CNV ? VT_XK_CNV : 0u;
}
// the VT_XK_* bits one extra-ALT word contributes to its record's word
inline uint32_t vt_xk_bits(uint32_t xw) {
    if (xw & VT_SYM) return VT_XK_SYM;
    const uint32_t c = (xw >> VT_CLASS_SHIFT) & 31u;
    uint32_t b = 0;
    for (uint32_t k = VT_DEL; k <= VT_CNV; ++k)
        if ((vt_class_mask(k) >> c) & 1u) b |= vt_xk_bit(k);
    return b;
}
// the 32-bit word of one ALT with class bits `cls` (C_*); false = not representable
inline bool vt_alt_word(uint32_t cls, uint64_t ref_len, uint64_t alt_len, uint32_t *w) {
    const uint32_t sym = cls >> C_SYM_SHIFT;
    const uint32_t rep = (cls >> C_REP_SHIFT) & 63u;
    if ((cls & C_AC_MISSING) || ref_len >= 255 || alt_len >= 255 || ((cls & C_SYMBOLIC) && sym >= 255)) return false;
    const uint32_t rc = rep == C_REP_NONE ? 0u : rep < 2 ? 1u : rep == 2 ? 2u : 3u;
    const uint32_t cmp = alt_len < ref_len ? 0u : alt_len == ref_len ? 1u : 2u;
    const uint32_t c = cmp * 8 + rc * 2 + ((cls & C_DOT) ? 1u : 0u);
    *w = static_cast<uint32_t>(alt_len) | (c << VT_CLASS_SHIFT);
    if (cls & C_SYMBOLIC) *w |= VT_SYM | (sym << 16);
    return true;
}

// ---- query modes -----------------------------------------------------------
enum : uint32_t {
    REF_ANY = 0,    // reference_bases == 'N' (:59)
    REF_EXACT = 1,  // REF.upper() == reference_bases
    REF_WILD = 2,   // samples variant regex with N -> [ACGTN] (svs:88-91)
    REF_NEVER = 3,  // None in search_variants (never equal)
    REF_ERROR = 4,  // raise ref_err at the first record passing the end filter
};
enum : uint32_t { ALT_N = 0, ALT_EXACT = 1, ALT_VTYPE = 2 };
// scan-kernel specialisations (query classes launched separately)
enum : int { MODE_GENERAL = 0, MODE_RANGE_N = 1, MODE_EXACT = 2, MODE_VTYPE = 3, MODE_RANGE_N8 = 4 };
enum : uint32_t {
    F_DETAILS = 1u << 0,         // include_details
    F_BOOL_BREAK = 1u << 1,      // granularity boolean in search_variants (:253)
    F_COLLECT = 1u << 2,         // collect sample indices (:235 / svs:231)
    F_SAMPLES_VARIANT = 1u << 3, // search_variants_in_samples
    F_STRICT_UNBOUND = 1u << 4,  // alt None, reproduce UnboundLocalError (:101)
    F_EMPTY = 1u << 5,           // bcftools emits nothing (unknown contig/sample)
    F_NONNEG = 1u << 6,          // every AC/GT count in the store is >= 0
};

struct alignas(8) XRow {
    uint32_t cls;  // C_* class bits + symbolic id (layout of RecHot::hot bits 6..31)
    int32_t ac;    // INFO AC entry, or its GT count when AC is absent
};

struct QDev;

struct DStore {
    // record-indexed
    const RecHot *rec;
    const RangeHot *rng;      // MODE_RANGE_N view of the same records
    const RangeHot8 *rng8;    // MODE_RANGE_N8 view (VCFs with a common AN)
    const VtHot *vth;         // MODE_VTYPE view of the same records
    const uint32_t *xvt;      // MODE_VTYPE word of each extra row
    const VtHot *vc_word;     // MODE_VTYPE candidates (see VcBlock)
    const uint32_t *vc_idx;
    const VcBlock *vc_blk;    // [kVtKinds][vc_nblk]
    uint64_t vc_nblk;
    const uint32_t *vc_pos;   // POS of each candidate (parallel to vc_word)
    const VcQ *vc_q;          // request_eval_kernel's copy of each candidate (parallel to vc_word)
    const uint32_t *vc_bucket;  // coarse POS index per (kind, segment) over candidates (ChainDev)
    const VcIndex *vcx;         // [segment (store-wide) * kVtKinds + kind]: the pair's coarse index
    const uint64_t *vc_altpre;  // ALTs of candidates [0, j) (a chain's hit capacity)
    const uint32_t *pos;
    const uint64_t *ref_key;  // key(REF.upper())
    const uint64_t *a0_key;   // key(ALT0.upper())
    const uint32_t *a0_len;
    const uint32_t *x_lo;     // [n_records + 1] first extra row of each record
    const uint64_t *ref_off;  // blob offsets (confirmation of hashed keys)
    const uint64_t *a0_off;
    const int64_t *fb_off;    // genotype fallback row (u32 words) or -1
    // extra-ALT rows (ALT index >= 1)
    const XRow *xrow;  // (class, AC) of each extra row: one 8-byte load
    const uint64_t *x_key;
    const uint32_t *x_len;
    const uint64_t *x_off;
    // bulk
    const uint8_t *blob;
    const uint64_t *planes;   // carrier bitplanes [alt row][words]
    const uint32_t *fb;       // fallback rows: per sample [n:8][v0:8][v1:8][v2:8]
    const uint32_t *bucket;   // coarse POS index of every segment
    const uint32_t *sym_lut;  // per query-distinct variantType: bitset over sym ids
    // per run: the batch's launch-ordered queries and the general-slice work
    // list ([0] = count, then launch indices); nullptr = the store has no
    // general record
    const QDev *q_all;
    uint32_t *gen_work;
};

struct QDev {
    uint32_t seg_lo, seg_hi;   // record range of the (vcf, contig) segment
    uint64_t bucket_off;       // this segment's coarse index: bucket[b] = first
    uint32_t bucket_base;      //   record with POS >= base + (b << shift), b <= nb
    uint32_t bucket_shift;
    uint32_t n_buckets;
    uint32_t flags;
    int64_t first_bp, last_bp;
    int64_t end_min, end_max;
    uint64_t ref_key;
    uint64_t alt_key;
    int64_t vmin, vmax;        // vmax = INT64_MAX when < 0 (:67)
    uint64_t plane0_base;      // word offset of this vcf's ALT-0 planes (row = r - rec_base)
    uint64_t planex_base;      // word offset of this vcf's extra-ALT planes (row = x - x_base)
    uint32_t rec_base, x_base;
    uint32_t words;            // ceil(n_samples / 64)
    uint32_t n_samples;
    uint32_t ref_len, alt_len;
    uint32_t ref_mode, alt_mode;
    uint32_t ref_err;          // SB_QERR_* for REF_ERROR
    uint32_t vt_kind;
    uint32_t lut_off;          // u32 word offset into sym_lut
    uint32_t qbytes_off;       // query REF bytes then ALT bytes
    uint64_t subset_off;       // word offset of subset mask (samples variant), ~0 = none
    uint64_t samples_out_off;  // word offset of the per-query sample bitset, ~0 = none
    uint64_t hit_off;          // this query's output region (host-planned upper bound)
    int64_t an_default;        // the VCF's common AN (MODE_RANGE_N8)
    uint32_t orig;             // the query's index in the batch (its QRes row); the device
    uint32_t pad_;             //   array is in launch order, so waves index it directly
};

struct QRes {
    int32_t error;
    int32_t exists;
    int64_t call_count;
    int64_t all_alleles_count;
    uint32_t n_hits;
    uint32_t n_scanned;
};

// one request row of sb_batch_reduce_requests (include/sbeacon.h
// sb_request_partial, same layout)
struct ReqPartial {
    int64_t exists;  // slices with exists = True
    int64_t n_variants;
    int64_t call_count;
    int64_t all_alleles_count;
    int64_t errors;  // slices whose performQuery raised
};

// A request row in the compact output (sb_requests_set_compact; the layout
// of sb_request_row32): the ReqPartial sums as u32, no error count
struct RowC {
    uint32_t exists, n_variants, call_count, all_alleles_count;
};
static_assert(sizeof(RowC) == 16, "RowC is one 16-byte word");

// Escapes of the compact outputs: a row the compact form cannot hold (a sum
// past 32 bits, a raising or inexact slice) is written as
// {kRowEscaped, n_variants, kRowEscaped, kRowEscaped} and its wide sums go to
// xrows[row]; a u32 hit whose ALT label does not fit 3 bits, or is 7, carries
// the label kHitLabelEscape and its ALT index goes to xlab[its output
// position].  request_eval_kernel / request_deliver_kernel set the batch's
// error word bits kErrRowEscapes / kErrHitEscapes when they wrote any.
struct ReqEsc {
    ReqPartial *xrows;        // n_rows (COMPACT_ALL batches)
    const uint8_t *row_flag;  // inexact rows of the per-slice part (or null)
    uint16_t *xlab;           // one label per output hit position (compact hits)
};
inline constexpr uint32_t kRowEscaped = 0xffffffffu;
inline constexpr uint32_t kHitLabelEscape = 7u;
inline constexpr uint32_t kErrRowEscapes = 8u, kErrHitEscapes = 16u;

// hit = record | (alt index << 32); alt index is the label index (the GT
// fallback labels with alts[i] for a 1-based i, search_variants.py:223)
inline constexpr uint64_t kHitAltShift = 32;

// ---- summariseSlice (lambda/summariseSlice/source/main.cpp:52-109,195-245)
// What one record contributes when the reference's VcfChunkReader visits it,
// precomputed at ingest from the record's own line:
//   rem = bytes from the cursor addCounts leaves (after the delimiter that
//         ended the AC/AN scan) to the end of the line incl. '\n'; the skip
//         heuristic (seek(skipSize) + skipPast('\n'), main.cpp:234-235) swallows
//         the next record iff skipSize >= rem;
//   nvf = numVariants contribution (1 + commas per AC= field seen) | bit 31 =
//         record the restatement cannot represent (its reads would leave the
//         line: INFO ending in '\n' before AC and AN were both seen, empty
//         CHROM/REF/ALT fields, AN= values longer than atoui64 handles);
//   nc  = numCalls contribution (atoui64 of each AN= field seen).
struct alignas(16) SumHot {
    uint32_t rem;
    uint32_t nvf;
    uint64_t nc;
};
inline constexpr uint32_t kSumUnsupported = 1u << 31;

// The same contribution packed into one 8-byte word for the phase-A stream:
// rem bits 0..23, numVariants bits 24..31, numCalls bits 32..62; bit 63 =
// escape (a field does not fit, or the record is unsupported): read SumHot.
inline constexpr uint64_t kSumEscape = 1ull << 63;
inline uint64_t pack_sum(const SumHot &h) {
    const uint64_t nv = h.nvf & ~kSumUnsupported;
    if ((h.nvf & kSumUnsupported) || h.rem >= (1u << 24) || nv >= 256 || h.nc >= (1ull << 31)) return kSumEscape;
    return static_cast<uint64_t>(h.rem) | (nv << 24) | (h.nc << 32);
}

inline constexpr uint32_t kSumChunk = 4096;  // records per phase-A workgroup

struct SDev {  // one summariseSlice invocation after host planning
    uint32_t lo, hi;        // records whose line starts in [U(vstart), U(vend))
    uint64_t bitmap_off;    // u64-word offset of this slice's overshoot bitmap
    uint32_t chunk_lo;      // first phase-A chunk of this slice
    uint32_t n_chunks;      // ceil((hi - lo) / kSumChunk)
};

struct SPart {  // phase-A partial of one chunk
    uint64_t nv, nc;
    uint32_t bad, overshoot_words;
};

struct SRes {
    int32_t error;
    int32_t pad;
    uint64_t num_variants;
    uint64_t num_calls;
    uint64_t records;  // records visited (the reference's `records` log count)
};

struct SStore {  // summary columns
    const uint64_t *sum8;   // pack_sum(sum[i]) — the phase-A stream
    const SumHot *sum;
    const uint64_t *start;  // line start, absolute offset in the VCF text stream
    const uint32_t *cur;    // cursor offset after addCounts, relative to start
    const uint32_t *dcount; // delimiters {\t / | ; :} from the cursor to '\n'
};

// ---- duplicateVariantSearch (lambda/duplicateVariantSearch/source/
// duplicateVariantSearch.cpp:31-84, readVcfData.cpp:3-38)
// A key is the string to_string(pos) + ref' + '_' + alt' (readVcfData.cpp:23,
// write_data_to_s3.h:30-37) where x' = compressSeq(x).  The store keeps, per
// key: pos, a 64-bit hash of the whole string and the tail ref'_alt' as one
// word: bit 63 clear = inline (bytes in bits 0..55, length in bits 56..62,
// length <= 7); bit 63 set = bytes in the key blob (offset bits 0..39,
// length bits 40..55).
inline constexpr uint64_t kTailBlob = 1ull << 63;
inline constexpr int kTailInlineMax = 7;

struct alignas(16) KBody {  // what the equality check reads: one 16-byte load
    uint64_t tail;
    uint32_t pos;
    uint32_t flags;  // kKeyDisplaced
};
// the tail starts with a decimal digit: the string's leading digit run (its
// "effective position" P) is longer than decimal(pos) and the same string
// may also be stored at a larger POS (a prefix of P's digits, or P itself)
inline constexpr uint32_t kKeyDisplaced = 1u;

// Window dedup (sb_dedup_count): a job's key runs (POS-sorted) cut at POS
// boundaries into windows [p0, p1) of at most kWinCap keys, each
// deduplicated on its own in LDS.  Equal strings at one POS meet in one
// window.  A string stored at several POS (displaced keys) counts only at its
// largest POS: a displaced key y with 10 POS > the job's largest POS can have
// no copy at a larger POS and is counted in its window like any key; the
// others (deferred keys) are listed and counted by a second kernel, one lane
// per key: y counts when no key of the job's runs holds its string at a
// larger POS (its twin, found through the record POS index) and no earlier
// key of the job's runs (earlier run, or earlier in its run) equals it.
// Window w's record (dedup_plan_kernel writes it; rec_words u32 per window):
// the KWin header, then run r's piece of the window's keys as [lo, hi) at
// words kWinRecHead + 2 r, + 1 -- one load round for the window kernel
// (header and pieces side by side, no dependent read of a run-start table)
inline constexpr uint32_t kWinRecHead = 8;
struct KWin {  // header of window w's record
    uint32_t i, nruns, job, p0;  // window i of its job; the job's runs; POS where it starts
    uint32_t run_lo;  // the job's first KRun
    uint32_t pmax;    // largest POS of the job's runs
    uint32_t pad;
    uint32_t nw;      // the job's windows
};
static_assert(sizeof(KWin) == 4 * kWinRecHead, "KWin is the record header");
// One job of a window-dedup call (host-built): its windows [w0, w0 + nw) cut
// its POS axis at the leader run's key ranks i * lead_n / nw, every run of the
// job split at the same POS (dedup_plan_kernel: a lower bound per run and cut)
struct KJob {
    uint32_t w0, nw, run_lo, nruns;
    uint32_t lead_lo, lead_n;  // the leader run's (the job's longest) keys
    uint32_t pmin, pmax;       // POS span of the job's runs
    uint32_t pad[4];
};
struct KRun {  // one POS-sorted key run of a job + its segment's POS index
    uint32_t key_lo, key_hi, pos_lo, pos_hi;  // keys, POS of the first / last
    uint32_t seg_lo, seg_hi, b_base, b_shift;  // segment records, bucket base / width
    uint64_t b_off;
    uint32_t b_n;
    uint32_t job;
    uint32_t run_lo, nruns;  // the job's runs [run_lo, run_lo + nruns)
    uint32_t pad[2];
};
#ifndef SBEACON_WIN_CAP
#define SBEACON_WIN_CAP 2048
#endif
inline constexpr uint32_t kWinCap = SBEACON_WIN_CAP;         // keys per window (LDS sets sized for it)
inline constexpr uint32_t kWinTarget = kWinCap / 4 * 3;      // keys a window is planned for (runs of a job differ in density)
inline constexpr uint32_t kWinPieces = 64;   // pieces (= runs) per window
inline constexpr uint32_t kWinSpanBits = 26; // p1 - p0 < 2^26 - 1: exact words fit 32 bits

// one 8-byte class word per key (the window dedup reads only this for
// almost every key): POS in bits 0..31, the tail's store-wide id in bits
// 32..60 (< 64: c1 << 3 | c2, the compressSeq codes of a single-base REF and
// ALT; 0: no id, the key is hashed), kWordDisplaced when the tail starts
// with a digit
inline constexpr uint64_t kWordDisplaced = 1ull << 62;
inline constexpr uint32_t kWordIdMask = (1u << 29) - 1;
struct KStore {
    const uint64_t *hash;
    const KBody *body;
    const uint64_t *word;
    const uint8_t *blob;
    // twin lookups of the window dedup: first key of each record (+ end), the
    // records' POS and the segments' coarse POS index (DStore::pos / bucket)
    const uint32_t *lo;
    const uint32_t *rpos;
    const uint32_t *bucket;
};

struct KSeg {  // one run of store keys gathered for a job
    uint64_t key_lo;   // first store key
    uint64_t out_lo;   // first gather index of the run
    uint32_t n;
    uint32_t job;
    uint32_t range_start;  // the job's rangeStart (exact words hold POS - rangeStart)
    uint32_t pad;
};

// Exact dedup words.  A key string decimal(pos) ++ tail parses uniquely as
// (P = its longest leading digit run read as a number, rest); when rest is
// c1 '_' c2 with c1, c2 compressSeq codes 1..7 (single-base REF and ALT: the
// bulk of every VCF) the string is determined by (P, c1, c2) and the word
// (job | P - rangeStart | c1 c2) identifies it exactly — equal words need no
// string comparison.  Every other key (and any P outside the job's window)
// goes to the hashed stream, whose equal words are confirmed byte-for-byte.
// Both streams partition the strings (a string's class is a function of the
// string), so the job's distinct count is the sum of the two streams'.

}  // namespace sb
