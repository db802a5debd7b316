// query_kernels.hip — CDNA4 (gfx950) kernel of the slice-query hot path.
//
// Reference semantics: lambda/performQuery/search_variants.py:33-271 and
// search_variants_in_samples.py:31-259 (restated in SURVEY.md §8a.1).  The
// reference walks `bcftools query` output record by record in a Python loop;
// here one 64-lane wavefront owns one slice query:
//   1. exact [lo, hi) bounds of the slice from the segment's coarse POS index
//      (two dependent rounds: scalar bucket loads, then 64-wide POS reads);
//   2. a walk over the records 64 at a time, one 16-byte RecHot word per lane
//      (global_load_dwordx4), the next chunk prefetched while this one is
//      evaluated;
//   3. the loop's order-dependent state — running call_count, `if
//      call_count:`, include_details / boolean early exits, the first
//      exception — as ballots, find-first-set and prefix sums;
//   4. hits written as packed u64 into the query's host-planned region,
//      positions from mbcnt (or a wave prefix sum for multi-hit lanes).
// One launch answers a whole splitQuery fan-out.  All arithmetic is integer;
// nothing here is a dense contraction, so no MFMA: the bound is memory
// bandwidth on the RecHot stream.
#include <hip/hip_runtime.h>
#include <type_traits>

#include <cstddef>
#include <cstdlib>
#include <stdexcept>

#include "../../include/sbeacon.h"
#include "config.hpp"
#include "devtypes.hpp"
#include "kernels.hpp"

namespace sb {

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
// chunks in flight per wave in the streaming kernels (stream_window)
constexpr int kRangeWindow = 8;  // 16-byte RangeHot: 32 VGPRs
constexpr int kRange8Window = 8;  // 8-byte RangeHot8: 16 VGPRs
constexpr int kVtWindow = 4;     // 16-byte VtHot: 16 VGPRs (a 1000G-shape slice is ~4 chunks)

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
    return (static_cast<uint64_t>(uniform(static_cast<uint32_t>(v >> 32))) << 32) | uniform(static_cast<uint32_t>(v));
}

// lane k's value, k wave-uniform (v_readlane into an SGPR)
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t k) {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v), static_cast<int>(k)));
}
__device__ __forceinline__ int64_t rdl64(int64_t v, uint32_t k) {
    const uint64_t u = static_cast<uint64_t>(v);
    return static_cast<int64_t>((static_cast<uint64_t>(rdl(static_cast<uint32_t>(u >> 32), k)) << 32) |
                                rdl(static_cast<uint32_t>(u), k));
}

__device__ __forceinline__ int ffs64(uint64_t m) { return __ffsll(static_cast<unsigned long long>(m)) - 1; }

__device__ __forceinline__ int64_t shfl_i64(int64_t v, int src) {
    const int lo = __shfl(static_cast<int>(static_cast<uint64_t>(v) & 0xffffffffu), src, kWave);
    const int hi = __shfl(static_cast<int>(static_cast<uint64_t>(v) >> 32), src, kWave);
    return static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) |
                                static_cast<uint32_t>(lo));
}

__device__ __forceinline__ int64_t shfl_up_i64(int64_t v, int d) {
    const int lo = __shfl_up(static_cast<int>(static_cast<uint64_t>(v) & 0xffffffffu), d, kWave);
    const int hi = __shfl_up(static_cast<int>(static_cast<uint64_t>(v) >> 32), d, kWave);
    return static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) |
                                static_cast<uint32_t>(lo));
}

__device__ __forceinline__ int64_t wave_incl_scan_i64(int64_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const int64_t t = shfl_up_i64(v, d);
        if (lane >= d) v += t;
    }
    return v;
}

// v of lane (DPP pattern CTRL); lanes the row / bank masks or the row edge
// exclude read 0
template <int CTRL, int ROW, int BANK>
__device__ __forceinline__ int64_t dpp_i64(int64_t v) {
    const uint64_t u = static_cast<uint64_t>(v);
    const uint32_t lo = static_cast<uint32_t>(
        __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(u)), CTRL, ROW, BANK, false));
    const uint32_t hi = static_cast<uint32_t>(
        __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(u >> 32)), CTRL, ROW, BANK, false));
    return static_cast<int64_t>((static_cast<uint64_t>(hi) << 32) | lo);
}

// sum over the wave, returned in every lane: DPP row reductions (quad_perm,
// row_shr 4 / 8, row_bcast 15 / 31) into lane 63, then one readlane -- no
// LDS round trips (ds_bpermute) on the per-slice path
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
    v += dpp_i64<0xb1, 0xf, 0xf>(v);   // quad_perm [1,0,3,2]
    v += dpp_i64<0x4e, 0xf, 0xf>(v);   // quad_perm [2,3,0,1]: quad sums
    v += dpp_i64<0x114, 0xf, 0xe>(v);  // row_shr:4 into banks 1..3
    v += dpp_i64<0x118, 0xf, 0xc>(v);  // row_shr:8 into banks 2..3: lane 15 of a row = row sum
    v += dpp_i64<0x142, 0xa, 0xf>(v);  // row_bcast:15 into rows 1, 3
    v += dpp_i64<0x143, 0xc, 0xf>(v);  // row_bcast:31 into rows 2, 3: lane 63 = total
    return rdl64(v, 63);
}

// number of lanes strictly below this one whose bit is set in m
__device__ __forceinline__ uint32_t popc_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}

__device__ __forceinline__ uint8_t up(uint8_t c) { return (c >= 'a' && c <= 'z') ? c - 32 : c; }

// XCD-aware workgroup order (cdna_hip_programming.md T1, bijective form):
// the dispatcher deals workgroups round-robin over the 8 XCDs, so block b
// shares an L2 with b + 8.  Remapping gives each XCD one contiguous run of
// the (position-sorted) query list: neighbouring slices scan overlapping or
// adjacent records, which then hit the same XCD's L2.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t nb) {
    const uint32_t q = nb / 8, r = nb % 8, x = b % 8;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// ---------------------------------------------------------------- bounds
// [lo, hi) = records of the segment with x1 <= POS < x2.  The bucket holding
// x brackets lower_bound(x) in [bucket[b], bucket[b+1]]; both searches issue
// their bucket loads and their 64-wide POS reads together, so the bounds cost
// two dependent memory rounds (a bucket longer than 64 records loops).
struct Bracket {
    uint32_t L, H;
    bool done;  // answer already known (= L)
};

__device__ __forceinline__ Bracket bracket(const DStore &st, const QDev &Q, int64_t x) {
    if (x <= static_cast<int64_t>(Q.bucket_base)) return {Q.seg_lo, Q.seg_lo, true};
    const uint64_t b = static_cast<uint64_t>(x - Q.bucket_base) >> Q.bucket_shift;
    if (b >= Q.n_buckets) return {Q.seg_hi, Q.seg_hi, true};
    return {st.bucket[Q.bucket_off + b], st.bucket[Q.bucket_off + b + 1], false};
}

__device__ __forceinline__ uint32_t finish_bound(const DStore &st, Bracket k, int64_t x, uint32_t v_first) {
    // v_first: this lane's POS at k.L + lane (already loaded), UINT32_MAX past H
    const int lane = lane_id();
    uint32_t L = k.L;
    uint32_t v = v_first;
    for (;;) {
        const uint64_t m = __ballot(static_cast<int64_t>(v) >= x || L + static_cast<uint32_t>(lane) >= k.H);
        if (m) {
            const uint32_t r = L + static_cast<uint32_t>(ffs64(m));
            return r < k.H ? r : k.H;
        }
        L += kWave;  // all 64 POS < x: the bucket is longer than one wave
        const uint32_t i = L + static_cast<uint32_t>(lane);
        v = i < k.H ? st.pos[i] : 0xffffffffu;
    }
}

__device__ __forceinline__ void slice_bounds(const DStore &st, const QDev &Q, uint32_t *lo, uint32_t *hi) {
    const Bracket a = bracket(st, Q, Q.first_bp), b = bracket(st, Q, Q.last_bp + 1);
    const uint32_t ia = a.L + static_cast<uint32_t>(lane_id()), ib = b.L + static_cast<uint32_t>(lane_id());
    const uint32_t va = (!a.done && ia < a.H) ? st.pos[ia] : 0xffffffffu;
    const uint32_t vb = (!b.done && ib < b.H) ? st.pos[ib] : 0xffffffffu;
    *lo = a.done ? a.L : finish_bound(st, a, Q.first_bp, va);
    *hi = b.done ? b.L : finish_bound(st, b, Q.last_bp + 1, vb);
    if (*hi < *lo) *hi = *lo;
}

// ---------------------------------------------------------------- predicates
__device__ __forceinline__ bool blob_eq_upper(const uint8_t *__restrict__ blob, uint64_t off, uint32_t len,
                                              const uint8_t *__restrict__ q, uint32_t qlen) {
    if (len != qlen) return false;
    for (uint32_t i = 0; i < len; ++i)
        if (up(blob[off + i]) != q[i]) return false;
    return true;
}

// svs:88-91: '^' + ref.replace('N', '[ACGTN]{1}') + '$' against REF.upper()
__device__ __forceinline__ bool wild_char(uint8_t c, uint8_t p) {
    if (p == 'N') return c == 'A' || c == 'C' || c == 'G' || c == 'T' || c == 'N';
    if (p == '.') return c != '\n';
    return c == p;
}

__device__ bool ref_wild_match(const DStore &st, uint32_t r, uint32_t ref_len, const uint8_t *__restrict__ pat,
                               uint32_t plen, uint64_t key) {
    if (ref_len != plen) return false;
    if (!(key >> 63)) {
        for (uint32_t i = 0; i < plen; ++i)
            if (!wild_char(static_cast<uint8_t>(key >> (8 * i)), pat[i])) return false;
        return true;
    }
    const uint64_t off = st.ref_off[r];
    for (uint32_t i = 0; i < plen; ++i)
        if (!wild_char(up(st.blob[off + i]), pat[i])) return false;
    return true;
}

// :100-166 variantType predicate of one non-None-alt-less query
__device__ __forceinline__ bool vtype_hit(const QDev &Q, const DStore &st, uint32_t cls, int64_t len,
                                          int64_t ref_len) {
    if (cls & C_SYMBOLIC) {
        const uint32_t sym = cls >> C_SYM_SHIFT;
        return (st.sym_lut[Q.lut_off + (sym >> 5)] >> (sym & 31)) & 1u;
    }
    const uint32_t rep = (cls >> C_REP_SHIFT) & 63u;
    switch (Q.vt_kind) {
        case VT_DEL: return len < ref_len;
        case VT_INS: return len > ref_len;
        case VT_DUP: return rep != C_REP_NONE && rep >= 2;
        case VT_DUPT: return rep == 2;
        case VT_CNV: return (cls & C_DOT) || rep != C_REP_NONE;
        default: return false;
    }
}

// genotype fallback over the selected samples (samples variant, record without
// AC / AN): search_variants_in_samples.py:211-222 / :239-245 with bcftools
// --samples restricting the GT text.  value = allele number (0 = every call).
__device__ int64_t fallback_count(const DStore &st, uint32_t r, const uint64_t *__restrict__ subset,
                                  uint32_t n_samples, uint32_t value) {
    const int64_t base = st.fb_off[r];
    int64_t n_match = 0;
    for (uint32_t s = 0; s < n_samples; ++s) {
        if (subset && !((subset[s >> 6] >> (s & 63)) & 1)) continue;
        const uint32_t w = st.fb[base + s];
        const uint32_t n = w & 0xffu;
        if (!value) {
            n_match += n;
            continue;
        }
        for (uint32_t t = 0; t < n; ++t)
            if (((w >> (8 + 8 * t)) & 0xffu) == value) ++n_match;
    }
    return n_match;
}

// ---------------------------------------------------------------- scan
// What one record contributes to its slice query (search_variants.py:84-226):
// hm = hit ALTs (bit k = ALT k), em = ALTs emitted as variant strings (bit =
// label index; the GT fallback labels with alts[k+1], :223), c = its call
// count contribution, anv = its all_alleles_count contribution, err = the
// exception the reference raises at this record (SB_QERR_*).
struct LaneOut {
    int err;
    uint64_t hm, em;
    int64_t c, anv;
};

struct QView {  // per-wave query constants, specialised by MODE
    uint32_t flags, ref_mode, alt_mode;
    bool samples_variant, strict_unbound;
    const uint8_t *qref, *qalt;
    const uint64_t *subset;
};

// General evaluation of record r (RecHot h already loaded); extra ALTs and
// hashed-key confirmations are loaded on demand.
// pre_pos / pre_key: POS and ref_key of record r when the caller streamed
// them ahead with the record word (have_pre), so REF_WILD costs no dependent load
__device__ __forceinline__ LaneOut eval_record(const DStore &st, const QDev &Q, const QView &V, uint32_t r,
                                            const RecHot h0, bool have_pre = false, uint32_t pre_pos = 0,
                                            uint64_t pre_key = 0) {
    LaneOut o{0, 0, 0, 0, 0};
    const uint32_t e = h0.end;
    const uint32_t h = h0.hot;
    bool pass = static_cast<int64_t>(e) >= Q.end_min && static_cast<int64_t>(e) <= Q.end_max;  // :90
    if (pass) {
        switch (V.ref_mode) {  // :94 / svs:88-91
            case REF_ANY:
                break;
            case REF_EXACT: {
                const uint64_t k = st.ref_key[r];
                pass = k == Q.ref_key;
                if (pass && (k >> 63)) pass = blob_eq_upper(st.blob, st.ref_off[r], e - st.pos[r] + 1, V.qref, Q.ref_len);
                break;
            }
            case REF_WILD:
                pass = have_pre ? ref_wild_match(st, r, e - pre_pos + 1, V.qref, Q.ref_len, pre_key)
                                : ref_wild_match(st, r, e - st.pos[r] + 1, V.qref, Q.ref_len, st.ref_key[r]);
                break;
            case REF_NEVER:
                pass = false;
                break;
            default:
                o.err = static_cast<int>(Q.ref_err);
                pass = false;
                break;
        }
    }
    if (pass && V.strict_unbound) {  // :101 in the unpatched reference
        o.err = SB_QERR_UNBOUND_LOCAL;
        pass = false;
    }
    if (!pass) return o;
    if ((h & H_AN_BAD) && h0.an == kAnUnrepresentable) {  // a general record: general_slice_kernel answers the slice
        o.err = SB_QERR_GENERAL;
        return o;
    }
    uint32_t x0 = 0, nx = 0;
    const int64_t ref_len = (V.alt_mode == ALT_VTYPE) ? static_cast<int64_t>(e) - st.pos[r] + 1 : 0;
    {  // ALT 0: class bits live in RecHot::hot
        bool ok;
        int64_t len = 1;
        if (V.alt_mode == ALT_N) {
            ok = h & C_SINGLE_BASE;
        } else if (V.alt_mode == ALT_EXACT) {
            const uint64_t k = st.a0_key[r];
            ok = k == Q.alt_key;
            len = Q.alt_len;
            if (ok && (k >> 63)) ok = blob_eq_upper(st.blob, st.a0_off[r], st.a0_len[r], V.qalt, Q.alt_len);
        } else {
            len = st.a0_len[r];
            ok = vtype_hit(Q, st, h, len, ref_len);
        }
        if (ok && len >= Q.vmin && len <= Q.vmax) o.hm = 1;
    }
    if (h & H_MULTI) {  // ALTs 1..n-1 of multiallelic records
        x0 = st.x_lo[r];
        nx = st.x_lo[r + 1] - x0;
        for (uint32_t k = 0; k < nx && k < 63; ++k) {
            const uint32_t x = x0 + k;
            const uint32_t cls = st.xrow[x].cls;
            bool ok;
            int64_t len = 1;
            if (V.alt_mode == ALT_N) {
                ok = cls & C_SINGLE_BASE;
            } else if (V.alt_mode == ALT_EXACT) {
                const uint64_t key = st.x_key[x];
                ok = key == Q.alt_key;
                len = Q.alt_len;
                if (ok && (key >> 63)) ok = blob_eq_upper(st.blob, st.x_off[x], st.x_len[x], V.qalt, Q.alt_len);
            } else {
                len = st.x_len[x];
                ok = vtype_hit(Q, st, cls, len, ref_len);
            }
            if (ok && len >= Q.vmin && len <= Q.vmax) o.hm |= 2ull << k;
        }
    }
    if (!o.hm) return o;
    const uint32_t na = 1 + nx;
    const bool sub = V.samples_variant && (h & H_HAS_FB);
    if (h & H_AN_BAD) {
        o.err = SB_QERR_VALUE;  // :199
    } else if (h & H_HAS_AC) {  // :205-214
        if (h & H_AC_BAD) {
            o.err = SB_QERR_VALUE;  // :206
        } else {
            for (uint64_t b = o.hm; b; b &= b - 1) {
                const int k = ffs64(b);
                const XRow xk = k ? st.xrow[x0 + k - 1] : XRow{h, h0.ac0};
                if (xk.cls & C_AC_MISSING) o.err = SB_QERR_INDEX;  // :207
                const int64_t v = xk.ac;
                o.c += v;
                if (v != 0) o.em |= 1ull << k;
            }
        }
    } else {  // :215-226 genotype fallback, labelled alts[i] with 1-based i
        for (uint64_t b = o.hm; b; b &= b - 1) {
            const int k = ffs64(b);
            const int64_t v = sub ? fallback_count(st, r, V.subset, Q.n_samples, k + 1)
                                  : (k ? st.xrow[x0 + k - 1].ac : h0.ac0);
            o.c += v;
            if (v > 0) {
                if (static_cast<uint32_t>(k + 1) >= na) o.err = SB_QERR_INDEX;  // :223
                else o.em |= 1ull << (k + 1);
            }
        }
    }
    o.anv = (h & H_HAS_AN) ? h0.an : (sub ? fallback_count(st, r, V.subset, Q.n_samples, 0) : h0.an);
    if (o.err) {
        o.hm = 0;
        o.em = 0;
        o.c = 0;
    }
    return o;
}

struct ScanState {
    int64_t carry = 0;      // running call_count (general path)
    bool carry_nz = false;  // running call_count != 0 (non-negative path)
    int64_t cc_acc = 0, an_acc = 0;  // per-lane partial sums, reduced once at the end
    uint32_t n_out = 0;
    bool exists = false;
    int err_out = 0;
    bool touched = false;  // some chunk had a hit or an error (else every total is 0)
};

// The reference loop's order-dependent state over one 64-record chunk
// (:229-254): running call_count, `if call_count:`, the include_details /
// boolean early exits and the first exception, then the compacted emission
// of variant strings (:209-213 / :222-225).  Returns the stop lane (kWave =
// none); *collectm = hit lanes whose samples are collected (:233-236).
template <bool NONNEG>
__device__ __forceinline__ int chunk_tail(ScanState &S, const LaneOut &o, uint32_t r, bool stop_on_exists,
                                          bool details, uint64_t *__restrict__ out, uint64_t *collectm) {
    const int lane = lane_id();
    const bool hit = o.hm != 0;
    const uint64_t errm = __ballot(o.err != 0);
    const uint64_t hitm = __ballot(hit);
    if (!(errm | hitm)) {  // nothing to emit, count or stop on: state unchanged
        *collectm = 0;
        return kWave;
    }
    S.touched = true;
    int64_t cum = 0;
    uint64_t trigm;  // hit lanes where the running call_count is non-zero
    if constexpr (NONNEG) {
        const uint64_t pm = __ballot(hit && o.c > 0);
        trigm = S.carry_nz ? hitm : (pm ? (hitm & ~((1ull << ffs64(pm)) - 1ull)) : 0ull);
    } else {
        cum = S.carry + wave_incl_scan_i64(hit ? o.c : 0);
        trigm = __ballot(hit && cum != 0);
    }
    const uint64_t stopm = errm | (stop_on_exists ? trigm : 0ull);
    const int s = stopm ? ffs64(stopm) : kWave;
    if (s < kWave && ((errm >> s) & 1ull)) {
        S.err_out = __shfl(o.err, s, kWave);
        *collectm = 0;
        return s;
    }
    const uint64_t upto = (s >= kWave - 1) ? ~0ull : ((2ull << s) - 1ull);
    const bool in = (upto >> lane) & 1ull;
    const uint32_t cnt = (hit && in) ? static_cast<uint32_t>(__popcll(o.em)) : 0u;
    const uint64_t multi = __ballot(cnt > 1);
    uint32_t pos0, total;
    if (!multi) {
        const uint64_t one = __ballot(cnt == 1);
        pos0 = popc_below(one);
        total = static_cast<uint32_t>(__popcll(one));
    } else {  // bit-sliced exclusive prefix of cnt: one ballot + mbcnt per bit, no LDS traffic
        pos0 = 0;
        total = 0;
        for (uint32_t b = 0; b < 7; ++b) {
            const uint64_t m = __ballot((cnt >> b) & 1u);
            pos0 += popc_below(m) << b;
            total += static_cast<uint32_t>(__popcll(m)) << b;
            if (!__ballot(cnt >> (b + 1))) break;
        }
    }
    if (cnt) {
        uint64_t *dst = out + S.n_out + pos0;
        for (uint64_t b = o.em; b; b &= b - 1)
            *dst++ = static_cast<uint64_t>(r) | (static_cast<uint64_t>(ffs64(b)) << kHitAltShift);
    }
    S.n_out += total;
    // call_count and all_alleles_count: lanes up to the stop; the stop lane's
    // AN only for the boolean break (after :244), not for :231
    if (hit && in) S.cc_acc += o.c;
    if (hit && (lane < s || (lane == s && details))) S.an_acc += o.anv;
    S.exists = S.exists || ((trigm & upto) != 0ull);
    if constexpr (NONNEG)
        S.carry_nz = S.exists;
    else
        S.carry = shfl_i64(cum, s < kWave ? s : kWave - 1);
    *collectm = trigm & upto;
    return s;
}

template <bool NONNEG>
__device__ __forceinline__ void finish_query(const ScanState &S, const DStore &st, const QDev &Q, uint32_t n_scanned,
                                             QRes *res) {
    const uint32_t q = Q.orig;
    if (!S.touched) {  // no hit and no error in the whole slice (most variantType slices)
        if (lane_id() == 0) res[q] = QRes{0, 0, 0, 0, 0, n_scanned};
        return;
    }
    if (S.err_out == SB_QERR_GENERAL && lane_id() == 0) {  // the scan reached a general record
        const uint32_t k = atomicAdd(st.gen_work, 1u);
        st.gen_work[1 + k] = static_cast<uint32_t>(&Q - st.q_all);
    }
    const int64_t call_count = NONNEG ? wave_sum_i64(S.cc_acc) : S.carry;
    const int64_t an_sum = wave_sum_i64(S.an_acc);
    if (lane_id() == 0) {
        QRes o;
        o.error = S.err_out;
        o.exists = S.exists ? 1 : 0;
        o.call_count = call_count;
        o.all_alleles_count = an_sum;
        o.n_hits = S.err_out ? 0u : S.n_out;
        o.n_scanned = n_scanned;
        res[q] = o;
    }
}

// Sliding-window stream over the chunks of [lo, hi): D chunks of packed words
// are in flight per wave, and chunk base + D*64 is requested as soon as chunk
// base is consumed (the window rotates by register name in the unrolled body,
// never by copy, so no load is waited on early).  `ld` must load
// unconditionally (clamped index, no exec-masked branch): a load under a
// divergent branch makes the waitcnt pass fall back to vmcnt(0).  `fast(base, word)` evaluates
// one chunk: 0 = go on, 1 = the query is done, 2 = the chunk holds lanes only
// the general path can decide (not consumed).  Returns that status; *at = the
// base of the chunk it stopped on.
template <int D, typename W, typename Load, typename Fast>
__device__ __forceinline__ int stream_window(uint32_t lo, uint32_t hi, uint32_t *at, Load ld, Fast fast) {
    const uint32_t ul = static_cast<uint32_t>(lane_id());
    uint32_t base = lo;
    int status = 0;
    if (lo >= hi) {
        *at = lo;
        return 0;
    }
    W a[D];
#pragma unroll
    for (int k = 0; k < D; ++k) a[k] = ld(lo + ul + static_cast<uint32_t>(k) * kWave);
    // The first D chunks are straight-line code: the waitcnt pass counts the
    // loads in flight exactly there (vmcnt(D-1-k)), while at a loop header it
    // falls back to vmcnt(0).  Most slices end inside this block; longer ones
    // continue in the loop, whose header drains once per D chunks.
#pragma unroll
    for (int k = 0; k < D; ++k) {
        status = fast(base, a[k]);
        if (status) goto done;
        if (base + static_cast<uint32_t>(D) * kWave < hi) a[k] = ld(base + ul + static_cast<uint32_t>(D) * kWave);
        base += kWave;
        if (base >= hi) goto done;
    }
    for (;;) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            status = fast(base, a[k]);
            if (status) goto done;
            a[k] = ld(base + ul + static_cast<uint32_t>(D) * kWave);
            base += kWave;
            if (base >= hi) goto done;
        }
    }
done:
    *at = base;
    return status;
}

// NACC: 64-bit sample-bitset words per lane (0 = no query in this launch
// collects samples); NONNEG: every AC in the store is >= 0, so the running
// call_count is monotone and `if call_count:` reduces to ballots.  MODE_EXACT
// specialises the predicates for REF/ALT point queries; MODE_GENERAL handles
// every payload (variantType, samples variant, strict mode, wildcards).
constexpr int kRowBatch = 16;  // carrier rows in flight per wave (sample path)

template <int NACC, bool NONNEG, int MODE>
__device__ __forceinline__ void scan_slice(
    DStore st, const QDev *__restrict__ qs, 
    const uint8_t *__restrict__ qbytes, const uint64_t *__restrict__ subsets, QRes *__restrict__ res,
    uint64_t *__restrict__ hits, uint64_t *__restrict__ samples_out, uint32_t q, uint32_t lo, uint32_t hi) {
    const int lane = lane_id();
    const QDev &Q = qs[q];
    constexpr bool kGeneral = MODE == MODE_GENERAL;
    QView V;
    V.flags = Q.flags;
    V.ref_mode = MODE == MODE_EXACT ? REF_EXACT : Q.ref_mode;
    V.alt_mode = MODE == MODE_EXACT ? ALT_EXACT : Q.alt_mode;
    V.samples_variant = kGeneral && (V.flags & F_SAMPLES_VARIANT);
    V.strict_unbound = kGeneral && (V.flags & F_STRICT_UNBOUND);
    V.qref = qbytes + Q.qbytes_off;
    V.qalt = V.qref + Q.ref_len;
    V.subset = (Q.subset_off != ~0ull) ? subsets + Q.subset_off : nullptr;
    const bool details = V.flags & F_DETAILS;
    const bool collect = NACC > 0 && (V.flags & F_COLLECT) && details;
    const bool stop_on_exists = !details || (V.flags & F_BOOL_BREAK);


    ScanState S;
    uint64_t acc[NACC > 0 ? NACC : 1];
#pragma unroll
    for (int j = 0; j < (NACC > 0 ? NACC : 1); ++j) acc[j] = 0;
    uint64_t *out = hits + Q.hit_off;

    RecHot cur = {0, 0, 0, 0}, nxt = {0, 0, 0, 0};
    // samples variant with a wildcard REF (svs:88-91): POS and ref_key are
    // streamed one chunk ahead with the record word
    const bool pre = kGeneral && V.ref_mode == REF_WILD;
    uint32_t cpos = 0, npos = 0;
    uint64_t ckey = 0, nkey = 0;
    if (lo + static_cast<uint32_t>(lane) < hi) {
        cur = st.rec[lo + lane];
        if (pre) {
            cpos = st.pos[lo + lane];
            ckey = st.ref_key[lo + lane];
        }
    }
    for (uint32_t base = lo; base < hi; base += kWave) {
        const uint32_t r = base + static_cast<uint32_t>(lane);
        if (r + kWave < hi) {
            nxt = st.rec[r + kWave];
            if (pre) {
                npos = st.pos[r + kWave];
                nkey = st.ref_key[r + kWave];
            }
        }
        LaneOut o{0, 0, 0, 0, 0};
        if (r < hi) o = eval_record(st, Q, V, r, cur, pre, cpos, ckey);
        uint64_t cm;
        const int s = chunk_tail<NONNEG>(S, o, r, stop_on_exists, details, out, &cm);
        if (s < kWave && S.err_out) break;
        // sample path (:233-236): OR the carrier planes of every hit allele.
        // Lanes whose only hit is ALT 0 (nearly all) go 8 rows at a time:
        // eight independent loads in flight per wave instead of one
        // dependent round trip per hit; other lanes take the per-allele loop.
        if constexpr (NACC > 0) if (collect) {
            // hit lane L scanned record base + L: its ALT-0 row is wave-uniform arithmetic
            const uint64_t row_base = Q.plane0_base + static_cast<uint64_t>(base - Q.rec_base) * Q.words;
            uint64_t m1 = cm & __ballot(o.hm == 1ull);
            cm &= ~m1;
            while (m1) {
                uint64_t rows[kRowBatch];
                int nb = 0;
#pragma unroll
                for (int u = 0; u < kRowBatch; ++u) {
                    rows[u] = ~0ull;
                    if (m1) {
                        const int L = ffs64(m1);
                        m1 &= m1 - 1;
                        rows[u] = row_base + static_cast<uint64_t>(L) * Q.words;
                        nb = u + 1;
                    }
                }
#pragma unroll
                for (int j = 0; j < NACC; ++j) {
                    const uint32_t wd = static_cast<uint32_t>(lane) + 64u * j;
                    if (wd < Q.words) {
                        uint64_t v[kRowBatch];
#pragma unroll
                        for (int u = 0; u < kRowBatch; ++u) v[u] = u < nb ? st.planes[rows[u] + wd] : 0ull;
#pragma unroll
                        for (int u = 0; u < kRowBatch; ++u) acc[j] |= v[u];
                    }
                }
                if (Q.words > 64u * NACC && Q.samples_out_off != ~0ull)  // beyond the register window
                    for (uint32_t wd = static_cast<uint32_t>(lane) + 64u * NACC; wd < Q.words; wd += 64u) {
                        uint64_t v = 0;
                        for (int u = 0; u < nb; ++u) v |= st.planes[rows[u] + wd];
                        samples_out[Q.samples_out_off + wd] |= v;
                    }
            }
            while (cm) {
                const int L = ffs64(cm);
                cm &= cm - 1;
                const uint64_t hml = static_cast<uint64_t>(shfl_i64(static_cast<int64_t>(o.hm), L));
                const uint32_t rl = static_cast<uint32_t>(__shfl(static_cast<int>(r), L, kWave));
                const uint32_t xl = (hml >> 1) ? st.x_lo[rl] : 0u;
                for (uint64_t b = hml; b; b &= b - 1) {
                    const int k = ffs64(b);
                    const uint64_t row = k ? Q.planex_base + static_cast<uint64_t>(xl + k - 1 - Q.x_base) * Q.words
                                           : Q.plane0_base + static_cast<uint64_t>(rl - Q.rec_base) * Q.words;
#pragma unroll
                    for (int j = 0; j < NACC; ++j) {
                        const uint32_t wd = static_cast<uint32_t>(lane) + 64u * j;
                        if (wd < Q.words) acc[j] |= st.planes[row + wd];
                    }
                    if (Q.words > 64u * NACC && Q.samples_out_off != ~0ull)
                        for (uint32_t wd = static_cast<uint32_t>(lane) + 64u * NACC; wd < Q.words; wd += 64u)
                            samples_out[Q.samples_out_off + wd] |= st.planes[row + wd];
                }
            }
        }
        cur = nxt;
        cpos = npos;
        ckey = nkey;
        if (s < kWave) break;
    }
    finish_query<NONNEG>(S, st, Q, hi - lo, res);
    if constexpr (NACC > 0) if (collect && Q.samples_out_off != ~0ull) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) {
            const uint32_t wd = static_cast<uint32_t>(lane) + 64u * j;
            if (wd < Q.words) {
                uint64_t v = S.err_out ? 0ull : acc[j];
                if (V.subset) v &= V.subset[wd];
                samples_out[Q.samples_out_off + wd] = v;
            }
        }
        // words past the register window were OR-ed into samples_out (zeroed
        // by the host) by the lane that owns them: mask them the same way
        for (uint32_t wd = static_cast<uint32_t>(lane) + 64u * NACC; wd < Q.words; wd += 64u) {
            uint64_t v = S.err_out ? 0ull : samples_out[Q.samples_out_off + wd];
            if (V.subset) v &= V.subset[wd];
            samples_out[Q.samples_out_off + wd] = v;
        }
    }
}

// MODE_RANGE_N / MODE_RANGE_N8: referenceBases 'N' + alternateBases 'N'
// range queries (the bulk of Beacon traffic).  Every per-record quantity such
// a query needs is query-independent and sits in one RangeHot word (16 bytes)
// or, for a VCF with a common AN, one RangeHot8 word (8 bytes; devtypes.hpp),
// so a record costs one coalesced load and a handful of VALU ops, streamed
// through a stream_window; chunks with RH_SLOW lanes (no AC, int() failures,
// > 8 ALTs, an uncommon AN in RangeHot8 ...) go to a tail loop with
// eval_record.
// the two record words of MODE_RANGE_N / MODE_RANGE_N8
template <typename W>
struct RangeWord;
template <>
struct RangeWord<RangeHot> {
    static constexpr int kWindow = kRangeWindow;
    static __device__ __forceinline__ const RangeHot *col(const DStore &st) { return st.rng; }
    static __device__ __forceinline__ uint32_t info(const RangeHot &h) { return h.info; }
    static __device__ __forceinline__ int64_t c(const RangeHot &h) { return h.c; }
    static __device__ __forceinline__ int64_t an(const RangeHot &h, int64_t) { return h.an; }
};
template <>
struct RangeWord<RangeHot8> {
    static constexpr int kWindow = kRange8Window;
    static __device__ __forceinline__ const RangeHot8 *col(const DStore &st) { return st.rng8; }
    static __device__ __forceinline__ uint32_t info(const RangeHot8 &h) { return h.w; }
    static __device__ __forceinline__ int64_t c(const RangeHot8 &h) { return h.w >> RH8_C_SHIFT; }
    static __device__ __forceinline__ int64_t an(const RangeHot8 &, int64_t an_default) { return an_default; }
};

template <bool NONNEG, typename W>
__device__ __forceinline__ void range_n_slice(DStore st, const QDev *__restrict__ qs,
                                                         
                                                         QRes *__restrict__ res, uint64_t *__restrict__ hits, uint32_t q, uint32_t lo, uint32_t hi) {
    const int lane = lane_id();
    const QDev &Q = qs[q];
    const uint32_t flags = Q.flags;
    const bool details = flags & F_DETAILS;
    const bool stop_on_exists = !details || (flags & F_BOOL_BREAK);
    ScanState S;
    // len(alt) = 1 for every ALT an 'N' query can hit (:174)
    const bool len_ok = Q.vmin <= 1 && Q.vmax >= 1;
    const bool end_void = Q.end_max < 0 || Q.end_min > 0xffffffffll || Q.end_min > Q.end_max;
    const uint32_t e0 = Q.end_min < 0 ? 0u : static_cast<uint32_t>(Q.end_min);  // END in [e0, e0 + espan]
    const uint32_t espan = (Q.end_max > 0xffffffffll ? 0xffffffffu : static_cast<uint32_t>(Q.end_max)) - e0;
    const uint32_t shi = (len_ok && !end_void) ? hi : lo;  // nothing can hit: nothing to scan
    uint64_t *out = hits + Q.hit_off;
    const QView V{flags, REF_ANY, ALT_N, false, false, nullptr, nullptr, nullptr};
    const uint32_t ul = static_cast<uint32_t>(lane);

    using RW = RangeWord<W>;
    const int64_t an_default = Q.an_default;
    const W *col = RW::col(st);
    auto lane_eval = [&](const W h, bool cand) -> LaneOut {
        LaneOut o{0, 0, 0, 0, 0};
        if (cand) {
            o.hm = 1;
            o.em = RW::info(h) & RH_EMIT_MASK;
            o.c = RW::c(h);
            o.anv = RW::an(h, an_default);
        }
        return o;
    };
    auto fast = [&](uint32_t base, const W h) -> int {
        const uint32_t r = base + ul;
        const bool cand = r < shi && (RW::info(h) & RH_HIT) && h.end - e0 <= espan;
        if (__ballot(cand && (RW::info(h) & RH_SLOW))) return 2;
        uint64_t cm;
        return chunk_tail<NONNEG>(S, lane_eval(h, cand), r, stop_on_exists, details, out, &cm) >= kWave ? 0 : 1;
    };
    // clamped, unconditional (used only when lo < shi); lanes past shi fail `cand`
    auto ld = [&](uint32_t i) -> W { return col[min(i, shi - 1)]; };
    uint32_t base = lo;
    if (lo < shi && stream_window<RW::kWindow, W>(lo, shi, &base, ld, fast) == 2) {
        // the rest one chunk at a time, eval_record for RH_SLOW lanes
        W h = ld(base + ul);
        for (; base < shi; base += kWave) {
            const uint32_t r = base + ul;
            const W nh = ld(r + kWave);
            const bool cand = r < shi && (RW::info(h) & RH_HIT) && h.end - e0 <= espan;
            const bool slow = cand && (RW::info(h) & RH_SLOW);
            LaneOut o = lane_eval(h, cand && !slow);
            if (__ballot(slow) && slow) o = eval_record(st, Q, V, r, st.rec[r]);
            uint64_t cm;
            if (chunk_tail<NONNEG>(S, o, r, stop_on_exists, details, out, &cm) < kWave) break;
            h = nh;
        }
    }
    finish_query<NONNEG>(S, st, Q, hi - lo, res);
}

// MODE_VTYPE: referenceBases 'N' + alternateBases None + variantType queries
// (search_variants.py:100-166, the patched-oracle branch selector; strict
// mode goes to MODE_GENERAL).  One 16-byte VtHot word per record carries END,
// the first ALT's class index (len(ALT0) vs len(REF), REF*k class, '.') or
// symbolic id, len(ALT0), AC0 and AN: the predicate, the length bounds
// (:177-183) and the AC / AN contributions (:205-214) of a biallelic record
// need no other load.  Multiallelic lanes read their extra rows' words
// (DStore::xvt) and AC; records flagged VT_SLOW (no AC, int() failures,
// missing AC entries, > 8 ALTs, lengths or symbolic ids >= 255) go to a
// one-chunk-at-a-time tail loop with eval_record.  The record stream is a
// stream_window of kVtWindow chunks.
// candidate word + its record index (MODE_VTYPE stream element)
struct VcWord {
    VtHot h;
    uint32_t r;
};

// candidates of variantType kind k among records [0, r): the VcBlock table
__device__ __forceinline__ uint32_t vc_count(const DStore &st, uint32_t k, uint32_t r) {
    const VcBlock b = st.vc_blk[k * st.vc_nblk + (r >> 6)];
    const uint32_t o = r & 63u;
    return b.pre + static_cast<uint32_t>(__popcll(o ? (b.mask & ((1ull << o) - 1ull)) : 0ull));
}

// The variantType predicate of one query over packed VtHot words
// (search_variants.py:100-183 + :205-214 for records that are not VT_SLOW):
// END in [e0, e0 + espan] and len(ALT) in [vlo, vlo + vspan] as one unsigned
// compare each (an empty length range never matches: vlo = 256), the class
// mask of the kind, and the symbolic-ALT LUT held in lanes 0..7.
struct VtPred {
    uint32_t e0, espan, vlo, vspan, cmask, xneed;
    bool end_void;  // no END can match
    const uint32_t *lut;
    uint32_t lutv;      // lane lut_lane + k (k < 8): LUT word k (symbolic ids in the words are < 255)
    uint32_t lut_lane;
    const uint32_t *llut = nullptr;  // the 8 LUT words in LDS (chain_pack_kernel) instead of lanes

    __device__ __forceinline__ void set_kind(uint32_t vk) {
        constexpr uint32_t kDel = vt_class_mask(VT_DEL), kIns = vt_class_mask(VT_INS), kDup = vt_class_mask(VT_DUP),
                           kDupT = vt_class_mask(VT_DUPT), kCnv = vt_class_mask(VT_CNV);
        cmask = vk == VT_DEL ? kDel : vk == VT_INS ? kIns : vk == VT_DUP ? kDup : vk == VT_DUPT ? kDupT
              : vk == VT_CNV ? kCnv : 0u;
        xneed = vt_xk_bit(vk) | VT_XK_SYM;  // an extra ALT might match
    }
    __device__ __forceinline__ VtPred(const DStore &st, const QDev &Q) {
        end_void = Q.end_max < 0 || Q.end_min > 0xffffffffll || Q.end_min > Q.end_max;
        e0 = Q.end_min < 0 ? 0u : static_cast<uint32_t>(Q.end_min);
        espan = (Q.end_max > 0xffffffffll ? 0xffffffffu : static_cast<uint32_t>(Q.end_max)) - e0;
        const int64_t vl = Q.vmin < 0 ? 0 : Q.vmin, vh = Q.vmax > 255 ? 255 : Q.vmax;
        vlo = vh < vl ? 256u : static_cast<uint32_t>(vl);
        vspan = vh < vl ? 0u : static_cast<uint32_t>(vh - vl);
        set_kind(Q.vt_kind);
        lut = st.sym_lut + Q.lut_off;
        // ALT0 lanes fetch their LUT word with ds_bpermute: no vector-memory
        // load inside a chunk, so a stream window is never drained for a symbolic ALT
        lutv = lut[min(static_cast<uint32_t>(lane_id()), 7u)];
        lut_lane = 0;
    }
    // the same from a chain descriptor's constants (ChainDev, computed on the
    // host exactly as above); LUT words already held in lanes lane0 .. lane0 + 7
    __device__ __forceinline__ VtPred(const DStore &st, uint32_t e0_, uint32_t espan_, uint32_t vlo_, uint32_t vspan_,
                                      uint32_t kind, uint32_t lut_off, uint32_t lutv_, uint32_t lane0) {
        e0 = e0_;
        espan = espan_;
        vlo = vlo_;
        vspan = vspan_;
        end_void = (kind & kChainEndVoid) != 0;
        set_kind(kind & 0xffu);
        lut = st.sym_lut + lut_off;
        lutv = lutv_;
        lut_lane = lane0;
    }
    // chain_pack_kernel: the constants precomputed per chain at setup, LUT words in LDS
    __device__ __forceinline__ VtPred(uint32_t e0_, uint32_t espan_, uint32_t vlo_, uint32_t vspan_, uint32_t cmask_,
                                      uint32_t xneed_, bool end_void_, const uint32_t *llut_) {
        e0 = e0_;
        espan = espan_;
        vlo = vlo_;
        vspan = vspan_;
        cmask = cmask_;
        xneed = xneed_;
        end_void = end_void_;
        lut = nullptr;
        lutv = 0;
        lut_lane = 0;
        llut = llut_;
    }
    __device__ __forceinline__ bool end_ok(uint32_t end) const { return !end_void && end - e0 <= espan; }
    // one ALT word + the LUT word its symbolic id falls in: predicate + length bounds
    __device__ __forceinline__ bool alt_ok(uint32_t aw, uint32_t lw) const {
        if ((aw & 0xffu) - vlo > vspan) return false;
        if (aw & VT_SYM) return (lw >> ((aw >> 16) & 31u)) & 1u;
        return (cmask >> ((aw >> VT_CLASS_SHIFT) & 31u)) & 1u;
    }
    // a lane whose word is not VT_SLOW (cand false: nothing); call with every lane active
    __device__ __forceinline__ LaneOut eval(const DStore &st, const VtHot h, uint32_t r, bool cand) const {
        LaneOut o{0, 0, 0, 0, 0};
        const uint32_t lw0 = llut ? llut[(h.w >> 21) & 7u]
                                  : static_cast<uint32_t>(__shfl(lutv, static_cast<int>(lut_lane + ((h.w >> 21) & 7u)), kWave));
        uint64_t hm = (cand && alt_ok(h.w, lw0)) ? 1ull : 0ull;
        const uint32_t nx = (cand && (h.w & xneed)) ? h.w >> VT_NX_SHIFT : 0u;
        uint32_t x0 = 0;
        if (__ballot(nx != 0) && nx) {  // ALTs 2..n (:124 loop)
            x0 = st.x_lo[r];
            for (uint32_t k = 0; k < nx; ++k) {
                const uint32_t xw = st.xvt[x0 + k];
                if (alt_ok(xw, (xw & VT_SYM) ? (llut ? llut[(xw >> 21) & 7u] : lut[(xw >> 21) & 7u]) : 0u))
                    hm |= 2ull << k;
            }
        }
        if (hm) {  // :205-214, AC of each matching ALT
            if (hm == 1ull) {
                o.c = h.ac0;
                o.em = h.ac0 != 0 ? 1ull : 0ull;
            } else {
                for (uint64_t b = hm; b; b &= b - 1) {
                    const int k = ffs64(b);
                    const int64_t v = k ? st.xrow[x0 + k - 1].ac : h.ac0;
                    o.c += v;
                    if (v != 0) o.em |= 1ull << k;
                }
            }
            o.hm = hm;
            o.anv = h.an;
        }
        return o;
    }
};

template <bool NONNEG>
__device__ __forceinline__ void vt_slice(DStore st, const QDev *__restrict__ qs, QRes *__restrict__ res,
                                         uint64_t *__restrict__ hits, uint32_t q, uint32_t lo, uint32_t hi,
                                         uint32_t c_lo, uint32_t c_hi_all) {
    const int lane = lane_id();
    const QDev &Q = qs[q];
    if (c_hi_all <= c_lo) {  // no candidate of this kind in the slice: nothing can hit or raise
        if (lane == 0) res[Q.orig] = QRes{0, 0, 0, 0, 0, hi - lo};
        return;
    }
    const uint32_t flags = Q.flags;
    const bool details = flags & F_DETAILS;
    const bool stop_on_exists = !details || (flags & F_BOOL_BREAK);
    ScanState S;
    const VtPred P(st, Q);
    uint64_t *out = hits + Q.hit_off;
    const QView V{flags, REF_ANY, ALT_VTYPE, false, false, nullptr, nullptr, nullptr};
    const uint32_t ul = static_cast<uint32_t>(lane);
    const uint32_t shi = P.end_void ? lo : hi;  // no END can match: nothing to scan
    auto lane_eval = [&](const VtHot h, uint32_t r, bool cand) -> LaneOut { return P.eval(st, h, r, cand); };
    // the slice's candidates of this variantType (VcBlock): positions [c_lo, c_hi),
    // mapped from [lo, hi) by the slice driver (VcAux); none if no END can match
    const uint32_t c_hi = shi > lo ? c_hi_all : c_lo;
    auto fast_chunk = [&](uint32_t base, const VcWord x) -> int {  // 0 go on, 1 stop, 2 has VT_SLOW lanes
        const bool cand = base + ul < c_hi && x.h.end - P.e0 <= P.espan;
        if (__ballot(cand && (x.h.w & VT_SLOW))) return 2;
        const LaneOut o = lane_eval(x.h, x.r, cand);
        uint64_t cm;
        return chunk_tail<NONNEG>(S, o, x.r, stop_on_exists, details, out, &cm) >= kWave ? 0 : 1;
    };
    // clamped, unconditional (used only when c_lo < c_hi); lanes past c_hi fail `cand`
    auto ld = [&](uint32_t i) -> VcWord {
        const uint32_t j = min(i, c_hi - 1);
        return VcWord{st.vc_word[j], st.vc_idx[j]};
    };
    uint32_t base = c_lo;
    const int status = c_lo < c_hi ? stream_window<kVtWindow, VcWord>(c_lo, c_hi, &base, ld, fast_chunk) : 0;
    if (status == 2) {  // the rest of the candidates one chunk at a time, eval_record for VT_SLOW lanes
        VcWord x = ld(base + ul);
        for (; base < c_hi; base += kWave) {
            const VcWord nx = ld(base + ul + kWave);
            const uint32_t r = x.r;
            const bool cand = base + ul < c_hi && x.h.end - P.e0 <= P.espan;
            const bool slow = cand && (x.h.w & VT_SLOW);
            LaneOut o = lane_eval(x.h, r, cand && !slow);
            if (__ballot(slow) && slow) o = eval_record(st, Q, V, r, st.rec[r]);
            uint64_t cm;
            if (chunk_tail<NONNEG>(S, o, r, stop_on_exists, details, out, &cm) < kWave) break;
            x = nx;
        }
    }
    finish_query<NONNEG>(S, st, Q, hi - lo, res);
}

// ---------------------------------------------------------------- packed variantType slices
// A variantType slice has a few candidates (about 3 % of its records), so a
// wave spent on one slice leaves most lanes idle and pays the chunk_tail /
// finish_query reductions per slice.  Here four slices of a run share one
// 64-lane pass, 16 lanes (candidates) each, with segmented sums and prefix
// counts over each 16-lane group.  A slice is packed only when its answer
// needs none of the order-dependent machinery: <= 16 candidates in its END
// window, include_details and no boolean break (nothing stops the loop,
// :229-232 / :253-254), a non-negative-AC store and no VT_SLOW candidate (no
// exception can occur).  Then exists = some hit has AC > 0 (the cumulative
// call_count of :229), call_count / all_alleles_count are sums over the hit
// records (:214, :244) and hits are written in record-then-ALT order --
// exactly what vt_slice + chunk_tail produce for it.  Other slices of the
// run go through vt_slice.
constexpr uint32_t kPackLanes = 16;
constexpr uint32_t kPackPasses = 2;  // a run's slices (kRun = 8) / 4 per pass

__device__ __forceinline__ int64_t seg16_sum_i64(int64_t v) {
#pragma unroll
    for (int m = 1; m < static_cast<int>(kPackLanes); m <<= 1) {
        const int lo = __shfl_xor(static_cast<int>(static_cast<uint64_t>(v) & 0xffffffffu), m, kWave);
        const int hi = __shfl_xor(static_cast<int>(static_cast<uint64_t>(v) >> 32), m, kWave);
        v += static_cast<int64_t>((static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
    }
    return v;
}

template <bool NONNEG>
struct VtPack {
    const DStore *st;
    const QDev *qs;
    QRes *res;
    uint64_t *hits;
    // q / bound / abound as run_slices holds them (lanes 2j, 2j+1 = slice j);
    // returns the mask of run slices answered here (wave-uniform)
    __device__ __forceinline__ uint32_t operator()(uint32_t n, uint32_t q, uint32_t bound, uint32_t abound) const {
        if constexpr (!NONNEG) {
            return 0u;
        } else {
            const DStore &D = *st;
            const uint32_t lane = static_cast<uint32_t>(lane_id());
            const uint32_t g = lane / kPackLanes, k = lane % kPackLanes;
            const uint64_t gm = 0xffffull << (kPackLanes * g);
            uint32_t handled = 0;
            // every load of both passes first (query fields, candidate words:
            // their addresses come from shuffles only), then the evaluation
            uint32_t a_lo[kPackPasses], a_hi[kPackPasses], a_alo[kPackPasses], a_ahi[kPackPasses];
            VcWord a_x[kPackPasses];
            QDev a_Q[kPackPasses];
#pragma unroll
            for (uint32_t p = 0; p < kPackPasses; ++p) {
                const uint32_t j = p * 4 + g;
                const bool vs = j < n;
                const int src = vs ? static_cast<int>(2 * j) : 0;
                const uint32_t qj = __shfl(q, src, kWave);
                a_lo[p] = __shfl(bound, src, kWave);
                a_hi[p] = max(a_lo[p], __shfl(bound, src + 1, kWave));
                a_alo[p] = __shfl(abound, src, kWave);
                a_ahi[p] = __shfl(abound, src + 1, kWave);
                const uint32_t span = a_ahi[p] > a_alo[p] ? a_ahi[p] - a_alo[p] : 0u;
                a_x[p] = VcWord{VtHot{0, 0, 0, 0}, 0};
                if (vs && k < span && span <= kPackLanes)  // inside the kind's list: safe to load early
                    a_x[p] = VcWord{D.vc_word[a_alo[p] + k], D.vc_idx[a_alo[p] + k]};
                const QDev &G = qs[qj];
                a_Q[p].flags = G.flags;
                a_Q[p].end_min = G.end_min;
                a_Q[p].end_max = G.end_max;
                a_Q[p].vmin = G.vmin;
                a_Q[p].vmax = G.vmax;
                a_Q[p].vt_kind = G.vt_kind;
                a_Q[p].lut_off = G.lut_off;
                a_Q[p].hit_off = G.hit_off;
                a_Q[p].orig = G.orig;
            }
#pragma unroll
            for (uint32_t p = 0; p < kPackPasses; ++p) {
                if (p * 4 >= n) break;
                const uint32_t j = p * 4 + g;
                const bool vs = j < n;
                const uint32_t lo = a_lo[p], hi = a_hi[p], alo = a_alo[p], ahi = a_ahi[p];
                const QDev &Q = a_Q[p];
                const uint32_t flags = Q.flags;
                const bool end_void = Q.end_max < 0 || Q.end_min > 0xffffffffll || Q.end_min > Q.end_max;
                // vt_slice: shi = end_void ? lo : hi; c_hi = shi > lo ? c_hi_all : c_lo
                const uint32_t c_hi = (!end_void && hi > lo) ? ahi : alo;
                const uint32_t ncand = c_hi > alo ? c_hi - alo : 0u;
                bool ok = vs && ncand <= kPackLanes && (flags & F_DETAILS) && !(flags & F_BOOL_BREAK);
                const bool has = ok && k < ncand;
                const VcWord x = a_x[p];
                const uint32_t e0 = Q.end_min < 0 ? 0u : static_cast<uint32_t>(Q.end_min);
                const uint32_t espan = (Q.end_max > 0xffffffffll ? 0xffffffffu : static_cast<uint32_t>(Q.end_max)) - e0;
                const bool cand = has && x.h.end - e0 <= espan;
                const uint64_t slowm = __ballot(cand && (x.h.w & VT_SLOW));
                ok = ok && !(slowm & gm);
                const uint64_t okm = __ballot(ok && k == 0);
                if (!okm) continue;
                // lane_eval of vt_slice with this lane's slice parameters
                LaneOut o{0, 0, 0, 0, 0};
                const int64_t vl = Q.vmin < 0 ? 0 : Q.vmin, vh = Q.vmax > 255 ? 255 : Q.vmax;
                const uint32_t vlo = vh < vl ? 256u : static_cast<uint32_t>(vl);
                const uint32_t vspan = vh < vl ? 0u : static_cast<uint32_t>(vh - vl);
                const uint32_t vk = Q.vt_kind;
                constexpr uint32_t kDel = vt_class_mask(VT_DEL), kIns = vt_class_mask(VT_INS),
                                   kDup = vt_class_mask(VT_DUP), kDupT = vt_class_mask(VT_DUPT),
                                   kCnv = vt_class_mask(VT_CNV);
                const uint32_t cmask = vk == VT_DEL ? kDel : vk == VT_INS ? kIns : vk == VT_DUP ? kDup
                                     : vk == VT_DUPT ? kDupT : vk == VT_CNV ? kCnv : 0u;
                const uint32_t xneed = vt_xk_bit(vk) | VT_XK_SYM;
                const uint32_t *lut = D.sym_lut + Q.lut_off;
                auto alt_ok = [&](uint32_t aw, uint32_t lw) -> bool {
                    if ((aw & 0xffu) - vlo > vspan) return false;
                    if (aw & VT_SYM) return (lw >> ((aw >> 16) & 31u)) & 1u;
                    return (cmask >> ((aw >> VT_CLASS_SHIFT) & 31u)) & 1u;
                };
                const bool ev = ok && cand;
                if (ev) {
                    const uint32_t lw0 = (x.h.w & VT_SYM) ? lut[(x.h.w >> 21) & 7u] : 0u;
                    uint64_t hm = alt_ok(x.h.w, lw0) ? 1ull : 0ull;
                    const uint32_t nx = (x.h.w & xneed) ? x.h.w >> VT_NX_SHIFT : 0u;
                    uint32_t x0 = 0;
                    if (nx) {  // ALTs 2..n (:124 loop)
                        x0 = D.x_lo[x.r];
                        for (uint32_t t = 0; t < nx; ++t) {
                            const uint32_t xw = D.xvt[x0 + t];
                            if (alt_ok(xw, (xw & VT_SYM) ? lut[(xw >> 21) & 7u] : 0u)) hm |= 2ull << t;
                        }
                    }
                    if (hm) {  // :205-214
                        if (hm == 1ull) {
                            o.c = x.h.ac0;
                            o.em = x.h.ac0 != 0 ? 1ull : 0ull;
                        } else {
                            for (uint64_t b = hm; b; b &= b - 1) {
                                const int a = ffs64(b);
                                const int64_t v = a ? D.xrow[x0 + a - 1].ac : x.h.ac0;
                                o.c += v;
                                if (v != 0) o.em |= 1ull << a;
                            }
                        }
                        o.hm = hm;
                        o.anv = x.h.an;
                    }
                }
                const bool hit = o.hm != 0;
                const uint32_t cnt = hit ? static_cast<uint32_t>(__popcll(o.em)) : 0u;
                uint32_t pos0, total;
                if (!__ballot(cnt > 1)) {
                    const uint64_t one = __ballot(cnt == 1) & gm;
                    pos0 = popc_below(one);
                    total = static_cast<uint32_t>(__popcll(one));
                } else {  // bit-sliced exclusive prefix within the 16-lane group
                    pos0 = 0;
                    total = 0;
                    for (uint32_t b = 0; b < 7; ++b) {
                        const uint64_t m = __ballot((cnt >> b) & 1u) & gm;
                        pos0 += popc_below(m) << b;
                        total += static_cast<uint32_t>(__popcll(m)) << b;
                        if (!__ballot(cnt >> (b + 1))) break;
                    }
                }
                if (cnt) {
                    uint64_t *dst = hits + Q.hit_off + pos0;
                    for (uint64_t b = o.em; b; b &= b - 1)
                        *dst++ = static_cast<uint64_t>(x.r) | (static_cast<uint64_t>(ffs64(b)) << kHitAltShift);
                }
                const int64_t cc = seg16_sum_i64(hit ? o.c : 0);
                const int64_t an = seg16_sum_i64(hit ? o.anv : 0);
                const bool ex = (__ballot(hit && o.c > 0) & gm) != 0ull;
                if (ok && k == 0) res[Q.orig] = QRes{0, ex ? 1 : 0, cc, an, total, hi - lo};
#pragma unroll
                for (uint32_t t = 0; t < 4; ++t)
                    if ((okm >> (kPackLanes * t)) & 1ull) handled |= 1u << (p * 4 + t);
            }
            return handled;
        }
    }
};

// no packed path
struct NoPack {
    __device__ __forceinline__ uint32_t operator()(uint32_t, uint32_t, uint32_t, uint32_t) const { return 0u; }
};

// Gather each query's hits from its planned region into a dense array
// (result shipping at fetch time; not part of the timed query step).
// ---------------------------------------------------------------- slice runs
// A wave answers `run` (<= kRun) consecutive entries of the (position-sorted)
// launch list; the host picks run per launch (run_for) so that a small batch
// still spreads over every SIMD.  One slice is only a few chunks of records, so a wave per slice would
// spend most of its life on dependent setup rounds (query, index bucket, POS
// probe) before its few data loads.  Here lanes 2j / 2j+1 fetch slice j's
// parameters and bracket its lower / upper bound together, the 64-wide POS
// probes of all 2*run bounds are issued at once, and the slices are then
// evaluated in order with their [lo, hi) already known: the setup latency is
// paid once per run.  Bounds are those of slice_bounds.
constexpr uint32_t kRun = 8;
static_assert(kPackPasses * (kWave / kPackLanes) == kRun, "packed passes cover a whole run");

template <class Body, class Aux, class Pack>
__device__ __forceinline__ void run_slices(const DStore &st, const QDev *__restrict__ qs,
                                           const uint32_t *__restrict__ qidx, uint32_t nq, uint32_t run, uint32_t w,
                                           Body body, Aux aux, Pack pack) {
    const uint32_t first = w * run;
    if (first >= nq) return;
    const uint32_t n = min(run, nq - first);
    const uint32_t lane = static_cast<uint32_t>(lane_id());
    const uint32_t j = lane >> 1;
    const bool upper = lane & 1u;
    uint32_t q = 0, L = 0, H = 0, done = 1;
    int64_t x = 0;
    if (j < n) {
        q = qidx ? qidx[first + j] : first + j;
        const QDev &Q = qs[q];
        if ((Q.flags & F_EMPTY) || Q.first_bp > Q.last_bp) {  // a <= POS <= b (:84-85)
            L = H = Q.seg_lo;
        } else {
            x = upper ? Q.last_bp + 1 : Q.first_bp;
            const Bracket k = bracket(st, Q, x);
            L = k.L;
            H = k.H;
            done = k.done ? 1u : 0u;
        }
    }
    const uint32_t nb = 2 * n;
    uint32_t v[2 * kRun];
#pragma unroll
    for (uint32_t k = 0; k < 2 * kRun; ++k) {
        v[k] = 0xffffffffu;
        if (k < nb) {
            const uint32_t i = rdl(L, k) + lane;
            if (!rdl(done, k) && i < rdl(H, k)) v[k] = st.pos[i];
        }
    }
    uint32_t bound = 0;  // lane k: bound k (record index)
#pragma unroll
    for (uint32_t k = 0; k < 2 * kRun; ++k) {
        if (k < nb) {
            const uint32_t Lk = rdl(L, k);
            const uint32_t b = rdl(done, k) ? Lk : finish_bound(st, Bracket{Lk, rdl(H, k), false}, rdl64(x, k), v[k]);
            if (lane == k) bound = b;
        }
    }
    // a per-bound companion value (aux(Q, bound), e.g. a candidate-list
    // position), computed by all bound lanes at once
    const uint32_t other = __shfl(bound, static_cast<int>(lane ^ 1u), kWave);  // the slice's other bound
    uint32_t abound = 0;
    if (lane < nb) abound = aux(qs[q], upper ? max(bound, other) : bound);
    const uint32_t packed = pack(n, q, bound, abound);  // run slices answered in packed passes
    for (uint32_t sj = 0; sj < n; ++sj) {
        if ((packed >> sj) & 1u) continue;
        const uint32_t lo = rdl(bound, 2 * sj);
        body(rdl(q, 2 * sj), lo, max(lo, rdl(bound, 2 * sj + 1)), rdl(abound, 2 * sj), rdl(abound, 2 * sj + 1));
    }
}

// one slice per wave (run == 1): fewer registers than run_slices, which
// matters when a launch has too few slices to amortise setup over runs
template <class Body, class Aux>
__device__ __forceinline__ void one_slice(const DStore &st, const QDev *__restrict__ qs,
                                          const uint32_t *__restrict__ qidx, uint32_t nq, uint32_t w, Body body,
                                          Aux aux) {
    if (w >= nq) return;
    const uint32_t q = qidx ? uniform(qidx[w]) : w;
    const QDev &Q = qs[q];
    uint32_t lo = Q.seg_lo, hi = Q.seg_lo;  // a <= POS <= b (:84-85)
    if (!(Q.flags & F_EMPTY) && Q.first_bp <= Q.last_bp) slice_bounds(st, Q, &lo, &hi);
    body(q, lo, hi, aux(Q, lo), aux(Q, hi));
}

// no companion value
struct NoAux {
    __device__ __forceinline__ uint32_t operator()(const QDev &, uint32_t) const { return 0; }
};

template <bool RUN, class Body, class Aux = NoAux, class Pack = NoPack>
__device__ __forceinline__ void slices(const DStore &st, const QDev *__restrict__ qs,
                                       const uint32_t *__restrict__ qidx, uint32_t nq, uint32_t run, uint32_t w,
                                       Body body, Aux aux = Aux(), Pack pack = Pack()) {
    if constexpr (RUN)
        run_slices(st, qs, qidx, nq, run, w, body, aux, pack);
    else
        one_slice(st, qs, qidx, nq, w, body, aux);
}

// MODE_VTYPE companion: a bound's position in the slice kind's candidate list
struct VcAux {
    const DStore *st;
    __device__ __forceinline__ uint32_t operator()(const QDev &Q, uint32_t r) const {
        return vc_count(*st, Q.vt_kind, r);
    }
};

// ---------------------------------------------------------------- launches
// wave index of this wave in a launch, XCD-aware (xcd_block)
__device__ __forceinline__ uint32_t launch_wave() {
    return uniform(xcd_block(blockIdx.x, gridDim.x) * kWavesPerBlock + (threadIdx.x >> 6));
}

template <int NACC, bool NONNEG, int MODE, bool RUN>
__global__ __launch_bounds__(kBlock) void scan_kernel(DStore st, const QDev *__restrict__ qs,
                                                      const uint32_t *__restrict__ qidx, uint32_t nq, uint32_t run,
                                                      const uint8_t *__restrict__ qbytes,
                                                      const uint64_t *__restrict__ subsets, QRes *__restrict__ res,
                                                      uint64_t *__restrict__ hits, uint64_t *__restrict__ samples_out) {
    slices<RUN>(st, qs, qidx, nq, run, launch_wave(), [&](uint32_t q, uint32_t lo, uint32_t hi, uint32_t alo, uint32_t ahi) {
        scan_slice<NACC, NONNEG, MODE>(st, qs, qbytes, subsets, res, hits, samples_out, q, lo, hi);
    });
}

// one specialisation per launch (a batch with a single sample-free group)
template <bool NONNEG, bool RUN>
__global__ __launch_bounds__(kBlock) void range_n_kernel(DStore st, const QDev *__restrict__ qs,
                                                         const uint32_t *__restrict__ qidx, uint32_t nq, uint32_t run,
                                                         QRes *__restrict__ res, uint64_t *__restrict__ hits) {
    slices<RUN>(st, qs, qidx, nq, run, launch_wave(), [&](uint32_t q, uint32_t lo, uint32_t hi, uint32_t alo, uint32_t ahi) {
        range_n_slice<NONNEG, RangeHot>(st, qs, res, hits, q, lo, hi);
    });
}

template <bool NONNEG, bool RUN>
__global__ __launch_bounds__(kBlock) void range_n8_kernel(DStore st, const QDev *__restrict__ qs,
                                                          const uint32_t *__restrict__ qidx, uint32_t nq, uint32_t run,
                                                          QRes *__restrict__ res, uint64_t *__restrict__ hits) {
    slices<RUN>(st, qs, qidx, nq, run, launch_wave(), [&](uint32_t q, uint32_t lo, uint32_t hi, uint32_t alo, uint32_t ahi) {
        range_n_slice<NONNEG, RangeHot8>(st, qs, res, hits, q, lo, hi);
    });
}

template <bool NONNEG, bool RUN>
__global__ __launch_bounds__(kBlock) void vt_kernel(DStore st, const QDev *__restrict__ qs,
                                                    const uint32_t *__restrict__ qidx, uint32_t nq, uint32_t run,
                                                    QRes *__restrict__ res, uint64_t *__restrict__ hits) {
    slices<RUN>(st, qs, qidx, nq, run, launch_wave(), [&](uint32_t q, uint32_t lo, uint32_t hi, uint32_t alo, uint32_t ahi) {
        vt_slice<NONNEG>(st, qs, res, hits, q, lo, hi, alo, ahi);
    }, VcAux{&st}, VtPack<NONNEG>{&st, qs, res, hits});
}

// All sample-free groups of a batch in one launch: group g owns waves
// [wave_begin[g], wave_begin[g+1]), rounded to whole workgroups so a block
// runs one specialisation.  Longest-running groups come first in the grid, so
// the short ones (point lookups) fill the others' tail instead of running
// after it in a second launch.
struct FusedGroups {
    const QDev *q[kFusedMax];  // group g's queries, in launch order
    uint32_t n[kFusedMax];
    uint32_t run[kFusedMax];
    uint32_t wave_begin[kFusedMax + 1];
    int mode[kFusedMax];
    int count;
};

template <bool NONNEG, bool RUN>
__global__ __launch_bounds__(kBlock) void fused_kernel(DStore st, FusedGroups G, const uint8_t *__restrict__ qbytes,
                                                       const uint64_t *__restrict__ subsets, QRes *__restrict__ res,
                                                       uint64_t *__restrict__ hits) {
    const uint32_t gw = launch_wave();
    int g = 0;
    while (g + 1 < G.count && gw >= G.wave_begin[g + 1]) ++g;
    const uint32_t w = gw - G.wave_begin[g];
    const int mode = G.mode[g];
    const QDev *qs = G.q[g];
    const auto aux = [&](const QDev &Q, uint32_t r) -> uint32_t {
        return mode == MODE_VTYPE ? vc_count(st, Q.vt_kind, r) : 0u;
    };
    slices<RUN>(st, qs, nullptr, G.n[g], G.run[g], w, [&](uint32_t q, uint32_t lo, uint32_t hi, uint32_t alo, uint32_t ahi) {
        switch (mode) {
            case MODE_RANGE_N: range_n_slice<NONNEG, RangeHot>(st, qs, res, hits, q, lo, hi); break;
            case MODE_RANGE_N8: range_n_slice<NONNEG, RangeHot8>(st, qs, res, hits, q, lo, hi); break;
            case MODE_VTYPE: vt_slice<NONNEG>(st, qs, res, hits, q, lo, hi, alo, ahi); break;
            case MODE_EXACT:
                scan_slice<0, NONNEG, MODE_EXACT>(st, qs, qbytes, subsets, res, hits, nullptr, q, lo, hi);
                break;
            default:
                scan_slice<0, NONNEG, MODE_GENERAL>(st, qs, qbytes, subsets, res, hits, nullptr, q, lo, hi);
                break;
        }
    }, aux);
}

// ---------------------------------------------------------------- slice chains
// A chain is the consecutive 10 kb slices one request was cut into by
// splitQuery, all with the same filters, none needing the order-dependent
// machinery (host-checked at prepare: include_details, no boolean break,
// non-negative AC, no VT_SLOW record in the window).  For such slices
// vt_slice's answer is: exists = some hit with AC > 0, call_count /
// all_alleles_count = sums over the hit records, hits in record-then-ALT
// order -- so a chain needs ONE candidate range, [C0, C1) from two entries of
// the (kind, segment) coarse POS index (chain_pack_kernel below).
struct ChainChunk {
    uint32_t p;  // candidate POS
    VtHot h;
    uint32_t r;  // candidate record
};

// Packed chain kernel: a run of up to kPackRun chains shares the wave's lanes
// (runs built on the host so a run's slices fit kPackSlots LDS slots).
// After the descriptor round (staged in LDS) and the bounds / LUT / corig
// round, the candidate ranges [C0_k, C1_k) of the run's chains are laid end
// to end (prefix pex); lane L of chunk c takes global candidate g = 64 c + L,
// i.e. the last chain k with pex_k <= g.  A run's candidates then fill few
// chunks, and every chunk load of the run is issued before the first is
// evaluated (kPackAhead in flight).  Per-slice sums live in LDS at the
// run-flattened slot of (chain, slice); each chain's hits stay dense and in
// record order: its lanes are contiguous within a chunk, so the in-chain
// prefix is a masked popcount and the chain's running count (lane k of
// noutv) advances by the popcount over its lane range.  exists =
// call_count > 0 (chains need a non-negative-AC store).  The slot and LUT
// tables keep the per-chain work off the VALU: the kernel is issue-bound
// (SQ counters, profiles/r02_pmc_chain).
constexpr int kPackAhead = 3;     // candidate chunks in flight (a chunk's load is issued kPackAhead chunks ahead)
constexpr uint32_t kPackRun = 32;  // chains per wave at most
constexpr uint32_t kPackSlots = 256;  // slices per run at most (host-enforced)

// SLICES: per-slice sums (the per-slice QRes rows); without them (request
// rows only) a slice keeps one "exists" bit and the chain its totals, which
// frees the LDS for occupancy
template <bool SLICES>
struct PackLds {
    uint4 desc[kPackRun * 5];  // the run's ChainDev descriptors
    unsigned long long cc[SLICES ? kPackSlots : 1], an[SLICES ? kPackSlots : 1];
    unsigned int nh[SLICES ? kPackSlots : 1];
    unsigned int exw[kPackSlots / 32];  // !SLICES: bit = the slot's slice exists
    uint32_t lut[kPackRun * 8];  // each chain's symbolic-ALT LUT words
    unsigned long long tcc[kPackRun], tan[kPackRun];
    unsigned int slow[kPackRun];
};

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

struct PackChunk {
    ChainChunk x;
    uint32_t k;  // the lane's chain
};

// last lane j < R <= RUN (lanes hold a nondecreasing prefix v) with v_j <= g
template <uint32_t RUN = kPackRun>
__device__ __forceinline__ uint32_t last_le(uint32_t v, uint32_t R, uint32_t g) {
    uint32_t lo = 0;
#pragma unroll
    for (uint32_t step = RUN / 2; step >= 1; step >>= 1) {
        const uint32_t t = lo + step;
        const uint32_t vt = static_cast<uint32_t>(__shfl(static_cast<int>(v), static_cast<int>(min(t, RUN - 1)), kWave));
        if (t < R && vt <= g) lo = t;
    }
    return lo;
}

template <bool SLICES>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(SLICES ? 4 : 8, 8))) void chain_pack_kernel(DStore st, const ChainDev *__restrict__ chains,
                                                            const uint32_t *__restrict__ runs, uint32_t n_runs,
                                                            const uint32_t *__restrict__ corig,
                                                            QRes *__restrict__ res, uint64_t *__restrict__ hits,
                                                            ReqPartial *__restrict__ cpart) {
    __shared__ PackLds<SLICES> lds_all[kWavesPerBlock];
    const uint32_t w = launch_wave();
    if (w >= n_runs) return;
    const uint32_t c_first = uniform(runs[w]);
    const uint32_t R = uniform(runs[w + 1]) - c_first;  // 1 .. kPackRun
    PackLds<SLICES> &L = lds_all[threadIdx.x >> 6];
    const uint32_t ul = static_cast<uint32_t>(lane_id());
    // round 1: the run's descriptors (5 x 16 B per chain), staged in LDS
    {
        const uint4 *cd = reinterpret_cast<const uint4 *>(chains + c_first);
        constexpr uint32_t kDw = (kPackRun * 5 + kWave - 1) / kWave;  // descriptor words per lane
        uint4 dw[kDw];
#pragma unroll
        for (uint32_t q = 0; q < kDw; ++q) dw[q] = ul + kWave * q < 5 * R ? cd[ul + kWave * q] : uint4{0, 0, 0, 0};
#pragma unroll
        for (uint32_t q = 0; q < kDw; ++q)
            if (ul + kWave * q < 5 * R) L.desc[ul + kWave * q] = dw[q];
        if (ul < kPackRun) {
            L.tcc[ul] = 0;
            L.tan[ul] = 0;
            L.slow[ul] = 0;
        }
        if (ul < kPackSlots / 32) L.exw[ul] = 0;
    }
    wave_lds_sync();
    // lane j < R: chain j's slice count and slot prefix (sex / sin)
    uint32_t nv = 0, sin = 0, sex = 0;
    {
        nv = ul < R ? L.desc[5 * ul].y : 0u;
        sin = nv;
#pragma unroll
        for (int d = 1; d < static_cast<int>(kPackRun); d <<= 1) {
            const uint32_t t = __shfl_up(sin, d, kWave);
            if (ul >= static_cast<uint32_t>(d)) sin += t;
        }
        sex = sin - nv;
    }
    const uint32_t S = rdl(sin, kPackRun - 1);  // slots in use (<= kPackSlots, host-enforced)
    // round 2: lanes 2k / 2k+1 = chain k's candidate bounds; every chain's
    // LUT words into LDS; lane t = corig of slot t; zero the used slots
    uint32_t bound = 0;
    {
        const uint32_t kb = min(ul >> 1, R - 1);
        const uint4 b0 = L.desc[5 * kb], b1 = L.desc[5 * kb + 1], b2 = L.desc[5 * kb + 2];
        if (ul < 2 * R) {
            const uint32_t up = ul & 1u;
            const uint64_t x = up ? static_cast<uint64_t>(b0.w) + 1 : b0.z;  // last + 1 / first
            const uint32_t c_lo = b1.y, c_hi = b1.z, cb_base = b1.w;
            const uint64_t cb_off = static_cast<uint64_t>(b2.x) | (static_cast<uint64_t>(b2.y) << 32);
            if (x <= cb_base) {
                bound = c_lo;
            } else {
                const uint64_t b = (x - cb_base) >> b2.z;
                bound = b >= b2.w ? c_hi : st.vc_bucket[cb_off + b + up];
            }
        }
#pragma unroll
        for (uint32_t h = 0; h < kPackRun * 8 / kWave; ++h) {
            const uint32_t t = ul + kWave * h;  // word t & 7 of chain t >> 3
            const uint32_t kl = min(t >> 3, R - 1);
            L.lut[t] = st.sym_lut[L.desc[5 * kl + 4].y + (t & 7u)];
        }
    }
    uint32_t orig[kPackSlots / kWave];  // slot ul + 64 t (res == nullptr: request rows only, no per-slice QRes)
#pragma unroll
    for (uint32_t t = 0; t < kPackSlots / kWave; ++t) {
        orig[t] = 0;
        if (kWave * t < S) {
            const uint32_t slot = min(ul + kWave * t, S - 1);
            if constexpr (SLICES) {
                const uint32_t k = last_le(sex, R, slot);
                const uint32_t sk = __shfl(sex, static_cast<int>(k), kWave);  // every lane active
                if (ul + kWave * t < S) {
                    orig[t] = corig[L.desc[5 * k].x + (slot - sk)];
                    L.cc[slot] = 0;
                    L.an[slot] = 0;
                    L.nh[slot] = 0;
                }
            }
        }
    }
    // the chains' candidate ranges laid end to end; lane j < R holds chain
    // j's first candidate (c0v), its prefix (pex: exclusive, pin: inclusive)
    uint32_t c0v = 0, pex = 0, pin = 0;
    {
        const uint32_t j = min(ul, R - 1);
        const uint32_t lo = __shfl(bound, static_cast<int>(2 * j), kWave);
        const uint32_t hi = __shfl(bound, static_cast<int>(2 * j + 1), kWave);
        const bool void_end = (L.desc[5 * j + 4].x & kChainEndVoid) != 0;
        c0v = lo;
        const uint32_t cnt = (ul < R && !void_end) ? max(lo, hi) - lo : 0u;
        pin = cnt;
#pragma unroll
        for (int d = 1; d < static_cast<int>(kPackRun); d <<= 1) {
            const uint32_t t = __shfl_up(pin, d, kWave);
            if (ul >= static_cast<uint32_t>(d)) pin += t;
        }
        pex = pin - cnt;
        // lane j < R: chain j's per-candidate constants in its descriptor's
        // setup-only words (read above, in program order): word 1.y = 1 /
        // width (f32), word 4.x = the kind's class mask, word 4.y = the
        // extra-ALT bits | end_void << 31 (the LUT offset is not needed: the
        // LUT words are in LDS)
        if (ul < R) {
            const uint32_t kind = L.desc[5 * ul + 4].x;
            VtPred q(st, 0u, 0u, 0u, 0u, kind, 0u, 0u, 0u);
            L.desc[5 * ul + 1].y = __float_as_uint(__frcp_rn(static_cast<float>(L.desc[5 * ul + 1].x)));
            L.desc[5 * ul + 4].x = q.cmask;
            L.desc[5 * ul + 4].y = q.xneed | (q.end_void ? 0x80000000u : 0u);
        }
    }
    wave_lds_sync();
    const uint32_t T = rdl(pin, kPackRun - 1);
    const uint32_t i_safe = rdl(c0v, 0);  // a valid slot (inside the kind lists + sentinel)
    auto load = [&](uint32_t base) -> PackChunk {
        const uint32_t g = base + ul;
        uint32_t k = 0, i = i_safe;
        if (base < T) {  // wave-uniform; the load itself is issued either way
            k = last_le(pex, R, g);
            const uint32_t c0 = __shfl(c0v, static_cast<int>(k), kWave), p = __shfl(pex, static_cast<int>(k), kWave);
            if (g < T) i = c0 + (g - p);
        }
        return PackChunk{ChainChunk{st.vc_pos[i], st.vc_word[i], st.vc_idx[i]}, k};
    };
    uint32_t noutv = 0;  // lane j: hits chain j has written so far
    auto lanes_from = [](uint32_t a) -> uint64_t { return a >= 64 ? 0ull : (~0ull << a); };
    auto lanes_below = [](uint32_t b) -> uint64_t { return b >= 64 ? ~0ull : ((1ull << b) - 1ull); };
    auto eval = [&](const PackChunk &c, uint32_t base) {
        const ChainChunk &x = c.x;
        const uint32_t k = c.k;
        const uint32_t g = base + ul;
        const bool valid = g < T;
        const uint4 e0 = L.desc[5 * k], e1 = L.desc[5 * k + 1], e3 = L.desc[5 * k + 3], e4 = L.desc[5 * k + 4];
        const uint32_t first = e0.z, last = e0.w, n = e0.y, width = e1.x;
        VtPred Pd(e3.x, e3.y, e3.z, e3.w, e4.x, e4.y & 0x7fffffffu, (e4.y >> 31) != 0, &L.lut[8 * k]);
        const bool inwin = valid && x.p >= first && x.p <= last;
        const bool cand = inwin && Pd.end_ok(x.h.end);
        if (cand && (x.h.w & VT_SLOW)) L.slow[k] = 1u;  // never: prepare dissolves such chains
        const LaneOut o = Pd.eval(st, x.h, x.r, cand && !(x.h.w & VT_SLOW));
        const bool hit = o.hm != 0;
        if (!__ballot(hit)) return;
        // slice = (POS - first) / width: f32 estimate within one of the quotient, then exact
        uint32_t sid = 0;
        if (inwin) {
            const uint32_t d = x.p - first;
            uint32_t q;
            if (d < (1u << 24)) {
                q = static_cast<uint32_t>(static_cast<float>(d) * __uint_as_float(e1.y));  // 1 / width (setup)
                if (static_cast<uint64_t>(q) * width > d) --q;
                else if (static_cast<uint64_t>(q + 1) * width <= d) ++q;
            } else {
                q = d / width;
            }
            sid = min(q, n - 1);
        }
        const uint32_t cnt = hit ? static_cast<uint32_t>(__popcll(o.em)) : 0u;
        const uint32_t pk = __shfl(pex, static_cast<int>(k), kWave);
        const uint32_t before = __shfl(noutv, static_cast<int>(k), kWave);
        const uint32_t slot = __shfl(sex, static_cast<int>(k), kWave) + sid;
        const uint64_t mine = lanes_from(pk > base ? pk - base : 0u) & ((1ull << ul) - 1ull);  // chain k's lanes below
        // lane j < R: chain j's lanes in this chunk
        const uint64_t mj = lanes_from(pex > base ? pex - base : 0u) & lanes_below(pin > base ? pin - base : 0u);
        uint32_t pre = 0, add = 0;
        if (!__ballot(cnt > 1)) {
            const uint64_t one = __ballot(cnt == 1);
            pre = static_cast<uint32_t>(__popcll(one & mine));
            add = static_cast<uint32_t>(__popcll(one & mj));
        } else {  // bit-sliced (multi-ALT hit lanes)
            for (uint32_t bb = 0; bb < 7; ++bb) {
                const uint64_t m = __ballot((cnt >> bb) & 1u);
                pre += static_cast<uint32_t>(__popcll(m & mine)) << bb;
                add += static_cast<uint32_t>(__popcll(m & mj)) << bb;
                if (!__ballot(cnt >> (bb + 1))) break;
            }
        }
        if (ul < R) noutv += add;
        if (cnt) {
            const uint64_t out = static_cast<uint64_t>(e4.z) | (static_cast<uint64_t>(e4.w) << 32);
            uint64_t *dst = hits + out + before + pre;
            for (uint64_t b = o.em; b; b &= b - 1)
                *dst++ = static_cast<uint64_t>(x.r) | (static_cast<uint64_t>(ffs64(b)) << kHitAltShift);
            if constexpr (SLICES) atomicAdd(&L.nh[slot], cnt);
        }
        if (hit) {
            if constexpr (SLICES) {
                atomicAdd(&L.cc[slot], static_cast<unsigned long long>(o.c));
                atomicAdd(&L.an[slot], static_cast<unsigned long long>(o.anv));
            } else {
                if (o.c > 0) atomicOr(&L.exw[slot >> 5], 1u << (slot & 31u));
                atomicAdd(&L.tcc[k], static_cast<unsigned long long>(o.c));
                atomicAdd(&L.tan[k], static_cast<unsigned long long>(o.anv));
            }
        }
    };
    // every chunk of the run issued before the first is evaluated
    {
        // software pipeline: chunk c + kPackAhead's loads are issued right
        // after chunk c is evaluated (static buffer slots: unrolled by kPackAhead)
        PackChunk buf[kPackAhead];
#pragma unroll
        for (int a = 0; a < kPackAhead; ++a) buf[a] = load(64u * a);
        for (uint32_t base = 0; base < T; base += 64u * kPackAhead) {
#pragma unroll
            for (int a = 0; a < kPackAhead; ++a) {
                const uint32_t b = base + 64u * a;
                if (b < T) {
                    eval(buf[a], b);
                    if (b + 64u * kPackAhead < T) buf[a] = load(b + 64u * kPackAhead);
                }
            }
        }
    }
    wave_lds_sync();
    if constexpr (SLICES) {
        // results: lane ul + 64 t = slot; chain totals by slot atomics
        uint64_t exm_all[kPackSlots / kWave];
#pragma unroll
        for (uint32_t t = 0; t < kPackSlots / kWave; ++t) {
            exm_all[t] = 0;
            if (kWave * t < S) {
                const uint32_t slot = min(ul + kWave * t, S - 1);
                const bool sl = ul + kWave * t < S;
                const uint32_t k = last_le(sex, R, slot);
                const int64_t cc = sl ? static_cast<int64_t>(L.cc[slot]) : 0;
                const int64_t an = sl ? static_cast<int64_t>(L.an[slot]) : 0;
                const uint32_t nh = sl ? L.nh[slot] : 0u;
                exm_all[t] = __ballot(sl && cc > 0);
                if (sl && res) {
                    QRes o{0, 0, 0, 0, 0, 0};  // n_scanned: filled on the host
                    if (L.slow[k]) {
                        o.error = SB_QERR_UNSUPPORTED;
                    } else {
                        o.exists = cc > 0 ? 1 : 0;
                        o.call_count = cc;
                        o.all_alleles_count = an;
                        o.n_hits = nh;
                    }
                    res[orig[t]] = o;
                }
                if (sl && cpart && (cc | an)) {
                    atomicAdd(&L.tcc[k], static_cast<unsigned long long>(cc));
                    atomicAdd(&L.tan[k], static_cast<unsigned long long>(an));
                }
            }
        }
        if (cpart) {
            wave_lds_sync();
            if (ul < R) {
                // exists count of chain ul: its slots [sex, sin) in the flattened order
                int64_t ex = 0;
#pragma unroll
                for (uint32_t t = 0; t < kPackSlots / kWave; ++t) {
                    const uint32_t a = sex > kWave * t ? sex - kWave * t : 0u, b = sin > kWave * t ? sin - kWave * t : 0u;
                    ex += __popcll(exm_all[t] & lanes_from(a) & lanes_below(b));
                }
                cpart[c_first + ul] = L.slow[ul] ? ReqPartial{0, 0, 0, 0, static_cast<int64_t>(nv)}
                                                 : ReqPartial{ex, static_cast<int64_t>(noutv),
                                                              static_cast<int64_t>(L.tcc[ul]),
                                                              static_cast<int64_t>(L.tan[ul]), 0};
            }
        }
    } else if (ul < R) {  // request rows only: chain ul's partial from its exists bits and totals
        int64_t ex = 0;
#pragma unroll
        for (uint32_t q = 0; q < kPackSlots / 32; ++q) {
            const uint32_t a = sex > 32 * q ? min(sex - 32 * q, 32u) : 0u, b = sin > 32 * q ? min(sin - 32 * q, 32u) : 0u;
            const uint32_t m = (b >= 32 ? ~0u : ((1u << b) - 1u)) & (a >= 32 ? 0u : (~0u << a));
            ex += __popc(L.exw[q] & m);
        }
        cpart[c_first + ul] = L.slow[ul] ? ReqPartial{0, 0, 0, 0, static_cast<int64_t>(nv)}
                                         : ReqPartial{ex, static_cast<int64_t>(noutv), static_cast<int64_t>(L.tcc[ul]),
                                                      static_cast<int64_t>(L.tan[ul]), 0};
    }
}

// Hit-region offsets of chained slices (their hits are dense per chain, in
// slice order): src[orig] = chain out + the n_hits of the chain's earlier slices.
__global__ __launch_bounds__(kBlock) void chain_src_kernel(const ChainDev *__restrict__ chains, uint32_t n_chains,
                                                           const uint32_t *__restrict__ corig,
                                                           const QRes *__restrict__ res, uint64_t *__restrict__ src) {
    const uint32_t c = blockIdx.x * kBlock + threadIdx.x;
    if (c >= n_chains) return;
    const ChainDev C = chains[c];
    uint64_t at = C.out;
    for (uint32_t j = 0; j < C.n; ++j) {
        const uint32_t q = corig[C.s0 + j];
        src[q] = at;
        at += res[q].error ? 0u : res[q].n_hits;
    }
}

// ---------------------------------------------------------------- request rows
// Request batches (sb_requests_run, devtypes.hpp RowRun), three launches:
//
// request_eval_kernel -- one wave per run of consecutive request rows with up
// to kReqRun (64) chains (XCD-aware block order; no inter-wave dependency).
// Lane k holds chain k: its candidate range laid end to end with the run's
// other chains (positions [pex, pin) of the run's T positions).  A chunk of 64
// positions is evaluated per step, lane L taking position 64 c + L:
//   * its chain: the chain-start bitmap of the chunk (built once per wave in
//     LDS, then held one word per lane; chunks past the 64th collect their
//     few starts by ballot) read with v_readlane into SGPRs; the lane's chain
//     = the chunk's first chain + v_mbcnt of the starts at or below it -- two
//     VALU, no LDS round trip, no search;
//   * its candidate: index = position + the chain's delta (one LDS read), the
//     three candidate columns loaded PIPE chunks ahead;
//   * the predicate of lambda/performQuery/search_variants.py:100-183 (the
//     variantType branch, patched-oracle intent) with the chain's constants
//     from two 16-byte LDS words; hits staged in candidate order = chain order
//     = row order (ballot + mbcnt);
//   * per-chain sums without atomics: inclusive DPP scans over the chunk of
//     the hit count, the new-slice count (a positive hit whose 10 kb slice
//     differs from the previous positive hit's: max-scan of slice keys), the
//     call count and the AN sum; lane k then pulls the scans at its chain's
//     last lane in the chunk (ds_bpermute) and subtracts chain k-1's (DPP
//     wave_shr) -- chain k's part of the chunk, added to lane-held totals.
// The wave writes its rows, each row's hit count (into row_cnt), the staging
// start of rows answered row by row, and the run's total as a status word.
//
// request_tile_scan_kernel -- the runs' totals, summed per tile of 16 runs, into tile offsets.
//
// request_deliver_kernel -- one wave per run: the run's output offset (its
// tile's offset + the earlier runs' totals of the tile), row offsets, and the
// hits copied to the dense output: one contiguous copy for a run of chain rows
// only; row by row where some rows were answered per slice (queries of the
// batch's slice part, reduced into `rows` by request_reduce before the first
// kernel).
//
// Measured forms this replaces: chains found by a
// binary search over lane-held prefixes (5 dependent ds_bpermutes per chunk)
// and per-chain sums by contended 64-bit LDS atomics, 32 chains per run.

// the batch's symbolic-ALT LUT words (8 per distinct variantType string) are
// staged in LDS once per workgroup when they fit: a predicate's LUT word is
// then an LDS read, not a dependent global load behind the candidate's load
constexpr uint32_t kReqLut = 512;
constexpr uint32_t kDeliverTile = 16;  // runs per request_deliver_kernel wave
#ifndef SBEACON_REQ_PIPE
#define SBEACON_REQ_PIPE 2
#endif
#ifndef SBEACON_REQ_WAVES
#define SBEACON_REQ_WAVES 8
#endif
constexpr int kReqPipe = SBEACON_REQ_PIPE;  // candidate chunks in flight per wave

// DPP lane moves (GFX9 controls; lanes without a source read 0)
template <int CTRL, int ROW = 0xf, int BANK = 0xf>
__device__ __forceinline__ uint32_t dpp32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROW, BANK, false));
}
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) { return dpp32<0x138>(v); }  // lane i <- lane i - 1 (lane 0: 0)
__device__ __forceinline__ uint64_t wave_shr1_64(uint64_t v) {
    return (static_cast<uint64_t>(wave_shr1(static_cast<uint32_t>(v >> 32))) << 32) | wave_shr1(static_cast<uint32_t>(v));
}
// inclusive scans over the wave: row_shr 1, 2, 4, 8 inside rows of 16, then
// row_bcast 15 / 31 across rows (the GFX9 sequence; no LDS)
__device__ __forceinline__ uint32_t incl_sum_u32(uint32_t v) {
    v += dpp32<0x111>(v);
    v += dpp32<0x112>(v);
    v += dpp32<0x114>(v);
    v += dpp32<0x118>(v);
    v += dpp32<0x142, 0xa>(v);
    v += dpp32<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ uint32_t incl_max_u32(uint32_t v) {
    v = max(v, dpp32<0x111>(v));
    v = max(v, dpp32<0x112>(v));
    v = max(v, dpp32<0x114>(v));
    v = max(v, dpp32<0x118>(v));
    v = max(v, dpp32<0x142, 0xa>(v));
    v = max(v, dpp32<0x143, 0xc>(v));
    return v;
}
// the two scans of a chunk side by side: inclusive max of m, inclusive sum of v
__device__ __forceinline__ void incl_max_sum_u32(uint32_t m, uint32_t v, uint32_t &mo, uint32_t &vo) {
    m = max(m, dpp32<0x111>(m));
    v += dpp32<0x111>(v);
    m = max(m, dpp32<0x112>(m));
    v += dpp32<0x112>(v);
    m = max(m, dpp32<0x114>(m));
    v += dpp32<0x114>(v);
    m = max(m, dpp32<0x118>(m));
    v += dpp32<0x118>(v);
    m = max(m, dpp32<0x142, 0xa>(m));
    v += dpp32<0x142, 0xa>(v);
    m = max(m, dpp32<0x143, 0xc>(m));
    v += dpp32<0x143, 0xc>(v);
    mo = m;
    vo = v;
}
__device__ __forceinline__ uint64_t incl_sum_u64(uint64_t v) {
    v += static_cast<uint64_t>(dpp_i64<0x111, 0xf, 0xf>(static_cast<int64_t>(v)));
    v += static_cast<uint64_t>(dpp_i64<0x112, 0xf, 0xf>(static_cast<int64_t>(v)));
    v += static_cast<uint64_t>(dpp_i64<0x114, 0xf, 0xf>(static_cast<int64_t>(v)));
    v += static_cast<uint64_t>(dpp_i64<0x118, 0xf, 0xf>(static_cast<int64_t>(v)));
    v += static_cast<uint64_t>(dpp_i64<0x142, 0xa, 0xf>(static_cast<int64_t>(v)));
    v += static_cast<uint64_t>(dpp_i64<0x143, 0xc, 0xf>(static_cast<int64_t>(v)));
    return v;
}
__device__ __forceinline__ uint32_t bperm(uint32_t v, uint32_t lane) {
    return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(static_cast<int>(lane << 2), static_cast<int>(v)));
}
__device__ __forceinline__ uint64_t bperm64(uint64_t v, uint32_t lane) {
    return (static_cast<uint64_t>(bperm(static_cast<uint32_t>(v >> 32), lane)) << 32) | bperm(static_cast<uint32_t>(v), lane);
}

struct ReqLds {
    // (a, b and wch hold a simple run's 64 rows of 40 B after the candidate loop)
    uint4 a[kReqRun];  // chain k: {candidate index - run position, first, last - first, e0}
    uint4 b[kReqRun];  // {espan, vlo | vspan << 9 | LUT offset << 17, class mask, extra-ALT bits that may match}
    unsigned long long wch[kReqStartChunks];  // chunk c: bit j = a chain's first position is 64 c + j
    unsigned int slow[kReqRun / 32];          // bit = a VT_SLOW candidate in the chain's window
    uint8_t rowchain[kRunRows];               // row (run-relative) -> its chain (0xff: not a chain row)
};

struct ReqChunk {
    VcQ q;       // the candidate's POS, END, VtHot word and ALT0 AC: one 16-byte load
    int32_t an;  // its record's AN (loaded only by runs without a common AN)
    uint32_t i;  // staged as the hit: the candidate's record (REC), else its index (the deliver maps it)
    uint32_t k;  // the lane's chain
};

static_assert(offsetof(ReqLds, b) == sizeof(uint4) * kReqRun && offsetof(ReqLds, wch) == 2 * sizeof(uint4) * kReqRun &&
                  offsetof(ReqLds, slow) >= kRunRows * sizeof(ReqPartial),
              "a, b, wch are one block that holds a run's rows");
// One run's planning (request_plan_kernel's, below, without the capacity
// sums): lane = row; the chain descriptors packed into slots (rows with
// candidates first, in row order, then those without, then first == 0 slots)
// and written to `slots` (LDS, 64 x 32 B); returns the run record
__device__ __forceinline__ RowRun plan_run(const DStore &st, const ReqIn *__restrict__ in, uint32_t n, uint32_t w,
                                           uint64_t stride, ReqChain *slots, uint32_t ul) {
    const uint32_t row = w * kRunRows + ul;
    ReqIn q{};
    if (row < n) q = in[row];
    const uint32_t cls = row < n ? (q.cls & 3u) : static_cast<uint32_t>(REQ_NONE);
    const bool chain = cls == REQ_CHAIN;
    uint32_t c0 = 0, c1 = 0, vi_xinfo = 0;
    if (chain) {
        const VcIndex vi = st.vcx[static_cast<uint64_t>(q.seg) * kVtKinds + ((q.bits >> 23) & 7u)];
        c0 = vc_bound(vi, st.vc_bucket, q.first, 0);
        c1 = (q.bits >> 26) & 1u ? c0 : max(c0, vc_bound(vi, st.vc_bucket, static_cast<uint64_t>(q.last) + 1, 1));
        vi_xinfo = vi.xinfo;
    }
    const bool ne = chain && c1 > c0;
    const uint64_t mne = __ballot(ne), mem = __ballot(chain && !ne);
    const uint32_t nne = static_cast<uint32_t>(__popcll(mne)), nslots = nne + static_cast<uint32_t>(__popcll(mem));
    if (chain) {
        const uint32_t slot = ne ? popc_below(mne) : nne + popc_below(mem);
        slots[slot] = ReqChain{q.first, q.last, c0, c1, q.e0, q.espan, q.bits | (ul << 17), q.lut_off};
    }
    if (ul >= nslots) slots[ul] = ReqChain{0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t nsl = chain ? q.cls >> 2 : 0u;
    const uint32_t slsum = rdl(incl_sum_u32(nsl), kWave - 1);
    const bool simple = __ballot(cls == REQ_SLICES) == 0;
    const uint32_t xi = ne ? vi_xinfo : kVcNarrow;
    const bool narrow = __ballot(!(xi & kVcNarrow)) == 0;
    const uint32_t a = xi & kVcAnMask;
    const uint32_t a0 = mne ? rdl(a, static_cast<uint32_t>(ffs64(mne))) : 1u;
    const bool anc = narrow && a0 != 0u && __ballot(ne && a != a0) == 0;
    const uint32_t flags = (simple ? kRunSimple : 0u) | (narrow ? kRunNarrow : 0u) |
                           (anc ? kRunAnCommon | (a0 - 1u) << kRunAnShift : 0u);
    wave_lds_sync();
    return RowRun{w * kRunRows, min(w * kRunRows + kRunRows, n), 0u, nslots, stride * w, slsum, flags};
}

// COMPACT (sb_requests_set_compact): rows as RowC (16 B), row counts /
// offsets as u32; only batches without a per-slice part (sres == nullptr)
// REC: hits are staged as their record numbers (the store's records fit 29
// bits): the record id is loaded with the candidate word, coalesced, and
// request_deliver_kernel copies without a per-hit gather; else the
// candidate index is staged and the deliver maps it (vc_idx)
// PLAN: the run is planned in the wave itself (a re-planning pass of a
// fixed-stride batch: plan_run below, request_plan_kernel's work) from the
// resident packed requests, its chain descriptors passed through LDS instead
// of HBM, its run record written for request_deliver_kernel -- one launch
// and 64 B per request fewer, the planner's dependent index loads hidden
// behind other waves' candidate work
template <bool LDS_LUT, bool COMPACT, bool REC, bool PLAN>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(SBEACON_REQ_WAVES, SBEACON_REQ_WAVES))) void request_eval_kernel(
    DStore st, const ReqChain *__restrict__ chains, RowRun *__restrict__ runs, uint32_t n_runs,
    unsigned long long *__restrict__ status, const QRes *__restrict__ sres, void *__restrict__ rows_out,
    void *__restrict__ row_cnt_out, uint64_t *__restrict__ row_src, uint32_t *__restrict__ stage, uint32_t n_lut,
    unsigned int *__restrict__ err, uint32_t inject, unsigned long long *__restrict__ gtot,
    const ReqIn *__restrict__ in, uint32_t n_in, uint64_t stride, ReqEsc esc) {
    ReqPartial *const rows = static_cast<ReqPartial *>(rows_out);
    uint64_t *const row_cnt = static_cast<uint64_t *>(row_cnt_out);
    __shared__ ReqLds lds_all[kWavesPerBlock];
    __shared__ uint32_t slut[LDS_LUT ? kReqLut : 1];
    // the workgroup's run totals: the last wave to finish writes their sum
    // (gtot[group], request_tile_scan_kernel), counted by an LDS atomic --
    // no barrier, a finished wave leaves at once
    __shared__ unsigned long long s_tot[kWavesPerBlock];
    __shared__ uint32_t s_done;
    ReqLds &L = lds_all[threadIdx.x >> 6];
    const uint32_t ul = static_cast<uint32_t>(lane_id());
    const uint32_t w = launch_wave();
    auto finish = [&](uint64_t H) {  // lane 0
        s_tot[threadIdx.x >> 6] = H;
        if (__hip_atomic_fetch_add(&s_done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP) == kWavesPerBlock - 1) {
            uint64_t t = 0;
#pragma unroll
            for (uint32_t k = 0; k < kWavesPerBlock; ++k) t += s_tot[k];
            gtot[w / kWavesPerBlock] = t;
        }
    };
    // the run record and the run's chain descriptors (lane k = slot k; the
    // non-empty chains first, then the empty ones, then first == 0 slots)
    // and the workgroup's LUT words: independent loads, one round trip
    const bool live = w < n_runs;
    RowRun rr{};
    ReqChain C{};
    if (live) {
        if constexpr (PLAN) {
            rr = plan_run(st, in, n_in, w, stride, reinterpret_cast<ReqChain *>(L.a), ul);
            if (ul == 0) runs[w] = rr;
            C = reinterpret_cast<const ReqChain *>(L.a)[ul];
            wave_lds_sync();  // (L.a / L.b are rewritten below)
        } else {
            rr = runs[w];
            C = chains[static_cast<uint64_t>(w) * kReqRun + ul];
        }
    }
    if (threadIdx.x == 0) s_done = 0;
    if constexpr (LDS_LUT)
        for (uint32_t i = threadIdx.x; i < n_lut; i += kBlock) slut[i] = st.sym_lut[i];
    __syncthreads();
    const uint32_t *lut_base = LDS_LUT ? slut : st.sym_lut;
    if (!live) {
        if (ul == 0) finish(0);
        return;
    }
    const uint32_t row_lo = uniform(rr.row_lo), row_hi = uniform(rr.row_hi);
    const uint64_t stage_at = uniform64(rr.stage);
    const uint32_t rflags = uniform(rr.flags);
    const bool simple = (rflags & kRunSimple) != 0;
    // request_plan_kernel's guarantees over every candidate the run's chains
    // can load: chunk sums fit 32 bits (no wide path); one AN, so a chain's
    // AN sum is its hit records times it (no AN scan)
    const bool narrow = (rflags & kRunNarrow) != 0;
    const bool anc = (rflags & kRunAnCommon) != 0;
    const uint64_t an_c = rflags >> kRunAnShift;
    const bool slot = C.first != 0;
    const uint32_t R = static_cast<uint32_t>(__popcll(__ballot(slot)));
    const uint32_t cnt = slot ? C.c_hi - C.c_lo : 0u;
    const uint32_t nrows = row_hi - row_lo;
    // ---- setup: candidate ranges end to end (lane k: [pex, pin))
    const uint32_t pin = incl_sum_u32(cnt), pex = pin - cnt;
    const uint32_t T = rdl(pin, kWave - 1);
    const uint32_t Rn = static_cast<uint32_t>(__popcll(__ballot(cnt != 0)));  // non-empty chains = lanes 0 .. Rn-1
    const uint32_t rowk = row_lo + ((C.bits >> 17) & 63u);
    const uint32_t kind = (C.bits >> 23) & 7u;
    const uint32_t nsl = slot ? (C.last - C.first) / kReqWidth + 1 : 0u;
    {
        constexpr uint32_t kDel = vt_class_mask(VT_DEL), kIns = vt_class_mask(VT_INS), kDup = vt_class_mask(VT_DUP),
                           kDupT = vt_class_mask(VT_DUPT), kCnv = vt_class_mask(VT_CNV);
        const uint32_t cm = kind == VT_DEL ? kDel : kind == VT_INS ? kIns : kind == VT_DUP ? kDup : kind == VT_DUPT ? kDupT
                          : kind == VT_CNV ? kCnv : 0u;
        L.a[ul] = uint4{C.c_lo - pex, C.first, C.last - C.first, C.e0};
        // lut_off < kReqLutMax (host-enforced) shares the length-bounds word
        L.b[ul] = uint4{C.espan, (C.bits & 0x1ffffu) | C.lut_off << 17, cm, VT_XK_SYM | vt_xk_bit(kind)};
    }
    L.wch[ul] = 0ull;  // kReqStartChunks == kWave
    L.rowchain[ul] = 0xffu;
    if (ul < kReqRun / 32) L.slow[ul] = 0u;
    wave_lds_sync();
    if (ul < R) L.rowchain[rowk - row_lo] = static_cast<uint8_t>(ul);
    // the chain-start bitmap of the first kReqStartChunks chunks (later chunks
    // find their chains' starts one by one)
    if (ul < Rn && pex < kWave * kReqStartChunks) atomicOr(&L.wch[pex >> 6], 1ull << (pex & 63u));
    wave_lds_sync();
    const uint64_t wl = L.wch[ul];  // lane c: chunk c's chain starts
    const uint32_t cumv = incl_sum_u32(static_cast<uint32_t>(__popcll(wl))) - static_cast<uint32_t>(__popcll(wl));
    const uint32_t nch = (T + kWave - 1) / kWave;
    const uint32_t i_safe = rdl(C.c_lo, 0);  // a valid candidate index (chain 0 is non-empty when T > 0)
    // the run's staging region (capacity planned with the batch): a hit is
    // staged as its candidate index | ALT label << 29 (4 bytes)
    uint32_t *const hdst = stage + stage_at;
    uint32_t hpos = 0;   // hits staged so far (wave-uniform)
    uint32_t carry = 0;  // the last positive hit's slice key + 1 (keys grow with the position)
    uint32_t run_ex = 0; // slices with exists = True so far (wave-uniform; the invariant check)
    uint32_t acc_nv = 0, acc_ex = 0, acc_hr = 0;
    uint64_t acc_cc = 0, acc_an = 0;
    // each lane's own totals over its positions (call count, AN, or under a
    // common AN its hit records), modulo 2^32: the per-chain pulls must add
    // up to their wave sum (the invariants below); plain per-lane adds, no
    // cross-lane step and no scalar state in the loop
    uint32_t lane_cc = 0, lane_an = 0;
    // one instantiation per AN mode (a wave-uniform run flag): under a
    // common AN no AN column is loaded and no AN sum is scanned
    auto pass = [&](auto anc_t) {
    constexpr bool ANC = decltype(anc_t)::value;
    // ---- candidates
    auto load = [&](uint32_t c) -> ReqChunk {
        const uint32_t g = kWave * c + ul;
        uint64_t W;
        uint32_t cum;
        if (c < kReqStartChunks) {
            W = (static_cast<uint64_t>(rdl(static_cast<uint32_t>(wl >> 32), c)) << 32) | rdl(static_cast<uint32_t>(wl), c);
            cum = rdl(cumv, c);
        } else {  // past the bitmap (a run with more than 4 k candidates): the chains starting here, one by one
            const uint32_t b0 = kWave * c;
            cum = static_cast<uint32_t>(__popcll(__ballot(ul < Rn && pex < b0)));
            W = 0;
            for (uint64_t m = __ballot(ul < Rn && pex >= b0 && pex - b0 < kWave); m; m &= m - 1)
                W |= 1ull << (rdl(pex, static_cast<uint32_t>(ffs64(m))) - b0);
        }
        // chain of position g: starts before the chunk + starts at chunk positions <= lane
        const uint32_t s0 = cum + static_cast<uint32_t>(W & 1ull) - 1u;
        const uint64_t W1 = W >> 1;
        ReqChunk q;
        q.k = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(W1 >> 32),
                                        __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(W1), s0));
        const uint32_t i = g < T ? g + L.a[q.k].x : i_safe;
        q.q = st.vc_q[i];
        if constexpr (ANC) q.an = 0;
        else q.an = st.vc_word[i].an;
        if constexpr (REC) q.i = st.vc_idx[i];
        else q.i = i;
        return q;
    };
    auto eval = [&](const ReqChunk &q, uint32_t c) {
        const VcQ &x = q.q;
        const uint32_t k = q.k;
        // every column of this chunk is waited for here, at once: the wait
        // counter pass then knows them ready on every path below.  Without
        // it the first use of the record id (the staging store) sits after
        // branches that may issue loads, where the pass can only wait for
        // vmcnt(0) -- the NEXT chunk's prefetch included, which serialised
        // the pipeline
        asm volatile("" ::"v"(x.pos), "v"(x.end), "v"(x.w), "v"(x.ac0));
        if constexpr (!ANC) asm volatile("" ::"v"(q.an));
        if constexpr (REC) asm volatile("" ::"v"(q.i));
        const uint32_t base = kWave * c;
        const uint32_t g = base + ul;
        const uint4 A = L.a[k], Bw = L.b[k];
        const uint32_t first = A.y;
        const uint32_t w = x.w;
        // window, END bounds: every operand evaluated (bitwise, not
        // short-circuit: no divergent LDS reads)
        uint32_t cand = static_cast<uint32_t>(g < T) & static_cast<uint32_t>(x.pos - first <= A.z) &
                        static_cast<uint32_t>(x.end - A.w <= Bw.x);
        if (__ballot(cand & (w >> 28))) {  // VT_SLOW: never (prepare sends such requests per slice)
            if (cand & (w >> 28)) atomicOr(&L.slow[k >> 5], 1u << (k & 31u));
            cand &= ~(w >> 28) & 1u;
        }
        const uint32_t vlo = Bw.y & 511u, vspan = (Bw.y >> 9) & 255u, lut_off = Bw.y >> 17;
        // ALT0 (search_variants.py:100-183): length bounds, then the class
        // mask of the kind or, for a symbolic ALT, the variantType's LUT bit
        uint32_t a0 = (Bw.z >> ((w >> VT_CLASS_SHIFT) & 31u)) & 1u;
        const uint32_t sym = (w >> 13) & 1u;  // VT_SYM
        if (__ballot(cand & sym)) {
            const uint32_t lw = sym ? lut_base[lut_off + ((w >> 21) & 7u)] : 0u;
            if (sym) a0 = (lw >> ((w >> 16) & 31u)) & 1u;
        }
        const uint32_t h0 = cand & static_cast<uint32_t>((w & 0xffu) - vlo <= vspan) & a0;
        // ALTs 2..n (:124 loop): only records whose word says an extra ALT
        // of an accepted class (or a symbolic one) might match (Bw.w = xneed)
        const uint32_t xl = cand & static_cast<uint32_t>((w >> VT_NX_SHIFT) != 0) & static_cast<uint32_t>((w & Bw.w) != 0);
        bool hit;
        uint32_t cn;      // variants emitted (ALTs with AC != 0)
        int64_t cv;       // call count contribution
        uint32_t anv;     // AN contribution
        uint32_t pre, tot;
        if (!__ballot(xl)) {  // every hit lane has one ALT: ALT0 (label 0) is the only variant
            hit = h0 != 0;
            cv = hit ? x.ac0 : 0;
            cn = static_cast<uint32_t>(hit & (x.ac0 != 0));
            anv = hit ? static_cast<uint32_t>(q.an) : 0u;
            const uint64_t one = __ballot(cn);
            pre = popc_below(one);
            tot = static_cast<uint32_t>(__popcll(one));
            if (cn) hdst[hpos + pre] = q.i;
        } else {
            uint64_t hm = h0;
            uint32_t x0 = 0;
            if (xl) {
                x0 = st.x_lo[REC ? q.i : st.vc_idx[q.i]];
                // consumed here: no load left pending on this register past
                // the branch (a later writer of the register would wait for
                // vmcnt(0) on every path)
                asm volatile("" ::"v"(x0));
                const uint32_t nx = w >> VT_NX_SHIFT;
                for (uint32_t j = 0; j < nx; ++j) {
                    const uint32_t xw = st.xvt[x0 + j];
                    bool ok = (xw & 0xffu) - vlo <= vspan;
                    if (ok) {
                        if (xw & VT_SYM) ok = ((lut_base[lut_off + ((xw >> 21) & 7u)] >> ((xw >> 16) & 31u)) & 1u) != 0;
                        else ok = ((Bw.z >> ((xw >> VT_CLASS_SHIFT) & 31u)) & 1u) != 0;
                    }
                    if (ok) hm |= 2ull << j;
                }
            }
            hit = hm != 0;
            cv = 0;
            uint64_t em = 0;  // labels of the emitted variants
            for (uint64_t b = hm; b; b &= b - 1) {  // :205-214, AC of each matching ALT
                const int j = ffs64(b);
                const int64_t v = j ? st.xrow[x0 + j - 1].ac : x.ac0;
                cv += v;
                if (v != 0) em |= 1ull << j;
            }
            cn = static_cast<uint32_t>(__popcll(em));
            anv = hit ? static_cast<uint32_t>(q.an) : 0u;
            // ---- staging: hits in candidate order, ALTs of a record in label order
            if (!__ballot(cn > 1)) {
                const uint64_t one = __ballot(cn == 1);
                pre = popc_below(one);
                tot = static_cast<uint32_t>(__popcll(one));
                if (cn == 1) hdst[hpos + pre] = q.i | static_cast<uint32_t>(ffs64(em)) << kStageAltShift;
            } else {  // bit-sliced prefix (multi-ALT hit lanes)
                pre = 0;
                tot = 0;
                for (uint32_t bb = 0; bb < 7; ++bb) {
                    const uint64_t m = __ballot((cn >> bb) & 1u);
                    pre += popc_below(m) << bb;
                    tot += static_cast<uint32_t>(__popcll(m)) << bb;
                    if (!__ballot(cn >> (bb + 1))) break;
                }
                uint32_t at = hpos + pre;
                for (uint64_t b = em; b; b &= b - 1)
                    hdst[at++] = q.i | static_cast<uint32_t>(ffs64(b)) << kStageAltShift;
            }
        }
        hpos += tot;
        // ---- slices with exists = True: a positive hit whose slice differs
        // from the previous positive hit's (keys: chain << 20 | slice, growing
        // with the position), the carry from the chunks before
        const bool pos = hit && cv > 0;
        const uint32_t key1 = pos ? (k << 20 | (x.pos - first) / kReqWidth) + 1u : 0u;
        // (under a common AN the call-count scan runs beside the slice-key
        // scan: two independent DPP chains interleave, no wait states)
        uint32_t mx, scc_anc = 0;
        if constexpr (ANC) {
            incl_max_sum_u32(key1, static_cast<uint32_t>(cv), mx, scc_anc);
        } else {
            mx = incl_max_u32(key1);
        }
        const uint32_t prev = max(wave_shr1(mx), carry);
        const bool isnew = pos && key1 != prev;
        carry = max(carry, rdl(mx, kWave - 1));
        const uint64_t nb = __ballot(isnew);
        run_ex += static_cast<uint32_t>(__popcll(nb));
        // inclusive per-lane counts of the chunk, three fields pulled and
        // subtracted at once (each field's prefix grows with the lane, so
        // no field borrows): variants (<= 8 ALTs x 64 lanes) | new slices
        // << 10 | hit records << 17 (only read under a common AN)
        uint32_t nvex = (pre + cn) | (popc_below(nb) + (isnew ? 1u : 0u)) << 10;
        lane_cc += static_cast<uint32_t>(cv);
        if constexpr (ANC) {
            nvex |= (popc_below(__ballot(hit)) + (hit ? 1u : 0u)) << 17;
            lane_an += hit ? 1u : 0u;
        } else {
            lane_an += anv;
        }
        // ---- chain k's part of the chunk, pulled by lane k from its last lane
        const uint32_t lim = min(base + kWave, T);
        const bool inter = pex < lim && pin > base;
        const uint32_t e = inter ? min(pin, base + kWave) - 1u - base : 0u;
        const bool opens = pex <= base;  // no earlier chain in the chunk
        const uint32_t pn = bperm(nvex, e);
        const uint32_t qn = wave_shr1(pn);
        const uint32_t dn = inter ? pn - (opens ? 0u : qn) : 0u;
        acc_nv += dn & 0x3ffu;
        acc_ex += (dn >> 10) & 0x7fu;
        acc_hr += dn >> 17;
        if constexpr (ANC) {  // (a common AN implies narrow) the chunk's sums fit 32 bits; AN sums from hit records
            const uint32_t scc = scc_anc;
            const uint32_t pc = bperm(scc, e);
            const uint32_t qc = wave_shr1(pc);
            if (inter) acc_cc += pc - (opens ? 0u : qc);
            return;
        }
        const bool big = !narrow &&
                         __ballot(hit && (cv < 0 || cv >= (1ll << 25) || q.an < 0 || q.an >= (1 << 25))) != 0;
        if (!big) {  // the chunk's sums fit 32 bits
            const uint32_t scc = incl_sum_u32(static_cast<uint32_t>(cv)), san = incl_sum_u32(anv);
            const uint32_t pc = bperm(scc, e), pa = bperm(san, e);
            const uint32_t qc = wave_shr1(pc), qa = wave_shr1(pa);
            if (inter) {
                acc_cc += pc - (opens ? 0u : qc);
                acc_an += pa - (opens ? 0u : qa);
            }

        } else {
            const uint64_t scc = incl_sum_u64(static_cast<uint64_t>(cv)),
                           san = incl_sum_u64(static_cast<uint64_t>(static_cast<int64_t>(static_cast<int32_t>(anv))));
            const uint64_t pc = bperm64(scc, e), pa = bperm64(san, e);
            const uint64_t qc = wave_shr1_64(pc), qa = wave_shr1_64(pa);
            if (inter) {
                acc_cc += pc - (opens ? 0ull : qc);
                acc_an += pa - (opens ? 0ull : qa);
            }

        }
    };
    if (nch) {
        // The prefetch is unconditional (past the run a load reads the valid
        // index i_safe, one cache line): every path of the steady loop then
        // issues the same loads, so the wait-counter pass can wait for chunk
        // c's columns with the next chunks' loads still in flight.  A
        // conditional prefetch leaves a path with no later load, where the
        // only safe wait is vmcnt(0) -- the pipeline serialised.
        ReqChunk buf[kReqPipe];
#pragma unroll
        for (int a = 0; a < kReqPipe; ++a) buf[a] = load(a);
        uint32_t c0 = 0;
        for (; c0 + kReqPipe <= nch; c0 += kReqPipe) {
#pragma unroll
            for (int a = 0; a < kReqPipe; ++a) {
                eval(buf[a], c0 + a);
                buf[a] = load(c0 + a + kReqPipe);
            }
        }
#pragma unroll
        for (int a = 0; a < kReqPipe; ++a)
            if (c0 + a < nch) eval(buf[a], c0 + a);
    }
    };
    if (anc) pass(std::true_type{});
    else pass(std::false_type{});
    wave_lds_sync();
    // (tests, SBEACON_REQ_INJECT=1/2/3: one chain's exists-slice count, call
    // count or AN pull perturbed -- the checks below must fire)
    if (inject && w == 0 && ul == 0) {
        if (inject == 1) ++acc_ex;
        else if (inject == 2) ++acc_cc;
        else if (anc) ++acc_hr;
        else ++acc_an;
    }
    // the run's rows staged over the candidate-loop LDS (a, b, wch: dead now)
    ReqPartial *const srow = reinterpret_cast<ReqPartial *>(&L.a[0]);
    if constexpr (!COMPACT) {
        if (simple) {
            if (ul < nrows) srow[ul] = ReqPartial{0, 0, 0, 0, 0};
            wave_lds_sync();
        }
    }
    // ---- per chain (lane k < R): staging start (scan of the hit counts), partial
    const uint32_t cs_incl = incl_sum_u32(acc_nv), cs = cs_incl - acc_nv;
    // invariants of the per-chain sums (the pulls are cross-lane: a lane
    // reading another's stale value would break them): the chains' variant
    // counts add up to the hits staged, their new-slice counts to the
    // wave's, and a chain has no more exists-slices than variants nor (under
    // a common AN) than hit records.  A violation fails the batch at sync
    // (SB_EINTERNAL), never a silent wrong row.
    {
        const uint32_t ex_tot = rdl(incl_sum_u32(acc_ex), kWave - 1);
        const bool bad_lane = acc_ex > acc_nv || (anc && acc_ex > acc_hr);
        // the call-count and AN pulls (the same cross-lane primitives) against
        // the lanes' own totals, modulo 2^32: two wave sums of pairs per run
        const uint32_t d_cc = static_cast<uint32_t>(acc_cc) - lane_cc;
        const uint32_t d_an = (anc ? acc_hr : static_cast<uint32_t>(acc_an)) - lane_an;
        if (rdl(cs_incl, kWave - 1) != hpos || ex_tot != run_ex || __ballot(bad_lane) ||
            rdl(incl_sum_u32(d_cc), kWave - 1) != 0u || rdl(incl_sum_u32(d_an), kWave - 1) != 0u)
            if (ul == 0) atomicOr(err, 1u);
        // (PLAN: the run's hits within its fixed-stride staging region; never
        // past it, the stride was sized on these requests)
        if (PLAN && hpos > stride && ul == 0) atomicOr(err, 1u);
    }
    if (ul < R) {
        const bool slow = (L.slow[ul >> 5] >> (ul & 31u)) & 1u;  // never for prepared chains
        const uint64_t an_sum = anc ? static_cast<uint64_t>(acc_hr) * an_c : acc_an;
        if constexpr (COMPACT) {
            // counts past 32 bits or a slow chain: the row escapes (its wide
            // sums in xrows, the compact row marked)
            if (slow || acc_cc > 0xffffffffull || an_sum > 0xffffffffull) {
                esc.xrows[rowk] = slow ? ReqPartial{0, static_cast<int64_t>(acc_nv), 0, 0, static_cast<int64_t>(nsl)}
                                       : ReqPartial{static_cast<int64_t>(acc_ex), static_cast<int64_t>(acc_nv),
                                                    static_cast<int64_t>(acc_cc), static_cast<int64_t>(an_sum), 0};
                static_cast<RowC *>(rows_out)[rowk] = RowC{kRowEscaped, acc_nv, kRowEscaped, kRowEscaped};
                atomicOr(err, kErrRowEscapes);
            } else {
                static_cast<RowC *>(rows_out)[rowk] = RowC{acc_ex, acc_nv, static_cast<uint32_t>(acc_cc),
                                                           static_cast<uint32_t>(an_sum)};
            }
        } else {
            const ReqPartial rp = slow ? ReqPartial{0, static_cast<int64_t>(acc_nv), 0, 0, static_cast<int64_t>(nsl)}
                                       : ReqPartial{static_cast<int64_t>(acc_ex), static_cast<int64_t>(acc_nv),
                                                    static_cast<int64_t>(acc_cc), static_cast<int64_t>(an_sum), 0};
            if (simple) srow[rowk - row_lo] = rp;  // (staged: written out below, coalesced)
            else rows[rowk] = rp;
        }
    }
    if constexpr (!COMPACT) {
        // a simple run's rows (chain rows and empty rows, nothing per slice)
        // leave as one contiguous block: 16-byte stores over the run's 64 x
        // 40 B instead of five 8-byte stores 40 B apart per lane
        if (simple) {
            wave_lds_sync();
            const uint4 *src = reinterpret_cast<const uint4 *>(srow);
            uint4 *dst = reinterpret_cast<uint4 *>(rows + row_lo);
            const uint32_t n16 = nrows * sizeof(ReqPartial) / 16;
            for (uint32_t i = ul; i < n16; i += kWave) dst[i] = src[i];
            if ((nrows & 1u) && ul == 0)  // an odd row count leaves 8 bytes
                reinterpret_cast<uint64_t *>(rows + row_lo)[nrows * sizeof(ReqPartial) / 8 - 1] =
                    reinterpret_cast<const uint64_t *>(srow)[nrows * sizeof(ReqPartial) / 8 - 1];
        }
    }
    // ---- rows (lane i < nrows = row row_lo + i): hit counts, staging starts
    const uint32_t row = row_lo + ul;
    const uint32_t ch = ul < nrows ? L.rowchain[ul] : 0xffu;
    const uint32_t chn = bperm(acc_nv, ch & 63u), chs = bperm(cs, ch & 63u);
    uint64_t nvr = 0;
    if constexpr (COMPACT) {
        if (ul < nrows) {
            if (ch != 0xffu) {
                nvr = chn;
            } else if (sres) {  // a row answered per slice: its wide sums (request_reduce_kernel wrote xrows)
                const ReqPartial p = esc.xrows[row];
                const bool fits = !(esc.row_flag && esc.row_flag[row]) && p.errors == 0 && p.exists >= 0 &&
                                  p.exists < kRowEscaped && p.n_variants >= 0 && p.call_count >= 0 &&
                                  p.call_count <= 0xffffffffll && p.all_alleles_count >= 0 &&
                                  p.all_alleles_count <= 0xffffffffll;
                nvr = static_cast<uint64_t>(p.n_variants);
                static_cast<RowC *>(rows_out)[row] =
                    fits ? RowC{static_cast<uint32_t>(p.exists), static_cast<uint32_t>(nvr),
                                static_cast<uint32_t>(p.call_count), static_cast<uint32_t>(p.all_alleles_count)}
                         : RowC{kRowEscaped, static_cast<uint32_t>(nvr), kRowEscaped, kRowEscaped};
                if (!fits) atomicOr(err, kErrRowEscapes);
                if (nvr > 0xffffffffull) atomicOr(err, 2u);  // (the u32 offsets cannot hold it)
            } else {  // no slice (or no candidate)
                static_cast<RowC *>(rows_out)[row] = RowC{0, 0, 0, 0};
            }
            static_cast<uint32_t *>(row_cnt_out)[row] = static_cast<uint32_t>(nvr);
            if (!simple && ch != 0xffu) row_src[row] = stage_at + chs;
        }
    } else {
        if (ul < nrows) nvr = ch != 0xffu ? chn : (sres ? static_cast<uint64_t>(rows[row].n_variants) : 0ull);
        if (!sres && !simple && ul < nrows && ch == 0xffu) rows[row] = ReqPartial{0, 0, 0, 0, 0};
        if (ul < nrows) {
            row_cnt[row] = nvr;
            if (!simple && ch != 0xffu) row_src[row] = stage_at + chs;
        }
    }
    const uint64_t H = static_cast<uint64_t>(rdl64(static_cast<int64_t>(incl_sum_u64(nvr)), kWave - 1));
    if (ul == 0) {
        status[w] = H;  // read by request_deliver_kernel (kernel boundary)
        finish(H);
    }
}

// ---- request planning on the device (sb_requests_prepare_columns)
// request_plan_kernel: one wave per run of 64 consecutive rows (row = lane).
// A chain row's candidate range is read from its (segment, kind) coarse
// index -- two bucket entries, the batched lower / upper bound of
// splitQuery's window -- and its hit capacity from the candidates' ALT
// prefix; the run's chains are packed into its 64 slots (rows with
// candidates first, in row order, then those without; first == 0 after),
// its capacity summed for request_stage_scan_kernel.  Rows answered per
// slice (REQ_SLICES) make the run non-simple; REQ_NONE rows have no slice.
__global__ __launch_bounds__(kBlock) void request_plan_kernel(DStore st, const ReqIn *__restrict__ in, uint32_t n,
                                                              uint32_t n_runs, ReqChain *__restrict__ chains,
                                                              RowRun *__restrict__ runs,
                                                              unsigned long long *__restrict__ rcap,
                                                              unsigned long long *__restrict__ gcap, uint64_t stride,
                                                              unsigned int *__restrict__ err) {
    __shared__ ulonglong2 wtot[kWavesPerBlock];
    const uint32_t w = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    const uint32_t ul = static_cast<uint32_t>(lane_id());
    if (w >= n_runs) {  // (no run: its part of the workgroup total is zero)
        if (ul == 0) wtot[threadIdx.x >> 6] = ulonglong2{0ull, 0ull};
        __syncthreads();
        return;
    }
    const uint32_t row = w * kRunRows + ul;
    ReqIn q{};
    if (row < n) q = in[row];
    const uint32_t cls = row < n ? (q.cls & 3u) : static_cast<uint32_t>(REQ_NONE);
    const bool chain = cls == REQ_CHAIN;
    uint32_t c0 = 0, c1 = 0, vi_xinfo = 0;
    uint64_t cap = 0;
    if (chain) {
        const VcIndex vi = st.vcx[static_cast<uint64_t>(q.seg) * kVtKinds + ((q.bits >> 23) & 7u)];
        c0 = vc_bound(vi, st.vc_bucket, q.first, 0);
        c1 = (q.bits >> 26) & 1u ? c0 : max(c0, vc_bound(vi, st.vc_bucket, static_cast<uint64_t>(q.last) + 1, 1));
        cap = st.vc_altpre[c1] - st.vc_altpre[c0];
        vi_xinfo = vi.xinfo;
    }
    const bool ne = chain && c1 > c0;
    const uint64_t mne = __ballot(ne), mem = __ballot(chain && !ne);
    const uint32_t nne = static_cast<uint32_t>(__popcll(mne)), nslots = nne + static_cast<uint32_t>(__popcll(mem));
    ReqChain *out = chains + static_cast<uint64_t>(w) * kReqRun;
    if (chain) {
        const uint32_t slot = ne ? popc_below(mne) : nne + popc_below(mem);
        out[slot] = ReqChain{q.first, q.last, c0, c1, q.e0, q.espan, q.bits | (ul << 17), q.lut_off};
    }
    if (ul >= nslots) out[ul] = ReqChain{0, 0, 0, 0, 0, 0, 0, 0};  // the unused slots (first == 0)
    const uint64_t capsum = static_cast<uint64_t>(rdl64(static_cast<int64_t>(incl_sum_u64(cap)), kWave - 1));
    const uint32_t nsl = chain ? q.cls >> 2 : 0u;
    const uint32_t slsum = rdl(incl_sum_u32(nsl), kWave - 1);
    const bool simple = __ballot(cls == REQ_SLICES) == 0;
    // what request_eval_kernel may assume of every chain with candidates
    // (VcIndex::xinfo): 32-bit chunk sums, one AN (AN sum = hit records x AN)
    const uint32_t xi = ne ? vi_xinfo : kVcNarrow;
    const bool narrow = __ballot(!(xi & kVcNarrow)) == 0;
    const uint32_t a = xi & kVcAnMask;  // AN + 1, 0 = no common AN
    const uint32_t a0 = mne ? rdl(a, static_cast<uint32_t>(ffs64(mne))) : 1u;
    const bool anc = narrow && a0 != 0u && __ballot(ne && a != a0) == 0;
    const uint32_t flags = (simple ? kRunSimple : 0u) | (narrow ? kRunNarrow : 0u) |
                           (anc ? kRunAnCommon | (a0 - 1u) << kRunAnShift : 0u);
    if (ul == 0) {  // (the batch's chain / slice totals: request_stage_scan_kernel -- one counter
                    // atomically bumped by every wave serialised the launch, ~350 us for 15.6 k runs)
        // staging: at a fixed stride per run when the batch has one (a
        // re-planning pass: no scan), else request_stage_scan_kernel's offset
        runs[w] = RowRun{w * kRunRows, min(w * kRunRows + kRunRows, n), 0u, nslots, stride * w, slsum, flags};
        if (stride && capsum > stride) atomicOr(err, 1u);  // (never: the prepare sized the stride on these requests)
        const unsigned long long cw = static_cast<unsigned long long>(slsum) << 32 | nslots;
        rcap[2 * w] = capsum;
        rcap[2 * w + 1] = cw;
        wtot[threadIdx.x >> 6] = ulonglong2{capsum, cw};
    }
    // the workgroup's totals (request_stage_scan_kernel sums these for the
    // runs before its tile: a quarter of the words per-run totals would be)
    __syncthreads();
    if (threadIdx.x == 0) {
        ulonglong2 t{0ull, 0ull};
#pragma unroll
        for (uint32_t k = 0; k < kWavesPerBlock; ++k) {
            t.x += wtot[k].x;
            t.y += wtot[k].y;
        }
        reinterpret_cast<ulonglong2 *>(gcap)[blockIdx.x] = t;
    }
}

static_assert(kDeliverTile == 16, "a delivery tile is 16 runs");

// request_stage_scan_kernel: each run's staging offset = the exclusive
// prefix of the runs' capacities; counters = (chains, chain slices, staging
// total).  request_plan_kernel left per run {capacity, slices << 32 |
// chains} (16 B) and the same per plan workgroup of kWavesPerBlock runs.
// One workgroup per tile of kStageTile runs: it sums the workgroup totals of
// every earlier tile (coalesced, all loads of a round in flight), then scans
// its own tile; the last workgroup, which reads every total anyway, writes
// the counters.  (Summing the earlier tiles' per-run words took 6.3 us: the
// last workgroup read 250 KB; one workgroup scanning all runs, 10.5 us.)
constexpr uint32_t kStageTile = 1024;
static_assert(kStageTile % kWavesPerBlock == 0, "a stage tile is whole plan workgroups");
__device__ __forceinline__ uint64_t block_sum_u64(uint64_t v, unsigned long long *wsum) {
    const uint32_t wave = threadIdx.x >> 6;
    const uint64_t t = static_cast<uint64_t>(rdl64(static_cast<int64_t>(incl_sum_u64(v)), kWave - 1));
    __syncthreads();
    if (lane_id() == 0) wsum[wave] = t;
    __syncthreads();
    uint64_t r = 0;
    for (uint32_t k = 0; k < blockDim.x / kWave; ++k) r += wsum[k];
    return r;
}
__global__ __launch_bounds__(kStageTile) void request_stage_scan_kernel(RowRun *__restrict__ runs,
                                                                        const unsigned long long *__restrict__ rcap,
                                                                        const unsigned long long *__restrict__ gcap,
                                                                        uint32_t n_runs,
                                                                        unsigned long long *__restrict__ counters) {
    __shared__ unsigned long long wsum[kStageTile / kWave];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, t0 = blockIdx.x * kStageTile;
    const bool last = blockIdx.x + 1 == gridDim.x;
    const ulonglong2 *rc2 = reinterpret_cast<const ulonglong2 *>(rcap);
    const ulonglong2 *gc2 = reinterpret_cast<const ulonglong2 *>(gcap);
    const uint32_t g0 = t0 / kWavesPerBlock;  // plan workgroups before this tile
    uint64_t pre = 0, nch = 0, nsl = 0;
    constexpr uint32_t kU = 4;
    for (uint32_t i0 = 0; i0 < g0; i0 += kStageTile * kU) {
        ulonglong2 x[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint32_t i = i0 + u * kStageTile + tid;
            x[u] = i < g0 ? gc2[i] : ulonglong2{0ull, 0ull};
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            pre += x[u].x;
            nch += x[u].y & 0xffffffffull;
            nsl += x[u].y >> 32;
        }
    }
    const uint32_t i = t0 + tid;
    const ulonglong2 me = i < n_runs ? rc2[i] : ulonglong2{0ull, 0ull};
    nch += me.y & 0xffffffffull;
    nsl += me.y >> 32;
    {  // the largest run capacity (counters[3]: sizes a fixed-stride staging layout)
        uint32_t mx = static_cast<uint32_t>(min(me.x, 0xffffffffull));
        for (uint32_t d = 1; d < kWave; d <<= 1) mx = max(mx, static_cast<uint32_t>(__shfl_xor(static_cast<int>(mx), d)));
        if (lane_id() == 0 && mx) atomicMax(reinterpret_cast<unsigned int *>(counters + 3), mx);
    }
    pre = block_sum_u64(pre, wsum);
    // the tile's exclusive scan
    const uint64_t incl = incl_sum_u64(me.x);
    __syncthreads();
    if (lane_id() == kWave - 1) wsum[wave] = incl;
    __syncthreads();
    uint64_t before = pre;
    for (uint32_t k = 0; k < wave; ++k) before += wsum[k];
    if (i < n_runs) runs[i].stage = before + incl - me.x;
    uint64_t tile = 0;
    for (uint32_t k = 0; k < kStageTile / kWave; ++k) tile += wsum[k];
    if (last) {
        const uint64_t ch = block_sum_u64(nch, wsum), sl = block_sum_u64(nsl, wsum);
        if (tid == 0) {
            counters[0] = ch;
            counters[1] = sl;
            counters[2] = pre + tile;
        }
    }
}

// request_tile_scan_kernel: the tiles' totals (a tile of kDeliverTile runs =
// kDeliverTile / kWavesPerBlock eval workgroups, whose totals
// request_eval_kernel left in gtot) scanned into exclusive tile offsets, one
// workgroup, rounds of 1,024 tiles with every load coalesced: a tile is a
// quad of lanes (DPP quad permutes sum it).  (Reading the runs' own totals:
// 6.3 us, one CU's loads of 8 B per run; tile totals by device atomics in
// request_eval_kernel needed a memset launch before every pass.)
static_assert(kDeliverTile == 4 * kWavesPerBlock, "a tile is four eval workgroups (a quad of lanes)");
constexpr uint32_t kTilePer = 4;  // group totals per thread per round: 1,024 tiles
__global__ __launch_bounds__(1024) void request_tile_scan_kernel(const unsigned long long *__restrict__ gtot,
                                                                 uint32_t n_groups,
                                                                 unsigned long long *__restrict__ tsum,
                                                                 uint32_t nt) {
    __shared__ unsigned long long tl[1024];
    __shared__ unsigned long long wsum[1024 / kWave];
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    uint64_t carry = 0;
    for (uint32_t base = 0; base < n_groups; base += 1024 * kTilePer) {
        uint64_t v[kTilePer];
#pragma unroll
        for (uint32_t u = 0; u < kTilePer; ++u) {
            const uint32_t g = base + u * 1024 + tid;
            v[u] = g < n_groups ? gtot[g] : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < kTilePer; ++u) {  // quad sums: [1,0,3,2] then [2,3,0,1]
            uint64_t q = v[u] + static_cast<uint64_t>(dpp_i64<0xB1, 0xf, 0xf>(static_cast<int64_t>(v[u])));
            q += static_cast<uint64_t>(dpp_i64<0x4E, 0xf, 0xf>(static_cast<int64_t>(q)));
            if ((lane_id() & 3u) == 0) tl[u * 256 + tid / 4] = q;
        }
        __syncthreads();
        const uint64_t x = tl[tid];
        const uint64_t inc = incl_sum_u64(x);
        if (lane_id() == kWave - 1) wsum[wave] = inc;
        __syncthreads();
        uint64_t before = carry, total = 0;
#pragma unroll
        for (uint32_t k = 0; k < 1024 / kWave; ++k) {
            const uint64_t ws = wsum[k];
            if (k < wave) before += ws;
            total += ws;
        }
        const uint32_t t = base / 4 + tid;
        if (t < nt) tsum[t] = before + inc - x;
        carry += total;
        __syncthreads();  // tl / wsum are rewritten by the next round
    }
}

// request_deliver_kernel: one wave per run.  Its output offset = its tile's
// offset + the totals of the earlier runs of its tile (<= 15 loads, one per
// lane); row offsets by a wave scan of the row counts request_eval_kernel
// left in row_off; the run's hits copied from its staging region (one
// contiguous range for a run of chain rows; row by row where some rows were
// answered per slice).  No inter-wave dependency.  (One wave per tile of 16
// runs, or a look-back, left the chip mostly idle: ~2 k waves, 0.1 ms.)
// COMPACT: row counts / offsets u32, hits u32 = (record + rec_base) | label
// << kStageAltShift (the host checks records + rec_base < 2^29; an offset
// past 32 bits fails the batch at sync)
// GSUM: no tile scan before it -- the workgroup (= one eval workgroup's 4
// runs) sums the eval workgroup totals before its own (gtot, <= 16 coalesced
// loads per thread from L2 per 4,096 groups) and each wave adds its group's
// earlier runs: one launch and its boundary fewer
// SLICED: the batch has a per-slice part (runs that are not simple); without
// one a compact-row batch's runs are all simple and the row-by-row path is
// not compiled in (registers of the common instantiation)
// LAB7: the store holds an 8-ALT record, so a chain hit can carry the label
// 7 that the compact hit form escapes (store_has_label7)
template <bool ROWC, bool HITC, bool REC, bool GSUM, bool SLICED, bool LAB7>
__global__ __launch_bounds__(kBlock) void request_deliver_kernel(
    const RowRun *__restrict__ runs, uint32_t n_runs, const unsigned long long *__restrict__ status,
    const unsigned long long *__restrict__ toff, const QRes *__restrict__ sres, const uint32_t *__restrict__ sseg,
    const uint64_t *__restrict__ shoff, const uint8_t *__restrict__ sherr, const uint64_t *__restrict__ shits,
    void *__restrict__ row_off_out, const uint64_t *__restrict__ row_src, const uint32_t *__restrict__ stage,
    const uint32_t *__restrict__ vc_idx, void *__restrict__ out_v, uint32_t n_rows, uint64_t rec_base,
    unsigned int *__restrict__ err, const unsigned long long *__restrict__ gtot, ReqEsc esc) {
    using Hit = std::conditional_t<HITC, uint32_t, uint64_t>;
    using Off = std::conditional_t<ROWC, uint32_t, uint64_t>;
    Hit *const out = static_cast<Hit *>(out_v);
    Off *const row_off = static_cast<Off *>(row_off_out);  // (counts in, offsets out)
    // a staged hit (candidate | ALT label << kStageAltShift) as the output's
    // (record + rec_base) | label << kHitAltShift
    auto hit_of = [&](uint32_t v) -> Hit {
        const uint32_t r = REC ? (v & kStageCandMask) : vc_idx[v & kStageCandMask];  // the staged record
        if constexpr (HITC)
            return (r + static_cast<uint32_t>(rec_base)) | (v & ~kStageCandMask);
        else
            return (static_cast<uint64_t>(r) + rec_base) | static_cast<uint64_t>(v >> kStageAltShift) << kHitAltShift;
    };
    const uint32_t w = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    // (GSUM: a wave past the last run still joins the workgroup's sum below)
    const bool live = w < n_runs;
    if (!GSUM && !live) return;
    const uint32_t ul = static_cast<uint32_t>(lane_id());
    constexpr uint32_t kTileRuns = GSUM ? kWavesPerBlock : kDeliverTile;
    const uint32_t t0 = (w / kTileRuns) * kTileRuns;
    // the run record and the run's total (status[w] = its staged hits, which
    // request_eval_kernel wrote) first: a simple run's first round of staged
    // hits is loaded before its output offset is known, so those loads and
    // the record-id gathers behind them overlap the offset scans
    const RowRun rr = live ? runs[w] : RowRun{};
    const uint64_t Hs = live ? uniform64(status[w]) : 0ull;
    const uint32_t row_lo = uniform(rr.row_lo), row_hi = uniform(rr.row_hi);
    const uint64_t stage_at = uniform64(rr.stage);
    const bool simple = (uniform(rr.flags) & kRunSimple) != 0;
    constexpr uint32_t kU = 8;  // 512 hits per round: most runs in one (~480 hits per run)
    uint32_t v0[kU];
    if (simple) {
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) {
            const uint64_t j = kWave * u + ul;
            v0[u] = j < Hs ? stage[stage_at + j] : 0u;
        }
    }
    const uint32_t row = row_lo + ul;
    const uint64_t c = row < row_hi ? static_cast<uint64_t>(row_off[row]) : 0ull;  // the counts request_eval_kernel left
    const uint64_t before = live && t0 + ul < w ? status[t0 + ul] : 0ull;
    // (GSUM: issued behind the run's own loads, so their latencies overlap)
    uint64_t gsum = 0;  // GSUM: the totals of the eval workgroups before this one
    if constexpr (GSUM) {
        __shared__ unsigned long long s_part[kWavesPerBlock];
        constexpr uint32_t kG = 16;
        uint64_t part = 0;
        for (uint32_t base = 0; base < blockIdx.x; base += kG * kBlock) {
            uint64_t v[kG];
#pragma unroll
            for (uint32_t u = 0; u < kG; ++u) {
                const uint32_t g = base + u * kBlock + threadIdx.x;
                v[u] = g < blockIdx.x ? gtot[g] : 0ull;
            }
#pragma unroll
            for (uint32_t u = 0; u < kG; ++u) part += v[u];
        }
        part = static_cast<uint64_t>(rdl64(static_cast<int64_t>(incl_sum_u64(part)), kWave - 1));
        if (lane_id() == 0) s_part[threadIdx.x >> 6] = part;
        __syncthreads();  // (every wave of the workgroup, live or not, reaches it)
#pragma unroll
        for (uint32_t k = 0; k < kWavesPerBlock; ++k) gsum += s_part[k];
    }
    if (!live) return;
    const uint64_t O = (GSUM ? uniform64(gsum) : uniform64(toff[w / kDeliverTile])) +
                       static_cast<uint64_t>(rdl64(wave_incl_scan_i64(static_cast<int64_t>(before)), kWave - 1));
    const uint64_t linc = static_cast<uint64_t>(wave_incl_scan_i64(static_cast<int64_t>(c)));
    const uint64_t H = static_cast<uint64_t>(rdl64(static_cast<int64_t>(linc), kWave - 1));
    const uint64_t off = O + linc - c;
    if constexpr (ROWC) {
        if (ul == 0 && O + H > 0xffffffffull) atomicOr(err, 2u);
    }
    if (row < row_hi) row_off[row] = static_cast<Off>(off);
    if (row_hi == n_rows && ul == 0) row_off[n_rows] = static_cast<Off>(O + H);
    if (simple) {  // chain rows (and empty rows) only: the staging region is the output, in order
        for (uint64_t j0 = 0; j0 < H; j0 += kWave * kU) {
            uint32_t v[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u) {
                const uint64_t j = j0 + kWave * u + ul;
                v[u] = j0 == 0 ? v0[u] : (j < H ? stage[stage_at + j] : 0u);
            }
            Hit h[kU];
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u) h[u] = hit_of(v[u]);
#pragma unroll
            for (uint32_t u = 0; u < kU; ++u) {
                const uint64_t j = j0 + kWave * u + ul;
                if (j < H) out[O + j] = h[u];
            }
            if constexpr (HITC && LAB7) {  // the label 7 escapes -- its ALT goes to xlab too
                bool lab7x = false;
#pragma unroll
                for (uint32_t u = 0; u < kU; ++u) {
                    const uint64_t j = j0 + kWave * u + ul;
                    if (j < H && (v[u] >> kStageAltShift) == kHitLabelEscape) {
                        esc.xlab[O + j] = static_cast<uint16_t>(kHitLabelEscape);
                        lab7x = true;
                    }
                }
                if (__ballot(lab7x) && ul == 0) atomicOr(err, kErrHitEscapes);
            }
        }
        return;
    }
    if constexpr (ROWC && !SLICED) return;  // (never reached: every run is simple)
    for (uint32_t i = 0; i < row_hi - row_lo; ++i) {  // row by row (some rows answered per slice)
        const uint64_t nv = static_cast<uint64_t>(rdl64(static_cast<int64_t>(c), i));
        if (!nv) continue;
        const uint64_t at = static_cast<uint64_t>(rdl64(static_cast<int64_t>(off), i));
        const uint32_t r = row_lo + i;
        const uint32_t q0 = uniform(sseg[r]), q1 = uniform(sseg[r + 1]);
        if (q1 == q0) {  // a chain row: its hits are contiguous in the staging region
            const uint64_t src = uniform64(row_src[r]);
            bool lab7x = false;
            for (uint64_t k = ul; k < nv; k += kWave) {
                const uint32_t v = stage[src + k];
                out[at + k] = hit_of(v);
                if (HITC && (v >> kStageAltShift) == kHitLabelEscape) {
                    esc.xlab[at + k] = static_cast<uint16_t>(kHitLabelEscape);
                    lab7x = true;
                }
            }
            if (HITC && __ballot(lab7x) && ul == 0) atomicOr(err, kErrHitEscapes);
        } else {
            uint64_t dst = at;
            for (uint32_t q = q0; q < q1; ++q) {
                const QRes rq = sres[q];
                if (rq.error || sherr[q]) continue;
                const uint64_t src = shoff[q];
                // HITC: an ALT label of 7 or more escapes (label 7, the index
                // in xlab); past 65,535 the side table cannot hold it (the batch fails)
                bool escd = false, wide_alt = false;
                for (uint32_t k = ul; k < rq.n_hits; k += kWave) {
                    const uint64_t h = shits[src + k];  // record | ALT << kHitAltShift
                    if constexpr (HITC) {
                        const uint64_t a = h >> kHitAltShift;
                        const bool x = a >= kHitLabelEscape;
                        escd |= x;
                        wide_alt |= a > 0xffffu;
                        if (x) esc.xlab[dst + k] = static_cast<uint16_t>(a);
                        out[dst + k] = (static_cast<uint32_t>(h) + static_cast<uint32_t>(rec_base)) |
                                       static_cast<uint32_t>(x ? kHitLabelEscape : a) << kStageAltShift;
                    } else
                        out[dst + k] = h + rec_base;
                }
                if constexpr (HITC) {
                    const bool any_x = __ballot(escd) != 0, any_w = __ballot(wide_alt) != 0;
                    if (ul == 0 && any_x) atomicOr(err, kErrHitEscapes);
                    if (ul == 0 && any_w) atomicOr(err, 4u);
                }
                dst += rq.n_hits;
            }
        }
    }
}

// ---------------------------------------------------------------- dense hit lists
// Device-side result delivery for a sharded fan-out (sb_batch_compact_hits):
// dense[q] = exclusive prefix over queries of their emitted hit counts (0 for
// a query that raised), in three launches (tile sums, one-block scan of the
// tile sums, tile scans); then every query's hits are copied from its region
// to dense[q] with the shard's global record base added, and each request
// row's first dense offset is read off at its first query.
constexpr uint32_t kScanPer = 4;                    // items per thread
constexpr uint32_t kScanTile = kBlock * kScanPer;  // items per workgroup

__device__ __forceinline__ uint64_t hit_count(const QRes &r) { return r.error ? 0u : r.n_hits; }

// inclusive sum over the workgroup of one value per thread (LDS of the wave totals)
__device__ __forceinline__ uint64_t block_incl_scan(uint64_t v, uint64_t *wsum) {
    const int wave = threadIdx.x >> 6;
    const uint64_t incl = static_cast<uint64_t>(wave_incl_scan_i64(static_cast<int64_t>(v)));
    if (lane_id() == kWave - 1) wsum[wave] = incl;
    __syncthreads();
    uint64_t before = 0;
    for (int w = 0; w < wave; ++w) before += wsum[w];
    __syncthreads();
    return incl + before;
}

__global__ __launch_bounds__(kBlock) void hit_tile_sum_kernel(const QRes *__restrict__ res, uint32_t nq,
                                                              uint64_t *__restrict__ tsum) {
    __shared__ uint64_t wsum[kWavesPerBlock];
    const uint32_t i0 = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint64_t v = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k)
        if (i0 + k < nq) v += hit_count(res[i0 + k]);
    const uint64_t t = block_incl_scan(v, wsum);
    if (threadIdx.x == kBlock - 1) tsum[blockIdx.x] = t;
}

// exclusive scan of tsum[0 .. nt) in place by one workgroup; tsum[nt] = total
__global__ __launch_bounds__(kBlock) void tile_scan_kernel(uint64_t *__restrict__ tsum, uint32_t nt) {
    __shared__ uint64_t wsum[kWavesPerBlock];
    uint64_t carry = 0;
    for (uint32_t base = 0; base < nt; base += kBlock) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t v = i < nt ? tsum[i] : 0u;
        const uint64_t incl = block_incl_scan(v, wsum);
        if (i < nt) tsum[i] = carry + incl - v;
        if (threadIdx.x == kBlock - 1) wsum[0] = incl;  // block_incl_scan's LDS is free again here
        __syncthreads();
        carry += wsum[0];
        __syncthreads();
    }
    if (threadIdx.x == 0) tsum[nt] = carry;
}

__global__ __launch_bounds__(kBlock) void hit_tile_scan_kernel(const QRes *__restrict__ res, uint32_t nq,
                                                               const uint64_t *__restrict__ tsum,
                                                               uint64_t *__restrict__ dense) {
    __shared__ uint64_t wsum[kWavesPerBlock];
    const uint32_t i0 = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint64_t c[kScanPer], v = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        c[k] = i0 + k < nq ? hit_count(res[i0 + k]) : 0u;
        v += c[k];
    }
    uint64_t at = tsum[blockIdx.x] + block_incl_scan(v, wsum) - v;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        if (i0 + k < nq) dense[i0 + k] = at;
        at += c[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) dense[nq] = tsum[gridDim.x];
}

// thread per query (most queries emit 0-3 hits)
__global__ __launch_bounds__(kBlock) void hit_gather_kernel(const QRes *__restrict__ res, uint32_t nq,
                                                            const uint64_t *__restrict__ src,
                                                            const uint64_t *__restrict__ dense,
                                                            const uint64_t *__restrict__ hits, uint64_t rec_base,
                                                            uint64_t *__restrict__ out) {
    const uint32_t q = blockIdx.x * kBlock + threadIdx.x;
    if (q >= nq) return;
    const uint64_t n = hit_count(res[q]), a = src[q], d = dense[q];
    for (uint64_t k = 0; k < n; ++k) out[d + k] = hits[a + k] + rec_base;
}

__global__ __launch_bounds__(kBlock) void row_off_kernel(const uint32_t *__restrict__ seg, uint32_t n_rows,
                                                         const uint64_t *__restrict__ dense,
                                                         uint64_t *__restrict__ row_off) {
    const uint32_t w = blockIdx.x * kBlock + threadIdx.x;
    if (w <= n_rows) row_off[w] = dense[seg[w]];
}

// ---------------------------------------------------------------- request rows by pieces
// When every chain lies in one request row (sb_batch_set_owners checks), a
// row is a list of pieces -- chains (their partial rows come from
// chain_kernel) and unchained queries (QRes) -- so the reduction, the scan of
// the rows' hit counts and the hit gather run over rows and pieces (10^6)
// instead of slices (5 x 10^6), and a chain's hits are one contiguous copy.
// piece p: bit 31 set = chain (p & 0x7fffffff), else a query index.
constexpr uint32_t kPieceChain = 1u << 31;

// rowsrc[w] = {hit region, count} of a single-piece row ({~0, 0} otherwise):
// the gather then needs no piece lookups for it
// one request row from its pieces (chains: their partial; slices: their QRes)
__device__ __forceinline__ ReqPartial reduce_row(uint32_t w, const ReqPartial *__restrict__ cpart,
                                                 const ChainDev *__restrict__ chains,
                                                 const uint64_t *__restrict__ hoff, const QRes *__restrict__ res,
                                                 const uint8_t *__restrict__ host_err,
                                                 const uint32_t *__restrict__ poff,
                                                 const uint32_t *__restrict__ piece, ulonglong2 *__restrict__ rowsrc) {
    ReqPartial P{0, 0, 0, 0, 0};
    const uint32_t k0 = poff[w], k1 = poff[w + 1];
    if (rowsrc) {
        ulonglong2 rs{~0ull, 0ull};
        if (k1 == k0 + 1) {
            const uint32_t p = piece[k0];
            if (p & kPieceChain) {
                rs.x = chains[p & ~kPieceChain].out;
                rs.y = static_cast<uint64_t>(cpart[p & ~kPieceChain].n_variants);
            } else {
                rs.x = hoff[p];
                rs.y = hit_count(res[p]);
            }
        } else if (k1 == k0) {
            rs.x = 0;
        }
        rowsrc[w] = rs;
    }
    for (uint32_t k = k0; k < k1; ++k) {
        const uint32_t p = piece[k];
        if (p & kPieceChain) {
            const ReqPartial c = cpart[p & ~kPieceChain];
            P.exists += c.exists;
            P.n_variants += c.n_variants;
            P.call_count += c.call_count;
            P.all_alleles_count += c.all_alleles_count;
            P.errors += c.errors;
        } else {
            const QRes r = res[p];
            if (r.error || host_err[p]) {
                ++P.errors;
                continue;
            }
            P.exists += r.exists != 0;
            P.n_variants += r.n_hits;
            P.call_count += r.call_count;
            P.all_alleles_count += r.all_alleles_count;
        }
    }
    return P;
}

__global__ __launch_bounds__(kBlock) void row_reduce_kernel(const ReqPartial *__restrict__ cpart,
                                                            const ChainDev *__restrict__ chains,
                                                            const uint64_t *__restrict__ hoff,
                                                            const QRes *__restrict__ res,
                                                            const uint8_t *__restrict__ host_err,
                                                            const uint32_t *__restrict__ poff,
                                                            const uint32_t *__restrict__ piece, uint32_t n_rows,
                                                            ReqPartial *__restrict__ out, ulonglong2 *__restrict__ rowsrc) {
    const uint32_t w = blockIdx.x * kBlock + threadIdx.x;
    if (w >= n_rows) return;
    out[w] = reduce_row(w, cpart, chains, hoff, res, host_err, poff, piece, rowsrc);
}

// sb_batch_deliver: the rows as above plus, for the hit-list offsets, each
// row's n_variants in a dense array and the per-tile sums of it (one tile =
// kScanTile rows = this block's rows), so the offset scan reads 8 B / row
__global__ __launch_bounds__(kBlock) void row_reduce_tiles_kernel(const ReqPartial *__restrict__ cpart,
                                                                  const ChainDev *__restrict__ chains,
                                                                  const uint64_t *__restrict__ hoff,
                                                                  const QRes *__restrict__ res,
                                                                  const uint8_t *__restrict__ host_err,
                                                                  const uint32_t *__restrict__ poff,
                                                                  const uint32_t *__restrict__ piece, uint32_t n_rows,
                                                                  ReqPartial *__restrict__ out,
                                                                  ulonglong2 *__restrict__ rowsrc,
                                                                  int64_t *__restrict__ nv, uint64_t *__restrict__ tsum) {
    __shared__ uint64_t wsum[kWavesPerBlock];
    uint64_t x = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        const uint32_t w = blockIdx.x * kScanTile + k * kBlock + threadIdx.x;  // coalesced per k
        if (w < n_rows) {
            const ReqPartial P = reduce_row(w, cpart, chains, hoff, res, host_err, poff, piece, rowsrc);
            out[w] = P;
            nv[w] = P.n_variants;
            x += static_cast<uint64_t>(P.n_variants);
        }
    }
    const uint64_t t = block_incl_scan(x, wsum);
    if (threadIdx.x == kBlock - 1) tsum[blockIdx.x] = t;
}

// tile sums / tile scans of one int64 field of a strided array (ReqPartial rows)
__global__ __launch_bounds__(kBlock) void field_tile_sum_kernel(const int64_t *__restrict__ v, uint32_t stride,
                                                                uint32_t n, uint64_t *__restrict__ tsum) {
    __shared__ uint64_t wsum[kWavesPerBlock];
    const uint32_t i0 = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint64_t x = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k)
        if (i0 + k < n) x += static_cast<uint64_t>(v[static_cast<size_t>(i0 + k) * stride]);
    const uint64_t t = block_incl_scan(x, wsum);
    if (threadIdx.x == kBlock - 1) tsum[blockIdx.x] = t;
}

__global__ __launch_bounds__(kBlock) void field_tile_scan_kernel(const int64_t *__restrict__ v, uint32_t stride,
                                                                 uint32_t n, const uint64_t *__restrict__ tsum,
                                                                 uint64_t *__restrict__ out) {
    __shared__ uint64_t wsum[kWavesPerBlock];
    const uint32_t i0 = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint64_t c[kScanPer], x = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        c[k] = i0 + k < n ? static_cast<uint64_t>(v[static_cast<size_t>(i0 + k) * stride]) : 0u;
        x += c[k];
    }
    uint64_t at = tsum[blockIdx.x] + block_incl_scan(x, wsum) - x;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        if (i0 + k < n) out[i0 + k] = at;
        at += c[k];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = tsum[gridDim.x];
}

// The same scan without the one-block tile_scan launch in front: block b
// sums the raw tile sums of the blocks before it itself (L2-resident, a few
// KB), and the last block writes the total at out[n]
__global__ __launch_bounds__(kBlock) void field_scan_fused_kernel(const int64_t *__restrict__ v, uint32_t n,
                                                                  const uint64_t *__restrict__ tsum,
                                                                  uint64_t *__restrict__ out) {
    __shared__ uint64_t wsum[kWavesPerBlock];
    __shared__ uint64_t s_pre;
    uint64_t part = 0;
    for (uint32_t i = threadIdx.x; i < blockIdx.x; i += kBlock) part += tsum[i];
    const uint64_t pincl = block_incl_scan(part, wsum);
    if (threadIdx.x == kBlock - 1) s_pre = pincl;
    __syncthreads();
    const uint64_t pre = s_pre;
    const uint32_t i0 = blockIdx.x * kScanTile + threadIdx.x * kScanPer;
    uint64_t c[kScanPer], x = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        c[k] = i0 + k < n ? static_cast<uint64_t>(v[i0 + k]) : 0u;
        x += c[k];
    }
    const uint64_t incl = block_incl_scan(x, wsum);
    uint64_t at = pre + incl - x;
#pragma unroll
    for (uint32_t k = 0; k < kScanPer; ++k) {
        if (i0 + k < n) out[i0 + k] = at;
        at += c[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == kBlock - 1) out[n] = pre + incl;
}

__global__ __launch_bounds__(kBlock) void row_gather_seg_kernel(const uint32_t *__restrict__ poff,
                                                                const uint32_t *__restrict__ piece, uint32_t n_rows,
                                                                const ChainDev *__restrict__ chains,
                                                                const ReqPartial *__restrict__ cpart,
                                                                const QRes *__restrict__ res,
                                                                const uint64_t *__restrict__ hoff,
                                                                const uint64_t *__restrict__ hits, uint64_t rec_base,
                                                                const uint64_t *__restrict__ row_off,
                                                                const uint64_t *__restrict__ srcx, uint32_t sstride,
                                                                uint64_t *__restrict__ out) {
    const uint32_t r0 = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * kWave;
    if (r0 >= n_rows) return;
    const uint32_t ul = static_cast<uint32_t>(lane_id());
    const uint32_t r = min(r0 + ul, n_rows - 1);
    const bool live = r0 + ul < n_rows;
    const uint64_t base = row_off[r0];
    const uint64_t end = row_off[min(r0 + kWave, n_rows)];
    const uint64_t my0 = row_off[r];
    const ulonglong2 rs{live ? srcx[static_cast<size_t>(r) * sstride] : 0ull, 0ull};  // x: the row's hit region
    const uint32_t e = static_cast<uint32_t>(live ? my0 - base : end - base);  // row start within the range
    const bool single = live && rs.x != ~0ull;
    const uint64_t total = end - base;
    // lane r's source offset of output slot j is off_r + j - 2^63 (its hit
    // region minus its row start, biased so it is never 0); 0 = a
    // several-piece row (copied below)
    constexpr uint64_t kBias = 1ull << 63;
    const uint64_t offr = single ? rs.x - e + kBias : 0ull;
    auto src_of = [&](uint32_t j) -> uint64_t {  // call with every lane active
        uint32_t l = 0;  // last lane l with e_l <= j (e is nondecreasing over the lanes)
#pragma unroll
        for (uint32_t step = kWave / 2; step >= 1; step >>= 1) {
            const uint32_t t = l + step;
            const uint32_t et = static_cast<uint32_t>(__shfl(static_cast<int>(e), static_cast<int>(t), kWave));
            if (et <= j) l = t;
        }
        return static_cast<uint64_t>(shfl_i64(static_cast<int64_t>(offr), static_cast<int>(l)));
    };
    // four output passes per round: their searches, then every load, then the stores
    constexpr uint32_t kGU = 4;
    for (uint64_t j0 = 0; j0 < total; j0 += kGU * kWave) {
        uint64_t so[kGU], hv[kGU];
#pragma unroll
        for (uint32_t q = 0; q < kGU; ++q)
            so[q] = j0 + q * kWave < total ? src_of(static_cast<uint32_t>(j0) + q * kWave + ul) : 0ull;
#pragma unroll
        for (uint32_t q = 0; q < kGU; ++q) {
            const uint64_t j = j0 + q * kWave + ul;
            hv[q] = (j < total && so[q] != 0ull) ? hits[so[q] - kBias + j] : 0ull;
        }
#pragma unroll
        for (uint32_t q = 0; q < kGU; ++q) {
            const uint64_t j = j0 + q * kWave + ul;
            if (j < total && so[q] != 0ull) out[base + j] = hv[q] + rec_base;
        }
    }
    if (live && !single) {  // several pieces: this lane copies its row
        uint64_t d = my0;
        for (uint32_t k = poff[r], ke = poff[r + 1]; k < ke; ++k) {
            const uint32_t p = piece[k];
            uint64_t a, n;
            if (p & kPieceChain) {
                const uint32_t c = p & ~kPieceChain;
                a = chains[c].out;
                n = static_cast<uint64_t>(cpart[c].n_variants);
            } else {
                a = hoff[p];
                n = hit_count(res[p]);
            }
            for (uint64_t jj = 0; jj < n; ++jj) out[d + jj] = hits[a + jj] + rec_base;
            d += n;
        }
    }
}

__global__ __launch_bounds__(kBlock) void compact_kernel(const uint64_t *__restrict__ hit_off,
                                                         const uint64_t *__restrict__ dense_off,
                                                         const QRes *__restrict__ res, uint32_t nq,
                                                         const uint64_t *__restrict__ hits,
                                                         uint64_t *__restrict__ out) {
    const uint32_t q = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    if (q >= nq) return;
    const uint64_t src = hit_off[q], dst = dense_off[q];
    const uint32_t n = res[q].n_hits;
    for (uint32_t i = static_cast<uint32_t>(lane_id()); i < n; i += kWave) out[dst + i] = hits[src + i];
}

// Route-level reduction of one shard's slice answers
// (lambda/getGenomicVariants/route_g_variants.py:144-171): request row w owns
// the contiguous queries [seg[w], seg[w+1]).  exists is OR-ed (kept as the
// number of slices that exist, so shard partials combine by sum), n_variants,
// call_count and all_alleles_count are summed; a slice that raised (device
// error or host-detected error flag) counts in `errors` and contributes
// nothing else.  A workgroup owns kBlock consecutive rows, whose queries are
// one contiguous QRes range: it stages that range through LDS in tiles with
// coalesced 16-byte loads (a thread-per-row walk of QRes directly would read
// 32-byte records at a ~5-record stride across the lanes), then each thread
// sums its row's part of the tile.
constexpr uint32_t kReduceTile = 1024;  // QRes per LDS tile (32 KiB)

// wide[q] = 1 for every slice whose counts needed more than 64 bits (the
// general path's big list; its QRes holds the low 64 bits)
__global__ __launch_bounds__(kBlock) void mark_wide_kernel(const uint32_t *__restrict__ big_n,
                                                           const GenBig *__restrict__ big, uint32_t cap,
                                                           uint8_t *__restrict__ wide) {
    const uint32_t n = min(*big_n, cap);
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) wide[big[i].orig] = 1;
}

// row w = the sums of slices [seg[w], seg[w + 1]); row_flag[w] (optional) = 1
// when a count is not exact in 64 bits (a wide slice, or the sum overflows):
// the row then holds the low 64 bits of the exact sums
__global__ __launch_bounds__(kBlock) void request_reduce_kernel(const QRes *__restrict__ res,
                                                                const uint32_t *__restrict__ seg,
                                                                const uint8_t *__restrict__ host_err,
                                                                const uint8_t *__restrict__ wide, uint32_t n_rows,
                                                                ReqPartial *__restrict__ out,
                                                                uint8_t *__restrict__ row_flag) {
    __shared__ uint4 tile[kReduceTile * (sizeof(QRes) / 16)];
    __shared__ uint8_t terr[kReduceTile];
    static_assert(sizeof(QRes) == 32, "QRes is two 16-byte words");
    const uint32_t r0 = blockIdx.x * kBlock, r1 = min(n_rows, r0 + kBlock);
    const uint32_t w = r0 + threadIdx.x;
    const uint32_t q_lo = seg[r0], q_hi = seg[r1];
    const uint32_t a = w < r1 ? seg[w] : 0u, e = w < r1 ? seg[w + 1] : 0u;
    ReqPartial P{0, 0, 0, 0, 0};
    bool inexact = false;
    const uint4 *src = reinterpret_cast<const uint4 *>(res);
    for (uint32_t t0 = q_lo; t0 < q_hi; t0 += kReduceTile) {
        const uint32_t t1 = min(q_hi, t0 + kReduceTile);
        for (uint32_t k = threadIdx.x; k < 2 * (t1 - t0); k += kBlock) tile[k] = src[2 * static_cast<size_t>(t0) + k];
        for (uint32_t k = threadIdx.x; k < t1 - t0; k += kBlock) terr[k] = host_err[t0 + k];
        __syncthreads();
        const QRes *T = reinterpret_cast<const QRes *>(tile);
        for (uint32_t q = max(a, t0), qe = min(e, t1); q < qe; ++q) {
            const QRes &r = T[q - t0];
            if (r.error || terr[q - t0]) {
                ++P.errors;
                continue;
            }
            P.exists += r.exists != 0;
            P.n_variants += r.n_hits;
            long long cc, an;
            inexact |= __builtin_add_overflow(static_cast<long long>(P.call_count), static_cast<long long>(r.call_count), &cc);
            inexact |= __builtin_add_overflow(static_cast<long long>(P.all_alleles_count),
                                              static_cast<long long>(r.all_alleles_count), &an);
            P.call_count = cc;
            P.all_alleles_count = an;
            if (wide && wide[q]) inexact = true;
        }
        __syncthreads();
    }
    if (w < r1) {
        out[w] = P;
        if (row_flag) row_flag[w] = inexact ? 1 : 0;
    }
}

inline uint32_t blocks_for(uint32_t nwaves) { return (nwaves + kWavesPerBlock - 1) / kWavesPerBlock; }
// slices per wave for a launch of nq slices: up to kRun while the launch
// still has >= 4 waves per slot of a full chip (256 CUs x 4 SIMDs x 8)
// (SBEACON_SLICES_PER_WAVE=k forces k, 1..kRun: tests drive run_slices with small batches)
inline uint32_t run_for(uint32_t nq) {
    if (const int k = config().slices_per_wave; k >= 1) return std::min<uint32_t>(kRun, static_cast<uint32_t>(k));
    return std::max(1u, std::min(kRun, nq / 32768u));
}
inline uint32_t run_waves(uint32_t nq, uint32_t run) { return (nq + run - 1) / run; }

// ------------------------------------------------------------ summariseSlice
// lambda/summariseSlice/source/main.cpp:195-245.  The reader visits the first
// record, then for every later record r: recordHeader + addCounts, seek
// (skipSize = 2 x delimiters after the first record's AC/AN cursor) and
// skipPast('\n').  That skips record r+1.. whenever skipSize >= rem_r (the
// bytes left on r's line).  Phase A sums every record of the slice and marks
// those overshoots; phase B (wave 0) walks the marks in order, keeps only the
// overshoots of visited records and subtracts the records their jumps skip.
// Phase A: one workgroup per chunk of kSumChunk records of one slice (chunks
// never straddle slices) — sums the chunk's contributions and writes its
// overshoot bitmap words.
__global__ __launch_bounds__(kBlock) void summarise_chunk_kernel(SStore ss, const SDev *__restrict__ slices,
                                                                 const uint32_t *__restrict__ chunk_slice,
                                                                 uint32_t nchunks, uint64_t *__restrict__ bitmap,
                                                                 SPart *__restrict__ part) {
    __shared__ uint64_t red_nv[kWavesPerBlock], red_nc[kWavesPerBlock];
    __shared__ uint32_t red_bad[kWavesPerBlock], red_ov[kWavesPerBlock];
    const uint32_t c = blockIdx.x;
    if (c >= nchunks) return;
    const SDev S = slices[chunk_slice[c]];
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const uint32_t c0 = S.lo + (c - S.chunk_lo) * kSumChunk;
    const uint32_t c1 = min(S.hi, c0 + kSumChunk);
    const uint64_t skip = 2ull * ss.dcount[S.lo];
    uint64_t nv = 0, nc = 0;
    uint32_t bad = 0, ov = 0;
    uint64_t *bm = bitmap + S.bitmap_off;
    constexpr int kPer = kSumChunk / kBlock;
    uint64_t h[kPer];  // all 8-byte loads in flight before any use
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t r = c0 + k * kBlock + threadIdx.x;
        h[k] = r < c1 ? ss.sum8[r] : 0ull;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t base = c0 + k * kBlock;
        const uint32_t r = base + threadIdx.x;
        uint64_t rem, vnv, vnc;
        uint32_t vbad = 0;
        if (h[k] & kSumEscape) {  // rare: the wide word
            const SumHot w = ss.sum[r];
            rem = w.rem;
            vnv = w.nvf & ~kSumUnsupported;
            vnc = w.nc;
            vbad = w.nvf >> 31;
        } else {
            rem = h[k] & 0xffffffull;
            vnv = (h[k] >> 24) & 0xffull;
            vnc = h[k] >> 32;
        }
        if (r < c1) {
            nv += vnv;
            nc += vnc;
            bad += vbad;
        }
        const uint64_t m = __ballot(r < c1 && r > S.lo && skip >= rem);
        ov += m != 0;
        if (lane == 0 && base + wave * kWave < c1) bm[(base - S.lo) / kWave + wave] = m;
    }
    nv = static_cast<uint64_t>(wave_sum_i64(static_cast<int64_t>(nv)));
    nc = static_cast<uint64_t>(wave_sum_i64(static_cast<int64_t>(nc)));
    bad = static_cast<uint32_t>(wave_sum_i64(bad));
    if (lane == 0) {
        red_nv[wave] = nv;
        red_nc[wave] = nc;
        red_bad[wave] = bad;
        red_ov[wave] = ov;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        SPart P{0, 0, 0, 0};
        for (int w = 0; w < kWavesPerBlock; ++w) {
            P.nv += red_nv[w];
            P.nc += red_nc[w];
            P.bad += red_bad[w];
            P.overshoot_words += red_ov[w];
        }
        part[c] = P;
    }
}

// Phase B: one wave per slice — totals of its chunks, then the in-order walk
// of the overshoot marks (only chunks that have any): a visited overshoot
// seeks to P = start + cursor + skipSize and skipPast('\n') resumes at the
// first record starting after P; the records in between are subtracted.
__global__ __launch_bounds__(kBlock) void summarise_finish_kernel(SStore ss, const SDev *__restrict__ slices,
                                                                  uint32_t ns, const uint64_t *__restrict__ bitmap,
                                                                  const SPart *__restrict__ part,
                                                                  SRes *__restrict__ out) {
    const uint32_t sid = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (sid >= ns) return;
    const SDev S = slices[sid];
    const int lane = lane_id();
    const uint32_t lo = S.lo, hi = S.hi;
    if (lo >= hi) {
        if (lane == 0) out[sid] = SRes{0, 0, 0, 0, 0};
        return;
    }
    const uint64_t skip = 2ull * ss.dcount[lo];
    uint64_t tnv = 0, tnc = 0, tbad = 0;
    for (uint32_t k = lane; k < S.n_chunks; k += kWave) {
        const SPart P = part[S.chunk_lo + k];
        tnv += P.nv;
        tnc += P.nc;
        tbad += P.bad;
    }
    tnv = static_cast<uint64_t>(wave_sum_i64(static_cast<int64_t>(tnv)));
    tnc = static_cast<uint64_t>(wave_sum_i64(static_cast<int64_t>(tnc)));
    tbad = static_cast<uint64_t>(wave_sum_i64(static_cast<int64_t>(tbad)));
    const uint64_t *bm = bitmap + S.bitmap_off;
    uint64_t sub_nv = 0, sub_nc = 0, sub_bad = 0, skipped = 0;
    uint32_t resume = lo;  // records >= resume are visited until the next jump
    constexpr uint32_t kWordsPerChunk = kSumChunk / kWave;
    for (uint32_t k = 0; k < S.n_chunks; ++k) {
        if (part[S.chunk_lo + k].overshoot_words == 0) continue;
        const uint32_t wbeg = k * kWordsPerChunk;
        const uint32_t wend = min((hi - lo + kWave - 1) / kWave, wbeg + kWordsPerChunk);
        for (uint32_t w0 = wbeg; w0 < wend; w0 += kWave) {
            const uint64_t word = (w0 + lane < wend) ? bm[w0 + lane] : 0ull;
            uint64_t nz = __ballot(word != 0ull);
            while (nz) {
                const int L = ffs64(nz);
                nz &= nz - 1;
                uint64_t bits = static_cast<uint64_t>(shfl_i64(static_cast<int64_t>(word), L));
                while (bits) {
                    const int b = ffs64(bits);
                    bits &= bits - 1;
                    const uint32_t r = lo + (w0 + static_cast<uint32_t>(L)) * kWave + static_cast<uint32_t>(b);
                    if (r < resume) continue;  // r itself was skipped: it never seeks
                    const uint64_t P = ss.start[r] + ss.cur[r] + skip;
                    uint32_t t = hi;
                    for (uint32_t q0 = r + 1; q0 < hi; q0 += kWave) {
                        const uint32_t i = q0 + static_cast<uint32_t>(lane);
                        const uint64_t m = __ballot(i < hi && ss.start[i] > P);
                        if (m) {
                            t = q0 + static_cast<uint32_t>(ffs64(m));
                            break;
                        }
                    }
                    for (uint32_t q0 = r + 1; q0 < t; q0 += kWave) {
                        const uint32_t i = q0 + static_cast<uint32_t>(lane);
                        uint64_t a = 0, c = 0, d = 0;
                        if (i < t) {
                            const SumHot h = ss.sum[i];
                            a = h.nvf & ~kSumUnsupported;
                            c = h.nc;
                            d = h.nvf >> 31;
                        }
                        sub_nv += static_cast<uint64_t>(wave_sum_i64(static_cast<int64_t>(a)));
                        sub_nc += static_cast<uint64_t>(wave_sum_i64(static_cast<int64_t>(c)));
                        sub_bad += static_cast<uint64_t>(wave_sum_i64(static_cast<int64_t>(d)));
                    }
                    skipped += t - (r + 1);
                    resume = t;
                }
            }
        }
    }
    if (lane == 0) {
        SRes o;
        o.error = (tbad - sub_bad) ? SB_QERR_UNSUPPORTED : 0;
        o.pad = 0;
        o.num_variants = tnv - sub_nv;
        o.num_calls = tnc - sub_nc;
        o.records = (hi - lo) - skipped;
        out[sid] = o;
    }
}

// ---------------------------------------------------------------- general records
// A slice whose scan reached a general record (devtypes.hpp GenRec) is
// answered here, one wave per slice, record by record in file order
// (search_variants.py:70-254 / search_variants_in_samples.py:63-245): the
// ordinary records of each 64-record chunk through eval_record in parallel,
// then the reference loop's state machine over the chunk's lanes in order; a
// general record is evaluated by the whole wave:
//   * ALT predicates over any number of ALTs, 64 per round (hit bitmap);
//   * AC / AN as Python ints: running sums are two's complement numbers of up
//     to kGenAccMax 32-bit limbs, limb j in lane j % 64 of group j / 64, added
//     with a carry-lookahead over the wave (generate / propagate ballots:
//     carry-in = (G + (G|P)) ^ (G|P) ^ G);
//   * the GT fallback (:215-226): token counts over the (subset) samples in
//     parallel; the variant order is CPython's iteration order of
//     set(all_calls) & hit_set (:223), emulated by one lane over scratch
//     tables exactly as Objects/setobject.c (3.10) builds them.

// per-lane limbs of a wave-wide number
using BigLimbs = uint32_t[kGenAccGroups];

__device__ __forceinline__ void big_zero(BigLimbs &a) {
#pragma unroll
    for (uint32_t t = 0; t < kGenAccGroups; ++t) a[t] = 0u;
}

// a += x over `groups` 64-limb groups (both sign-extended to the full width)
__device__ __forceinline__ void big_add(BigLimbs &a, const BigLimbs &x, uint32_t groups) {
    const uint32_t lane = static_cast<uint32_t>(lane_id());
    uint32_t cg = 0;  // carry into limb 0 of the group
#pragma unroll
    for (uint32_t t = 0; t < kGenAccGroups; ++t) {
        if (t < groups) {
            const uint64_t s = static_cast<uint64_t>(a[t]) + x[t] + (lane == 0 ? cg : 0u);
            const uint64_t G = __ballot((s >> 32) != 0);
            const uint64_t P = __ballot(static_cast<uint32_t>(s) == 0xffffffffu);
            const uint64_t X = G | P, sum = G + X;
            const uint64_t cin = sum ^ X ^ G;  // bit i: carry into limb i
            a[t] = static_cast<uint32_t>(s) + static_cast<uint32_t>((cin >> lane) & 1u);
            cg = sum < X ? 1u : 0u;  // out of the group's top limb
        }
    }
}

__device__ __forceinline__ void big_add_i64(BigLimbs &a, int64_t v, uint32_t groups) {
    const uint32_t lane = static_cast<uint32_t>(lane_id());
    const uint32_t sgn = v < 0 ? 0xffffffffu : 0u;
    BigLimbs x;
#pragma unroll
    for (uint32_t t = 0; t < kGenAccGroups; ++t) x[t] = sgn;
    const uint64_t u = static_cast<uint64_t>(v);
    if (lane == 0) x[0] = static_cast<uint32_t>(u);
    if (lane == 1) x[0] = static_cast<uint32_t>(u >> 32);
    big_add(a, x, groups);
}

// GStore number k (limbs of it past gs.limbs: its sign)
__device__ __forceinline__ void big_add_num(BigLimbs &a, const GStore &gs, uint64_t k, uint32_t groups) {
    const uint32_t lane = static_cast<uint32_t>(lane_id());
    const uint32_t *p = gs.num + k * gs.limbs;
    const uint32_t sgn = (p[gs.limbs - 1] >> 31) ? 0xffffffffu : 0u;
    BigLimbs x;
#pragma unroll
    for (uint32_t t = 0; t < kGenAccGroups; ++t) {
        const uint32_t j = t * kWave + lane;
        x[t] = (t < groups && j < gs.limbs) ? p[j] : sgn;
    }
    big_add(a, x, groups);
}

__device__ __forceinline__ bool big_nonzero(const BigLimbs &a, uint32_t groups) {
    bool nz = false;
#pragma unroll
    for (uint32_t t = 0; t < kGenAccGroups; ++t)
        if (t < groups) nz = nz || __ballot(a[t] != 0u);
    return nz;
}

__device__ __forceinline__ int64_t big_low64(const BigLimbs &a) {
    return static_cast<int64_t>((static_cast<uint64_t>(rdl(a[0], 1)) << 32) | rdl(a[0], 0));
}

__device__ __forceinline__ bool big_fits64(const BigLimbs &a, uint32_t groups) {
    const uint32_t lane = static_cast<uint32_t>(lane_id());
    const uint32_t sgn = (rdl(a[0], 1) >> 31) ? 0xffffffffu : 0u;
    bool bad = false;
#pragma unroll
    for (uint32_t t = 0; t < kGenAccGroups; ++t)
        if (t < groups) bad = bad || __ballot((t > 0 || lane >= 2) && a[t] != sgn);
    return !bad;
}

// one slot of an emulated CPython set: key bit 31 = a hit allele number
// (hit_set), else a value id of the record's GT digit runs (set(all_calls))
struct SetEnt {
    uint64_t hash;
    uint32_t key;
    uint32_t used;
};
struct PySetD {
    SetEnt *t;
    uint64_t mask, fill, used;
};
constexpr uint32_t kHitKey = 0x80000000u;

__device__ __forceinline__ bool set_key_eq(const GenVal *val, uint32_t a, uint32_t b) {
    if (a == b) return true;
    if ((a ^ b) < kHitKey) return false;  // same domain, different keys
    const uint32_t vid = (a & kHitKey) ? b : a, al = ((a & kHitKey) ? a : b) & ~kHitKey;
    return val[vid].allele == al;
}

__device__ void set_init(PySetD &s, SetEnt *t) {
    s.t = t;
    s.mask = 7;
    s.fill = s.used = 0;
    for (int i = 0; i < 8; ++i) t[i] = SetEnt{0, 0, 0};
}

__device__ void set_insert_clean(SetEnt *t, uint64_t mask, uint64_t hash, uint32_t key) {
    uint64_t perturb = hash, i = hash & mask;
    SetEnt *e;
    for (;;) {
        e = &t[i];
        if (!e->used) break;
        bool found = false;
        if (i + 9 <= mask)
            for (int j = 0; j < 9; ++j) {
                ++e;
                if (!e->used) {
                    found = true;
                    break;
                }
            }
        if (found) break;
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
    *e = SetEnt{hash, key, 1u};
}

// set_add_entry (with set_table_resize through `tmp`, tcap entries)
__device__ void set_add(PySetD &s, SetEnt *tmp, const GenVal *val, uint64_t hash, uint32_t key) {
    uint64_t mask = s.mask, i = hash & mask, perturb = hash;
    SetEnt *e = nullptr;
    for (;;) {
        e = &s.t[i];
        int probes = (i + 9 <= mask) ? 9 : 0;
        bool unused = false;
        do {
            if (!e->used) {
                unused = true;
                break;
            }
            if (e->hash == hash && set_key_eq(val, e->key, key)) return;
            ++e;
        } while (probes--);
        if (unused) break;
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
    *e = SetEnt{hash, key, 1u};
    ++s.fill;
    ++s.used;
    if (s.fill * 5 < mask * 3) return;
    const uint64_t minused = s.used > 50000 ? s.used * 2 : s.used * 4;
    uint64_t newsize = 8;
    while (newsize <= minused) newsize <<= 1;
    for (uint64_t k = 0; k < newsize; ++k) tmp[k] = SetEnt{0, 0, 0};
    for (uint64_t k = 0; k <= mask; ++k)
        if (s.t[k].used) set_insert_clean(tmp, newsize - 1, s.t[k].hash, s.t[k].key);
    for (uint64_t k = 0; k < newsize; ++k) s.t[k] = tmp[k];
    s.mask = newsize - 1;
    s.fill = s.used;
}

__device__ bool set_contains(const PySetD &s, const GenVal *val, uint64_t hash, uint32_t key) {
    uint64_t mask = s.mask, i = hash & mask, perturb = hash;
    for (;;) {
        const SetEnt *e = &s.t[i];
        int probes = (i + 9 <= mask) ? 9 : 0;
        do {
            if (!e->used) return false;
            if (e->hash == hash && set_key_eq(val, e->key, key)) return true;
            ++e;
        } while (probes--);
        perturb >>= 5;
        i = (i * 5 + 1 + perturb) & mask;
    }
}

// ALT k of record r against the query's ALT predicate + length bounds
// (search_variants.py:100-183; the ALT half of eval_record)
__device__ __forceinline__ bool gen_alt_ok(const DStore &st, const QDev &Q, const QView &V, uint32_t r, uint32_t k,
                                           uint32_t x0, uint32_t a0_cls, int64_t ref_len) {
    const uint32_t x = x0 + k - 1;
    const uint32_t cls = k ? st.xrow[x].cls : a0_cls;
    int64_t len = 1;
    bool ok;
    if (V.alt_mode == ALT_N) {
        ok = cls & C_SINGLE_BASE;
    } else if (V.alt_mode == ALT_EXACT) {
        const uint64_t key = k ? st.x_key[x] : st.a0_key[r];
        ok = key == Q.alt_key;
        len = Q.alt_len;
        if (ok && (key >> 63))
            ok = k ? blob_eq_upper(st.blob, st.x_off[x], st.x_len[x], V.qalt, Q.alt_len)
                   : blob_eq_upper(st.blob, st.a0_off[r], st.a0_len[r], V.qalt, Q.alt_len);
    } else {
        len = k ? st.x_len[x] : st.a0_len[r];
        ok = vtype_hit(Q, st, cls, len, ref_len);
    }
    return ok && len >= Q.vmin && len <= Q.vmax;
}

struct GenSlice {  // one wave's state over one slice
    BigLimbs cc, an;
    uint32_t n_out;
    bool exists;
};

enum : int { GEN_GO = 0, GEN_STOP = -1 };  // > 0: the SB_QERR_* the reference raises

__device__ __forceinline__ void or_planes(const DStore &st, const QDev &Q, uint64_t row, uint64_t *samples_out) {
    for (uint32_t w = static_cast<uint32_t>(lane_id()); w < Q.words; w += kWave)
        samples_out[Q.samples_out_off + w] |= st.planes[row + w];
}

// one general record reached by the slice's loop
__device__ int general_record(const DStore &st, const GStore &gs, const QDev &Q, const QView &V, uint32_t r,
                              GenSlice &S, uint64_t *out, uint64_t *samples_out, bool collect, uint32_t groups,
                              uint64_t *hbits, SetEnt *tabs, uint32_t tcap) {
    const uint32_t lane = static_cast<uint32_t>(lane_id());
    const GenRec G = gs.rec[static_cast<uint32_t>(st.rec[r].ac0)];
    const uint32_t n_alt = G.n_alt, x0 = st.x_lo[r];
    const int64_t ref_len = static_cast<int64_t>(st.rec[r].end) - st.pos[r] + 1;
    // ---- hit_indexes (:100-183)
    uint32_t nh = 0, maxhit = 0;
    for (uint32_t k0 = 0; k0 < n_alt; k0 += kWave) {
        const uint32_t k = k0 + lane;
        const bool ok = k < n_alt && gen_alt_ok(st, Q, V, r, k, x0, G.a0_cls, ref_len);
        const uint64_t m = __ballot(ok);
        if (lane == 0) hbits[k0 / kWave] = m;
        if (m) {
            nh += static_cast<uint32_t>(__popcll(m));
            maxhit = k0 + 63u - static_cast<uint32_t>(__clzll(m));
        }
    }
    if (!nh) return GEN_GO;  // :184
    __threadfence();  // hbits: lane 0's stores, every lane's loads
    auto is_hit = [&](uint32_t k) -> bool { return (hbits[k / kWave] >> (k % kWave)) & 1ull; };
    if (G.flags & GR_AN_BAD) return SB_QERR_VALUE;  // :199
    const uint64_t *subset = V.subset;
    if (G.flags & GR_HAS_AC) {  // :205-214
        if (G.flags & GR_AC_BAD) return SB_QERR_VALUE;
        if (maxhit >= G.n_ac) return SB_QERR_INDEX;  // :207
        for (uint32_t k0 = 0; k0 < n_alt; k0 += kWave) {
            const uint64_t m = static_cast<uint64_t>(rdl64(static_cast<int64_t>(hbits[k0 / kWave]), 0));
            if (!m) continue;
            const uint32_t k = k0 + lane;
            bool nz = false;
            if ((m >> lane) & 1ull) {
                const uint32_t *p = gs.num + (G.ac_num + k) * gs.limbs;
                for (uint32_t j = 0; j < gs.limbs; ++j) nz = nz || p[j] != 0u;
            }
            const uint64_t nzm = __ballot(nz);
            if (nz) out[S.n_out + popc_below(nzm)] = static_cast<uint64_t>(r) | (static_cast<uint64_t>(k) << kHitAltShift);
            S.n_out += static_cast<uint32_t>(__popcll(nzm));
            for (uint64_t b = m; b; b &= b - 1) big_add_num(S.cc, gs, G.ac_num + k0 + ffs64(b), groups);
        }
    } else if (G.flags & GR_FB) {  // :215-226 genotype fallback over the (subset) samples
        const uint64_t *toff = gs.tok_off + G.tok_off;
        const GenVal *val = gs.val + G.val_off;
        int64_t cnt = 0;
        bool huge = false, last = false;  // last: the value n_alt occurs (alts[n_alt] -> IndexError)
        for (uint32_t s = lane; s < Q.n_samples; s += kWave) {
            if (subset && !((subset[s >> 6] >> (s & 63)) & 1ull)) continue;
            for (uint64_t t = toff[s]; t < toff[s + 1]; ++t) {
                const GenVal v = val[gs.tok[t]];
                huge = huge || v.huge;
                if (v.allele && is_hit(v.allele - 1)) {
                    ++cnt;
                    last = last || v.allele == n_alt;
                }
            }
        }
        if (__ballot(huge)) return SB_QERR_VALUE;  // :218 int(g) past 4300 digits
        if (__ballot(last)) return SB_QERR_INDEX;  // :223 alts[i] with 1-based i
        const int64_t cc = wave_sum_i64(cnt);
        uint32_t ne = 0;
        if (lane == 0) {  // variants in the iteration order of set(all_calls) & hit_set
            SetEnt *tmp = tabs + 3ull * tcap;
            PySetD sc, hs, rs;
            set_init(sc, tabs);
            set_init(hs, tabs + tcap);
            set_init(rs, tabs + 2ull * tcap);
            if (!subset) {  // value ids are numbered in first-occurrence order over all samples
                for (uint32_t v = 0; v < G.n_vals; ++v) set_add(sc, tmp, val, val[v].hash, v);
            } else {
                for (uint32_t s = 0; s < Q.n_samples; ++s)
                    if ((subset[s >> 6] >> (s & 63)) & 1ull)
                        for (uint64_t t = toff[s]; t < toff[s + 1]; ++t) {
                            const uint32_t v = gs.tok[t];
                            set_add(sc, tmp, val, val[v].hash, v);
                        }
            }
            for (uint32_t k = 0; k < n_alt; ++k)
                if (is_hit(k)) set_add(hs, tmp, val, k + 1, kHitKey | (k + 1));
            const PySetD *so = &sc, *other = &hs;  // set_intersection: iterate the smaller
            if (hs.used > sc.used) {
                so = &hs;
                other = &sc;
            }
            for (uint64_t i = 0; i <= other->mask; ++i) {
                const SetEnt e = other->t[i];
                if (e.used && set_contains(*so, val, e.hash, e.key)) set_add(rs, tmp, val, e.hash, e.key);
            }
            for (uint64_t i = 0; i <= rs.mask; ++i)
                if (rs.t[i].used) {
                    const uint32_t key = rs.t[i].key;
                    const uint32_t a = (key & kHitKey) ? key & ~kHitKey : val[key].allele;
                    out[S.n_out + ne++] = static_cast<uint64_t>(r) | (static_cast<uint64_t>(a) << kHitAltShift);
                }
        }
        S.n_out += rdl(ne, 0);
        big_add_i64(S.cc, cc, groups);
    }
    // :229-236
    if (big_nonzero(S.cc, groups)) {
        S.exists = true;
        if (!(V.flags & F_DETAILS)) return GEN_STOP;  // :231-232, before AN
        if (collect)
            for (uint32_t k = 0; k < n_alt; ++k)
                if (is_hit(k))
                    or_planes(st, Q,
                              k ? Q.planex_base + static_cast<uint64_t>(x0 + k - 1 - Q.x_base) * Q.words
                                : Q.plane0_base + static_cast<uint64_t>(r - Q.rec_base) * Q.words,
                              samples_out);
    }
    // :244-250
    if (G.flags & GR_HAS_AN) {
        big_add_num(S.an, gs, G.an_num, groups);
    } else if (G.flags & GR_FB) {  // len(get_all_calls(genotypes))
        const uint64_t *toff = gs.tok_off + G.tok_off;
        int64_t n = 0;
        for (uint32_t s = lane; s < Q.n_samples; s += kWave)
            if (!subset || ((subset[s >> 6] >> (s & 63)) & 1ull)) n += static_cast<int64_t>(toff[s + 1] - toff[s]);
        big_add_i64(S.an, wave_sum_i64(n), groups);
    }
    if ((V.flags & F_BOOL_BREAK) && S.exists) return GEN_STOP;  // :253-254
    return GEN_GO;
}

__global__ __launch_bounds__(kWave) void general_slice_kernel(
    DStore st, GStore gs, const uint32_t *__restrict__ work, const uint8_t *__restrict__ qbytes,
    const uint64_t *__restrict__ subsets, QRes *__restrict__ res, uint64_t *__restrict__ hits,
    uint64_t *__restrict__ samples_out, uint8_t *__restrict__ scratch, uint64_t wave_bytes, uint32_t hwords,
    uint32_t tcap, uint32_t *__restrict__ big_n, GenBig *__restrict__ big, uint32_t *__restrict__ big_limbs,
    uint32_t big_cap) {
    const uint32_t lane = static_cast<uint32_t>(lane_id());
    const uint32_t n_work = work[0];
    uint64_t *hbits = reinterpret_cast<uint64_t *>(scratch + blockIdx.x * wave_bytes);
    SetEnt *tabs = reinterpret_cast<SetEnt *>(hbits + hwords);
    const uint32_t groups = (gs.acc_limbs + kWave - 1) / kWave;
    for (uint32_t w = blockIdx.x; w < n_work; w += gridDim.x) {
        const QDev &Q = st.q_all[work[1 + w]];
        QView V;
        V.flags = Q.flags;
        V.ref_mode = Q.ref_mode;
        V.alt_mode = Q.alt_mode;
        V.samples_variant = (V.flags & F_SAMPLES_VARIANT) != 0;
        V.strict_unbound = (V.flags & F_STRICT_UNBOUND) != 0;
        V.qref = qbytes + Q.qbytes_off;
        V.qalt = V.qref + Q.ref_len;
        V.subset = (Q.subset_off != ~0ull) ? subsets + Q.subset_off : nullptr;
        const bool collect = (V.flags & F_COLLECT) && (V.flags & F_DETAILS) && Q.samples_out_off != ~0ull;
        uint32_t lo = Q.seg_lo, hi = Q.seg_lo;
        if (!(Q.flags & F_EMPTY) && Q.first_bp <= Q.last_bp) slice_bounds(st, Q, &lo, &hi);
        if (collect)
            for (uint32_t wd = lane; wd < Q.words; wd += kWave) samples_out[Q.samples_out_off + wd] = 0ull;
        GenSlice S;
        big_zero(S.cc);
        big_zero(S.an);
        S.n_out = 0;
        S.exists = false;
        uint64_t *out = hits + Q.hit_off;
        int err = 0;
        bool stop = false;
        for (uint32_t base = lo; base < hi && !stop; base += kWave) {
            const uint32_t r = base + lane;
            LaneOut o{0, 0, 0, 0, 0};
            if (r < hi) o = eval_record(st, Q, V, r, st.rec[r]);
            const uint32_t nin = min(static_cast<uint32_t>(kWave), hi - base);
            for (uint32_t L = 0; L < nin && !stop; ++L) {
                const int e = static_cast<int>(rdl(static_cast<uint32_t>(o.err), L));
                const uint32_t rr = base + L;
                if (e == SB_QERR_GENERAL) {
                    const int g = general_record(st, gs, Q, V, rr, S, out, samples_out, collect, groups, hbits, tabs,
                                                 tcap);
                    if (g > 0) err = g;
                    if (g != GEN_GO) stop = true;
                    continue;
                }
                if (e) {
                    err = e;
                    stop = true;
                    continue;
                }
                const uint64_t hm = static_cast<uint64_t>(rdl64(static_cast<int64_t>(o.hm), L));
                if (!hm) continue;
                const uint64_t em = static_cast<uint64_t>(rdl64(static_cast<int64_t>(o.em), L));
                if (lane == 0) {
                    uint32_t k = 0;
                    for (uint64_t b = em; b; b &= b - 1)
                        out[S.n_out + k++] = static_cast<uint64_t>(rr) | (static_cast<uint64_t>(ffs64(b)) << kHitAltShift);
                }
                S.n_out += static_cast<uint32_t>(__popcll(em));
                big_add_i64(S.cc, rdl64(o.c, L), groups);
                if (big_nonzero(S.cc, groups)) {
                    S.exists = true;
                    if (!(V.flags & F_DETAILS)) {
                        stop = true;
                        continue;
                    }
                    if (collect) {
                        const uint32_t xl = (hm >> 1) ? st.x_lo[rr] : 0u;
                        for (uint64_t b = hm; b; b &= b - 1) {
                            const int k = ffs64(b);
                            or_planes(st, Q,
                                      k ? Q.planex_base + static_cast<uint64_t>(xl + k - 1 - Q.x_base) * Q.words
                                        : Q.plane0_base + static_cast<uint64_t>(rr - Q.rec_base) * Q.words,
                                      samples_out);
                        }
                    }
                }
                big_add_i64(S.an, rdl64(o.anv, L), groups);
                if ((V.flags & F_BOOL_BREAK) && S.exists) stop = true;
            }
        }
        const int64_t cc = big_low64(S.cc), an = big_low64(S.an);
        const bool wide = !err && !(big_fits64(S.cc, groups) && big_fits64(S.an, groups));
        if (lane == 0)
            res[Q.orig] = QRes{err, (!err && S.exists) ? 1 : 0, err ? 0 : cc, err ? 0 : an, err ? 0u : S.n_out, hi - lo};
        if (wide) {  // Python ints past 64 bits: the exact limbs beside the row
            uint32_t slot = 0;
            if (lane == 0) slot = atomicAdd(big_n, 1u);
            slot = rdl(slot, 0);
            if (slot < big_cap) {
                if (lane == 0) big[slot] = GenBig{Q.orig, 0u};
                uint32_t *dst = big_limbs + static_cast<uint64_t>(slot) * 2u * kGenAccMax;
#pragma unroll
                for (uint32_t t = 0; t < kGenAccGroups; ++t)
                    if (t < groups) {
                        dst[t * kWave + lane] = S.cc[t];
                        dst[kGenAccMax + t * kWave + lane] = S.an[t];
                    }
            }
        }
        if (collect)
            for (uint32_t wd = lane; wd < Q.words; wd += kWave) {
                uint64_t v = err ? 0ull : samples_out[Q.samples_out_off + wd];
                if (V.subset) v &= V.subset[wd];
                samples_out[Q.samples_out_off + wd] = v;
            }
    }
}

}  // namespace

void launch_summarise(const SStore &ss, const SDev *slices, uint32_t ns, const uint32_t *chunk_slice, uint32_t nchunks,
                      uint64_t *bitmap, SPart *part, SRes *out, hipStream_t s) {
    if (!ns) return;
    if (nchunks)
        hipLaunchKernelGGL(summarise_chunk_kernel, dim3(nchunks), dim3(kBlock), 0, s, ss, slices, chunk_slice, nchunks,
                           bitmap, part);
    hipLaunchKernelGGL(summarise_finish_kernel, dim3((ns + kWavesPerBlock - 1) / kWavesPerBlock), dim3(kBlock), 0, s,
                       ss, slices, ns, bitmap, part, out);
}

void launch_chains(const DStore &st, const ChainDev *chains, uint32_t n_chains, const uint32_t *runs, uint32_t n_runs,
                   const uint32_t *corig, QRes *res, uint64_t *hits, ReqPartial *cpart, hipStream_t s) {
    if (!n_chains) return;
    if (res || !cpart)
        hipLaunchKernelGGL(chain_pack_kernel<true>, dim3(blocks_for(n_runs)), dim3(kBlock), 0, s, st, chains, runs, n_runs,
                           corig, res, hits, cpart);
    else
        hipLaunchKernelGGL(chain_pack_kernel<false>, dim3(blocks_for(n_runs)), dim3(kBlock), 0, s, st, chains, runs,
                           n_runs, corig, res, hits, cpart);
}

uint64_t general_wave_bytes(const GStore &gs, uint32_t *hwords, uint32_t *tcap) {
    *hwords = std::max<uint32_t>(1u, (gs.max_alt + kWave - 1) / kWave);
    uint64_t t = 8;
    while (t <= 4ull * std::max(gs.max_vals, gs.max_alt)) t <<= 1;
    *tcap = static_cast<uint32_t>(t);
    const uint64_t b = 8ull * *hwords + 4ull * t * sizeof(SetEnt);
    return (b + 255) & ~255ull;
}

void launch_general(const DStore &st, const GStore &gs, const uint32_t *work, uint32_t grid, const uint8_t *qbytes,
                    const uint64_t *subsets, QRes *res, uint64_t *hits, uint64_t *samples_out, uint8_t *scratch,
                    uint32_t *big_n, GenBig *big, uint32_t *big_limbs, uint32_t big_cap, hipStream_t s) {
    if (!grid) return;
    uint32_t hwords, tcap;
    const uint64_t wb = general_wave_bytes(gs, &hwords, &tcap);
    hipLaunchKernelGGL(general_slice_kernel, dim3(grid), dim3(kWave), 0, s, st, gs, work, qbytes, subsets, res, hits,
                       samples_out, scratch, wb, hwords, tcap, big_n, big, big_limbs, big_cap);
}

void launch_request_rows(const DStore &st, const ReqChain *chains, RowRun *runs, uint32_t n_runs,
                         unsigned long long *status, unsigned long long *tstatus, const QRes *sres,
                         const uint32_t *sseg, const uint64_t *shoff, const uint8_t *sherr, const uint64_t *shits,
                         ReqPartial *rows, uint64_t *row_off, uint64_t *row_src, uint32_t *stage, uint64_t *out,
                         uint32_t n_rows, uint64_t rec_base, uint32_t n_lut, uint32_t run, unsigned int *err,
                         int compact, bool rec_staged, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                         const ReqIn *plan_in, uint32_t n_in, uint64_t stride, int inject, bool tile_scan,
                         const ReqEsc &esc, bool lab7) {
    const bool rowc = compact == SB_COMPACT_ALL, hitc = compact != 0;  // u32 rows / offsets; u32 hits
    if (!n_runs) {
        (void)hipMemsetAsync(row_off, 0, rowc ? 4 : 8, s);
        return;
    }
    const dim3 grid(blocks_for(n_runs));
    const uint32_t n_tiles = request_tiles(n_runs), n_groups = blocks_for(n_runs);
    unsigned long long *const gtot = tstatus + n_tiles;  // eval workgroup totals (request_tstatus_words)
    if (ev0) (void)hipEventRecord(ev0, s);
    auto eval = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(kBlock), 0, s, st, chains, runs, n_runs, status, sres,
                           static_cast<void *>(rows), static_cast<void *>(row_off), row_src, stage, n_lut, err,
                           static_cast<uint32_t>(inject), gtot, plan_in, n_in, stride, esc);
    };
    (void)run;
    auto eval_rec = [&](auto rec, auto plan) {
        constexpr bool R = decltype(rec)::value, P = decltype(plan)::value;
        if (rowc) {
            if (n_lut <= kReqLut) eval(request_eval_kernel<true, true, R, P>);
            else eval(request_eval_kernel<false, true, R, P>);
        } else {
            if (n_lut <= kReqLut) eval(request_eval_kernel<true, false, R, P>);
            else eval(request_eval_kernel<false, false, R, P>);
        }
    };
    // (the planning fused only with record staging: the form every store
    // below 2^29 records takes)
    if (plan_in && rec_staged) eval_rec(std::true_type{}, std::true_type{});
    else if (rec_staged) eval_rec(std::true_type{}, std::false_type{});
    else eval_rec(std::false_type{}, std::false_type{});
    if (ev1) (void)hipEventRecord(ev1, s);
    // record staging: the delivery sums the eval workgroup totals itself (no
    // tile scan launch; SBEACON_REQ_TILE_SCAN=1 keeps it).  Each delivery
    // workgroup reads every earlier group's total, so the reads grow with the
    // square of the groups: 7.6 M words per pass at 3,906 groups (1 M
    // requests), 4x that at twice the groups -- past kGsumMaxGroups the
    // one-launch tile scan (linear) is cheaper than its saved launch
    constexpr uint32_t kGsumMaxGroups = 4096;
    const bool gsum = rec_staged && !tile_scan && n_groups <= kGsumMaxGroups;
    if (!gsum)
        hipLaunchKernelGGL(request_tile_scan_kernel, dim3(1), dim3(1024), 0, s, gtot, n_groups, tstatus, n_tiles);
    auto deliver = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(kBlock), 0, s, runs, n_runs, status, tstatus, sres, sseg, shoff, sherr,
                           shits, static_cast<void *>(row_off), row_src, stage, st.vc_idx, static_cast<void *>(out),
                           n_rows, rec_base, err, gtot, esc);
    };
    auto deliver_rec = [&](auto rec, auto gs) {
        constexpr bool R = decltype(rec)::value, G = decltype(gs)::value;
        auto lab = [&](auto l) {
            constexpr bool L7 = decltype(l)::value;
            if (rowc && sres) deliver(request_deliver_kernel<true, true, R, G, true, L7>);
            else if (rowc) deliver(request_deliver_kernel<true, true, R, G, false, L7>);
            else if (hitc) deliver(request_deliver_kernel<false, true, R, G, true, L7>);
            else deliver(request_deliver_kernel<false, false, R, G, true, false>);
        };
        if (lab7) lab(std::true_type{});
        else lab(std::false_type{});
    };
    if (gsum) deliver_rec(std::true_type{}, std::true_type{});
    else if (rec_staged) deliver_rec(std::true_type{}, std::false_type{});
    else deliver_rec(std::false_type{}, std::false_type{});
}

void launch_request_plan(const DStore &st, const ReqIn *in, uint32_t n, ReqChain *chains, RowRun *runs,
                         unsigned long long *rcap, unsigned long long *counters, hipStream_t s, uint64_t stride,
                         unsigned int *err) {
    const uint32_t n_runs = (n + kRunRows - 1) / kRunRows;
    if (!n_runs) return;
    // per plan workgroup totals after the counters (requests.cpp sizes the buffer: request_plan_words)
    unsigned long long *gcap = counters + 4;
    hipLaunchKernelGGL(request_plan_kernel, dim3(blocks_for(n_runs)), dim3(kBlock), 0, s, st, in, n, n_runs, chains,
                       runs, rcap, gcap, stride, err);
    if (!stride)  // (a fixed-stride batch re-planning: the offsets are w x stride, the totals known)
        hipLaunchKernelGGL(request_stage_scan_kernel, dim3((n_runs + kStageTile - 1) / kStageTile), dim3(kStageTile),
                           0, s, runs, rcap, gcap, n_runs, counters);
}

// planning scratch (u64 words): per run {capacity, slices | chains}, the
// three batch counters (+ pad), per plan workgroup the same two totals
size_t request_plan_words(uint32_t n_runs) { return size_t(n_runs) * 2 + 4 + size_t(blocks_for(n_runs)) * 2; }

// run totals (request_eval_kernel) -> tile offsets (request_tile_scan_kernel)
uint32_t request_tiles(uint32_t n_runs) { return (n_runs + kDeliverTile - 1) / kDeliverTile; }
// tile offsets, then the eval workgroups' totals
size_t request_tstatus_words(uint32_t n_runs) { return size_t(request_tiles(n_runs)) + blocks_for(n_runs); }

uint32_t pack_run_max() { return kPackRun; }
uint32_t req_run_max() { return kReqRun; }
uint32_t pack_slots_max() { return kPackSlots; }

void launch_chain_src(const ChainDev *chains, uint32_t n_chains, const uint32_t *corig, const QRes *res,
                      uint64_t *src, hipStream_t s) {
    if (!n_chains) return;
    hipLaunchKernelGGL(chain_src_kernel, dim3((n_chains + kBlock - 1) / kBlock), dim3(kBlock), 0, s, chains, n_chains,
                       corig, res, src);
}

size_t hit_scan_words(uint32_t nq) { return (nq + kScanTile - 1) / kScanTile + 1; }

void launch_hit_lists(const QRes *res, uint32_t nq, const uint64_t *src, const uint64_t *hits, uint64_t rec_base,
                      const uint32_t *seg, uint32_t n_rows, uint64_t *tsum, uint64_t *dense, uint64_t *out,
                      uint64_t *row_off, hipStream_t s) {
    const uint32_t nt = (nq + kScanTile - 1) / kScanTile;
    if (nt) hipLaunchKernelGGL(hit_tile_sum_kernel, dim3(nt), dim3(kBlock), 0, s, res, nq, tsum);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kBlock), 0, s, tsum, nt);
    if (nt) {
        hipLaunchKernelGGL(hit_tile_scan_kernel, dim3(nt), dim3(kBlock), 0, s, res, nq, tsum, dense);
        hipLaunchKernelGGL(hit_gather_kernel, dim3((nq + kBlock - 1) / kBlock), dim3(kBlock), 0, s, res, nq, src, dense,
                           hits, rec_base, out);
    } else {
        (void)hipMemsetAsync(dense, 0, 8, s);
    }
    if (seg && row_off)
        hipLaunchKernelGGL(row_off_kernel, dim3((n_rows + 1 + kBlock - 1) / kBlock), dim3(kBlock), 0, s, seg, n_rows,
                           dense, row_off);
}

void launch_row_reduce(const ReqPartial *cpart, const ChainDev *chains, const uint64_t *hoff, const QRes *res,
                       const uint8_t *host_err, const uint32_t *poff, const uint32_t *piece, uint32_t n_rows,
                       ReqPartial *out, ulonglong2 *rowsrc, hipStream_t s) {
    if (!n_rows) return;
    hipLaunchKernelGGL(row_reduce_kernel, dim3((n_rows + kBlock - 1) / kBlock), dim3(kBlock), 0, s, cpart, chains,
                       hoff, res, host_err, poff, piece, n_rows, out, rowsrc);
}

void launch_row_deliver(const ReqPartial *cpart, const ChainDev *chains, const uint64_t *hoff, const QRes *res,
                        const uint8_t *host_err, const uint32_t *poff, const uint32_t *piece, uint32_t n_rows,
                        ReqPartial *rows, ulonglong2 *rowsrc, const uint64_t *rowout, int64_t *nv, uint64_t *tsum,
                        const uint64_t *hits, uint64_t rec_base, uint64_t *row_off, uint64_t *out, hipStream_t s) {
    const uint32_t nt = (n_rows + kScanTile - 1) / kScanTile;
    if (!nt) {
        (void)hipMemsetAsync(row_off, 0, 8, s);
        return;
    }
    // rowout (static hit region of each single-piece row, ~0 for several
    // pieces): the reduction skips the scattered chain-descriptor reads and the
    // rowsrc writes
    hipLaunchKernelGGL(row_reduce_tiles_kernel, dim3(nt), dim3(kBlock), 0, s, cpart, chains, hoff, res, host_err, poff,
                       piece, n_rows, rows, rowout ? nullptr : rowsrc, nv, tsum);
    hipLaunchKernelGGL(field_scan_fused_kernel, dim3(nt), dim3(kBlock), 0, s, nv, n_rows, tsum, row_off);
    hipLaunchKernelGGL(row_gather_seg_kernel, dim3(blocks_for((n_rows + kWave - 1) / kWave)), dim3(kBlock), 0, s, poff,
                       piece, n_rows, chains, cpart, res, hoff, hits, rec_base, row_off,
                       rowout ? rowout : reinterpret_cast<const uint64_t *>(rowsrc), rowout ? 1u : 2u, out);
}

void launch_row_hit_lists(const ReqPartial *rows, const ulonglong2 *rowsrc, const uint32_t *poff,
                          const uint32_t *piece, uint32_t n_rows, const ChainDev *chains, const ReqPartial *cpart,
                          const QRes *res, const uint64_t *hoff, const uint64_t *hits, uint64_t rec_base,
                          uint64_t *tsum, uint64_t *row_off, uint64_t *out, hipStream_t s) {
    const uint32_t nt = (n_rows + kScanTile - 1) / kScanTile;
    const int64_t *nv = reinterpret_cast<const int64_t *>(rows) + 1;  // ReqPartial::n_variants
    constexpr uint32_t stride = sizeof(ReqPartial) / sizeof(int64_t);
    if (nt) hipLaunchKernelGGL(field_tile_sum_kernel, dim3(nt), dim3(kBlock), 0, s, nv, stride, n_rows, tsum);
    hipLaunchKernelGGL(tile_scan_kernel, dim3(1), dim3(kBlock), 0, s, tsum, nt);
    if (!nt) {
        (void)hipMemsetAsync(row_off, 0, 8, s);
        return;
    }
    hipLaunchKernelGGL(field_tile_scan_kernel, dim3(nt), dim3(kBlock), 0, s, nv, stride, n_rows, tsum, row_off);
    hipLaunchKernelGGL(row_gather_seg_kernel, dim3(blocks_for((n_rows + kWave - 1) / kWave)), dim3(kBlock), 0, s, poff,
                       piece, n_rows, chains, cpart, res, hoff, hits, rec_base, row_off,
                       reinterpret_cast<const uint64_t *>(rowsrc), 2u, out);
}

void mark_wide(const uint32_t *big_n, const GenBig *big, uint32_t cap, uint8_t *wide, hipStream_t s) {
    hipLaunchKernelGGL(mark_wide_kernel, dim3(std::max<uint32_t>(1, std::min<uint32_t>(64, (cap + kBlock - 1) / kBlock))),
                       dim3(kBlock), 0, s, big_n, big, cap, wide);
}

void launch_request_reduce(const QRes *res, const uint32_t *seg, const uint8_t *host_err, const uint8_t *wide,
                           uint32_t n_rows, ReqPartial *out, uint8_t *row_flag, hipStream_t s) {
    if (!n_rows) return;
    hipLaunchKernelGGL(request_reduce_kernel, dim3((n_rows + kBlock - 1) / kBlock), dim3(kBlock), 0, s, res, seg,
                       host_err, wide, n_rows, out, row_flag);
}

void launch_compact(const uint64_t *hit_off, const uint64_t *dense_off, const QRes *res, uint32_t nq,
                    const uint64_t *hits, uint64_t *out, hipStream_t s) {
    if (!nq) return;
    hipLaunchKernelGGL(compact_kernel, dim3(blocks_for(nq)), dim3(kBlock), 0, s, hit_off, dense_off, res, nq, hits,
                       out);
}

template <bool NONNEG>
void launch_variant(int nacc, int mode, dim3 g, const DStore &st, const QDev *q, const uint32_t *qidx, uint32_t n,
                    uint32_t run,
                    const uint8_t *qbytes, const uint64_t *subsets, QRes *res, uint64_t *hits, uint64_t *samples_out,
                    hipStream_t s) {
    const dim3 b(kBlock);
#define SB_SCAN(NA, MO) hipLaunchKernelGGL((scan_kernel<NA, NONNEG, MO, false>), g, b, 0, s, st, q, qidx, n, run, qbytes, subsets, res, hits, samples_out)
    switch (nacc) {
        case 0: SB_SCAN(0, MODE_GENERAL); break;
        case 1: SB_SCAN(1, MODE_GENERAL); break;
        case 4: SB_SCAN(4, MODE_GENERAL); break;
        default: SB_SCAN(16, MODE_GENERAL); break;
    }
#undef SB_SCAN
}

void launch_scan(const DStore &st, const QDev *q, const uint32_t *qidx, uint32_t n, bool nonneg, uint32_t max_words,
                 int mode, const uint8_t *qbytes, const uint64_t *subsets, QRes *res, uint64_t *hits,
                 uint64_t *samples_out, hipStream_t s) {
    if (!n) return;
    int nacc = max_words == 0 ? 0 : max_words <= 64 ? 1 : max_words <= 256 ? 4 : 16;
    // SBEACON_MAX_NACC (tests): shrink the register window so small cohorts
    // exercise the words-beyond-the-window path of >65,536-sample VCFs
    const int cap = config().max_nacc;
    if (nacc > 0 && cap >= 1) nacc = std::min(nacc, cap >= 16 ? 16 : cap >= 4 ? 4 : 1);
    if (nacc == 0) {  // every sample-free specialisation goes through the fused kernel
        if (qidx) throw std::runtime_error("launch_scan: sample-free queries must be contiguous (qidx = null)");
        const FusedGroup one{q, n, mode};
        launch_fused(st, &one, 1, nonneg, qbytes, subsets, res, hits, s);
        return;
    }
    const uint32_t run = 1;  // the sample path keeps one slice per wave
    const dim3 g(blocks_for(n));
    if (nonneg)
        launch_variant<true>(nacc, mode, g, st, q, qidx, n, run, qbytes, subsets, res, hits, samples_out, s);
    else
        launch_variant<false>(nacc, mode, g, st, q, qidx, n, run, qbytes, subsets, res, hits, samples_out, s);
}

void launch_fused(const DStore &st, const FusedGroup *groups, int count, bool nonneg, const uint8_t *qbytes,
                  const uint64_t *subsets, QRes *res, uint64_t *hits, hipStream_t s) {
    FusedGroups G{};
    uint32_t waves = 0;
    int c = 0;
    for (int i = 0; i < count; ++i) {
        if (!groups[i].n) continue;
        if (c == kFusedMax) throw std::runtime_error("launch_fused: too many groups");
        G.q[c] = groups[i].q;
        G.n[c] = groups[i].n;
        G.mode[c] = groups[i].mode;
        G.run[c] = run_for(groups[i].n);
        ++c;
    }
    // slice runs only when some group is large enough to use them (run_slices
    // costs registers); otherwise every group runs one slice per wave
    bool run = false;
    for (int i = 0; i < c; ++i) run = run || G.run[i] > 1;
    for (int i = 0; i < c; ++i) {
        G.wave_begin[i] = waves;
        waves += blocks_for(run_waves(G.n[i], G.run[i])) * kWavesPerBlock;
    }
    if (!c) return;
    G.count = c;
    G.wave_begin[c] = waves;
    const dim3 g(waves / kWavesPerBlock), b(kBlock);
    if (c == 1) {  // a single group: its own specialisation (smaller code, no group dispatch)
        const QDev *q = G.q[0];
        const uint32_t *qi = nullptr;  // the group's queries are contiguous in launch order
        const uint32_t n = G.n[0], rn = G.run[0];
#define SB_ONE(NN, RR)                                                                                         \
        switch (G.mode[0]) {                                                                                   \
            case MODE_RANGE_N: hipLaunchKernelGGL((range_n_kernel<NN, RR>), g, b, 0, s, st, q, qi, n, rn, res, hits); break; \
            case MODE_RANGE_N8: hipLaunchKernelGGL((range_n8_kernel<NN, RR>), g, b, 0, s, st, q, qi, n, rn, res, hits); break; \
            case MODE_VTYPE: hipLaunchKernelGGL((vt_kernel<NN, RR>), g, b, 0, s, st, q, qi, n, rn, res, hits); break;        \
            case MODE_EXACT:                                                                                   \
                hipLaunchKernelGGL((scan_kernel<0, NN, MODE_EXACT, RR>), g, b, 0, s, st, q, qi, n, rn, qbytes, subsets, res, hits, nullptr); \
                break;                                                                                         \
            default:                                                                                           \
                hipLaunchKernelGGL((scan_kernel<0, NN, MODE_GENERAL, RR>), g, b, 0, s, st, q, qi, n, rn, qbytes, subsets, res, hits, nullptr); \
                break;                                                                                         \
        }
        if (nonneg) {
            if (run) { SB_ONE(true, true) } else { SB_ONE(true, false) }
        } else {
            if (run) { SB_ONE(false, true) } else { SB_ONE(false, false) }
        }
#undef SB_ONE
        return;
    }
    if (nonneg) {
        if (run) hipLaunchKernelGGL((fused_kernel<true, true>), g, b, 0, s, st, G, qbytes, subsets, res, hits);
        else hipLaunchKernelGGL((fused_kernel<true, false>), g, b, 0, s, st, G, qbytes, subsets, res, hits);
    } else {
        if (run) hipLaunchKernelGGL((fused_kernel<false, true>), g, b, 0, s, st, G, qbytes, subsets, res, hits);
        else hipLaunchKernelGGL((fused_kernel<false, false>), g, b, 0, s, st, G, qbytes, subsets, res, hits);
    }
}

}  // namespace sb
