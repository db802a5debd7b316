// query_kernels.hip — CDNA4 (gfx950) kernels of the slice-query hot path.
//
// Reference semantics: lambda/performQuery/search_variants.py:33-271 and
// search_variants_in_samples.py:31-259 (restated in SURVEY.md §8a.1).  The
// reference walks `bcftools query` output record by record in a Python loop;
// here one 64-lane wavefront owns one slice query and walks its records 64 at
// a time with coalesced SoA loads, turning the loop's order-dependent state
// (cumulative call_count, include_details/boolean early exits, first error)
// into ballots and wave prefix sums.
//
// All arithmetic is integer; nothing here is a dense contraction, so no MFMA.
// The bound is HBM/Infinity-Cache bandwidth on the record columns.
#include <hip/hip_runtime.h>

#include "../../include/sbeacon.h"
#include "devtypes.hpp"
#include "kernels.hpp"

namespace sb {

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

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

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t t = __shfl_up(v, d, kWave);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += shfl_i64(v, lane_id() ^ d);
    return v;
}

__device__ __forceinline__ uint8_t up(uint8_t c) { return (c >= 'a' && c <= 'z') ? c - 32 : c; }

// 64-ary search: first idx in [L, H) with pos[idx] >= x, H if none.  Each
// step is one dependent round of 64 independent loads (the
// lower_bound term 4 B x ceil(log2 N) per query).
__device__ uint32_t wave_lower_bound(const uint32_t *__restrict__ pos, uint32_t L, uint32_t H, int64_t x) {
    const int lane = lane_id();
    while (H - L > kWave) {
        const uint32_t step = (H - L + kWave - 1) / kWave;
        const uint32_t s = L + static_cast<uint32_t>(lane) * step;
        const bool ge = (s < H) ? (static_cast<int64_t>(pos[s]) >= x) : true;
        const uint64_t m = __ballot(ge);
        const int f = m ? __ffsll(static_cast<unsigned long long>(m)) - 1 : kWave;
        if (f == 0) return L;
        const uint32_t prev = L + static_cast<uint32_t>(f - 1) * step;
        uint32_t nh = H;
        if (f < kWave) {
            const uint32_t sf = L + static_cast<uint32_t>(f) * step;
            nh = sf < H ? sf : H;
        }
        L = prev + 1;
        H = nh;
    }
    const uint32_t i = L + static_cast<uint32_t>(lane);
    const bool ge = (i < H) ? (static_cast<int64_t>(pos[i]) >= x) : true;
    const uint64_t m = __ballot(ge);
    if (!m) return H;
    const uint32_t r = L + static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(m)) - 1);
    return r < H ? r : H;
}

__global__ __launch_bounds__(kBlock) void bounds_kernel(DStore st, const QDev *__restrict__ qs, uint32_t nq,
                                                        uint32_t *__restrict__ lohi, uint32_t *__restrict__ caps) {
    const uint32_t q = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    if (q >= nq) return;
    const QDev &Q = qs[q];
    uint32_t lo = Q.seg_lo, hi = Q.seg_lo;
    if (!(Q.flags & F_EMPTY) && Q.first_bp <= Q.last_bp) {
        lo = wave_lower_bound(st.pos, Q.seg_lo, Q.seg_hi, Q.first_bp);
        hi = wave_lower_bound(st.pos, lo, Q.seg_hi, Q.last_bp + 1);
    }
    if (lane_id() == 0) {
        lohi[2 * q] = lo;
        lohi[2 * q + 1] = hi;
        caps[q] = st.alt_lo[hi] - st.alt_lo[lo];
    }
}

// ---------------------------------------------------------------- prefix sum
constexpr uint32_t kScanItems = 8;
constexpr uint32_t kScanTile = kBlock * kScanItems;

__device__ __forceinline__ uint64_t block_excl_scan_u64(uint64_t v, uint64_t *lds, uint64_t *total) {
    // wave scan then scan of wave totals
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    uint64_t x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint64_t t = static_cast<uint64_t>(shfl_up_i64(static_cast<int64_t>(x), d));
        if (lane >= d) x += t;
    }
    if (lane == kWave - 1) lds[wave] = x;
    __syncthreads();
    uint64_t off = 0, tot = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) {
        if (w < wave) off += lds[w];
        tot += lds[w];
    }
    __syncthreads();
    *total = tot;
    return off + x - v;
}

__global__ __launch_bounds__(kBlock) void scan_reduce_kernel(const uint32_t *__restrict__ in, uint32_t n,
                                                             uint64_t *__restrict__ block_sums) {
    __shared__ uint64_t lds[kWavesPerBlock];
    const uint32_t base = blockIdx.x * kScanTile;
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanItems; ++k) {
        const uint32_t i = base + k * kBlock + threadIdx.x;
        if (i < n) s += in[i];
    }
    uint64_t tot;
    block_excl_scan_u64(s, lds, &tot);
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void scan_blocks_kernel(uint64_t *__restrict__ block_sums, uint32_t nb) {
    __shared__ uint64_t lds[kWavesPerBlock];
    uint64_t carry = 0;
    for (uint32_t base = 0; base < nb; base += kBlock) {
        const uint32_t i = base + threadIdx.x;
        const uint64_t v = i < nb ? block_sums[i] : 0;
        uint64_t tot;
        const uint64_t ex = block_excl_scan_u64(v, lds, &tot);
        if (i < nb) block_sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) block_sums[nb] = carry;
}

__global__ __launch_bounds__(kBlock) void scan_apply_kernel(const uint32_t *__restrict__ in, uint32_t n,
                                                            const uint64_t *__restrict__ block_off,
                                                            uint32_t nb, uint64_t *__restrict__ out) {
    __shared__ uint64_t lds[kWavesPerBlock];
    // each thread owns kScanItems consecutive elements of the tile
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t v[kScanItems];
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < kScanItems; ++k) {
        v[k] = (base + k < n) ? in[base + k] : 0u;
        s += v[k];
    }
    uint64_t tot;
    uint64_t run = block_off[blockIdx.x] + block_excl_scan_u64(s, lds, &tot);
#pragma unroll
    for (uint32_t k = 0; k < kScanItems; ++k) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
    }
    if (blockIdx.x == nb - 1 && threadIdx.x == 0) out[n] = block_off[nb];
}

// ---------------------------------------------------------------- scan kernel
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
                               uint32_t plen) {
    if (ref_len != plen) return false;
    const uint64_t key = st.ref_key[r];
    if (!(st.meta[r] & M_REF_HASHED)) {
        for (uint32_t i = 0; i < plen; ++i)
            if (!wild_char(static_cast<uint8_t>(key >> (8 * i)), pat[i])) return false;
        return true;
    }
    const uint64_t off = st.ref_off[r];
    for (uint32_t i = 0; i < plen; ++i)
        if (!wild_char(up(st.blob[off + i]), pat[i])) return false;
    return true;
}

// genotype fallback over the selected samples (samples variant, record
// without AC / AN): search_variants_in_samples.py:211-222 and :239-245 with
// bcftools --samples restricting the GT text.  `value` = allele number to
// count (0 = count every call).  Rare path: one lane walks the subset.
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

template <int NACC>
__global__ __launch_bounds__(kBlock) void scan_kernel(DStore st, const QDev *__restrict__ qs, uint32_t nq,
                                                      const uint32_t *__restrict__ lohi,
                                                      const uint64_t *__restrict__ hit_off,
                                                      const uint8_t *__restrict__ qbytes,
                                                      const uint64_t *__restrict__ subsets,
                                                      QRes *__restrict__ res, uint32_t *__restrict__ nhits,
                                                      uint32_t *__restrict__ hit_rec,
                                                      uint32_t *__restrict__ hit_alt,
                                                      uint64_t *__restrict__ samples_out) {
    const uint32_t q = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    if (q >= nq) return;
    const int lane = lane_id();
    const QDev &Q = qs[q];
    const uint32_t lo = lohi[2 * q], hi = lohi[2 * q + 1];
    const uint64_t out = hit_off[q];
    const uint32_t flags = Q.flags;
    const bool details = flags & F_DETAILS;
    const bool samples_variant = flags & F_SAMPLES_VARIANT;
    const bool collect = (flags & F_COLLECT) && details;
    const bool stop_on_exists = !details || (flags & F_BOOL_BREAK);
    const uint8_t *qref = qbytes + Q.qbytes_off;
    const uint8_t *qalt = qref + Q.ref_len;
    const uint64_t *subset = (Q.subset_off != ~0ull) ? subsets + Q.subset_off : nullptr;

    int64_t carry = 0, an_sum = 0;
    uint32_t n_out = 0;
    bool exists = false;
    int err_out = 0;
    uint64_t acc[NACC];
#pragma unroll
    for (int j = 0; j < NACC; ++j) acc[j] = 0;

    for (uint32_t base = lo; base < hi; base += kWave) {
        const uint32_t r = base + static_cast<uint32_t>(lane);
        int err = 0;
        uint64_t hm = 0, em = 0;
        int64_t c = 0, anv = 0;
        uint32_t a0 = 0;
        if (r < hi) {
            const uint32_t e = st.end[r];
            bool pass = static_cast<int64_t>(e) >= Q.end_min && static_cast<int64_t>(e) <= Q.end_max; // :90
            if (pass) {
                switch (Q.ref_mode) {  // :94 / svs:88-91
                    case REF_ANY:
                        break;
                    case REF_EXACT: {
                        const uint64_t k = st.ref_key[r];
                        pass = k == Q.ref_key;
                        if (pass && (k >> 63)) {
                            const uint32_t rl = e - st.pos[r] + 1;
                            pass = blob_eq_upper(st.blob, st.ref_off[r], rl, qref, Q.ref_len);
                        }
                        break;
                    }
                    case REF_WILD:
                        pass = ref_wild_match(st, r, e - st.pos[r] + 1, qref, Q.ref_len);
                        break;
                    case REF_NEVER:
                        pass = false;
                        break;
                    default:
                        err = static_cast<int>(Q.ref_err);
                        pass = false;
                        break;
                }
            }
            if (pass && (flags & F_STRICT_UNBOUND)) {  // :101 in the unpatched reference
                err = SB_QERR_UNBOUND_LOCAL;
                pass = false;
            }
            if (pass) {
                a0 = st.alt_lo[r];
                const uint32_t na = st.alt_lo[r + 1] - a0;
                const int64_t ref_len = (Q.alt_mode == ALT_VTYPE) ? static_cast<int64_t>(e) - st.pos[r] + 1 : 0;
                for (uint32_t k = 0; k < na && k < 64; ++k) {  // :100-183 hit_indexes
                    const uint32_t a = a0 + k;
                    const uint32_t cls = st.alt_cls[a];
                    bool ok;
                    int64_t len = 1;
                    if (Q.alt_mode == ALT_N) {
                        ok = cls & A_SINGLE_BASE;
                    } else if (Q.alt_mode == ALT_EXACT) {
                        ok = st.alt_key[a] == Q.alt_key;
                        len = st.alt_len[a];
                        if (ok && (cls & A_HASHED))
                            ok = blob_eq_upper(st.blob, st.alt_off[a], static_cast<uint32_t>(len), qalt, Q.alt_len);
                    } else {
                        len = st.alt_len[a];
                        if (cls & A_SYMBOLIC) {
                            const uint32_t sym = cls >> A_SYM_SHIFT;
                            ok = (st.sym_lut[Q.lut_off + (sym >> 5)] >> (sym & 31)) & 1u;
                        } else {
                            const uint32_t rep = (cls >> A_REP_SHIFT) & 63u;
                            switch (Q.vt_kind) {
                                case VT_DEL: ok = len < ref_len; break;
                                case VT_INS: ok = len > ref_len; break;
                                case VT_DUP: ok = rep != A_REP_NONE && rep >= 2; break;
                                case VT_DUPT: ok = rep == 2; break;
                                case VT_CNV: ok = (cls & A_DOT) || rep != A_REP_NONE; break;
                                default: ok = false; break;
                            }
                        }
                    }
                    if (ok && len >= Q.vmin && len <= Q.vmax) hm |= 1ull << k;
                }
                if (hm) {
                    const uint32_t m = st.meta[r];
                    const bool sub = samples_variant && (m & M_HAS_FB);
                    if (m & M_AN_BAD) {
                        err = SB_QERR_VALUE;  // :199
                    } else if (m & M_HAS_AC) {  // :205-214
                        if (m & M_AC_BAD) {
                            err = SB_QERR_VALUE;  // :206
                        } else {
                            for (uint64_t b = hm; b; b &= b - 1) {
                                const int k = __ffsll(static_cast<unsigned long long>(b)) - 1;
                                if (st.alt_cls[a0 + k] & A_AC_MISSING) err = SB_QERR_INDEX;  // :207
                                const int64_t v = st.ac[a0 + k];
                                c += v;
                                if (v != 0) em |= 1ull << k;
                            }
                        }
                    } else {  // :215-226 genotype fallback (1-based alts[] label)
                        for (uint64_t b = hm; b; b &= b - 1) {
                            const int k = __ffsll(static_cast<unsigned long long>(b)) - 1;
                            const int64_t v = sub ? fallback_count(st, r, subset, Q.n_samples, k + 1) : st.ac[a0 + k];
                            c += v;
                            if (v > 0) {
                                if (static_cast<uint32_t>(k + 1) >= na) err = SB_QERR_INDEX;  // :223
                                else em |= 1ull << (k + 1);
                            }
                        }
                    }
                    // :244-250
                    anv = (m & M_HAS_AN) ? st.an[r] : (sub ? fallback_count(st, r, subset, Q.n_samples, 0) : st.an[r]);
                    if (err) {
                        hm = 0;
                        em = 0;
                        c = 0;
                    }
                }
            }
        }
        // ---- order-dependent loop state (:229-254) as wave operations
        const bool hit = hm != 0;
        const uint64_t errm = __ballot(err != 0);
        const int64_t cum = carry + wave_incl_scan_i64(hit ? c : 0);
        const bool trig = hit && cum != 0;  // `if call_count:` on the running total
        const uint64_t trigm = __ballot(trig);
        const uint64_t stopm = errm | (stop_on_exists ? trigm : 0ull);
        const int s = stopm ? __ffsll(static_cast<unsigned long long>(stopm)) - 1 : kWave;
        if (s < kWave && ((errm >> s) & 1ull)) {
            err_out = __shfl(err, s, kWave);
            break;
        }
        const uint64_t upto = (s >= kWave - 1) ? ~0ull : ((2ull << s) - 1ull);
        const bool in = (upto >> lane) & 1ull;
        // compacted emission of variant strings (:209-213 / :222-225)
        const uint32_t cnt = (hit && in) ? static_cast<uint32_t>(__popcll(em)) : 0u;
        const uint32_t incl = wave_incl_scan_u32(cnt);
        if (cnt) {
            uint64_t dst = out + n_out + (incl - cnt);
            for (uint64_t b = em; b; b &= b - 1) {
                hit_rec[dst] = r;
                hit_alt[dst] = static_cast<uint32_t>(__ffsll(static_cast<unsigned long long>(b)) - 1);
                ++dst;
            }
        }
        n_out += __shfl(incl, kWave - 1, kWave);
        // all_alleles_count: lanes before the stop, plus the stop lane when the
        // stop is the boolean break (AN added before :253) rather than :231
        const bool an_in = hit && (lane < s || (lane == s && details));
        an_sum += wave_sum_i64(an_in ? anv : 0);
        exists = exists || ((trigm & upto) != 0ull);
        carry = shfl_i64(cum, s < kWave ? s : kWave - 1);
        // sample path (:233-236): OR the carrier planes of every hit allele
        if (collect) {
            uint64_t cm = trigm & upto;
            while (cm) {
                const int L = __ffsll(static_cast<unsigned long long>(cm)) - 1;
                cm &= cm - 1;
                const uint64_t hml = static_cast<uint64_t>(shfl_i64(static_cast<int64_t>(hm), L));
                const uint32_t a0l = static_cast<uint32_t>(__shfl(static_cast<int>(a0), L, kWave));
                for (uint64_t b = hml; b; b &= b - 1) {
                    const int k = __ffsll(static_cast<unsigned long long>(b)) - 1;
                    const uint64_t row = Q.plane_base + static_cast<uint64_t>(a0l + k - Q.alt_base) * Q.words;
#pragma unroll
                    for (int j = 0; j < NACC; ++j) {
                        const uint32_t w = static_cast<uint32_t>(lane) + 64u * j;
                        if (w < Q.words) acc[j] |= st.planes[row + w];
                    }
                }
            }
        }
        if (s < kWave) break;
    }

    if (lane == 0) {
        QRes o;
        o.error = err_out;
        o.exists = exists ? 1 : 0;
        o.call_count = carry;
        o.all_alleles_count = an_sum;
        o.n_hits = err_out ? 0u : n_out;
        o.n_scanned = hi - lo;
        res[q] = o;
        nhits[q] = o.n_hits;
    }
    if (collect && Q.samples_out_off != ~0ull) {
#pragma unroll
        for (int j = 0; j < NACC; ++j) {
            const uint32_t w = static_cast<uint32_t>(lane) + 64u * j;
            if (w < Q.words) {
                uint64_t v = err_out ? 0ull : acc[j];
                if (subset) v &= subset[w];
                samples_out[Q.samples_out_off + w] = v;
            }
        }
    }
}

__global__ __launch_bounds__(kBlock) void compact_kernel(const uint64_t *__restrict__ hit_off,
                                                         const uint64_t *__restrict__ dense_off,
                                                         const uint32_t *__restrict__ nhits, uint32_t nq,
                                                         const uint32_t *__restrict__ hit_rec,
                                                         const uint32_t *__restrict__ hit_alt,
                                                         uint32_t *__restrict__ out_rec,
                                                         uint32_t *__restrict__ out_alt) {
    const uint32_t q = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
    if (q >= nq) return;
    const uint64_t src = hit_off[q], dst = dense_off[q];
    const uint32_t n = nhits[q];
    for (uint32_t i = static_cast<uint32_t>(lane_id()); i < n; i += kWave) {
        out_rec[dst + i] = hit_rec[src + i];
        out_alt[dst + i] = hit_alt[src + i];
    }
}

inline uint32_t blocks_for(uint32_t nq) { return (nq + kWavesPerBlock - 1) / kWavesPerBlock; }

}  // namespace

void launch_bounds(const DStore &st, const QDev *q, uint32_t nq, uint32_t *lohi, uint32_t *caps, hipStream_t s) {
    if (!nq) return;
    hipLaunchKernelGGL(bounds_kernel, dim3(blocks_for(nq)), dim3(kBlock), 0, s, st, q, nq, lohi, caps);
}

size_t scan_tmp_words(uint32_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

void launch_exclusive_scan(const uint32_t *in, uint32_t n, uint64_t *out, uint64_t *tmp, hipStream_t s) {
    const uint32_t nb = n ? (n + kScanTile - 1) / kScanTile : 1;
    if (!n) {
        (void)hipMemsetAsync(out, 0, sizeof(uint64_t), s);
        return;
    }
    hipLaunchKernelGGL(scan_reduce_kernel, dim3(nb), dim3(kBlock), 0, s, in, n, tmp);
    hipLaunchKernelGGL(scan_blocks_kernel, dim3(1), dim3(kBlock), 0, s, tmp, nb);
    hipLaunchKernelGGL(scan_apply_kernel, dim3(nb), dim3(kBlock), 0, s, in, n, tmp, nb, out);
}

void launch_scan(const DStore &st, const QDev *q, uint32_t nq, const uint32_t *lohi, const uint64_t *hit_off,
                 const uint8_t *qbytes, const uint64_t *subsets, uint32_t max_words, QRes *res, uint32_t *nhits,
                 uint32_t *hit_rec, uint32_t *hit_alt, uint64_t *samples_out, hipStream_t s) {
    if (!nq) return;
    const dim3 g(blocks_for(nq)), b(kBlock);
    if (max_words <= 64)
        hipLaunchKernelGGL(scan_kernel<1>, g, b, 0, s, st, q, nq, lohi, hit_off, qbytes, subsets, res, nhits, hit_rec,
                           hit_alt, samples_out);
    else if (max_words <= 256)
        hipLaunchKernelGGL(scan_kernel<4>, g, b, 0, s, st, q, nq, lohi, hit_off, qbytes, subsets, res, nhits, hit_rec,
                           hit_alt, samples_out);
    else
        hipLaunchKernelGGL(scan_kernel<16>, g, b, 0, s, st, q, nq, lohi, hit_off, qbytes, subsets, res, nhits,
                           hit_rec, hit_alt, samples_out);
}

void launch_compact(const uint64_t *hit_off, const uint64_t *dense_off, const uint32_t *nhits, uint32_t nq,
                    const uint32_t *hit_rec, const uint32_t *hit_alt, uint32_t *out_rec, uint32_t *out_alt,
                    hipStream_t s) {
    if (!nq) return;
    hipLaunchKernelGGL(compact_kernel, dim3(blocks_for(nq)), dim3(kBlock), 0, s, hit_off, dense_off, nhits, nq,
                       hit_rec, hit_alt, out_rec, out_alt);
}

}  // namespace sb
