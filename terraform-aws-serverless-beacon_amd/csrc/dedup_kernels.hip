// dedup_kernels.hip — duplicateVariantSearch on the device.
//
// The reference (lambda/duplicateVariantSearch/source/duplicateVariantSearch.cpp
// :31-84) inflates every region file of a (dataset, contig, range) job and
// inserts to_string(pos) + ref'_alt' into an unordered_set<string>; the job's
// answer is the set size.  Here the region keys already sit in HBM (one 64-bit
// hash + a tail word per key, devtypes.hpp KStore), and a batch of jobs is
// answered with
//   1. gather:   the keys of every job's VCF ranges, split into two streams
//      (devtypes.hpp, exact dedup words): EXACT words (job | P - rangeStart |
//      REF/ALT codes) for single-base REF/ALT keys, keys only; HASHED words
//      (job | hash) with their key ids for everything else;
//   2. LSD radix sort of each stream, 8-bit digits, only as many passes as
//      the stream's words have bits (exact: job + window + 6 bits, typically
//      5 passes; hashed: 8), each pass = tile histogram (upsweep) + exclusive
//      scan + stable rank-and-scatter (downsweep: wave-level match via 8
//      ballots, per-wave LDS counters, LDS-staged coalesced writes);
//   3. unique:   adjacent compare per stream.  Exact words are the strings;
//      equal hashed words are confirmed byte-for-byte on the key strings, and
//      pairs whose strings differ (hash collisions) are listed for the host's
//      exact recount of that group.
// Sorting by (job, word) keeps every job contiguous, so the whole batch is one
// sort per stream.  All passes are HBM-streaming integer work: 256-thread
// workgroups, one tile of 4096 keys each, coalesced 64-lane loads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "config.hpp"
#include "kernels.hpp"

namespace sb {
namespace {

constexpr int kThreads = 256;
constexpr int kItems = 16;
constexpr int kTile = kThreads * kItems;  // keys per workgroup
constexpr int kWaves = kThreads / 64;
constexpr int kWaveKeys = 64 * kItems;

__device__ __forceinline__ uint32_t popc_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                     __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
}

// ------------------------------------------------------------------ gather
// canonical exact code of a key (devtypes.hpp): 0 = hashed stream
__device__ __forceinline__ uint32_t exact_word(const KBody &b, uint32_t rs, uint32_t pos_bits, uint64_t *rel) {
    const uint64_t t = b.tail;
    if ((t & kTailBlob) || b.pos == 0) return 0;
    const uint32_t len = static_cast<uint32_t>(t >> 56);
    uint64_t P = b.pos;
    uint32_t d = 0;
    while (d < len) {
        const uint32_t c = static_cast<uint32_t>(t >> (8 * d)) & 0xffu;
        if (c < '0' || c > '9') break;
        P = P * 10 + (c - '0');
        ++d;
    }
    if (len - d != 3) return 0;
    const uint32_t c1 = static_cast<uint32_t>(t >> (8 * d)) & 0xffu;
    const uint32_t us = static_cast<uint32_t>(t >> (8 * d + 8)) & 0xffu;
    const uint32_t c2 = static_cast<uint32_t>(t >> (8 * d + 16)) & 0xffu;
    if (us != '_' || c1 < 1 || c1 > 7 || c2 < 1 || c2 > 7) return 0;
    if (P < rs || ((P - rs) >> pos_bits) != 0) return 0;  // outside the window: hashed stream
    *rel = P - rs;
    return (c1 << 3) | c2;
}

// One workgroup per host-planned tile of kTile keys of ONE segment (no
// per-key segment search): every body load is issued first, then the class of
// each key, then the hash loads of the (rare) hashed keys.  Each tile writes
// its exact words and its hashed (word, key id) pairs compacted at the start
// of its OWN kTile-slot region of the two streams and its two counts into
// tcnt[tile] / tcnt[ntiles + tile]: no cross-workgroup atomics.  The first
// radix pass reads the streams tile by tile (tile_n = tcnt) and leaves them
// dense.
constexpr int kGItems = kItems;
constexpr uint32_t kGTile = kThreads * kGItems;
static_assert(kGTile == static_cast<uint32_t>(kTile), "gather tiles are radix tiles");
__global__ __launch_bounds__(kThreads) void gather_kernel(KStore ks, const KSeg *segs, const uint2 *tiles,
                                                          uint32_t ntiles, uint32_t pos_bits,
                                                          uint32_t exact_job_shift, uint32_t job_bits, uint64_t mask,
                                                          uint64_t *ke, uint64_t *kh, uint32_t *vh, uint32_t *tcnt) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint2 T = tiles[blockIdx.x];  // (segment, first key offset in it)
    const KSeg g = segs[T.x];
    // two halves of kGItems / 2 keys: their body loads are issued together,
    // then classified; words are staged in LDS (slot r * kThreads + tid) so
    // only two flag masks stay live across the phases
    __shared__ uint64_t s_word[kGTile];
    __shared__ uint32_t s_off[2][kGItems][kWaves];
    constexpr int kHalf = kGItems / 2;
    uint32_t exm = 0, okm = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        KBody body[kHalf];
#pragma unroll
        for (int q = 0; q < kHalf; ++q) {
            const uint32_t j = T.y + static_cast<uint32_t>(h * kHalf + q) * kThreads + threadIdx.x;
            body[q] = j < g.n ? ks.body[g.key_lo + j] : KBody{0, 0, 0};
        }
#pragma unroll
        for (int q = 0; q < kHalf; ++q) {
            const int r = h * kHalf + q;
            const uint32_t j = T.y + static_cast<uint32_t>(r) * kThreads + threadIdx.x;
            if (j >= g.n) continue;
            okm |= 1u << r;
            uint64_t rel = 0;
            const uint32_t code = pos_bits ? exact_word(body[q], g.range_start, pos_bits, &rel) : 0u;
            if (code) {
                exm |= 1u << r;
                s_word[r * kThreads + threadIdx.x] =
                    (static_cast<uint64_t>(g.job) << exact_job_shift) | (rel << 6) | code;
            }
        }
    }
    const uint32_t hm = okm & ~exm;
    if (hm) {
        uint64_t hv[kGItems];
#pragma unroll
        for (int r = 0; r < kGItems; ++r)
            hv[r] = ((hm >> r) & 1u) ? ks.hash[g.key_lo + T.y + static_cast<uint32_t>(r) * kThreads + threadIdx.x] : 0;
#pragma unroll
        for (int r = 0; r < kGItems; ++r) {
            if ((hm >> r) & 1u) {
                const uint64_t x = hv[r] & mask;
                s_word[r * kThreads + threadIdx.x] =
                    job_bits ? ((static_cast<uint64_t>(g.job) << (64 - job_bits)) | (x >> job_bits)) : x;
            }
        }
    }
    // tile-local positions in (item, wave, lane) order so that every store
    // instruction writes consecutive slots: per-(item, wave) counts from
    // ballots, a serial exclusive scan over the 2 x kGItems x kWaves counts,
    // popc_below inside the wave
#pragma unroll
    for (int r = 0; r < kGItems; ++r) {
        const uint64_t me = __ballot((exm >> r) & 1u);
        const uint64_t mh = __ballot((hm >> r) & 1u);
        if (lane == 0) {
            s_off[0][r][w] = static_cast<uint32_t>(__popcll(me));
            s_off[1][r][w] = static_cast<uint32_t>(__popcll(mh));
        }
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        uint32_t run = 0;
        uint32_t *o = &s_off[threadIdx.x][0][0];
        for (int x = 0; x < kGItems * kWaves; ++x) {
            const uint32_t c = o[x];
            o[x] = run;
            run += c;
        }
        tcnt[threadIdx.x * ntiles + blockIdx.x] = run;
    }
    __syncthreads();
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kTile;
#pragma unroll
    for (int r = 0; r < kGItems; ++r) {
        const bool e = (exm >> r) & 1u, hh = (hm >> r) & 1u;
        const uint64_t me = __ballot(e), mh = __ballot(hh);
        if (e) {
            ke[t0 + s_off[0][r][w] + popc_below(me)] = s_word[r * kThreads + threadIdx.x];
        } else if (hh) {
            const uint64_t d = t0 + s_off[1][r][w] + popc_below(mh);
            kh[d] = s_word[r * kThreads + threadIdx.x];
            vh[d] = static_cast<uint32_t>(g.key_lo + T.y + static_cast<uint32_t>(r) * kThreads + threadIdx.x);
        }
    }
}

// ------------------------------------------------------------- radix sort
// splitmix64 finalizer: the bucket partition of the exact stream sorts on
// bits of mix(word) (a bijection), so buckets are uniform whatever the words
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27;
    x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}

template <bool MIX>
__device__ __forceinline__ uint32_t digit_of(uint64_t k, uint32_t shift) {
    return static_cast<uint32_t>((MIX ? mix64(k) : k) >> shift) & 255u;
}

// hist layout: digit-major, hist[d * ntiles + tile]
// keys of tile b: dense (tile_n == nullptr) = [b * kTile, min(n, ..+kTile));
// sparse (the first pass after gather) = the first tile_n[b] slots of tile b
__device__ __forceinline__ uint32_t tile_count(uint64_t n, const uint32_t *tile_n) {
    if (tile_n) return tile_n[blockIdx.x];
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kTile;
    return static_cast<uint32_t>(min(static_cast<uint64_t>(kTile), n - t0));
}

template <bool MIX>
__global__ __launch_bounds__(kThreads) void upsweep_kernel(const uint64_t *keys, uint64_t n, const uint32_t *tile_n,
                                                           uint32_t shift, uint32_t *hist, uint32_t ntiles) {
    __shared__ uint32_t h[kWaves][256];
    const int w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kWaves * 256; i += kThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile;
    const uint32_t tn = tile_count(n, tile_n);
    uint32_t dg[kItems];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint32_t j = static_cast<uint32_t>(r) * kThreads + threadIdx.x;
        dg[r] = j < tn ? digit_of<MIX>(keys[base + j], shift) : 256u;
    }
#pragma unroll
    for (int r = 0; r < kItems; ++r)
        if (dg[r] < 256u) atomicAdd(&h[w][dg[r]], 1u);
    __syncthreads();
    const int d = threadIdx.x;
    hist[static_cast<uint64_t>(d) * ntiles + blockIdx.x] = h[0][d] + h[1][d] + h[2][d] + h[3][d];
}

// exclusive scan of m u32 (block sums, top scan, down-sweep); kTile per block
__device__ __forceinline__ uint32_t block_exclusive(uint32_t x, uint32_t *lds, uint32_t *total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) lds[w] = inc;
    __syncthreads();
    uint32_t wofs = 0, tot = 0;
#pragma unroll
    for (int ww = 0; ww < kWaves; ++ww) {
        const uint32_t t = lds[ww];
        if (ww < w) wofs += t;
        tot += t;
    }
    __syncthreads();
    *total = tot;
    return wofs + inc - x;
}

template <bool VALS, bool MIX>
__global__ __launch_bounds__(kThreads) void downsweep_kernel(const uint64_t *kin, const uint32_t *vin,
                                                             uint64_t *kout, uint32_t *vout, uint64_t n,
                                                             const uint32_t *tile_n, uint32_t shift,
                                                             const uint32_t *off, uint32_t ntiles) {
    __shared__ uint32_t cnt[kWaves][256];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < kWaves * 256; i += kThreads) (&cnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t tile0 = static_cast<uint64_t>(blockIdx.x) * kTile;
    const uint32_t tn = tile_count(n, tile_n);
    const uint32_t wbase = static_cast<uint32_t>(w) * kWaveKeys;  // tile-local
    uint64_t k[kItems];
    uint32_t v[kItems], rank[kItems];
    // all of the wave's loads in flight first, then rank in index order
    // (wave w owns a contiguous quarter of the tile)
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint32_t j = wbase + static_cast<uint32_t>(r) * 64 + lane;
        k[r] = j < tn ? kin[tile0 + j] : 0;
        v[r] = (VALS && j < tn) ? vin[tile0 + j] : 0;
    }
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        if (wbase + static_cast<uint32_t>(r) * 64 >= tn) break;  // wave-uniform: the rest of the wave's slots are empty
        const bool ok = wbase + static_cast<uint32_t>(r) * 64 + lane < tn;
        const uint32_t d = digit_of<MIX>(k[r], shift);
        uint64_t peers = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const bool bit = (d >> b) & 1u;
            const uint64_t m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        const uint32_t before = popc_below(peers);
        uint32_t c = 0;
        if (ok) c = cnt[w][d];
        rank[r] = c + before;
        __builtin_amdgcn_wave_barrier();
        if (ok && before == 0) cnt[w][d] = c + static_cast<uint32_t>(__popcll(peers));
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    __shared__ uint32_t gbase[256], lds_scan[kWaves];
    {  // per digit: exclusive over waves, tile-local start, global start
        const int d = threadIdx.x;
        uint32_t run = 0;
#pragma unroll
        for (int ww = 0; ww < kWaves; ++ww) {
            const uint32_t t = cnt[ww][d];
            cnt[ww][d] = run;
            run += t;
        }
        uint32_t tot;
        const uint32_t local0 = block_exclusive(run, lds_scan, &tot);  // keys of smaller digits in this tile
#pragma unroll
        for (int ww = 0; ww < kWaves; ++ww) cnt[ww][d] += local0;
        gbase[d] = off[static_cast<uint64_t>(d) * ntiles + blockIdx.x] - local0;
    }
    __syncthreads();
    // stage the tile in digit order, then write runs of equal digits
    // contiguously (avg. 16 keys = 128 B per digit run)
    __shared__ uint64_t sk[kTile];
    __shared__ uint32_t sv[VALS ? kTile : 1];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        if (wbase + static_cast<uint32_t>(r) * 64 + lane < tn) {
            const uint32_t d = digit_of<MIX>(k[r], shift);
            const uint32_t loc = cnt[w][d] + rank[r];
            sk[loc] = k[r];
            if (VALS) sv[loc] = v[r];
        }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint32_t loc = static_cast<uint32_t>(r) * kThreads + threadIdx.x;
        if (loc < tn) {
            const uint64_t key = sk[loc];
            const uint32_t dst = gbase[digit_of<MIX>(key, shift)] + loc;
            kout[dst] = key;
            if (VALS) vout[dst] = sv[loc];
        }
    }
}

__global__ __launch_bounds__(kThreads) void scan_reduce_kernel(const uint32_t *a, uint64_t m, uint32_t *bsum) {
    __shared__ uint32_t lds[kWaves];
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile;
    uint32_t s = 0;
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = base + static_cast<uint64_t>(r) * kThreads + threadIdx.x;
        if (i < m) s += a[i];
    }
    uint32_t tot;
    block_exclusive(s, lds, &tot);
    if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kThreads) void scan_top_kernel(uint32_t *bsum, uint32_t nb) {
    __shared__ uint32_t lds[kWaves];
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += kThreads) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t x = i < nb ? bsum[i] : 0u;
        uint32_t tot;
        const uint32_t e = block_exclusive(x, lds, &tot);
        if (i < nb) bsum[i] = carry + e;
        carry += tot;
    }
}

__global__ __launch_bounds__(kThreads) void scan_down_kernel(uint32_t *a, uint64_t m, const uint32_t *bsum) {
    __shared__ uint32_t lds[kWaves];
    // thread t owns kItems consecutive entries
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile + static_cast<uint64_t>(threadIdx.x) * kItems;
    uint32_t x[kItems], s = 0;
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        x[r] = base + r < m ? a[base + r] : 0u;
        s += x[r];
    }
    uint32_t tot;
    uint32_t run = bsum[blockIdx.x] + block_exclusive(s, lds, &tot);
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        if (base + r < m) a[base + r] = run;
        run += x[r];
    }
}

// ------------------------------------------------------------------ unique
// key string = decimal(pos) ++ tail bytes
struct KeyStr {
    char dig[10];
    uint32_t nd, tl;
    uint64_t tail;
    const uint8_t *blob;
    __device__ uint8_t at(uint32_t j) const {
        if (j < nd) return static_cast<uint8_t>(dig[j]);
        j -= nd;
        if (tail & kTailBlob) return blob[(tail & ((1ull << 40) - 1)) + j];
        return static_cast<uint8_t>(tail >> (8 * j));
    }
};

__device__ KeyStr key_str(const KStore &ks, const KBody &k) {
    KeyStr s;
    uint32_t p = k.pos;
    char tmp[10];
    uint32_t nd = 0;
    do {
        tmp[nd++] = static_cast<char>('0' + p % 10);
        p /= 10;
    } while (p);
    for (uint32_t j = 0; j < nd; ++j) s.dig[j] = tmp[nd - 1 - j];
    s.nd = nd;
    s.tail = k.tail;
    s.tl = (s.tail & kTailBlob) ? static_cast<uint32_t>((s.tail >> 40) & 0xffff) : static_cast<uint32_t>(s.tail >> 56);
    s.blob = ks.blob;
    return s;
}

__device__ __noinline__ bool key_equal_slow(const KStore &ks, const KBody &x, const KBody &y) {
    const KeyStr u = key_str(ks, x), v = key_str(ks, y);
    if (u.nd + u.tl != v.nd + v.tl) return false;
    for (uint32_t j = 0; j < u.nd + u.tl; ++j)
        if (u.at(j) != v.at(j)) return false;
    return true;
}

// equal key strings?  Same POS (the common case of an equal hashed word):
// the tails must match — inline words directly, blob tails byte by byte;
// different POS: the general decimal-concatenation comparison.
__device__ bool key_equal(const KStore &ks, uint32_t a, uint32_t b) {
    if (a == b) return true;
    const KBody x = ks.body[a], y = ks.body[b];
    if (x.pos == y.pos) {
        if (x.tail == y.tail) return true;
        if (!((x.tail & y.tail) & kTailBlob)) return false;  // inline vs other: different bytes or lengths
        const uint32_t lx = static_cast<uint32_t>((x.tail >> 40) & 0xffff), ly = static_cast<uint32_t>((y.tail >> 40) & 0xffff);
        if (lx != ly) return false;
        const uint8_t *p = ks.blob + (x.tail & ((1ull << 40) - 1)), *q = ks.blob + (y.tail & ((1ull << 40) - 1));
        for (uint32_t j = 0; j < lx; ++j)
            if (p[j] != q[j]) return false;
        return true;
    }
    return key_equal_slow(ks, x, y);
}

// kItems sorted positions per thread (coalesced: item r of the block is
// r * kThreads + threadIdx.x); the block's distinct count goes out with one
// atomic per job it touches (one in the common single-job block)
// Per block: the fresh (distinct) keys of its first and last job go to
// part[block] = {job_first, count_first, job_last, count_last} (the host sums
// them: no same-address atomics across workgroups); jobs strictly inside a
// block (a job with fewer keys than a tile) take a global atomic.
template <bool VERIFY>
__global__ __launch_bounds__(kThreads) void unique_kernel(const uint64_t *keys, const uint32_t *vals, uint64_t n,
                                                          KStore ks, uint32_t job_shift, unsigned long long *counts,
                                                          uint4 *part, uint32_t *coll, uint32_t *ncoll) {
    __shared__ uint32_t s_job[2];
    __shared__ unsigned int s_cnt[2];
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile;
    const int lane = threadIdx.x & 63;
    if (threadIdx.x == 0) {
        s_cnt[0] = s_cnt[1] = 0;
        const uint64_t last = min(n, base + kTile) - 1;
        s_job[0] = job_shift < 64 ? static_cast<uint32_t>(keys[base] >> job_shift) : 0u;
        s_job[1] = job_shift < 64 ? static_cast<uint32_t>(keys[last] >> job_shift) : 0u;
    }
    // all loads in flight first: item r of the block is r * kThreads + tid;
    // its predecessor is lane - 1's item (shuffle), lane 0 loads its own
    uint64_t k[kItems], kp0[kItems];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = base + static_cast<uint64_t>(r) * kThreads + threadIdx.x;
        k[r] = i < n ? keys[i] : 0ull;
        kp0[r] = (lane == 0 && i > 0 && i < n) ? keys[i - 1] : 0ull;
    }
    __syncthreads();
    const uint32_t jf = s_job[0], jl = s_job[1];
    uint32_t cf = 0, cl = 0;
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = base + static_cast<uint64_t>(r) * kThreads + threadIdx.x;
        const uint32_t plo = __shfl_up(static_cast<uint32_t>(k[r]), 1, 64);
        const uint32_t phi = __shfl_up(static_cast<uint32_t>(k[r] >> 32), 1, 64);
        const uint64_t prev = lane ? ((static_cast<uint64_t>(phi) << 32) | plo) : kp0[r];
        if (i >= n) continue;
        bool fresh = false;
        if (i == 0 || prev != k[r]) {
            fresh = true;
        } else if (VERIFY && !key_equal(ks, vals[i - 1], vals[i])) {
            fresh = true;  // a different string under the same word: the host recounts its group
            coll[atomicAdd(ncoll, 1u)] = static_cast<uint32_t>(i);
        }
        if (!fresh) continue;
        const uint32_t j = job_shift < 64 ? static_cast<uint32_t>(k[r] >> job_shift) : 0u;
        if (j == jf) ++cf;
        else if (j == jl) ++cl;
        else atomicAdd(&counts[j], 1ull);
    }
    for (int d = 32; d >= 1; d >>= 1) {
        cf += __shfl_xor(cf, d, 64);
        cl += __shfl_xor(cl, d, 64);
    }
    if (lane == 0) {
        if (cf) atomicAdd(&s_cnt[0], cf);
        if (cl) atomicAdd(&s_cnt[1], cl);
    }
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = uint4{jf, s_cnt[0], jl, s_cnt[1]};
}

// ------------------------------------------------------------- bucket dedupe
// The exact stream after two radix passes on the top 16 bits of mix(word):
// equal words are in one bucket and buckets are contiguous.  Workgroup w owns
// the buckets that start in [w * kBTile, (w + 1) * kBTile) and counts their
// distinct words with an LDS hash set (one successful insert per distinct
// word), adding each to its job.  A set that would overflow raises *overflow
// (the host then takes the radix path).  8 B / key after the partition.
constexpr uint32_t kBTile = 2048;          // keys per workgroup (nominal)
constexpr uint32_t kBSlots = 8192;         // LDS hash set (64 KB)
constexpr uint64_t kBEmpty = ~0ull;        // exact words never reach all ones (job | window | 6 bits < 64 bits)

__device__ __forceinline__ uint32_t bucket_of(uint64_t k) { return static_cast<uint32_t>(mix64(k) >> 48); }

// first index in [at, n) whose bucket is above b (buckets are nondecreasing):
// two rounds of block-wide loads, 256 samples 16 apart then the 16 keys of
// the span that holds the boundary; a bucket longer than 4096 keys takes
// further rounds.  Every thread gets the answer.
__device__ uint64_t bucket_end(const uint64_t *keys, uint64_t n, uint64_t at, uint32_t b, uint32_t *lds) {
    for (uint64_t base = at; base < n; base += kThreads * 16) {
        const uint64_t i = base + threadIdx.x * 16;
        const bool past = i < n && bucket_of(keys[i]) > b;
        if (threadIdx.x == 0) lds[0] = 0xffffffffu;
        __syncthreads();
        if (past) atomicMin(&lds[0], threadIdx.x);
        __syncthreads();
        const uint32_t f = lds[0];
        __syncthreads();
        if (f == 0xffffffffu) continue;  // not in this 4096-key span
        // the boundary lies in (base + 16 (f - 1), base + 16 f]
        const uint64_t lo = f ? base + 16 * static_cast<uint64_t>(f - 1) + 1 : base;
        const uint64_t j = lo + threadIdx.x;
        const bool past2 = threadIdx.x < 16 && j < n && bucket_of(keys[j]) > b;
        if (threadIdx.x == 0) lds[0] = 0xffffffffu;
        __syncthreads();
        if (past2) atomicMin(&lds[0], threadIdx.x);
        __syncthreads();
        const uint32_t g = lds[0];
        __syncthreads();
        return g == 0xffffffffu ? base + 16 * static_cast<uint64_t>(f) : lo + g;
    }
    return n;
}

// VALS (the hashed stream: words are job | 64-bit hash, vals the key ids):
// a word already in the set is confirmed on the key strings; two different
// strings under one word (a 64-bit collision, or the SBEACON_DEDUP_HASH_BITS
// test hook) raise *overflow so the host recounts with the sorted path,
// whose exact collision recount needs adjacent groups.  Keys are handled in
// rounds of kBPer per thread, every load of a round issued first.
constexpr uint32_t kBPer = 8;

template <bool VALS, uint32_t SLOTS>
__global__ __launch_bounds__(kThreads) void bucket_dedupe_kernel(const uint64_t *keys, const uint32_t *vals, uint64_t n,
                                                                 KStore ks, uint32_t job_shift, uint32_t nj_lds,
                                                                 unsigned long long *counts, uint32_t *overflow,
                                                                 uint32_t cap, uint32_t dbg) {
    __shared__ unsigned long long set[SLOTS];
    __shared__ uint32_t ids[VALS ? SLOTS : 1];
    __shared__ unsigned int jc[256];
    __shared__ uint32_t s_ins;
    if (threadIdx.x == 0) s_ins = 0;
    for (uint32_t i = threadIdx.x; i < SLOTS; i += kThreads) set[i] = kBEmpty;
    for (uint32_t i = threadIdx.x; i < 256; i += kThreads) jc[i] = 0;
    // this workgroup owns tile [t0, t0 + kBTile) minus the leading keys of the
    // bucket that started in an earlier tile, plus the rest of its last bucket
    // beyond the tile's end (both ends found by bucket_end)
    const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * kBTile;
    const uint64_t te = min(n, t0 + kBTile);
    const uint32_t b_prev = t0 ? bucket_of(keys[t0 - 1]) : 0xffffffffu;
    const uint32_t b_last = bucket_of(keys[te - 1]);
    __syncthreads();
    // owned range [s0, s1): from the end of the bucket running into the tile
    // (if any) to the end of the tile's last bucket
    __shared__ uint32_t s_tmp[1];
    if (b_prev == b_last && t0) return;  // the whole tile lies in a bucket owned by an earlier workgroup
    const uint64_t s0 = t0 && b_prev != 0xffffffffu ? bucket_end(keys, n, t0, b_prev, s_tmp) : t0;
    const uint64_t s1 = te < n ? bucket_end(keys, n, te, b_last, s_tmp) : n;
    for (uint64_t r0 = s0; r0 < s1; r0 += kThreads * kBPer) {  // uniform trip count
        uint64_t k[kBPer];
        uint32_t v[kBPer], slot[kBPer];
        bool mine[kBPer], ok[kBPer];
#pragma unroll
        for (uint32_t u = 0; u < kBPer; ++u) {
            const uint64_t j = r0 + u * kThreads + threadIdx.x;
            ok[u] = j < s1;
            k[u] = ok[u] ? keys[j] : 0ull;
            v[u] = (VALS && ok[u]) ? vals[j] : 0u;
        }
        uint64_t mx[kBPer];  // mix(word): low bits = set slot
        uint32_t nok = 0;
#pragma unroll
        for (uint32_t u = 0; u < kBPer; ++u) {
            mx[u] = mix64(k[u]);
            nok += ok[u] ? 1u : 0u;
        }
        if (nok) atomicAdd(&s_ins, nok);
        __syncthreads();
        if (s_ins > cap) {  // the set cannot hold this workgroup's keys: the sorted path
            if (threadIdx.x == 0) atomicOr(overflow, 1u);
            return;
        }
        // first probe of every key issued back to back (independent slots),
        // then the (rare) keys whose slot held another word probe on
        uint32_t h[kBPer];
        unsigned long long was[kBPer];
#pragma unroll
        for (uint32_t u = 0; u < kBPer; ++u) {
            mine[u] = false;
            slot[u] = 0;
            h[u] = static_cast<uint32_t>(mx[u]) & (SLOTS - 1);
            if (ok[u] && k[u] == kBEmpty) {  // the set's empty marker (a hashed word of all ones): the sorted path
                atomicOr(overflow, 1u);
                ok[u] = false;
            }
            if (dbg) ok[u] = false;  // timing ablation (SBEACON_DEDUP_BUCKET_DBG): no inserts
            was[u] = ok[u] ? atomicCAS(&set[h[u]], kBEmpty, static_cast<unsigned long long>(k[u])) : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < kBPer; ++u) {
            if (!ok[u]) continue;
            for (uint32_t probe = 1; was[u] != kBEmpty && was[u] != k[u] && probe < SLOTS; ++probe) {
                h[u] = (h[u] + 1) & (SLOTS - 1);
                was[u] = atomicCAS(&set[h[u]], kBEmpty, static_cast<unsigned long long>(k[u]));
            }
            mine[u] = was[u] == kBEmpty;  // first copy of this word
            slot[u] = h[u];
            if (mine[u]) {
                const uint32_t j = job_shift < 64 ? static_cast<uint32_t>(k[u] >> job_shift) : 0u;
                if (j < nj_lds) atomicAdd(&jc[j], 1u);
                else atomicAdd(&counts[j], 1ull);
            }
        }
        if constexpr (VALS) {  // the inserters publish their key ids, the rest compare strings
            __syncthreads();
#pragma unroll
            for (uint32_t u = 0; u < kBPer; ++u)
                if (mine[u]) ids[slot[u]] = v[u];
            __syncthreads();
#pragma unroll
            for (uint32_t u = 0; u < kBPer; ++u)
                if (ok[u] && !mine[u] && !key_equal(ks, ids[slot[u]], v[u])) atomicOr(overflow, 1u);
        }
        __syncthreads();
    }
    for (uint32_t j = threadIdx.x; j < nj_lds; j += kThreads)
        if (jc[j]) atomicAdd(&counts[j], static_cast<unsigned long long>(jc[j]));
}

// ------------------------------------------------------------- window dedupe
// One workgroup per host-planned window (devtypes.hpp KWin): its keys are
// read ONCE from the store (16 B body; the 8 B hash only for keys outside
// the exact class) and counted in one LDS hash set of 64-bit entries:
//   exact keys   (POS - p0) << 6 | c1 c2          (< 2^32: the string itself)
//   hashed keys  1 << 63 | hash bits 13..62 << 12 | window-local key index
// A hashed key meeting an entry with its hash bits is confirmed on the key
// strings against the inserter (named by the entry's index).  Displaced keys
// with 10 POS > the job's largest POS are hashed like any key; the other
// displaced keys are deferred to deferred_dedupe_kernel (a list of (key, run)
// pairs).  Two strings under one hash, or a full deferred list, raise
// *overflow and the host recounts the call on the sorted path.  No gather
// stream, no radix pass: 16 B/key + 8 B per hashed key.
// A window's keys are deduplicated without LDS atomics: every key's
// identity word (identified: 1 << 63 | (POS - p0) << 29 | id, exact;
// hashed: the 64-bit hash with bit 63 clear) is staged at its window-local
// index, and in rounds every unresolved key writes its index to the slot of
// its identity (a per-round salted hash; plain 16-bit stores, one of the
// writers wins), then reads the winner back: the winner's identity equal to
// its own resolves it (the winner counts itself, an equal key is a
// duplicate -- for hashed identities after the strings are confirmed); a
// different identity (a collision) leaves it for the next round.  Equal
// identities always meet in one slot, so a value is counted once.
// LDS per workgroup (identities 16 KB + winners 5.5 KB + pieces) <= 22.7 KB:
// 7 workgroups per CU (4,096 slots and 128 confirmations: 6, and 4 % slower,
// profiles/r05_dedup/slots.log); the set's load is <= 0.73 (1,024 distinct
// identities in a config-4 window: ~0.36)
#ifndef SBEACON_WIN_THREADS
#define SBEACON_WIN_THREADS 256  // threads of window_dedupe_kernel (64: one wave per window, no cross-wave barriers)
#endif
constexpr uint32_t kWT = SBEACON_WIN_THREADS;
#ifndef SBEACON_WIN_SLOTS
#define SBEACON_WIN_SLOTS (kWinCap / 8 * 11)
#endif
constexpr uint32_t kWSlots = SBEACON_WIN_SLOTS;  // 16-bit winners
constexpr uint32_t kWRounds = 24;    // unresolved after that: the sorted path
#ifndef SBEACON_WIN_CONFIRM
#define SBEACON_WIN_CONFIRM 32
#endif
constexpr uint32_t kWConfirm = SBEACON_WIN_CONFIRM;  // hashed duplicate pairs confirmed per window
constexpr uint32_t kWPer = kWinCap / kWT;
static_assert(kWPer * kWT == kWinCap && kWT % 64 == 0, "window keys per thread");
static_assert(kWinCap <= kWSlots && kWinCap <= 65536, "window slot load / 16-bit winners");
static_assert(kWinPieces == 64, "one wave scans the pieces");

// wave-wide sums (DPP row shifts, then the row broadcasts)
template <int CTRL, int ROW = 0xf>
__device__ __forceinline__ uint32_t dppm(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), CTRL, ROW, 0xf, false));
}
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += dppm<0x111>(v);
    v += dppm<0x112>(v);
    v += dppm<0x114>(v);
    v += dppm<0x118>(v);
    v += dppm<0x142, 0xa>(v);
    v += dppm<0x143, 0xc>(v);
    return v;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
    return static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(wave_incl_sum(v)), 63));
}

// len bytes at blob offsets oa and ob equal?  Aligned 8-byte words (every
// load of a 32-byte round issued first) funnel-shifted into place; the blob
// is padded by 16 bytes, so the word past the last byte is readable.
__device__ bool blob_equal(const uint8_t *__restrict__ blob, uint64_t oa, uint64_t ob, uint32_t len) {
    const uint64_t *w = reinterpret_cast<const uint64_t *>(blob);
    auto word_at = [&](uint64_t lo_w, uint64_t hi_w, uint32_t sh) {
        return sh ? (lo_w >> (8 * sh)) | (hi_w << (64 - 8 * sh)) : lo_w;
    };
    for (uint32_t j = 0; j < len; j += 32) {
        uint64_t wa[5], wb[5];
        const uint64_t ia = (oa + j) >> 3, ib = (ob + j) >> 3;
        const uint32_t nw = min(len - j, 32u);
        const uint32_t na = static_cast<uint32_t>((((oa + j) & 7) + nw + 7) >> 3);
        const uint32_t nb = static_cast<uint32_t>((((ob + j) & 7) + nw + 7) >> 3);
#pragma unroll
        for (uint32_t q = 0; q < 5; ++q) {
            wa[q] = q < na ? w[ia + q] : 0ull;
            wb[q] = q < nb ? w[ib + q] : 0ull;
        }
        const uint32_t sa = static_cast<uint32_t>((oa + j) & 7), sb = static_cast<uint32_t>((ob + j) & 7);
#pragma unroll
        for (uint32_t q = 0; q < 4; ++q) {
            if (8 * q >= nw) break;
            uint64_t d = word_at(wa[q], wa[q + 1], sa) ^ word_at(wb[q], wb[q + 1], sb);
            const uint32_t rem = nw - 8 * q;
            if (rem < 8) d &= (1ull << (8 * rem)) - 1ull;
            if (d) return false;
        }
    }
    return true;
}

// two key bodies' strings equal (same POS: the tails; else the general
// decimal-concatenation comparison)
__device__ bool body_equal(const KStore &ks, const KBody &x, const KBody &y) {
    if (x.pos == y.pos) {
        if (x.tail == y.tail) return true;
        if (!((x.tail & y.tail) & kTailBlob)) return false;  // inline vs other: different bytes or lengths
        const uint32_t lx = static_cast<uint32_t>((x.tail >> 40) & 0xffff), ly = static_cast<uint32_t>((y.tail >> 40) & 0xffff);
        return lx == ly && blob_equal(ks.blob, x.tail & ((1ull << 40) - 1), y.tail & ((1ull << 40) - 1), lx);
    }
    return key_equal_slow(ks, x, y);
}

__device__ bool key_equal_body(const KStore &ks, uint32_t a, const KBody &y) { return body_equal(ks, ks.body[a], y); }

// byte j of a key's tail (j < its length)
__device__ __forceinline__ uint32_t tail_byte(const KStore &ks, uint64_t t, uint32_t j) {
    if (t & kTailBlob) return ks.blob[(t & ((1ull << 40) - 1)) + j];
    return static_cast<uint32_t>(t >> (8 * j)) & 0xffu;
}

// a key of run R at POS X, with index below klim, holding y's string?
__device__ bool run_has_equal(const KStore &ks, const KRun &R, uint64_t X, const KBody &y, uint32_t klim) {
    if (X < R.pos_lo || X > R.pos_hi) return false;
    // records of the segment with POS == X: bucket bracket + binary search
    const uint64_t b = (X - R.b_base) >> R.b_shift;
    uint32_t lo = b >= R.b_n ? R.seg_hi : ks.bucket[R.b_off + b];
    uint32_t hi = b >= R.b_n ? R.seg_hi : ks.bucket[R.b_off + b + 1];
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ks.rpos[mid] < X) lo = mid + 1;
        else hi = mid;
    }
    for (uint32_t rec = lo; rec < R.seg_hi && ks.rpos[rec] == X; ++rec) {
        const uint32_t k0 = max(ks.lo[rec], R.key_lo), k1 = min(min(ks.lo[rec + 1], R.key_hi), klim);
        for (uint32_t k = k0; k < k1; ++k)
            if (key_equal_body(ks, k, y)) return true;
    }
    return false;
}

// One lane per deferred key (kid, run): it counts for its job when no key of
// the job's runs holds its string at a larger POS (decimal(POS) ++ the first
// j >= 1 tail digits) and no earlier key of the job's runs equals it.
// Grid-stride over the list length the window kernel left in *n_list.
__global__ __launch_bounds__(kThreads) void deferred_dedupe_kernel(KStore ks, const KRun *runs, const uint2 *list,
                                                                   const uint32_t *n_list, uint32_t cap,
                                                                   unsigned long long *counts) {
    const uint32_t n = min(*n_list, cap);
    for (uint32_t i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        const uint2 e = list[i];
        const KRun R = runs[e.y];
        const KBody y = ks.body[e.x];
        bool skip = false;
        // a copy at a larger POS
        const uint64_t t = y.tail;
        const uint32_t len = (t & kTailBlob) ? static_cast<uint32_t>((t >> 40) & 0xffff) : static_cast<uint32_t>(t >> 56);
        uint64_t P = y.pos;
        for (uint32_t j = 0; j < len && !skip; ++j) {
            const uint32_t c = tail_byte(ks, t, j);
            if (c < '0' || c > '9') break;
            P = P * 10 + (c - '0');
            if (P > 0xffffffffull) break;
            for (uint32_t r = 0; r < R.nruns && !skip; ++r) skip = run_has_equal(ks, runs[R.run_lo + r], P, y, ~0u);
        }
        // an earlier copy at this POS: earlier runs of the job, or earlier in this run
        for (uint32_t r = R.run_lo; r <= e.y && !skip; ++r) skip = run_has_equal(ks, runs[r], y.pos, y, r == e.y ? e.x : ~0u);
        if (!skip) atomicAdd(&counts[R.job], 1ull);
    }
}

// first key of run R with POS >= x: the segment's coarse POS index
// brackets the records (as run_has_equal), a binary search over their POS
// names the record, its first key is the bound (keys are in record order)
__device__ uint32_t key_lower_bound(const KStore &ks, const KRun &R, uint32_t x) {
    if (x <= R.pos_lo) return R.key_lo;
    if (x > R.pos_hi) return R.key_hi;
    const uint64_t b = (static_cast<uint64_t>(x) - R.b_base) >> R.b_shift;
    uint32_t lo = b >= R.b_n ? R.seg_hi : ks.bucket[R.b_off + b];
    uint32_t hi = b >= R.b_n ? R.seg_hi : ks.bucket[R.b_off + b + 1];
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ks.rpos[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return min(max(ks.lo[lo], R.key_lo), R.key_hi);
}

// Window planning on the device (replaces the host walk): one thread per
// window.  Window i of job J starts at POS P_i = the POS of the leader
// run's key i * lead_n / nw (P_0 = the job's smallest POS); every run of the
// job starts it at its lower bound of P_i, so windows are POS ranges and the
// keys of one POS meet in one window.  Thread w writes window w's record
// (devtypes.hpp kWinRecHead): the header, each run's piece start, and the
// same start as the end of window w - 1's piece (the job's last window ends
// at the run's end).
__global__ __launch_bounds__(kThreads) void dedup_plan_kernel(KStore ks, const KJob *__restrict__ jobs, uint32_t nj,
                                                              const KRun *__restrict__ runs, uint32_t nw_total,
                                                              uint32_t *__restrict__ rec, uint32_t rec_words) {
    const uint32_t w = blockIdx.x * kThreads + threadIdx.x;
    if (w >= nw_total) return;
    uint32_t lo = 0, hi = nj;  // the last job with w0 <= w
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (jobs[mid].w0 <= w) lo = mid;
        else hi = mid;
    }
    const KJob J = jobs[lo];
    const uint32_t i = w - J.w0;
    const uint32_t P = i == 0 ? J.pmin
                              : static_cast<uint32_t>(ks.word[J.lead_lo + static_cast<uint64_t>(i) * J.lead_n / J.nw]);
    uint32_t *const me = rec + static_cast<uint64_t>(w) * rec_words;
    for (uint32_t r = 0; r < J.nruns; ++r) {
        const KRun R = runs[J.run_lo + r];
        const uint32_t at = i == 0 ? R.key_lo : key_lower_bound(ks, R, P);
        me[kWinRecHead + 2 * r] = at;
        if (i > 0) (me - rec_words)[kWinRecHead + 2 * r + 1] = at;  // window w - 1 of the job ends here
        if (i + 1 == J.nw) me[kWinRecHead + 2 * r + 1] = R.key_hi;
    }
    *reinterpret_cast<uint4 *>(me) = uint4{i, J.nruns, runs[J.run_lo].job, P};
    *reinterpret_cast<uint4 *>(me + 4) = uint4{J.run_lo, J.pmax, 0u, J.nw};
}

#ifndef SBEACON_WIN_WAVES
#define SBEACON_WIN_WAVES 7
#endif
// a barrier over the window's workgroup (a single wave: its LDS operations
// are ordered by the fence alone)
__device__ __forceinline__ void win_sync() {
    if constexpr (kWT == 64) {
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __builtin_amdgcn_wave_barrier();
    } else {
        __syncthreads();
    }
}

__global__ __launch_bounds__(kWT) __attribute__((amdgpu_waves_per_eu(SBEACON_WIN_WAVES, 8))) void window_dedupe_kernel(KStore ks, const uint32_t *__restrict__ rec, uint32_t rec_words,
                                                                 unsigned long long *counts, uint2 *list,
                                                                 uint32_t *n_list, uint32_t cap, uint32_t *overflow,
                                                                 uint32_t *wfresh, uint32_t dbg) {
    __shared__ __attribute__((aligned(16))) unsigned long long s_id[kWinCap];  // identity of window key f
    __shared__ __attribute__((aligned(16))) uint16_t s_win[kWSlots];            // a round's winner per slot
    __shared__ uint32_t s_pre[kWinPieces + 1], s_base[kWinPieces];  // piece p = run W.run_lo + p
    __shared__ uint32_t s_conf[kWConfirm];  // hashed duplicate pairs (winner | key << 16) to confirm
    __shared__ uint32_t s_fresh, s_def, s_def0, s_nconf, s_pend;
    // the window's record: its header and (wave 0, lane = run) the pieces,
    // loaded side by side (lanes past the call's largest run count load nothing)
    const uint32_t *const me = rec + static_cast<uint64_t>(blockIdx.x) * rec_words;
    const KWin W = *reinterpret_cast<const KWin *>(me);
    const uint32_t lane = threadIdx.x & 63u;
    if (threadIdx.x < 64) {  // wave 0: the pieces' inclusive prefix (DPP scan)
        uint2 pr{0u, 0u};
        if (kWinRecHead + 2 * lane < rec_words) pr = *reinterpret_cast<const uint2 *>(me + kWinRecHead + 2 * lane);
        const uint32_t klo = pr.x, len = lane < W.nruns ? pr.y - pr.x : 0u;
        const uint32_t inc = wave_incl_sum(len);
        s_pre[lane + 1] = inc;
        s_base[lane] = klo - (inc - len);  // key id = window-local index + base
        if (lane == 0) {
            s_pre[0] = 0;
            s_fresh = 0;
            s_def = 0;
            s_nconf = 0;
            s_pend = 0;
        }
    }
    win_sync();
    const uint32_t np = W.nruns, total = s_pre[np];
    if (total > kWinCap) {  // a pile-up past the window (the host recounts on the sorted path)
        if (threadIdx.x == 0) {
            atomicOr(overflow, 1u);
            wfresh[blockIdx.x] = 0;
        }
        return;
    }
    // every key's 8-byte class word (key u = u * kWT + tid): POS, the
    // tail's id, displaced flag -- the 8-byte hash and 16-byte body only for
    // the few keys without an id.  The lane's piece only moves forward with
    // u (f grows by kWT): a short catch-up walk per key, the pieces kept
    // 6 bits each for later
    uint32_t wlo[kWPer], whi[kWPer];  // the class words' halves
    uint32_t okm = 0;
    uint64_t pk = 0;  // piece of key u in bits 6u..6u+5
    if (np <= 4) {
        // (jobs of <= 4 runs: two VCFs per dataset is the common case) the
        // pieces' bounds in registers, read once: each key's piece is three
        // compares and its load issues at once, with no LDS round trip per
        // key before it.  s_pre[j] = total for j >= np, so those compares
        // are false for every key
        const uint32_t p1 = s_pre[1], p2 = s_pre[2], p3 = s_pre[3];
        const uint32_t b0 = s_base[0], b1 = s_base[1], b2 = s_base[2], b3 = s_base[3];
#pragma unroll
        for (uint32_t u = 0; u < kWPer; ++u) {
            const uint32_t f = u * kWT + threadIdx.x;
            wlo[u] = 0;
            whi[u] = 0;
            if (f < total) {
                const uint32_t pc = static_cast<uint32_t>(f >= p1) + static_cast<uint32_t>(f >= p2) +
                                    static_cast<uint32_t>(f >= p3);
                const uint32_t base = pc == 0 ? b0 : pc == 1 ? b1 : pc == 2 ? b2 : b3;
                const uint64_t wv = ks.word[f + base];
                wlo[u] = static_cast<uint32_t>(wv);
                whi[u] = static_cast<uint32_t>(wv >> 32);
                okm |= 1u << u;
                pk |= static_cast<uint64_t>(pc) << (6 * u);
            }
        }
    } else {
        uint32_t pc = 0;
#pragma unroll
        for (uint32_t u = 0; u < kWPer; ++u) {
            const uint32_t f = u * kWT + threadIdx.x;
            wlo[u] = 0;
            whi[u] = 0;
            if (f < total) {
                while (pc + 1 < np && s_pre[pc + 1] <= f) ++pc;
                const uint64_t wv = ks.word[f + s_base[pc]];
                wlo[u] = static_cast<uint32_t>(wv);
                whi[u] = static_cast<uint32_t>(wv >> 32);
                okm |= 1u << u;
                pk |= static_cast<uint64_t>(pc) << (6 * u);
            }
        }
    }
    if (dbg & 4u) {  // timing ablation (SBEACON_DEDUP_WIN_DBG): loads only
        uint32_t x = 0;
#pragma unroll
        for (uint32_t u = 0; u < kWPer; ++u) x += wlo[u] ^ whi[u];
        if (x == 0xdeadbeefu) atomicOr(overflow, x);
        if (threadIdx.x == 0) wfresh[blockIdx.x] = 0;
        return;
    }
    auto kid_of = [&](uint32_t u) { return u * kWT + threadIdx.x + s_base[static_cast<uint32_t>(pk >> (6 * u)) & 63u]; };
    // classes: identified (the tail has an id), hashed (no id), deferred
    // (displaced keys that may have a copy at a larger POS of the job).  A
    // displaced key with no such copy meets its equal strings at its own POS
    uint32_t em = 0, hm = 0, dm = 0;
    uint64_t idv[kWPer];  // the keys' identities, also kept in registers (the rounds read only the winners')
    const uint32_t pm10 = W.pmax / 10;
#pragma unroll
    for (uint32_t u = 0; u < kWPer; ++u) {
        const uint32_t pos = wlo[u];
        const uint32_t id = whi[u] & kWordIdMask;
        const bool ok = (okm >> u) & 1u;
        const bool disp = (whi[u] & static_cast<uint32_t>(kWordDisplaced >> 32)) != 0;
        const bool big = pos > pm10;  // 10 POS > the job's largest POS
        const bool ex = ok && (!disp || big) && id && pos >= W.p0 && ((pos - W.p0) >> kWinSpanBits) == 0;
        em |= (ex ? 1u : 0u) << u;
        hm |= ((ok && !ex && (!disp || big)) ? 1u : 0u) << u;
        dm |= ((ok && disp && !big) ? 1u : 0u) << u;
        idv[u] = (1ull << 63) | (static_cast<uint64_t>(pos - W.p0) << 29) | id;
    }
#pragma unroll
    for (uint32_t u = 0; u < kWPer; ++u)
        if ((hm >> u) & 1u) idv[u] = ks.hash[kid_of(u)] & ~(1ull << 63);
#pragma unroll
    for (uint32_t u = 0; u < kWPer; ++u)
        if (((em | hm) >> u) & 1u) s_id[u * kWT + threadIdx.x] = idv[u];
    // deferred keys: one reservation per workgroup in the global list
    const uint32_t nd = static_cast<uint32_t>(__popc(dm));
    uint32_t dofs = 0;
    if (nd) dofs = atomicAdd(&s_def, nd);
    win_sync();
    if (threadIdx.x == 0 && s_def) {
        const uint32_t at = atomicAdd(n_list, s_def);
        s_def0 = at;
        if (at + s_def > cap) atomicOr(overflow, 1u);
    }
    uint32_t pend = (dbg & 1u) ? 0u : (em | hm);  // timing ablation: no dedup rounds
    uint32_t fresh = 0;
    bool bad = false;
    for (uint32_t round = 0; round < kWRounds; ++round) {
        // write: every unresolved key's index to its identity's slot
        uint32_t sl[kWPer];
#pragma unroll
        for (uint32_t u = 0; u < kWPer; ++u)
            if ((pend >> u) & 1u) {
                const uint64_t v = idv[u];
                const uint32_t m = (static_cast<uint32_t>(v) ^ static_cast<uint32_t>(v >> 32) * 0x85EBCA6Bu ^
                                    round * 0xC2B2AE35u) * 0x9E3779B1u;
                sl[u] = static_cast<uint32_t>((static_cast<uint64_t>(m ^ (m >> 15)) * kWSlots) >> 32);
                s_win[sl[u]] = static_cast<uint16_t>(u * kWT + threadIdx.x);
            }
        win_sync();
        // read the winners back
#pragma unroll
        for (uint32_t u = 0; u < kWPer; ++u)
            if ((pend >> u) & 1u) {
                const uint32_t f = u * kWT + threadIdx.x;
                const uint32_t w = s_win[sl[u]];
                const uint64_t v = idv[u];
                // resolved: the winner counts, an equal identity is its
                // duplicate (a key that won its own slot reads nothing)
                if (w == f || s_id[w] == v) {
                    pend &= ~(1u << u);
                    if (w == f) {
                        ++fresh;
                    } else if (!(v >> 63)) {  // equal hashes: the strings are confirmed below
                        const uint32_t at = atomicAdd(&s_nconf, 1u);
                        if (at < kWConfirm) s_conf[at] = w | f << 16;
                    }
                }
            }
        // any key left?  (round + 1 in one LDS word: no earlier round's
        // value reads as this one's)
        if (pend) s_pend = round + 1;
        win_sync();  // also orders this round's reads before the next writes
        if (s_pend != round + 1) break;
        if (round + 1 == kWRounds && threadIdx.x == 0) atomicOr(overflow, 1u);  // unresolved: the sorted path
    }
    // hashed duplicates: the strings of every pair (winner, key) must be equal
    // (the general decimal-concatenation comparison only for different POS
    // or two blob tails); more pairs than the list: the sorted path
    {
        const uint32_t nc = s_nconf;
        if (nc > kWConfirm && threadIdx.x == 0) bad = true;
        for (uint32_t i = threadIdx.x; i < min(nc, kWConfirm); i += kWT) {
            const uint32_t w = s_conf[i] & 0xffffu, f = s_conf[i] >> 16;
            uint32_t q = 0, r = 0;
            while (q + 1 < np && s_pre[q + 1] <= w) ++q;
            while (r + 1 < np && s_pre[r + 1] <= f) ++r;
            const KBody xb = ks.body[w + s_base[q]], b = ks.body[f + s_base[r]];
            if (!(xb.pos == b.pos && xb.tail == b.tail)) {
                if (xb.pos == b.pos && !((xb.tail & b.tail) & kTailBlob)) bad = true;
                else if (!body_equal(ks, xb, b)) bad = true;
            }
        }
    }
    if (nd) {
        uint32_t at = s_def0 + dofs;
#pragma unroll
        for (uint32_t u = 0; u < kWPer; ++u)
            if ((dm >> u) & 1u) {
                const uint32_t pc = static_cast<uint32_t>(pk >> (6 * u)) & 63u;
                if (at < cap) list[at] = uint2{u * kWT + threadIdx.x + s_base[pc], W.run_lo + pc};
                ++at;
            }
    }
    if (bad) atomicOr(overflow, 1u);
    const uint32_t fw = wave_sum_u32(fresh);
    if (lane == 0 && fw) atomicAdd(&s_fresh, fw);
    win_sync();
    // the window's count, folded per job by window_fold_kernel: one device
    // atomic per window on the jobs' few counter lines (73 k windows for 50
    // jobs) serialised in L2
    if (threadIdx.x == 0) wfresh[blockIdx.x] = s_fresh;
}

// one wave per planned job: its windows' counts [w0, w0 + nw) summed into
// counts[its runs' job] (the job each of its windows counted for)
__global__ __launch_bounds__(kThreads) void window_fold_kernel(const KJob *__restrict__ jobs, uint32_t nj,
                                                               const KRun *__restrict__ runs,
                                                               const uint32_t *__restrict__ wfresh,
                                                               unsigned long long *__restrict__ counts) {
    const uint32_t j = (blockIdx.x * kThreads + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
    if (j >= nj) return;
    const KJob J = jobs[j];
    uint32_t sum = 0;
    for (uint32_t i = lane; i < J.nw; i += 64) sum += wfresh[J.w0 + i];
    const uint32_t tot = wave_sum_u32(sum);
    if (lane == 0 && tot) atomicAdd(&counts[runs[J.run_lo].job], static_cast<unsigned long long>(tot));
}

uint32_t tiles_of(uint64_t n) { return static_cast<uint32_t>((n + kTile - 1) / kTile); }

void exclusive_scan(uint32_t *a, uint64_t m, uint32_t *bsum, hipStream_t s) {
    const uint32_t nb = static_cast<uint32_t>((m + kTile - 1) / kTile);
    scan_reduce_kernel<<<nb, kThreads, 0, s>>>(a, m, bsum);
    scan_top_kernel<<<1, kThreads, 0, s>>>(bsum, nb);
    scan_down_kernel<<<nb, kThreads, 0, s>>>(a, m, bsum);
}

}  // namespace

size_t radix_hist_words(uint64_t n) { return static_cast<size_t>(tiles_of(n)) * 256; }
size_t radix_bsum_words(uint64_t n) { return (radix_hist_words(n) + kTile - 1) / kTile + 1; }

uint32_t dedup_gather_tile() { return kGTile; }

void launch_dedup_gather(const KStore &ks, const KSeg *segs, const uint2 *tiles, uint32_t ntiles, uint32_t pos_bits,
                         uint32_t exact_job_shift, uint32_t job_bits, uint64_t mask, uint64_t *ke, uint64_t *kh,
                         uint32_t *vh, uint32_t *tcnt, hipStream_t s) {
    if (!ntiles) return;
    gather_kernel<<<ntiles, kThreads, 0, s>>>(ks, segs, tiles, ntiles, pos_bits, exact_job_shift, job_bits, mask, ke,
                                              kh, vh, tcnt);
}

namespace {
template <bool MIX>
int radix_passes(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint64_t n, uint32_t shift0, uint32_t bits,
                 uint32_t *hist, uint32_t *bsum, hipStream_t s, const uint32_t *tile_n, uint32_t sparse_tiles) {
    uint64_t *kin = k0, *kout = k1;
    uint32_t *vin = v0, *vout = v1;
    for (uint32_t shift = shift0; shift < bits || (tile_n && shift == shift0); shift += 8) {
        const bool sparse = tile_n && shift == shift0;  // the first pass compacts the gather tiles
        const uint32_t nt = sparse ? sparse_tiles : tiles_of(n);
        const uint32_t *tn = sparse ? tile_n : nullptr;
        upsweep_kernel<MIX><<<nt, kThreads, 0, s>>>(kin, n, tn, shift, hist, nt);
        exclusive_scan(hist, static_cast<uint64_t>(nt) * 256, bsum, s);
        if (vin)
            downsweep_kernel<true, MIX><<<nt, kThreads, 0, s>>>(kin, vin, kout, vout, n, tn, shift, hist, nt);
        else
            downsweep_kernel<false, MIX><<<nt, kThreads, 0, s>>>(kin, vin, kout, vout, n, tn, shift, hist, nt);
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    return kin == k0 ? 0 : 1;
}
}  // namespace

int launch_radix_sort(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint64_t n, uint32_t bits,
                      uint32_t *hist, uint32_t *bsum, hipStream_t s, const uint32_t *tile_n, uint32_t sparse_tiles) {
    if (n == 0) return 0;
    if (n <= 1 && !tile_n) return 0;
    return radix_passes<false>(k0, v0, k1, v1, n, 0, bits, hist, bsum, s, tile_n, sparse_tiles);
}

int launch_bucket_dedupe(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint64_t n, const KStore &ks,
                         uint32_t job_shift, uint32_t nj, unsigned long long *counts, uint32_t *overflow,
                         uint32_t *hist, uint32_t *bsum, hipStream_t s, const uint32_t *tile_n, uint32_t sparse_tiles) {
    if (n == 0) return 0;
    // two stable passes on bits 48..63 of mix(word): buckets contiguous
    const int r = radix_passes<true>(k0, v0, k1, v1, n, 48, 64, hist, bsum, s, tile_n, sparse_tiles);
    const uint64_t *keys = r ? k1 : k0;
    const uint32_t *vals = v0 ? (r ? v1 : v0) : nullptr;
    const uint32_t nb = static_cast<uint32_t>((n + kBTile - 1) / kBTile);
    // SBEACON_DEDUP_BUCKET_CAP (tests): a smaller cap forces the overflow fallback
    const uint32_t slots = v0 ? 4096u : kBSlots;
    uint32_t cap = slots * 3 / 4;
    if (const int k = config().dedup_bucket_cap) cap = std::min<uint32_t>(cap, static_cast<uint32_t>(k));
    const uint32_t njl = nj < 256 ? nj : 256u;
    const uint32_t dbg = static_cast<uint32_t>(config().dedup_bucket_dbg);
    if (v0)
        bucket_dedupe_kernel<true, 4096><<<nb, kThreads, 0, s>>>(keys, vals, n, ks, job_shift, njl, counts, overflow, cap,
                                                                 dbg);
    else
        bucket_dedupe_kernel<false, kBSlots><<<nb, kThreads, 0, s>>>(keys, nullptr, n, ks, job_shift, njl, counts, overflow,
                                                                     cap, dbg);
    return r;
}

void launch_window_dedupe(const KStore &ks, const KJob *jobs, uint32_t nj, uint32_t *rec, uint32_t rec_words, uint32_t nw,
                          const KRun *runs, unsigned long long *counts, uint2 *list, uint32_t *n_list, uint32_t cap,
                          uint32_t *overflow, uint32_t *wfresh, hipStream_t s) {
    if (!nw) return;
    const uint32_t dbg = static_cast<uint32_t>(config().dedup_win_dbg);  // timing ablations (never set by the benches)
    dedup_plan_kernel<<<(nw + kThreads - 1) / kThreads, kThreads, 0, s>>>(ks, jobs, nj, runs, nw, rec, rec_words);
    window_dedupe_kernel<<<nw, kWT, 0, s>>>(ks, rec, rec_words, counts, list, n_list, cap, overflow, wfresh, dbg);
    window_fold_kernel<<<(nj * 64 + kThreads - 1) / kThreads, kThreads, 0, s>>>(jobs, nj, runs, wfresh, counts);
    deferred_dedupe_kernel<<<1024, kThreads, 0, s>>>(ks, runs, list, n_list, cap, counts);
}

uint32_t dedup_unique_blocks(uint64_t n) { return n ? tiles_of(n) : 0; }

void launch_dedup_unique(const uint64_t *keys, const uint32_t *vals, uint64_t n, const KStore &ks, uint32_t job_shift,
                         bool verify, unsigned long long *counts, uint4 *part, uint32_t *coll, uint32_t *ncoll,
                         hipStream_t s) {
    if (!n) return;
    if (verify)
        unique_kernel<true><<<tiles_of(n), kThreads, 0, s>>>(keys, vals, n, ks, job_shift, counts, part, coll, ncoll);
    else
        unique_kernel<false><<<tiles_of(n), kThreads, 0, s>>>(keys, vals, n, ks, job_shift, counts, part, coll, ncoll);
}

}  // namespace sb
