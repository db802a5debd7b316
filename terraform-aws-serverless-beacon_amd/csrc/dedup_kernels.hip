// dedup_kernels.hip — duplicateVariantSearch on the device.
//
// The reference (lambda/duplicateVariantSearch/source/duplicateVariantSearch.cpp
// :31-84) inflates every region file of a (dataset, contig, range) job and
// inserts to_string(pos) + ref'_alt' into an unordered_set<string>; the job's
// answer is the set size.  Here the region keys already sit in HBM (one 64-bit
// hash + a tail word per key, devtypes.hpp KStore), and a batch of jobs is
// answered with
//   1. gather:   the keys of every job's VCF ranges -> (job | hash, key id)
//   2. LSD radix sort of the 64-bit words, 8 passes of 8 bits, each pass =
//      tile histogram (upsweep) + exclusive scan + stable rank-and-scatter
//      (downsweep: wave-level match via 8 ballots, per-wave LDS counters)
//   3. unique:   adjacent compare; equal words are confirmed byte-for-byte on
//      the key strings, and pairs whose strings differ (hash collisions) are
//      listed for the host's exact recount of that group.
// Sorting by (job, hash) keeps every job contiguous, so the whole batch is one
// sort.  All passes are HBM-streaming integer work: 256-thread workgroups, one
// tile of 4096 keys each, coalesced 64-lane loads.
#include <hip/hip_runtime.h>

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
__global__ __launch_bounds__(kThreads) void gather_kernel(KStore ks, const KSeg *segs, uint32_t nseg, uint64_t n,
                                                          uint32_t job_bits, uint64_t mask, uint64_t *keys,
                                                          uint32_t *vals) {
    const uint64_t i = static_cast<uint64_t>(blockIdx.x) * kThreads + threadIdx.x;
    if (i >= n) return;
    uint32_t lo = 0, hi = nseg;  // last segment with out_lo <= i
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (segs[m].out_lo <= i) lo = m; else hi = m;
    }
    const KSeg g = segs[lo];
    const uint64_t k = g.key_lo + (i - g.out_lo);
    const uint64_t h = ks.hash[k] & mask;
    keys[i] = job_bits ? ((static_cast<uint64_t>(g.job) << (64 - job_bits)) | (h >> job_bits)) : h;
    vals[i] = static_cast<uint32_t>(k);
}

// ------------------------------------------------------------- radix sort
// hist layout: digit-major, hist[d * ntiles + tile]
__global__ __launch_bounds__(kThreads) void upsweep_kernel(const uint64_t *keys, uint64_t n, uint32_t shift,
                                                           uint32_t *hist, uint32_t ntiles) {
    __shared__ uint32_t h[kWaves][256];
    const int w = threadIdx.x >> 6;
    for (int i = threadIdx.x; i < kWaves * 256; i += kThreads) (&h[0][0])[i] = 0;
    __syncthreads();
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile;
    uint32_t dg[kItems];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = base + static_cast<uint64_t>(r) * kThreads + threadIdx.x;
        dg[r] = i < n ? static_cast<uint32_t>(keys[i] >> shift) & 255u : 256u;
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

__global__ __launch_bounds__(kThreads) void downsweep_kernel(const uint64_t *kin, const uint32_t *vin,
                                                             uint64_t *kout, uint32_t *vout, uint64_t n,
                                                             uint32_t shift, const uint32_t *off, uint32_t ntiles) {
    __shared__ uint32_t cnt[kWaves][256];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < kWaves * 256; i += kThreads) (&cnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile + static_cast<uint64_t>(w) * kWaveKeys;
    uint64_t k[kItems];
    uint32_t v[kItems], rank[kItems];
    // all of the wave's loads in flight first, then rank in index order
    // (wave w owns a contiguous quarter of the tile)
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = base + static_cast<uint64_t>(r) * 64 + lane;
        k[r] = i < n ? kin[i] : 0;
        v[r] = i < n ? vin[i] : 0;
    }
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const bool ok = base + static_cast<uint64_t>(r) * 64 + lane < n;
        const uint32_t d = static_cast<uint32_t>(k[r] >> shift) & 255u;
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
    __shared__ uint32_t sv[kTile];
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = base + static_cast<uint64_t>(r) * 64 + lane;
        if (i < n) {
            const uint32_t d = static_cast<uint32_t>(k[r] >> shift) & 255u;
            const uint32_t loc = cnt[w][d] + rank[r];
            sk[loc] = k[r];
            sv[loc] = v[r];
        }
    }
    __syncthreads();
    const uint64_t tile0 = static_cast<uint64_t>(blockIdx.x) * kTile;
    const uint32_t tn = static_cast<uint32_t>(min(static_cast<uint64_t>(kTile), n - tile0));
#pragma unroll
    for (int r = 0; r < kItems; ++r) {
        const uint32_t loc = static_cast<uint32_t>(r) * kThreads + threadIdx.x;
        if (loc < tn) {
            const uint64_t key = sk[loc];
            const uint32_t dst = gbase[static_cast<uint32_t>(key >> shift) & 255u] + loc;
            kout[dst] = key;
            vout[dst] = sv[loc];
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

__device__ bool key_equal(const KStore &ks, uint32_t a, uint32_t b) {
    if (a == b) return true;
    const KBody x = ks.body[a], y = ks.body[b];
    if (x.pos == y.pos && x.tail == y.tail) return true;  // same pos and same inline bytes / same blob bytes
    const KeyStr u = key_str(ks, x), v = key_str(ks, y);
    if (u.nd + u.tl != v.nd + v.tl) return false;
    for (uint32_t j = 0; j < u.nd + u.tl; ++j)
        if (u.at(j) != v.at(j)) return false;
    return true;
}

// kItems sorted positions per thread (coalesced: item r of the block is
// r * kThreads + threadIdx.x); the block's distinct count goes out with one
// atomic per job it touches (one in the common single-job block)
__global__ __launch_bounds__(kThreads) void unique_kernel(const uint64_t *keys, const uint32_t *vals, uint64_t n,
                                                          KStore ks, uint32_t job_bits, unsigned long long *counts,
                                                          uint32_t *coll, uint32_t *ncoll) {
    __shared__ uint32_t s_job[2];
    __shared__ unsigned int s_cnt;
    const uint64_t base = static_cast<uint64_t>(blockIdx.x) * kTile;
    if (threadIdx.x == 0) {
        s_cnt = 0;
        const uint64_t last = min(n, base + kTile) - 1;
        s_job[0] = job_bits ? static_cast<uint32_t>(keys[base] >> (64 - job_bits)) : 0u;
        s_job[1] = job_bits ? static_cast<uint32_t>(keys[last] >> (64 - job_bits)) : 0u;
    }
    __syncthreads();
    const bool one_job = s_job[0] == s_job[1];
    uint32_t mine = 0;
#pragma unroll 4
    for (int r = 0; r < kItems; ++r) {
        const uint64_t i = base + static_cast<uint64_t>(r) * kThreads + threadIdx.x;
        if (i >= n) break;
        const uint64_t k = keys[i];
        bool fresh = false;
        if (i == 0 || keys[i - 1] != k) {
            fresh = true;
        } else if (!key_equal(ks, vals[i - 1], vals[i])) {
            fresh = true;  // a different string under the same word: the host recounts its group
            coll[atomicAdd(ncoll, 1u)] = static_cast<uint32_t>(i);
        }
        if (!fresh) continue;
        if (one_job) {
            ++mine;
        } else {
            atomicAdd(&counts[job_bits ? static_cast<uint32_t>(k >> (64 - job_bits)) : 0u], 1ull);
        }
    }
    if (one_job) {
        // wave sum, then one LDS add per wave and one global atomic per block
        for (int d = 32; d >= 1; d >>= 1) mine += __shfl_xor(mine, d, 64);
        if ((threadIdx.x & 63) == 0 && mine) atomicAdd(&s_cnt, mine);
        __syncthreads();
        if (threadIdx.x == 0 && s_cnt) atomicAdd(&counts[s_job[0]], static_cast<unsigned long long>(s_cnt));
    }
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

void launch_dedup_gather(const KStore &ks, const KSeg *segs, uint32_t nseg, uint64_t n, uint32_t job_bits,
                         uint64_t mask, uint64_t *keys, uint32_t *vals, hipStream_t s) {
    if (!n) return;
    gather_kernel<<<static_cast<uint32_t>((n + kThreads - 1) / kThreads), kThreads, 0, s>>>(ks, segs, nseg, n,
                                                                                           job_bits, mask, keys, vals);
}

int launch_radix_sort(uint64_t *k0, uint32_t *v0, uint64_t *k1, uint32_t *v1, uint64_t n, uint32_t *hist,
                      uint32_t *bsum, hipStream_t s) {
    if (n <= 1) return 0;
    const uint32_t nt = tiles_of(n);
    uint64_t *kin = k0, *kout = k1;
    uint32_t *vin = v0, *vout = v1;
    for (uint32_t shift = 0; shift < 64; shift += 8) {
        upsweep_kernel<<<nt, kThreads, 0, s>>>(kin, n, shift, hist, nt);
        exclusive_scan(hist, static_cast<uint64_t>(nt) * 256, bsum, s);
        downsweep_kernel<<<nt, kThreads, 0, s>>>(kin, vin, kout, vout, n, shift, hist, nt);
        std::swap(kin, kout);
        std::swap(vin, vout);
    }
    return kin == k0 ? 0 : 1;  // 8 passes: the result is back in (k0, v0)
}

void launch_dedup_unique(const uint64_t *keys, const uint32_t *vals, uint64_t n, const KStore &ks, uint32_t job_bits,
                         unsigned long long *counts, uint32_t *coll, uint32_t *ncoll, hipStream_t s) {
    if (!n) return;
    unique_kernel<<<tiles_of(n), kThreads, 0, s>>>(keys, vals, n, ks,
                                                                                           job_bits, counts, coll,
                                                                                           ncoll);
}

}  // namespace sb
