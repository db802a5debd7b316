// api.cpp — the C ABI (include/sbeacon.h): builder, HBM store, query batches.
//
// The query path mirrors one splitQuery fan-out (lambda/splitQuery/
// lambda_function.py:74-110) handed to the device as ONE batch: every
// PerformQueryPayload becomes a QDev; the host plans each query's output
// region from the store's coarse POS index (an upper bound on its hits), so
// a query step is a single kernel launch (query_kernels.hip).  Result strings
// are formatted on the host from the store's allele blob in the reference's
// exact format.
#include <algorithm>
#include <deque>
#include <atomic>
#include <array>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <thread>
#include <tuple>
#include <string_view>
#include <unordered_map>
#include <unordered_set>

#include <zlib.h>

#include "config.hpp"
#include "jsonesc.hpp"
#include "kernels.hpp"
#include "store.hpp"

namespace sb {
void builder_add_text(sb_builder &b, uint32_t vcf_id, const char *text, size_t len);
void builder_add_file(sb_builder &b, uint32_t vcf_id, const char *path);
void builder_flush(sb_builder &b, uint32_t vcf_id);
void vcf_scan_file(const char *path, VcfScan &out);
void builder_attach_carriers(sb_builder &b, uint32_t vcf_id, const char *const *names, const uint32_t *name_len,
                             uint32_t n_samples, const uint64_t *planes, uint64_t n_rows);

namespace {
thread_local std::string g_last_error;

#define HIP_OK(expr)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            throw ::sb::Error(SB_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_));            \
    } while (0)

template <class F>
int guard(F &&f) {
    try {
        f();
        return SB_OK;
    } catch (const Error &e) {
        set_last_error(e.what());
        return e.code;
    } catch (const std::bad_alloc &) {
        set_last_error("out of host memory");
        return SB_ENOMEM;
    } catch (const std::exception &e) {
        set_last_error(e.what());
        return SB_EINVAL;
    }
}

template <class T>
T *dev_upload(sb_store &s, const std::vector<T> &v) {
    if (s.device < 0) return nullptr;  // a host-only store (SB_HOST_ONLY): no device image
    DeviceBuffer b;
    b.bytes = std::max<size_t>(v.size() * sizeof(T), 16);
    HIP_OK(hipMalloc(&b.p, b.bytes));
    if (!v.empty()) {
        HIP_OK(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s.stream));
        HIP_OK(hipStreamSynchronize(s.stream));  // callers free pageable temporaries right after
    }
    s.bufs.push_back(b);
    s.device_bytes += b.bytes;
    return static_cast<T *>(b.p);
}

struct DevMem {  // RAII device allocation for batches (move-only)
    void *p = nullptr;
    size_t bytes = 0;
    DevMem() = default;
    DevMem(const DevMem &) = delete;
    DevMem &operator=(const DevMem &) = delete;
    DevMem(DevMem &&o) noexcept : p(o.p), bytes(o.bytes) {
        o.p = nullptr;
        o.bytes = 0;
    }
    DevMem &operator=(DevMem &&o) noexcept {
        if (this != &o) {
            release();
            p = o.p;
            bytes = o.bytes;
            o.p = nullptr;
            o.bytes = 0;
        }
        return *this;
    }
    void alloc(size_t n) {
        release();
        bytes = std::max<size_t>(n, 16);
        HIP_OK(hipMalloc(&p, bytes));
    }
    // keep the allocation when it is large enough (per-store scratch reused
    // across calls: hipMalloc / hipFree of ~1 GB per call cost more than the
    // kernels)
    void reserve(size_t n) {
        if (p && bytes >= n) return;
        alloc(n + n / 4);
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <class T>
    T *as() const { return static_cast<T *>(p); }
    ~DevMem() { release(); }
};

struct ParsedRegion {
    std::string chrom;
    int64_t first = 0, last = 0;
    bool ok = false;
};

// search_variants.py:56-58 — chrom up to the first ':', first_bp up to the
// first '-', last_bp after it (Python int()).
ParsedRegion parse_region(const char *p, size_t n) {
    ParsedRegion r;
    const std::string s(p, n);
    const size_t c = s.find(':'), d = s.find('-');
    if (c == std::string::npos || d == std::string::npos || d < c) return r;
    r.chrom = s.substr(0, c);
    if (!py_int(s.data() + c + 1, d - c - 1, &r.first)) return r;
    if (!py_int(s.data() + d + 1, s.size() - d - 1, &r.last)) return r;
    r.ok = true;
    return r;
}

bool starts(const std::string &s, const char *pre) { return s.compare(0, strlen(pre), pre) == 0; }

// Host-side evaluation of the symbolic-ALT predicates of :101-166 for one
// variantType string over the store's symbolic dictionary.
std::vector<uint32_t> sym_lut(const sb_store &s, uint32_t kind, const std::string &vprefix) {
    std::vector<uint32_t> lut((s.sym.items.size() + 31) / 32 + 1, 0u);
    for (size_t i = 0; i < s.sym.items.size(); ++i) {
        const std::string &a = s.sym.items[i];
        bool ok = starts(a, vprefix.c_str());
        switch (kind) {
            case VT_DEL: ok = ok || a == "<CN0>"; break;
            case VT_DUP: ok = ok || (starts(a, "<CN") && a != "<CN0>" && a != "<CN1>"); break;
            case VT_DUPT: ok = ok || a == "<CN2>"; break;
            case VT_CNV: ok = ok || starts(a, "<CN") || starts(a, "<DEL") || starts(a, "<DUP"); break;
            default: break;
        }
        if (ok) lut[i / 32] |= 1u << (i % 32);
    }
    return lut;
}

}  // namespace

void set_last_error(const std::string &msg) { g_last_error = msg; }
const char *last_error_cstr() { return g_last_error.c_str(); }

}  // namespace sb

using namespace sb;

namespace sb {
void store_save(sb_store &s, const std::string &dir);                         // persist.cpp
sb_store *store_open(const std::string &path, int device, std::string *stale);  // persist.cpp
sb_store *store_hold(sb_store *s) {
    s->holders.fetch_add(1, std::memory_order_acq_rel);
    return s;
}
void store_release(sb_store *s) {
    if (s->holders.fetch_sub(1, std::memory_order_acq_rel) == 1) delete s;
}
}  // namespace sb

sb_store::~sb_store() {
    if (device >= 0) (void)hipSetDevice(device);
    for (auto &b : bufs) (void)hipFree(b.p);
    if (stream) (void)hipStreamDestroy(stream);
}

// ------------------------------------------------------------------ batch
// Request batches' buffers, pooled per store (sb_store::req_pool): planning
// stages descriptors in pinned host memory and a pass needs seven device
// buffers; allocating them per batch (hipHostMalloc pins pages, hipFree
// synchronises the device) cost more than the pass itself.  Best fit among
// the free buffers no more than twice the size asked for; bounded.
struct ReqPool {
    struct Pinned {
        void *p = nullptr;
        size_t bytes = 0;
    };
    std::mutex mu;
    std::vector<Pinned> pinned;
    std::vector<DevMem> dev;
    static constexpr size_t kKeep = 256;                     // buffers kept per kind at most (a pipelined caller holds ~10 per chunk batch)
    static constexpr size_t kKeepDevBytes = size_t(4) << 30;  // and bytes: the largest go first
    static constexpr size_t kKeepPinnedBytes = size_t(2) << 30;
    ~ReqPool() { trim(); }
    template <class V>
    static size_t total(const V &v) {
        size_t t = 0;
        for (const auto &x : v) t += x.bytes;
        return t;
    }
    template <class V>
    static size_t largest(const V &v) {
        size_t b = 0;
        for (size_t i = 1; i < v.size(); ++i)
            if (v[i].bytes > v[b].bytes) b = i;
        return b;
    }
    void trim() {  // free every cached buffer (sb_store_trim)
        std::lock_guard<std::mutex> lk(mu);
        for (Pinned &x : pinned) (void)hipHostFree(x.p);
        pinned.clear();
        dev.clear();
    }
    template <class V>
    static ptrdiff_t fit(const V &v, size_t n) {
        ptrdiff_t best = -1;
        for (size_t i = 0; i < v.size(); ++i)
            if (v[i].bytes >= n && v[i].bytes <= 2 * n + (1u << 20) && (best < 0 || v[i].bytes < v[best].bytes))
                best = static_cast<ptrdiff_t>(i);
        return best;
    }
    Pinned get_pinned(size_t n) {
        {
            std::lock_guard<std::mutex> lk(mu);
            const ptrdiff_t i = fit(pinned, n);
            if (i >= 0) {
                Pinned x = pinned[i];
                pinned.erase(pinned.begin() + i);
                return x;
            }
        }
        Pinned x;
        x.bytes = std::max<size_t>(n + n / 4, 4096);
        HIP_OK(hipHostMalloc(&x.p, x.bytes, hipHostMallocDefault));
        return x;
    }
    void put_pinned(Pinned x) {
        std::lock_guard<std::mutex> lk(mu);
        pinned.push_back(x);
        if (pinned.size() > kKeep) {
            (void)hipHostFree(pinned.front().p);
            pinned.erase(pinned.begin());
        }
        while (pinned.size() > 1 && total(pinned) > kKeepPinnedBytes) {
            const size_t i = largest(pinned);
            (void)hipHostFree(pinned[i].p);
            pinned.erase(pinned.begin() + static_cast<ptrdiff_t>(i));
        }
    }
    DevMem get_dev(size_t n) {
        {
            std::lock_guard<std::mutex> lk(mu);
            const ptrdiff_t i = fit(dev, n);
            if (i >= 0) {
                DevMem x = std::move(dev[i]);
                dev.erase(dev.begin() + i);
                return x;
            }
        }
        DevMem x;
        x.alloc(n + n / 4);
        return x;
    }
    void put_dev(DevMem &&x) {
        std::lock_guard<std::mutex> lk(mu);
        dev.push_back(std::move(x));
        if (dev.size() > kKeep) dev.erase(dev.begin());
        while (dev.size() > 1 && total(dev) > kKeepDevBytes) dev.erase(dev.begin() + static_cast<ptrdiff_t>(largest(dev)));
    }
};

std::shared_ptr<ReqPool> req_pool(sb_store &s) {
    std::call_once(s.req_pool_once, [&] {
        s.req_pool = std::shared_ptr<void>(new ReqPool, [](void *w) { delete static_cast<ReqPool *>(w); });
    });
    return std::shared_ptr<ReqPool>(s.req_pool, static_cast<ReqPool *>(s.req_pool.get()));
}

struct sb_batch {
    sb_store *s = nullptr;
    uint32_t nq = 0;
    std::vector<QDev> hq;
    std::vector<int32_t> host_err;               // errors raised before any record is read
    std::vector<std::string> chrom;              // region chrom per query (variant strings)
    std::vector<std::vector<uint32_t>> emitted;  // header indices of the emitted samples
    std::vector<uint8_t> samples_variant;
    std::vector<uint32_t> vcf;
    uint64_t cap_total = 0, samples_words = 0;
    DevMem q, hoff, qbytes, subsets, lut, res, hits, samples_out;
    // queries split by kernel variant: the sample path compiled in or out
    // queries grouped by kernel specialisation: one launch per non-empty group
    struct Group {
        int mode;
        uint32_t max_words;  // 0 = sample path compiled out
        std::vector<uint32_t> idx;
        uint32_t base;  // first entry of the group in the launch-ordered device array
    };
    std::vector<Group> groups;
    // slice chains (ChainDev): their slices sit after the groups in the
    // launch-ordered array; n_scanned of a chained slice is known on the host
    std::vector<ChainDev> hchains;
    DevMem chains;
    std::vector<uint32_t> hruns;  // first chain of each chain_pack_kernel wave (+ end)
    DevMem runs;
    // chained slices also write their per-slice QRes rows (sb_batch_set_slice_results);
    // off = request rows + hit lists only (row pieces), fetch refused
    bool slice_rows = true;
    bool slice_rows_stale = false;  // a run without them since the last run with them
    std::vector<uint8_t> chained;
    std::vector<uint32_t> nscan;
    std::vector<uint32_t> chain_members;  // chained queries, chain by chain (device copy: corig)
    uint32_t chain_base = 0;              // first chained slice in the launch-ordered array
    DevMem corig;
    DevMem srcoff;  // each query's hit-region offset (chained slices: rewritten by chain_src_kernel)
    DevMem tsum, dense;  // dense hit lists (sb_batch_compact_hits)
    DevMem cpart;        // per-chain request-row partials (chain_kernel)
    std::vector<uint64_t> chain_cap;  // hit capacity of each chain (ALTs of its coarse candidate range)
    // request rows as pieces (sb_batch_set_owners, when every chain lies in one row)
    bool row_pieces = false;
    DevMem poff, piece, rows_scratch, rowsrc, rowout;
    DevMem nvs;  // sb_batch_deliver: each row's n_variants (8 B / row) for the offset scan
    uint64_t cand_loaded = 0, cand_window = 0, cand_unique = 0;  // chain candidate statistics
    hipStream_t stream = nullptr;  // sb_batch_set_stream (nullptr: the store's stream)
    hipStream_t strm() const { return stream ? stream : s->stream; }
    bool nonneg = true;
    // per-request rows (sb_batch_set_owners): seg = n_rows + 1 query offsets
    uint32_t n_rows = 0;
    DevMem seg, herr;
    bool no_chains = false;  // the slice part of a request batch: every slice answered on its own
    // request batches (sb_requests_prepare): rows = requests
    struct Req {
        uint32_t n_rows = 0;
        std::vector<RowRun> runs;
        uint64_t cap = 0;              // output hit capacity
        uint64_t n_chain_slices = 0;
        uint32_t n_lut = 0;            // LUT words (request_eval_kernel stages them in LDS when they fit)
        uint64_t n_chains = 0;         // chain-answered requests (dchains holds them padded per run)
        uint32_t n_runs = 0;           // runs (runs: their host copy when planned on the host)
        // sb_requests_time_eval: events around every pass's request_eval_kernel
        bool time_eval = false;
        std::vector<std::array<hipEvent_t, 2>> eval_ev;
        size_t eval_used = 0;
        double last_eval_ms = 0;
        ~Req() {
            for (auto &p : eval_ev)
                for (auto e : p) (void)hipEventDestroy(e);
        }
        // dchains: ReqChain slots (kReqRun per run), then the RowRuns at runs_at
        DevMem dchains, status, tstatus, stage, row_src, lut, sseg, sherr;
        // device-planned batches: the packed requests (ReqIn) and the
        // planner's per-run capacities + counters stay resident, so a pass can
        // re-run the planning kernels first (sb_requests_set_replan)
        DevMem din, rcap;
        uint32_t n_in = 0;
        bool replan = false;
        bool compact = false;  // sb_requests_set_compact
        // request_eval_kernel's invariant word (sticky; checked at sync: SB_EINTERNAL)
        DevMem err;
        ReqPool::Pinned err_h;
        // rows whose counts are not exact in int64 (sb_requests_inexact_rows):
        // per-slice wide marks + one flag per row (batches with general records)
        DevMem wide, row_flag;
        std::vector<char> hplan;  // host-only stores: the descriptors + runs (as dchains would hold them)
        size_t runs_at = 0;
        uint32_t run = kReqRun;        // chain slots per run (request_eval_kernel: one lane each)
        std::shared_ptr<ReqPool> pool;  // where the device buffers go back when the batch is freed
        bool slices = false;           // some rows answered per slice (the batch's query part)
        void give_back() {
            for (DevMem *m : {&dchains, &status, &tstatus, &stage, &row_src, &lut, &sseg, &sherr, &wide, &row_flag, &din,
                              &rcap, &err})
                if (m->p) pool->put_dev(std::move(*m));
            if (err_h.p) {
                pool->put_pinned(err_h);
                err_h = ReqPool::Pinned{};
            }
        }
    };
    std::unique_ptr<Req> req;
    // slice batches: device buffers from the store's pool (a steady stream
    // of batches then allocates nothing), given back when the batch is freed
    std::shared_ptr<ReqPool> pool;
    // general records (general_slice_kernel): work list [count, launch
    // indices], per-wave scratch, slices with counts past 64 bits
    DevMem gen_work, gen_scratch, gen_big_n, gen_big, gen_limbs;
    uint32_t gen_grid = 0, gen_big_cap = 0;
    // events around the runs since the last sync (run() records [0], sync() [1])
    std::array<hipEvent_t, 2> ev{};
    size_t runs_pending = 0;
    float last_total_ms = 0;
    std::mutex mu;  // request batches: one pass at a time per batch
    ~sb_batch() {
        for (auto e : ev)
            if (e) (void)hipEventDestroy(e);
        if ((req && req->pool) || pool) (void)hipStreamSynchronize(strm());  // a pass may still be in flight
        if (req && req->pool) req->give_back();
        if (pool)
            for (DevMem *m : {&q, &hoff, &qbytes, &subsets, &lut, &res, &hits, &samples_out, &chains, &runs, &corig,
                              &srcoff, &cpart, &gen_work, &gen_scratch, &gen_big_n, &gen_big, &gen_limbs})
                if (m->p) pool->put_dev(std::move(*m));
    }
};

// a batch buffer: from the batch's pool when it has one
void palloc(sb_batch &B, DevMem &m, size_t n) {
    if (!B.pool) {
        m.alloc(n);
        return;
    }
    if (m.p) B.pool->put_dev(std::move(m));
    m = B.pool->get_dev(std::max<size_t>(n, 16));
}

// a result set's dense hit list: pinned host memory from the store's pool
// (the D2H lands there directly; no zero-filled pageable copy)
struct HitBuf {
    std::shared_ptr<ReqPool> pool;
    ReqPool::Pinned mem;
    size_t n = 0;
    HitBuf() = default;
    HitBuf(const HitBuf &) = delete;
    HitBuf &operator=(const HitBuf &) = delete;
    ~HitBuf() {
        if (mem.p) pool->put_pinned(mem);
    }
    uint64_t *data() { return static_cast<uint64_t *>(mem.p); }
    const uint64_t &operator[](size_t i) const { return static_cast<const uint64_t *>(mem.p)[i]; }
    size_t size() const { return n; }
};

struct sb_result_set {
    sb_store *s = nullptr;  // held (store_hold) while the set lives
    ~sb_result_set() {
        if (s) store_release(s);
    }
    std::vector<QRes> res;
    std::vector<uint64_t> dense_off;
    HitBuf hit;                                 // rec | alt << 32
    std::vector<std::vector<uint32_t>> sidx;    // emitted-list positions
    std::vector<std::vector<uint32_t>> emitted;
    std::vector<uint32_t> vcf_of;
    std::vector<uint8_t> samples_variant;
    std::vector<std::string> chrom;
    std::vector<std::string> vtext, ntext;
    std::vector<uint8_t> vbuilt, nbuilt;
    std::string distinct;                       // sb_result_distinct_variants
    std::vector<std::string> vt_json;           // escaped VT strings (sb::result_prepare_json)
    // per VCF of the set, per header sample: its name as JSON list items
    // (sb::result_prepare_json; "\x01" = not UTF-8)
    std::vector<std::vector<std::string>> names_json;
    // views for sb_result_get, split out of `hit` on its first call
    mutable std::vector<uint32_t> tmp_rec, tmp_alt;
    mutable std::once_flag tmp_once;
    // queries whose counts need more than 64 bits: 2 x big_limbs limbs each
    uint32_t big_limbs = 0;
    std::unordered_map<uint32_t, std::vector<uint32_t>> big;
    sb_batch_stats stats{};
};

namespace {


// coarse POS index of one segment: bucket[b] = first record with
// POS >= base + (b << shift), for b in [0, n]; bucket[n] = segment end
void build_buckets(const std::vector<uint32_t> &pos, const Segment &sg, BucketIndex &bi,
                   std::vector<uint32_t> &bucket) {
    bi.off = bucket.size();
    if (sg.hi <= sg.lo) {
        bi.base = 0;
        bi.shift = 31;
        bi.n = 1;
        bucket.push_back(sg.lo);
        bucket.push_back(sg.hi);
        return;
    }
    const uint32_t base = pos[sg.lo];
    const uint64_t span = static_cast<uint64_t>(pos[sg.hi - 1]) - base;
    const uint64_t n = sg.hi - sg.lo;
    // aim for ~32 records per bucket on average
    const double gap = n > 1 ? static_cast<double>(span) / static_cast<double>(n - 1) : 1.0;
    uint32_t shift = 0;
    while (shift < 31 && static_cast<double>(1ull << (shift + 1)) <= gap * 32.0) ++shift;
    const uint64_t nb = (span >> shift) + 1;
    bi.base = base;
    bi.shift = shift;
    bi.n = static_cast<uint32_t>(nb);
    uint32_t r = sg.lo;
    for (uint64_t b = 0; b <= nb; ++b) {
        const uint64_t x = static_cast<uint64_t>(base) + (b << shift);
        while (r < sg.hi && pos[r] < x) ++r;
        bucket.push_back(r);
    }
    bucket.back() = sg.hi;
}

void upload_store(sb_builder &b, sb_store &s) {
    std::vector<RecHot> rec;
    std::vector<RangeHot> rng;
    std::vector<uint32_t> pos, a0_len, x_lo, x_cls, x_len, fb, bucket;
    std::vector<int32_t> x_ac;
    std::vector<uint64_t> ref_key, a0_key, ref_off, a0_off, x_key, x_off, planes;
    std::vector<int64_t> fb_off;
    std::vector<uint16_t> vt;
    std::vector<uint8_t> blob;
    std::vector<uint64_t> start;
    std::vector<SumHot> sum;
    std::vector<uint32_t> cur, dcount;
    std::vector<uint32_t> dk_pos, dk_lo, dk_bad;
    std::vector<uint64_t> dk_hash, dk_tail;
    std::vector<uint8_t> dk_blob;
    // general records (GenRec side table), global indexing
    std::vector<GenRec> gen;
    std::vector<uint64_t> gnum_off{0}, gtok_off;
    std::vector<uint32_t> gnum, gtok;
    std::vector<GenVal> gval;
    uint64_t nr = 0, nx = 0, np = 0, nk = 0;
    for (auto &v : b.vcfs) {
        nr += v.c.pos.size();
        nx += v.c.x_key.size();
        nk += v.c.dk_hash.size();
        np += v.c.planes0.size() + v.c.planesx.size();
    }
    if (nr >= 0xfffffff0ull || nx >= 0xfffffff0ull || nk >= 0xfffffff0ull)
        throw Error(SB_EINVAL, "store exceeds 2^32 records per device; shard it across devices");
    rec.reserve(nr);
    pos.reserve(nr);
    planes.reserve(np);
    for (auto &v : b.vcfs) {
        VcfCols &c = v.c;
        const uint32_t rec_base = static_cast<uint32_t>(pos.size());
        const uint32_t x_base = static_cast<uint32_t>(x_key.size());
        const uint64_t blob_base = blob.size();
        const int64_t fb_base = static_cast<int64_t>(fb.size());
        const size_t n = c.pos.size();
        v.rec_base = rec_base;
        v.x_base = x_base;
        v.nonneg = !c.any_negative;
        v.has_planes = !c.planes0.empty();
        v.sample_pos.clear();
        for (uint32_t k = 0; k < v.samples.size(); ++k) v.sample_pos[v.samples[k]].push_back(k);
        v.plane0_base = planes.size();
        planes.insert(planes.end(), c.planes0.begin(), c.planes0.end());
        v.planex_base = planes.size();
        planes.insert(planes.end(), c.planesx.begin(), c.planesx.end());
        std::vector<uint64_t>().swap(c.planes0);  // the device copy is the only one used after upload
        std::vector<uint64_t>().swap(c.planesx);
        rec.insert(rec.end(), c.rec.begin(), c.rec.end());
        {  // general records: global record / number / token / value indices
            const uint32_t gen0 = static_cast<uint32_t>(gen.size());
            const uint64_t num0 = gnum_off.size() - 1, tok0 = gtok_off.size(), gt0 = gtok.size();
            const uint32_t val0 = static_cast<uint32_t>(gval.size());
            const uint64_t limb0 = gnum.size();
            for (size_t k = 0; k < c.gen.size(); ++k) {
                GenRec g = c.gen[k];
                rec[rec_base + g.rec].ac0 = static_cast<int32_t>(gen0 + k);
                g.rec += rec_base;
                g.ac_num += num0;
                g.an_num += num0;
                if (g.flags & GR_FB) {
                    g.tok_off += tok0;
                    g.val_off += val0;
                }
                gen.push_back(g);
            }
            for (size_t k = 1; k < c.gnum_off.size(); ++k) gnum_off.push_back(c.gnum_off[k] + limb0);
            gnum.insert(gnum.end(), c.gnum.begin(), c.gnum.end());
            for (uint64_t o : c.gtok_off) gtok_off.push_back(o + gt0);
            gtok.insert(gtok.end(), c.gtok.begin(), c.gtok.end());
            gval.insert(gval.end(), c.gval.begin(), c.gval.end());
        }
        rng.insert(rng.end(), c.rng.begin(), c.rng.end());
        pos.insert(pos.end(), c.pos.begin(), c.pos.end());
        a0_len.insert(a0_len.end(), c.a0_len.begin(), c.a0_len.end());
        ref_key.insert(ref_key.end(), c.ref_key.begin(), c.ref_key.end());
        a0_key.insert(a0_key.end(), c.a0_key.begin(), c.a0_key.end());
        vt.insert(vt.end(), c.vt.begin(), c.vt.end());
        start.insert(start.end(), c.start.begin(), c.start.end());
        sum.insert(sum.end(), c.sum.begin(), c.sum.end());
        cur.insert(cur.end(), c.cur.begin(), c.cur.end());
        dcount.insert(dcount.end(), c.dcount.begin(), c.dcount.end());
        for (size_t i = 0; i < n; ++i) {
            ref_off.push_back(c.ref_off[i] + blob_base);
            a0_off.push_back(c.a0_off[i] + blob_base);
            fb_off.push_back(c.fb_off[i] < 0 ? -1 : c.fb_off[i] + fb_base);
            x_lo.push_back(c.x_lo[i] + x_base);
        }
        x_cls.insert(x_cls.end(), c.x_cls.begin(), c.x_cls.end());
        x_len.insert(x_len.end(), c.x_len.begin(), c.x_len.end());
        x_ac.insert(x_ac.end(), c.x_ac.begin(), c.x_ac.end());
        x_key.insert(x_key.end(), c.x_key.begin(), c.x_key.end());
        for (size_t i = 0; i < c.x_off.size(); ++i) x_off.push_back(c.x_off[i] + blob_base);
        blob.insert(blob.end(), c.blob.begin(), c.blob.end());
        fb.insert(fb.end(), c.fb.begin(), c.fb.end());
        {
            const uint32_t kbase = static_cast<uint32_t>(dk_hash.size());
            const uint64_t kblob = dk_blob.size();
            for (size_t i = 0; i < n; ++i) dk_lo.push_back(c.dk_lo[i] + kbase);
            dk_pos.insert(dk_pos.end(), c.dk_pos.begin(), c.dk_pos.end());
            dk_hash.insert(dk_hash.end(), c.dk_hash.begin(), c.dk_hash.end());
            for (uint64_t t : c.dk_tail) dk_tail.push_back((t & kTailBlob) ? t + kblob : t);
            dk_blob.insert(dk_blob.end(), c.dk_blob.begin(), c.dk_blob.end());
            for (uint32_t r : c.dk_bad) dk_bad.push_back(r + rec_base);
        }
        for (auto &sg : v.segments) {
            sg.lo += rec_base;
            sg.hi += rec_base;
        }
        s.max_words = std::max(s.max_words, v.has_planes ? v.words : 0u);
        c = VcfCols();  // release the per-vcf copy
    }
    x_lo.push_back(static_cast<uint32_t>(x_key.size()));
    dk_lo.push_back(static_cast<uint32_t>(dk_hash.size()));
    for (auto &v : b.vcfs) {
        v.buckets.resize(v.segments.size());
        for (size_t i = 0; i < v.segments.size(); ++i) build_buckets(pos, v.segments[i], v.buckets[i], bucket);
    }
    s.n_records = pos.size();
    s.n_extra = x_key.size();
    if (gen.size() > 0xffffffffull) throw Error(SB_EINVAL, "more than 2^32 general records");
    {  // general records: numbers repacked to one limb count (sign-extended)
        uint32_t L = 2;
        for (size_t k = 0; k + 1 < gnum_off.size(); ++k)
            L = std::max<uint32_t>(L, static_cast<uint32_t>(gnum_off[k + 1] - gnum_off[k]));
        if (L + 2 > kGenAccMax) throw Error(SB_EPARSE, "an INFO integer beyond the general path's width");
        const size_t nn = gnum_off.size() - 1;
        std::vector<uint32_t> num(nn * L);
        for (size_t k = 0; k < nn; ++k) {
            const uint64_t a = gnum_off[k], e = gnum_off[k + 1];
            const uint32_t sgn = (gnum[e - 1] >> 31) ? 0xffffffffu : 0u;
            for (uint32_t j = 0; j < L; ++j) num[k * L + j] = a + j < e ? gnum[a + j] : sgn;
        }
        s.g.n = static_cast<uint32_t>(gen.size());
        s.g.limbs = L;
        s.g.acc_limbs = std::max<uint32_t>(L + 2, 4);
        s.g.max_alt = s.g.max_vals = 0;
        for (const GenRec &g : gen) {
            s.g.max_alt = std::max(s.g.max_alt, g.n_alt);
            s.g.max_vals = std::max(s.g.max_vals, g.n_vals);
        }
        s.g.rec = dev_upload(s, gen);
        s.g.num = dev_upload(s, num);
        s.g.tok_off = dev_upload(s, gtok_off);
        s.g.tok = dev_upload(s, gtok);
        s.g.val = dev_upload(s, gval);
    }

    s.d.rec = dev_upload(s, rec);
    s.d.rng = dev_upload(s, rng);
    {  // RangeHot8 per VCF: its most common AN, and whether the 8-byte words cover it
        std::vector<RangeHot8> rng8(rng.size());
        for (size_t vi = 0; vi < b.vcfs.size(); ++vi) {
            VcfData &v = b.vcfs[vi];
            const size_t r0 = v.rec_base, r1 = vi + 1 < b.vcfs.size() ? b.vcfs[vi + 1].rec_base : rng.size();
            std::unordered_map<int32_t, uint64_t> freq;
            for (size_t r = r0; r < r1; ++r) ++freq[rng[r].an];
            int32_t mode = 0;
            uint64_t best = 0;
            for (const auto &kv : freq)
                if (kv.second > best || (kv.second == best && kv.first < mode)) {
                    best = kv.second;
                    mode = kv.first;
                }
            uint64_t hit = 0, slow = 0;
            for (size_t r = r0; r < r1; ++r) {
                const RangeHot &h = rng[r];
                uint32_t info = h.info & (RH_EMIT_MASK | RH_HIT | RH_SLOW);
                if (h.an != mode || h.c < 0 || static_cast<uint32_t>(h.c) > RH8_C_MAX) info |= RH_SLOW;
                rng8[r] = RangeHot8{h.end, (info & RH_SLOW) ? info : (info | (static_cast<uint32_t>(h.c) << RH8_C_SHIFT))};
                if (info & RH_HIT) {
                    ++hit;
                    if ((info & RH_SLOW) && !(h.info & RH_SLOW)) ++slow;
                }
            }
            v.an_default = mode;
            // SBEACON_NO_RANGE8=1 keeps every VCF on RangeHot (tests cover both paths)
            const bool no8 = config().no_range8;
            v.range8 = !no8 && slow * 50 <= hit;
        }
        s.d.rng8 = dev_upload(s, rng8);
    }
    std::vector<RangeHot>().swap(rng);
    {
        std::vector<VtHot> vth(rec.size());
        std::vector<uint32_t> xvt(std::max<size_t>(x_cls.size(), 1), 0);
        for (size_t i = 0; i < rec.size(); ++i) {
            const RecHot &h = rec[i];
            const uint64_t rl = static_cast<uint64_t>(h.end) - pos[i] + 1;
            uint32_t w = 0;
            bool ok = !(h.hot & (H_AC_BAD | H_AN_BAD)) && (h.hot & H_HAS_AC) && vt_alt_word(h.hot, rl, a0_len[i], &w);
            if (ok && (h.hot & H_MULTI)) {
                const uint32_t nx = x_lo[i + 1] - x_lo[i];
                ok = nx <= VT_MAX_NX;
                for (uint32_t k = 0; ok && k < nx; ++k) {
                    const uint32_t x = x_lo[i] + k;
                    ok = vt_alt_word(x_cls[x], rl, x_len[x], &xvt[x]);
                    w |= vt_xk_bits(xvt[x]);
                }
                w |= nx << VT_NX_SHIFT;
            }
            vth[i] = VtHot{h.end, ok ? w : VT_SLOW, h.ac0, h.an};
        }
        s.d.vth = dev_upload(s, vth);
        s.d.xvt = dev_upload(s, xvt);
        // per-kind candidate lists + block tables (VcBlock)
        const size_t n = vth.size(), nblk = n / 64 + 1;
        std::vector<VcBlock> blk(kVtKinds * nblk, VcBlock{0, 0, 0});
        std::vector<VtHot> cw;
        std::vector<uint32_t> ci;
        constexpr uint32_t kXk[kVtKinds] = {VT_XK_DEL, VT_XK_INS, VT_XK_DUP, VT_XK_DUPT, VT_XK_CNV, 0u};
        for (uint32_t k = 0; k < kVtKinds; ++k) {
            const uint32_t cm = vt_class_mask(k), xk = kXk[k] | VT_XK_SYM;
            for (size_t i = 0; i < n; ++i) {
                VcBlock &b = blk[k * nblk + i / 64];
                if (i % 64 == 0) b.pre = static_cast<uint32_t>(cw.size());
                const uint32_t w = vth[i].w;
                const bool cand = (w & (VT_SLOW | VT_SYM | xk)) ||
                                  ((cm >> ((w >> VT_CLASS_SHIFT) & 31u)) & 1u);
                if (!cand) continue;
                b.mask |= 1ull << (i % 64);
                cw.push_back(vth[i]);
                ci.push_back(static_cast<uint32_t>(i));
            }
            if (n % 64 == 0) blk[k * nblk + n / 64].pre = static_cast<uint32_t>(cw.size());
        }
        if (cw.size() > 0xffffffffull) throw Error(SB_EINVAL, "variantType candidate index exceeds 2^32 entries");
        // candidate POS column + the coarse candidate index of every (segment,
        // kind) pair, aiming at ~2 candidates per bucket (chain_pack_kernel)
        std::vector<uint32_t> cpos(cw.size() + 1, 0u);
        for (size_t j = 0; j < ci.size(); ++j) cpos[j] = pos[ci[j]];
        {  // request_eval_kernel's 16-byte candidate words; staged hits carry the candidate index
            if (cw.size() > kStageCandMask) throw Error(SB_EINVAL, "variantType candidate index exceeds 2^29 entries");
            std::vector<VcQ> cq(std::max<size_t>(cw.size(), 1), VcQ{0, 0, VT_SLOW, 0});
            for (size_t j = 0; j < cw.size(); ++j) cq[j] = VcQ{cpos[j], cw[j].end, cw[j].w, cw[j].ac0};
            s.d.vc_q = dev_upload(s, cq);
        }
        // ALTs of the candidates, as a prefix (a chain's hit capacity: every
        // ALT of every candidate its coarse-index range can load)
        s.h_vc_altpre.assign(ci.size() + 1, 0);
        for (size_t j = 0; j < ci.size(); ++j) s.h_vc_altpre[j + 1] = s.h_vc_altpre[j] + 1 + (x_lo[ci[j] + 1] - x_lo[ci[j]]);
        auto cand_before = [&](uint32_t k, uint64_t r) -> uint32_t {  // global list index
            const VcBlock &b = blk[k * nblk + r / 64];
            const uint32_t o = static_cast<uint32_t>(r % 64);
            return b.pre + static_cast<uint32_t>(__builtin_popcountll(o ? (b.mask & ((1ull << o) - 1ull)) : 0ull));
        };
        std::vector<uint32_t> vcb;
        // candidates per bucket: a chain loads about this many outside its
        // window at each end (SBEACON_VC_BUCKET overrides)
        double per_bucket = 1.0;  // round 5: 2 -> 1 (request eval 69.5 -> 66.7 us: ~15 % of its loads were bucket overfetch)
        per_bucket = config().vc_bucket;
        for (auto &v : b.vcfs) {
            v.vc_index.assign(v.segments.size(), std::array<VcIndex, kVtKinds>{});
            for (size_t g = 0; g < v.segments.size(); ++g) {
                const Segment &sg = v.segments[g];
                for (uint32_t k = 0; k < kVtKinds; ++k) {
                    VcIndex &x = v.vc_index[g][k];
                    x.c_lo = cand_before(k, sg.lo);
                    x.c_hi = cand_before(k, sg.hi);
                    {  // kVcNarrow / common AN of the pair's (non-VT_SLOW) candidates
                        bool narrow = true, common = true;
                        int32_t an0 = -1;
                        for (uint32_t j = x.c_lo; j < x.c_hi && narrow; ++j) {
                            const VtHot &h = cw[j];
                            if (h.w & VT_SLOW) continue;
                            int64_t sac = h.ac0 < 0 ? -int64_t(h.ac0) : h.ac0;
                            for (uint32_t e = x_lo[ci[j]]; e < x_lo[ci[j] + 1]; ++e)
                                sac += x_ac[e] < 0 ? -int64_t(x_ac[e]) : x_ac[e];
                            narrow = h.an >= 0 && h.an < (1 << 25) && sac < (1 << 25);
                            if (an0 < 0) an0 = h.an;
                            common = common && h.an == an0;
                        }
                        x.xinfo = narrow ? kVcNarrow | (common && an0 >= 0 ? static_cast<uint32_t>(an0) + 1u : 0u) : 0u;
                    }
                    x.off = vcb.size();
                    const uint32_t nc = x.c_hi - x.c_lo;
                    if (nc == 0) {
                        x.base = 0;
                        x.shift = 31;
                        x.n = 1;
                        vcb.push_back(x.c_lo);
                        vcb.push_back(x.c_hi);
                        continue;
                    }
                    x.base = cpos[x.c_lo];
                    const uint64_t span = static_cast<uint64_t>(cpos[x.c_hi - 1]) - x.base;
                    const double gap = nc > 1 ? static_cast<double>(span) / static_cast<double>(nc - 1) : 1.0;
                    uint32_t shift = 0;
                    while (shift < 31 && static_cast<double>(1ull << (shift + 1)) <= gap * per_bucket) ++shift;
                    const uint64_t nb = (span >> shift) + 1;
                    x.shift = shift;
                    x.n = static_cast<uint32_t>(nb);
                    uint32_t j = x.c_lo;
                    for (uint64_t bb = 0; bb <= nb; ++bb) {
                        const uint64_t at = static_cast<uint64_t>(x.base) + (bb << shift);
                        while (j < x.c_hi && cpos[j] < at) ++j;
                        vcb.push_back(j);
                    }
                    vcb.back() = x.c_hi;
                }
            }
        }
        {  // the (segment, kind) indexes and the ALT prefix on the device (request_plan_kernel)
            std::vector<VcIndex> vcx;
            for (auto &v : b.vcfs) {
                v.seg_base = static_cast<uint32_t>(vcx.size() / kVtKinds);
                for (const auto &a : v.vc_index) vcx.insert(vcx.end(), a.begin(), a.end());
            }
            if (vcx.empty()) vcx.resize(kVtKinds);
            s.d.vcx = dev_upload(s, vcx);
            s.d.vc_altpre = dev_upload(s, s.h_vc_altpre);
        }
        s.h_vt_slow.clear();
        for (size_t i = 0; i < n; ++i)
            if (vth[i].w & VT_SLOW) s.h_vt_slow.push_back(static_cast<uint32_t>(i));
        s.seg_slow_pos.assign(b.vcfs.size(), {});
        for (size_t vi = 0; vi < b.vcfs.size(); ++vi) {
            const auto &segs = b.vcfs[vi].segments;
            auto &out = s.seg_slow_pos[vi];
            out.assign(segs.size(), {});
            for (size_t g = 0; g < segs.size(); ++g) {
                auto a = std::lower_bound(s.h_vt_slow.begin(), s.h_vt_slow.end(), segs[g].lo);
                for (; a != s.h_vt_slow.end() && *a < segs[g].hi; ++a) out[g].push_back(pos[*a]);
            }
        }
        cw.push_back(VtHot{0, 0, 0, 0});  // clamp target of an empty candidate range
        ci.push_back(0);
        s.d.vc_word = dev_upload(s, cw);
        s.d.vc_idx = dev_upload(s, ci);
        s.d.vc_blk = dev_upload(s, blk);
        s.d.vc_nblk = nblk;
        s.d.vc_pos = dev_upload(s, cpos);
        s.d.vc_bucket = dev_upload(s, vcb);
        s.h_vc_pos = std::move(cpos);
        s.h_vc_bucket = std::move(vcb);
    }
    s.d.pos = dev_upload(s, pos);
    s.d.ref_key = dev_upload(s, ref_key);
    s.d.a0_key = dev_upload(s, a0_key);
    s.d.a0_len = dev_upload(s, a0_len);
    s.d.x_lo = dev_upload(s, x_lo);
    s.d.ref_off = dev_upload(s, ref_off);
    s.d.a0_off = dev_upload(s, a0_off);
    s.d.fb_off = dev_upload(s, fb_off);
    {
        std::vector<XRow> xrow(x_cls.size());
        for (size_t i = 0; i < xrow.size(); ++i) xrow[i] = XRow{x_cls[i], x_ac[i]};
        s.d.xrow = dev_upload(s, xrow);
    }
    s.d.x_key = dev_upload(s, x_key);
    s.d.x_len = dev_upload(s, x_len);
    s.d.x_off = dev_upload(s, x_off);
    s.d.blob = dev_upload(s, blob);
    s.d.planes = dev_upload(s, planes);
    s.d.fb = dev_upload(s, fb);
    s.d.bucket = dev_upload(s, bucket);
    {
        std::vector<uint64_t> sum8(sum.size());
        for (size_t i = 0; i < sum.size(); ++i) sum8[i] = pack_sum(sum[i]);
        s.ds.sum8 = dev_upload(s, sum8);
    }
    s.ds.sum = dev_upload(s, sum);
    s.ds.start = dev_upload(s, start);
    s.ds.cur = dev_upload(s, cur);
    s.ds.dcount = dev_upload(s, dcount);
    s.dk.hash = dev_upload(s, dk_hash);
    {
        std::vector<KBody> body(dk_hash.size());
        std::vector<uint64_t> word(dk_hash.size());
        // every distinct tail string gets a store-wide id (kWordIdMask): the
        // window dedup then compares keys as (POS, id) words, exactly, with
        // no hash and no string confirmation (a displaced key's equal strings
        // in its window are at its own POS too: the others are deferred).  Single-base REF/ALT tails
        // c1 '_' c2 are ids c1 << 3 | c2 (< 64); the others are numbered from
        // 64 in key order; past the id space a key stays hashed (id 0)
        std::unordered_map<std::string_view, uint32_t> tail_id;
        uint32_t next_id = 64;
        for (size_t k = 0; k < body.size(); ++k) {
            const uint64_t t = dk_tail[k];
            uint32_t c0 = 0x100;  // first tail byte (none: 0x100)
            if (t & kTailBlob) {
                if ((t >> 40) & 0xffff) c0 = dk_blob[t & ((1ull << 40) - 1)];
            } else if (t >> 56) {
                c0 = static_cast<uint32_t>(t & 0xff);
            }
            const bool disp = c0 >= '0' && c0 <= '9';
            body[k] = KBody{t, dk_pos[k], disp ? kKeyDisplaced : 0u};
            uint64_t code = 0;
            if (dk_pos[k] != 0) {
                if (!(t & kTailBlob) && (t >> 56) == 3 && ((t >> 8) & 0xff) == '_' && (t & 0xff) >= 1 && (t & 0xff) <= 7 &&
                    ((t >> 16) & 0xff) >= 1 && ((t >> 16) & 0xff) <= 7) {
                    code = ((t & 0xff) << 3) | ((t >> 16) & 0xff);
                } else {
                    std::string_view sv;
                    if (t & kTailBlob)
                        sv = std::string_view(reinterpret_cast<const char *>(dk_blob.data() + (t & ((1ull << 40) - 1))),
                                              (t >> 40) & 0xffff);
                    else
                        sv = std::string_view(reinterpret_cast<const char *>(&dk_tail[k]), static_cast<size_t>(t >> 56));
                    auto it = tail_id.find(sv);
                    if (it != tail_id.end()) {
                        code = it->second;
                    } else if (next_id <= kWordIdMask) {
                        tail_id.emplace(sv, next_id);
                        code = next_id++;
                    }
                }
            }
            word[k] = dk_pos[k] | (code << 32) | (disp ? kWordDisplaced : 0ull);
        }
        s.dk.body = dev_upload(s, body);
        s.dk.word = dev_upload(s, word);
    }
    dk_blob.resize(dk_blob.size() + 16, 0);  // padding: the device compares blob tails by aligned words
    s.dk.blob = dev_upload(s, dk_blob);
    s.dk.lo = dev_upload(s, dk_lo);
    s.dk.rpos = s.d.pos;
    s.dk.bucket = s.d.bucket;
    s.n_keys = dk_hash.size();
    if (s.stream) HIP_OK(hipStreamSynchronize(s.stream));
    s.h_dk_pos = std::move(dk_pos);
    s.h_dk_lo = std::move(dk_lo);
    s.h_dk_bad = std::move(dk_bad);
    s.h_dk_tail = std::move(dk_tail);
    s.h_dk_blob = std::move(dk_blob);
    s.h_start = std::move(start);
    s.h_rem.resize(sum.size());
    s.h_sum_bad.resize(sum.size());
    for (size_t i = 0; i < sum.size(); ++i) {
        s.h_rem[i] = sum[i].rem;
        s.h_sum_bad[i] = (sum[i].nvf & kSumUnsupported) ? 1 : 0;
    }
    s.h_cur = std::move(cur);
    s.h_dcount = std::move(dcount);
    // host copies for output planning and result formatting
    s.h_pos = std::move(pos);
    s.h_end.resize(rec.size());
    for (size_t i = 0; i < rec.size(); ++i) s.h_end[i] = rec[i].end;
    s.h_a0_len = std::move(a0_len);
    s.h_x_lo = std::move(x_lo);
    s.h_x_len = std::move(x_len);
    s.h_bucket = std::move(bucket);
    s.h_vt = std::move(vt);
    s.h_ref_off = std::move(ref_off);
    s.h_a0_off = std::move(a0_off);
    s.h_x_off = std::move(x_off);
    s.h_blob = std::move(blob);
}

const char *kRegexMeta = "^$*+?{}[]\\|()";

// coarse bracket used to plan the output region: first record of the bucket
// holding x (<= the exact lower bound) / end of that bucket (>= it)
uint32_t bucket_floor(const sb_store &s, const QDev &d, int64_t x) {
    if (x <= static_cast<int64_t>(d.bucket_base)) return d.seg_lo;
    const uint64_t b = static_cast<uint64_t>(x - d.bucket_base) >> d.bucket_shift;
    if (b >= d.n_buckets) return d.seg_hi;
    return s.h_bucket[d.bucket_off + b];
}
uint32_t bucket_ceil(const sb_store &s, const QDev &d, int64_t x) {
    if (x <= static_cast<int64_t>(d.bucket_base)) return d.seg_lo;
    const uint64_t b = static_cast<uint64_t>(x - d.bucket_base) >> d.bucket_shift;
    if (b >= d.n_buckets) return d.seg_hi;
    return s.h_bucket[d.bucket_off + b + 1];
}

// A persistent host worker pool (planning runs once per call: spawning
// threads per call cost a few hundred microseconds).  run(n, fn) calls fn(i)
// for i < n on the pool and the calling thread; one run at a time (try_run:
// parallel_for falls back to its own threads when the pool is taken).
class WorkerPool {
  public:
    static WorkerPool &get() {
        static WorkerPool pool(std::max(1u, std::min(16u, std::thread::hardware_concurrency())) - 1);
        return pool;
    }
    // a second, smaller pool for a concurrent caller (two pipelined
    // preparers): spawning threads per call costs more than the work
    static WorkerPool &second() {
        static WorkerPool pool(std::max(1u, std::min(8u, std::thread::hardware_concurrency() / 2)) - 1);
        return pool;
    }
    template <class F>
    void run(size_t n, F fn) {
        std::unique_lock<std::mutex> one(run_mu_);
        run_locked(n, fn);
    }
    // the same, or false at once when another run holds the pool (a
    // concurrent caller, or a call from inside a task)
    template <class F>
    bool try_run(size_t n, F fn) {
        std::unique_lock<std::mutex> one(run_mu_, std::try_to_lock);
        if (!one.owns_lock()) return false;
        run_locked(n, fn);
        return true;
    }

  private:
    template <class F>
    void run_locked(size_t n, F fn) {
        std::function<void(size_t)> f = fn;
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &f;
            n_ = n;
            next_ = 0;
            busy_ = workers_.size();
            ++gen_;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return busy_ == 0; });
        fn_ = nullptr;
    }

  public:
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
            ++gen_;
        }
        cv_.notify_all();
        for (auto &t : workers_) t.join();
    }

  private:
    explicit WorkerPool(unsigned k) {
        for (unsigned i = 0; i < k; ++i) workers_.emplace_back([this] { loop(); });
    }
    void drain() {
        for (size_t i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            drain();
            std::lock_guard<std::mutex> lk(mu_);
            if (--busy_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_, run_mu_;
    std::condition_variable cv_, done_;
    std::function<void(size_t)> *fn_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    size_t busy_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

// run fn(i) for i in [0, n) on up to `threads` host threads (the worker
// pool's when it is free)
template <class F>
void parallel_for(size_t n, F fn, unsigned threads = 16, size_t grain = 4096) {
    const unsigned t = static_cast<unsigned>(std::min<size_t>(threads, std::max<size_t>(1, n / grain)));
    if (t <= 1) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    auto part = [&](size_t k) {
        for (size_t i = n * k / t, e = n * (k + 1) / t; i < e; ++i) fn(i);
    };
    if (WorkerPool::get().try_run(t, part) || WorkerPool::second().try_run(t, part)) return;
    std::vector<std::thread> th;
    for (unsigned k = 0; k < t; ++k)
        th.emplace_back([&, k] {
            for (size_t i = n * k / t, e = n * (k + 1) / t; i < e; ++i) fn(i);
        });
    for (auto &x : th) x.join();
}

}  // namespace

namespace sb {
// n tasks on the persistent worker pool (own threads when it is taken):
// the wire formatter's phases (csrc/wire.cpp)
void run_tasks(size_t n, const std::function<void(size_t)> &fn) {
    if (n <= 1) {
        for (size_t i = 0; i < n; ++i) fn(i);
        return;
    }
    if (WorkerPool::get().try_run(n, [&](size_t k) { fn(k); })) return;
    std::vector<std::thread> th;
    for (size_t k = 0; k < n; ++k) th.emplace_back([&, k] { fn(k); });
    for (auto &x : th) x.join();
}
}  // namespace sb

namespace {

// Chains of consecutive variantType slices (devtypes.hpp ChainDev).  vt =
// the MODE_VTYPE queries in input order; returns those left to vt_slice.
// Slices chain when they share the VCF segment and every filter, each starts
// one base past the previous one, the chain's first slice sets the width and
// only its last may be shorter (splitQuery's [a, min(a + 9999, start_max)]),
// interleaved with other VCFs' slices or not; a slice qualifies only without
// order-dependent semantics (include_details, no boolean break, a VCF without
// negative AC) and a chain is dissolved when a VT_SLOW record lies in its window.
std::vector<uint32_t> plan_chains(sb_batch &B, const std::vector<uint32_t> &segi, const std::vector<uint32_t> &vt) {
    sb_store &s = *B.s;
    std::vector<uint32_t> rest;
    if (config().no_chains || B.no_chains) return vt;
    struct Ch {
        std::vector<uint32_t> m;
        int64_t first = 0, last = 0, width = 0;
    };
    std::vector<Ch> ch;
    std::unordered_map<std::string, uint32_t> open;  // filter signature + next first_bp -> chain
    auto key = [&](const QDev &d, uint32_t i, int64_t next) {  // field bytes only (no struct padding)
        std::string k;
        k.reserve(60);
        auto put = [&](const auto &v) { k.append(reinterpret_cast<const char *>(&v), sizeof v); };
        put(B.vcf[i]);
        put(d.seg_lo);
        put(d.end_min);
        put(d.end_max);
        put(d.vmin);
        put(d.vmax);
        put(next);
        put(d.vt_kind);
        put(d.lut_off);
        put(d.flags);
        return k;
    };
    for (uint32_t i : vt) {
        const QDev &d = B.hq[i];
        const bool ok = (d.flags & F_DETAILS) && (d.flags & F_NONNEG) &&
                        !(d.flags & (F_BOOL_BREAK | F_EMPTY | F_STRICT_UNBOUND | F_SAMPLES_VARIANT)) &&
                        d.samples_out_off == ~0ull && segi[i] != UINT32_MAX && d.first_bp >= 0 &&
                        d.first_bp <= d.last_bp && d.last_bp <= 0xfffffffell;
        if (!ok) {
            rest.push_back(i);
            continue;
        }
        const int64_t w = d.last_bp - d.first_bp + 1;
        uint32_t c = UINT32_MAX;
        auto it = open.find(key(d, i, d.first_bp));
        if (it != open.end()) {
            c = it->second;
            open.erase(it);
            if (w > ch[c].width) c = UINT32_MAX;  // wider than the chain's slices: a new chain
        }
        if (c == UINT32_MAX) {
            c = static_cast<uint32_t>(ch.size());
            ch.push_back(Ch{{}, d.first_bp, d.last_bp, w});
        }
        ch[c].m.push_back(i);
        ch[c].last = d.last_bp;
        if (w == ch[c].width && ch[c].m.size() < kChainMax) open[key(d, i, d.last_bp + 1)] = c;
    }
    // exact record range of every chained slice (n_scanned) and the VT_SLOW check
    B.chained.assign(B.nq, 0);
    B.nscan.assign(B.nq, 0);
    std::vector<uint8_t> dissolve(ch.size(), 0);
    parallel_for(ch.size(), [&](size_t c) {
        const Ch &x = ch[c];
        const QDev &d0 = B.hq[x.m[0]];
        auto pb = s.h_pos.begin();
        auto lb = [&](int64_t p) {
            return static_cast<uint32_t>(std::lower_bound(pb + d0.seg_lo, pb + d0.seg_hi, static_cast<uint64_t>(p),
                                                          [](uint32_t a, uint64_t b) { return a < b; }) - pb);
        };
        const uint32_t lo = lb(x.first), hi = lb(x.last + 1);
        auto sl = std::lower_bound(s.h_vt_slow.begin(), s.h_vt_slow.end(), lo);
        if (sl != s.h_vt_slow.end() && *sl < hi) {
            dissolve[c] = 1;
            return;
        }
        uint32_t a = lo;
        for (uint32_t i : x.m) {
            const uint32_t e = lb(B.hq[i].last_bp + 1);
            B.nscan[i] = e - a;
            a = e;
        }
    });
    // chains in (segment, first base) order; ChainDev.q0 is set at upload
    std::vector<uint32_t> order;
    for (uint32_t c = 0; c < ch.size(); ++c) {
        if (dissolve[c])
            rest.insert(rest.end(), ch[c].m.begin(), ch[c].m.end());
        else
            order.push_back(c);
    }
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        const QDev &x = B.hq[ch[a].m[0]], &y = B.hq[ch[b].m[0]];
        return x.seg_lo != y.seg_lo ? x.seg_lo < y.seg_lo : ch[a].first < ch[b].first;
    });
    B.hchains.clear();
    B.chain_members.clear();
    for (uint32_t c : order) {
        const Ch &x = ch[c];
        const uint32_t i0 = x.m[0];
        const QDev &d = B.hq[i0];
        const VcIndex &vi = s.vcfs[B.vcf[i0]].vc_index[segi[i0]][d.vt_kind];
        ChainDev cd{};
        cd.s0 = static_cast<uint32_t>(B.chain_members.size());
        cd.n = static_cast<uint32_t>(x.m.size());
        cd.first = static_cast<uint32_t>(x.first);
        cd.last = static_cast<uint32_t>(x.last);
        cd.width = static_cast<uint32_t>(x.width);
        cd.c_lo = vi.c_lo;
        cd.c_hi = vi.c_hi;
        cd.cb_base = vi.base;
        cd.cb_off = vi.off;
        cd.cb_shift = vi.shift;
        cd.cb_n = vi.n;
        // VtPred's compare constants (query_kernels.hip), from the chain's common filters
        const bool end_void = d.end_max < 0 || d.end_min > 0xffffffffll || d.end_min > d.end_max;
        cd.e0 = d.end_min < 0 ? 0u : static_cast<uint32_t>(d.end_min);
        cd.espan = (d.end_max > 0xffffffffll ? 0xffffffffu : static_cast<uint32_t>(d.end_max)) - cd.e0;
        const int64_t vl = d.vmin < 0 ? 0 : d.vmin, vh = d.vmax > 255 ? 255 : d.vmax;
        cd.vlo = vh < vl ? 256u : static_cast<uint32_t>(vl);
        cd.vspan = vh < vl ? 0u : static_cast<uint32_t>(vh - vl);
        cd.kind = d.vt_kind | (end_void ? kChainEndVoid : 0u);
        cd.lut_off = d.lut_off;
        cd.out = 0;  // set with the hit regions
        B.hchains.push_back(cd);
        for (uint32_t i : x.m) {
            B.chained[i] = 1;
            B.chain_members.push_back(i);
        }
    }
    // candidate statistics (roofline pricing of the chain kernel): the
    // coarse-index superset each chain loads, its exact window, and the union
    // of the windows (the candidates a step must bring in at least once)
    std::vector<std::pair<uint32_t, uint32_t>> win(B.hchains.size());
    std::vector<uint64_t> loaded(B.hchains.size());
    B.chain_cap.assign(B.hchains.size(), 0);
    parallel_for(B.hchains.size(), [&](size_t c) {
        const ChainDev &d = B.hchains[c];
        auto cb = [&](uint64_t x, uint32_t up) -> uint32_t {
            if (x <= d.cb_base) return d.c_lo;
            const uint64_t b = (x - d.cb_base) >> d.cb_shift;
            return b >= d.cb_n ? d.c_hi : s.h_vc_bucket[d.cb_off + b + up];
        };
        const uint32_t C0 = cb(d.first, 0), C1 = (d.kind & kChainEndVoid) ? C0 : std::max(C0, cb(uint64_t(d.last) + 1, 1));
        loaded[c] = C1 - C0;
        B.chain_cap[c] = s.h_vc_altpre[C1] - s.h_vc_altpre[C0];
        auto pb = s.h_vc_pos.begin();
        const uint32_t a = static_cast<uint32_t>(std::lower_bound(pb + d.c_lo, pb + d.c_hi, d.first) - pb);
        const uint32_t e = static_cast<uint32_t>(std::upper_bound(pb + d.c_lo, pb + d.c_hi, d.last) - pb);
        win[c] = {a, std::max(a, e)};
    });
    B.cand_loaded = B.cand_window = B.cand_unique = 0;
    for (size_t c = 0; c < win.size(); ++c) {
        B.cand_loaded += loaded[c];
        B.cand_window += win[c].second - win[c].first;
    }
    std::sort(win.begin(), win.end());
    uint64_t reach = 0;
    for (const auto &w : win) {  // kinds' lists are disjoint ranges of one index space
        const uint64_t a = std::max<uint64_t>(w.first, reach);
        if (w.second > a) B.cand_unique += w.second - a;
        reach = std::max<uint64_t>(reach, w.second);
    }
    std::sort(rest.begin(), rest.end());
    return rest;
}

void prepare(sb_batch &B, const sb_query *qs, size_t nq) {
    sb_store &s = *B.s;
    if (nq >= (1u << 31)) throw Error(SB_EINVAL, "batch too large");
    static const bool trace = config().wire_trace;  // phase times (bench diagnostics)
    auto t_last = std::chrono::steady_clock::now();
    auto tick = [&](const char *what) {
        if (!trace) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[prepare] %-8s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    B.nq = static_cast<uint32_t>(nq);
    std::vector<uint32_t> segi(nq, UINT32_MAX);  // segment index of each query in its VCF
    std::vector<uint64_t> cap(nq, 0);           // hit-region capacity of each query
    B.hq.assign(nq, QDev{});
    B.host_err.assign(nq, 0);
    B.chrom.assign(nq, std::string());
    B.emitted.assign(nq, std::vector<uint32_t>());
    struct SubsetEntry {
        uint64_t off = 0;
        bool empty = false;
        std::vector<uint32_t> emitted;
    };
    std::unordered_map<std::string, SubsetEntry> subset_cache;
    B.samples_variant.assign(nq, 0);
    B.vcf.assign(nq, 0);
    std::vector<uint8_t> qbytes;
    std::vector<uint64_t> subsets;
    std::vector<uint32_t> lut_all;
    std::unordered_map<std::string, uint32_t> lut_cache;
    uint64_t samples_words = 0;
    for (size_t i = 0; i < nq; ++i) {  // what raises for the whole batch, first
        if (qs[i].vcf_id >= s.vcfs.size()) throw Error(SB_ENOSTORE, "query " + std::to_string(i) + ": unknown vcf id");
        if (!qs[i].region) throw Error(SB_EINVAL, "query " + std::to_string(i) + ": region is NULL");
    }
    // per query, in parallel: region, segment, bounds, predicates (no shared state)
    parallel_for(nq, [&](size_t i) {
        const sb_query &x = qs[i];
        QDev &d = B.hq[i];
        d.subset_off = ~0ull;
        d.samples_out_off = ~0ull;
        const VcfData &v = s.vcfs[x.vcf_id];
        B.vcf[i] = x.vcf_id;
        const ParsedRegion rg = parse_region(x.region, x.region_len);
        B.chrom[i] = rg.chrom;
        if (!rg.ok) {
            B.host_err[i] = SB_QERR_VALUE;  // int() of the region bounds (:56-57)
            d.flags |= F_EMPTY;
        }
        d.first_bp = rg.first;
        d.last_bp = rg.last;
        auto it = v.seg_index.find(rg.chrom);
        if (it == v.seg_index.end()) {
            d.flags |= F_EMPTY;
        } else {
            const Segment &sg = v.segments[it->second];
            const BucketIndex &bi = v.buckets[it->second];
            segi[i] = it->second;
            d.seg_lo = sg.lo;
            d.seg_hi = sg.hi;
            d.bucket_off = bi.off;
            d.bucket_base = bi.base;
            d.bucket_shift = bi.shift;
            d.n_buckets = bi.n;
        }
        d.end_min = x.end_min;
        d.end_max = x.end_max;
        const bool samples_variant = x.selected_samples_only != 0;
        B.samples_variant[i] = samples_variant;
        d.words = v.words;
        d.n_samples = static_cast<uint32_t>(v.samples.size());
        d.rec_base = v.rec_base;
        d.x_base = v.x_base;
        d.an_default = v.an_default;
        d.plane0_base = v.plane0_base;
        d.planex_base = v.planex_base;
        if (v.nonneg) d.flags |= F_NONNEG;
        // REF predicate (:59, :94 / svs:87-91)
        if (!x.reference_bases) {
            if (samples_variant) {
                d.ref_mode = REF_ERROR;
                d.ref_err = SB_QERR_ATTRIBUTE;
            } else {
                d.ref_mode = REF_NEVER;
            }
        } else {
            const char *rb = x.reference_bases;
            const size_t rn = x.reference_len;
            d.ref_len = static_cast<uint32_t>(rn);
            auto has_any = [&](const char *set) {
                for (size_t k = 0; k < rn; ++k)
                    if (std::strchr(set, rb[k]) && rb[k]) return true;
                return false;
            };
            if (rn == 1 && rb[0] == 'N') {
                d.ref_mode = REF_ANY;
            } else if (samples_variant && has_any(kRegexMeta)) {
                d.ref_mode = REF_ERROR;
                d.ref_err = SB_QERR_UNSUPPORTED;
            } else if (samples_variant && has_any("N.")) {
                d.ref_mode = REF_WILD;
            } else {
                d.ref_mode = REF_EXACT;
                bool h;
                d.ref_key = allele_key(reinterpret_cast<const uint8_t *>(rb), rn, false, &h);
            }
        }
        // ALT predicate (:100-183)
        if (!x.alternate_bases) {
            d.alt_mode = ALT_VTYPE;
            if (x.strict_variant_type) d.flags |= F_STRICT_UNBOUND;
            const std::string_view vt = x.variant_type ? std::string_view(x.variant_type, x.variant_type_len)
                                                       : std::string_view("None");
            const bool has = x.variant_type != nullptr;
            d.vt_kind = !has                 ? VT_OTHER
                        : vt == "DEL"        ? VT_DEL
                        : vt == "INS"        ? VT_INS
                        : vt == "DUP"        ? VT_DUP
                        : vt == "DUP:TANDEM" ? VT_DUPT
                        : vt == "CNV"        ? VT_CNV
                                             : VT_OTHER;
        } else {
            const char *ab = x.alternate_bases;
            const size_t an = x.alternate_len;
            d.alt_len = static_cast<uint32_t>(an);
            if (an == 1 && ab[0] == 'N') {
                d.alt_mode = ALT_N;
            } else {
                d.alt_mode = ALT_EXACT;
                bool h;
                d.alt_key = allele_key(reinterpret_cast<const uint8_t *>(ab), an, false, &h);
            }
        }
        d.vmin = x.variant_min_length;
        d.vmax = x.variant_max_length < 0 ? INT64_MAX : x.variant_max_length;
        if (x.include_details) d.flags |= F_DETAILS;
        if (samples_variant) d.flags |= F_SAMPLES_VARIANT;
        if (x.granularity == SB_GRAN_BOOLEAN && !samples_variant) d.flags |= F_BOOL_BREAK;
        // output region: every ALT row of the records in the coarse bracket
        // (offsets assigned below, once the chains are known)
        if (!(d.flags & F_EMPTY) && d.first_bp <= d.last_bp) {
            const uint32_t lo = bucket_floor(s, d, d.first_bp);
            const uint32_t hi = std::max(lo, bucket_ceil(s, d, d.last_bp + 1));
            cap[i] = static_cast<uint64_t>(hi - lo) + (s.h_x_lo[hi] - s.h_x_lo[lo]);
        }
    }, 16, 1024);
    // in batch order: the shared tables (sample subsets, predicate bytes,
    // variantType LUTs, sample output words)
    const char *last_vt = nullptr;
    size_t last_vt_len = 0;
    uint32_t last_vt_kind = ~0u, last_lut = 0;
    for (size_t i = 0; i < nq; ++i) {
        const sb_query &x = qs[i];
        QDev &d = B.hq[i];
        const VcfData &v = s.vcfs[x.vcf_id];
        const bool samples_variant = B.samples_variant[i] != 0;
        const uint32_t n_samples = d.n_samples;
        if (samples_variant) {  // bcftools --samples (svs:36-42), header order
            const std::string names = x.sample_names ? std::string(x.sample_names, x.sample_names_len) : std::string("_");
            // requests of one batch often share a sampleNames list: one mask each
            const std::string ck = std::to_string(x.vcf_id) + '\n' + names;
            auto hit = subset_cache.find(ck);
            if (hit == subset_cache.end()) {
                std::vector<uint8_t> sel(n_samples, 0);
                bool empty = false;
                size_t p = 0;
                for (;;) {
                    const size_t c = names.find(',', p);
                    const std::string nm = names.substr(p, c == std::string::npos ? std::string::npos : c - p);
                    auto f = v.sample_pos.find(nm);
                    if (f == v.sample_pos.end()) empty = true;  // unknown sample: bcftools exits, no output
                    else
                        for (uint32_t k : f->second) sel[k] = 1;
                    if (c == std::string::npos) break;
                    p = c + 1;
                }
                SubsetEntry e;
                e.off = subsets.size();
                e.empty = empty;
                subsets.resize(subsets.size() + std::max(1u, v.words), 0ull);
                for (uint32_t k = 0; k < n_samples; ++k)
                    if (sel[k]) {
                        e.emitted.push_back(k);
                        subsets[e.off + (k >> 6)] |= 1ull << (k & 63);
                    }
                hit = subset_cache.emplace(ck, std::move(e)).first;
            }
            if (hit->second.empty) d.flags |= F_EMPTY;
            d.subset_off = hit->second.off;
            B.emitted[i] = hit->second.emitted;
        }
        d.qbytes_off = static_cast<uint32_t>(qbytes.size());
        if (x.reference_bases) qbytes.insert(qbytes.end(), x.reference_bases, x.reference_bases + x.reference_len);
        if (!x.alternate_bases) {
            const char *vt = x.variant_type ? x.variant_type : "None";
            const size_t vl = x.variant_type ? x.variant_type_len : 4;
            if (!(d.vt_kind == last_vt_kind && vl == last_vt_len && last_vt &&
                  (vt == last_vt || std::memcmp(vt, last_vt, vl) == 0))) {  // a new (kind, variantType) pair
                const std::string key = std::to_string(d.vt_kind) + "|" + std::string(vt, vl);
                auto lt = lut_cache.find(key);
                if (lt == lut_cache.end()) {
                    const auto lut = sym_lut(s, d.vt_kind, "<" + std::string(vt, vl));
                    const uint32_t off = static_cast<uint32_t>(lut_all.size());
                    lut_all.insert(lut_all.end(), lut.begin(), lut.end());
                    lt = lut_cache.emplace(key, off).first;
                }
                last_vt = vt;
                last_vt_len = vl;
                last_vt_kind = d.vt_kind;
                last_lut = lt->second;
            }
            d.lut_off = last_lut;
        } else {
            qbytes.insert(qbytes.end(), x.alternate_bases, x.alternate_bases + x.alternate_len);
        }
        const bool collect = (x.granularity == SB_GRAN_RECORD || x.granularity == SB_GRAN_AGGREGATED) &&
                             (samples_variant || x.include_samples);
        if (collect) {
            d.flags |= F_COLLECT;
            if (x.include_details && v.words) {
                if (!v.has_planes) throw Error(SB_EINVAL, "sample path requested but the store was built without genotypes");
                d.samples_out_off = samples_words;
                samples_words += v.words;
            }
        }
    }
    B.samples_words = samples_words;
    tick("queries");
    {
        // collect -> general kernel with the sample path; otherwise the
        // narrowest specialisation whose predicates cover the query
        B.groups.clear();
        // groups 0..4 = MODE_GENERAL/RANGE_N/EXACT/VTYPE/RANGE_N8 without the
        // sample path; group 5 = MODE_GENERAL with the sample planes compiled in
        constexpr int kCollect = 5;
        for (int g = 0; g <= kCollect; ++g)
            B.groups.push_back(sb_batch::Group{g == kCollect ? MODE_GENERAL : g, g == kCollect ? s.max_words : 0u, {}, 0});
        for (uint32_t i = 0; i < B.nq; ++i) {
            const QDev &d = B.hq[i];
            if (!(d.flags & F_NONNEG)) B.nonneg = false;
            int g;
            if (d.samples_out_off != ~0ull) {
                g = kCollect;
            } else if (d.flags & (F_STRICT_UNBOUND | F_SAMPLES_VARIANT)) {
                g = MODE_GENERAL;
            } else if (d.ref_mode == REF_ANY && d.alt_mode == ALT_N) {
                g = s.vcfs[B.vcf[i]].range8 ? MODE_RANGE_N8 : MODE_RANGE_N;
            } else if (d.ref_mode == REF_EXACT && d.alt_mode == ALT_EXACT) {
                g = MODE_EXACT;
            } else if (d.ref_mode == REF_ANY && d.alt_mode == ALT_VTYPE) {
                g = MODE_VTYPE;
            } else {
                g = MODE_GENERAL;
            }
            B.groups[static_cast<size_t>(g)].idx.push_back(i);
        }
        {  // variantType slices of one request -> chains (chain_kernel); the rest stay with vt_slice
            auto &vg = B.groups[MODE_VTYPE].idx;
            vg = plan_chains(B, segi, vg);
        }
        tick("chains");
        std::vector<sb_batch::Group> keep;
        for (auto &g : B.groups)
            if (!g.idx.empty()) keep.push_back(std::move(g));
        B.groups = std::move(keep);
        // launch order = (segment, first base): neighbouring waves scan
        // neighbouring records (with the kernels' XCD-aware block order,
        // one XCD's L2 serves a contiguous stretch of the store).  Sorted as
        // packed (segment, first base, position) words: the same order as a
        // stable sort on (seg_lo, first_bp)
        for (auto &g : B.groups) {
            const size_t m = g.idx.size();
            bool packable = true;
            for (uint32_t i : g.idx) {
                const QDev &x = B.hq[i];
                packable = packable && x.first_bp >= 0 && x.first_bp < (int64_t(1) << 32);
            }
            if (!packable || m >= (size_t(1) << 31)) {
                std::stable_sort(g.idx.begin(), g.idx.end(), [&](uint32_t a, uint32_t b) {
                    const QDev &x = B.hq[a], &y = B.hq[b];
                    return x.seg_lo != y.seg_lo ? x.seg_lo < y.seg_lo : x.first_bp < y.first_bp;
                });
                continue;
            }
            // (seg_lo, first_bp) words; a stable LSD radix sort over their
            // used bits (11-bit digits) keeps equal words in input order --
            // std::sort of the (word, position) pairs took ~2 ms for 32 k
            // slices; already ordered input (slices of sorted requests) is
            // detected and left alone
            std::vector<uint64_t> key(m);
            uint64_t any = 0;
            bool sorted = true;
            for (size_t k = 0; k < m; ++k) {
                const QDev &x = B.hq[g.idx[k]];
                key[k] = static_cast<uint64_t>(x.seg_lo) << 32 | static_cast<uint64_t>(x.first_bp);
                any |= key[k];
                sorted = sorted && (k == 0 || key[k - 1] <= key[k]);
            }
            if (sorted) continue;
            std::vector<uint64_t> key2(m);
            std::vector<uint32_t> idx2(m);
            std::vector<uint32_t> &idx = g.idx;
            const int bits = 64 - __builtin_clzll(any | 1);
            for (int sh = 0; sh < bits; sh += 11) {
                uint32_t cnt[2049] = {0};
                for (size_t k = 0; k < m; ++k) ++cnt[((key[k] >> sh) & 2047u) + 1];
                for (int d = 0; d < 2048; ++d) cnt[d + 1] += cnt[d];
                for (size_t k = 0; k < m; ++k) {
                    const uint32_t at = cnt[(key[k] >> sh) & 2047u]++;
                    key2[at] = key[k];
                    idx2[at] = idx[k];
                }
                key.swap(key2);
                idx.swap(idx2);
            }
        }
    }
    tick("groups");
    {  // hit regions: unchained queries in batch order, then each chain's slices
        // back to back (a chain writes its hits densely from its first slot)
        uint64_t at = 0;
        for (uint32_t i = 0; i < nq; ++i)
            if (B.chained.empty() || !B.chained[i]) {
                B.hq[i].hit_off = at;
                at += cap[i];
            }
        size_t m = 0;
        for (size_t k = 0; k < B.hchains.size(); ++k) {
            ChainDev &c = B.hchains[k];
            c.out = at;
            for (uint32_t j = 0; j < c.n; ++j, ++m) B.hq[B.chain_members[m]].hit_off = at;
            at += B.chain_cap[k];
        }
        B.cap_total = at;
    }
    // 8 words of slack: vt_kernel reads words 0..7 of its LUT unconditionally
    // (packed symbolic ids are < 255; words past a LUT's end are never consulted)
    lut_all.insert(lut_all.end(), 8, 0u);
    // ---- device buffers
    if (s.device < 0) return;  // a host-only store: the plan stays on the host
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    if (!B.pool) B.pool = req_pool(s);
    // device query array in launch order (groups back to back, each sorted by
    // segment and first base): a wave reads its query at qs + w, with no index
    // load in front; QDev::orig names the QRes row
    std::vector<QDev> lq;
    lq.reserve(nq);
    for (uint32_t i = 0; i < nq; ++i) B.hq[i].orig = i;
    for (auto &g : B.groups) {
        g.base = static_cast<uint32_t>(lq.size());
        for (uint32_t i : g.idx) lq.push_back(B.hq[i]);
    }
    B.chain_base = static_cast<uint32_t>(lq.size());
    for (uint32_t i : B.chain_members) lq.push_back(B.hq[i]);
    // chain runs: consecutive chains, at most pack_run_max() per wave and
    // pack_slots_max() slices (the wave's LDS slots)
    B.hruns.clear();
    {
        uint32_t slots = 0, cnt = 0, run_max = pack_run_max();
        if (const int k = config().pack_run)  // A/B: shorter runs
            run_max = std::max(1u, std::min(run_max, static_cast<uint32_t>(k)));
        for (uint32_t c = 0; c < B.hchains.size(); ++c) {
            const uint32_t n = B.hchains[c].n;
            if (cnt == 0 || cnt == run_max || slots + n > pack_slots_max()) {
                B.hruns.push_back(c);
                slots = 0;
                cnt = 0;
            }
            slots += n;
            ++cnt;
        }
        B.hruns.push_back(static_cast<uint32_t>(B.hchains.size()));
    }
    palloc(B, B.runs, B.hruns.size() * 4);
    HIP_OK(hipMemcpyAsync(B.runs.p, B.hruns.data(), B.hruns.size() * 4, hipMemcpyHostToDevice, st));
    palloc(B, B.chains, B.hchains.size() * sizeof(ChainDev));
    palloc(B, B.corig, B.chain_members.size() * 4);
    palloc(B, B.cpart, B.hchains.size() * sizeof(ReqPartial));
    if (!B.hchains.empty()) {
        HIP_OK(hipMemcpyAsync(B.chains.p, B.hchains.data(), B.hchains.size() * sizeof(ChainDev), hipMemcpyHostToDevice,
                              st));
        HIP_OK(hipMemcpyAsync(B.corig.p, B.chain_members.data(), B.chain_members.size() * 4, hipMemcpyHostToDevice,
                              st));
    }
    std::vector<uint64_t> hoff(nq);
    for (uint32_t i = 0; i < nq; ++i) hoff[i] = B.hq[i].hit_off;
    palloc(B, B.q, nq * sizeof(QDev));
    palloc(B, B.hoff, nq * 8);
    palloc(B, B.qbytes, qbytes.size());
    palloc(B, B.subsets, subsets.size() * 8);
    palloc(B, B.lut, lut_all.size() * 4);
    if (nq) HIP_OK(hipMemcpyAsync(B.q.p, lq.data(), nq * sizeof(QDev), hipMemcpyHostToDevice, st));
    if (nq) HIP_OK(hipMemcpyAsync(B.hoff.p, hoff.data(), nq * 8, hipMemcpyHostToDevice, st));
    if (!B.hchains.empty()) {
        palloc(B, B.srcoff, nq * 8);
        HIP_OK(hipMemcpyAsync(B.srcoff.p, hoff.data(), nq * 8, hipMemcpyHostToDevice, st));
    }
    if (!qbytes.empty()) HIP_OK(hipMemcpyAsync(B.qbytes.p, qbytes.data(), qbytes.size(), hipMemcpyHostToDevice, st));
    if (!subsets.empty()) HIP_OK(hipMemcpyAsync(B.subsets.p, subsets.data(), subsets.size() * 8, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(B.lut.p, lut_all.data(), lut_all.size() * 4, hipMemcpyHostToDevice, st));

    palloc(B, B.res, size_t(nq) * sizeof(QRes));
    palloc(B, B.hits, B.cap_total * 8);
    palloc(B, B.samples_out, samples_words * 8);
    if (s.g.n && nq) {  // general records: work list + scratch (general_slice_kernel)
        uint32_t hw, tc;
        const uint64_t wb = general_wave_bytes(s.g, &hw, &tc);
        const uint64_t budget = uint64_t(256) << 20;
        B.gen_grid = static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>({nq, 1024, budget / wb})));
        palloc(B, B.gen_work, (size_t(nq) + 1) * 4);
        palloc(B, B.gen_scratch, size_t(B.gen_grid) * wb);
        B.gen_big_cap = std::min<uint32_t>(nq, 4096);
        palloc(B, B.gen_big_n, 4);
        palloc(B, B.gen_big, size_t(B.gen_big_cap) * sizeof(GenBig));
        palloc(B, B.gen_limbs, size_t(B.gen_big_cap) * 2 * kGenAccMax * 4);
    }
    tick("buffers");
    HIP_OK(hipStreamSynchronize(st));
    tick("upload");
}

// timing: one event before the first run since the last sync and one at the
// sync (sync()); no marker between back-to-back runs (a marker pair per run
// measured ~8 us of stream gap per run on MI355X)
void mark_run(sb_batch &B) {
    if (!B.ev[0]) {
        for (auto &e : B.ev) HIP_OK(hipEventCreate(&e));
    }
    if (B.runs_pending++ == 0) HIP_OK(hipEventRecord(B.ev[0], B.strm()));
}

void run_kernels(sb_batch &B);

void run(sb_batch &B) {
    HIP_OK(hipSetDevice(B.s->device));
    mark_run(B);
    run_kernels(B);
}

void run_kernels(sb_batch &B) {
    sb_store &s = *B.s;
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = B.strm();
    DStore d = s.d;
    d.sym_lut = B.lut.as<uint32_t>();
    d.q_all = B.q.as<QDev>();
    d.gen_work = B.gen_grid ? B.gen_work.as<uint32_t>() : nullptr;
    if (B.gen_grid) {
        HIP_OK(hipMemsetAsync(B.gen_work.p, 0, 4, st));
        HIP_OK(hipMemsetAsync(B.gen_big_n.p, 0, 4, st));
    }
    // chains of variantType slices (one wave per request's slices)
    launch_chains(d, B.chains.as<ChainDev>(), static_cast<uint32_t>(B.hchains.size()), B.runs.as<uint32_t>(),
                  static_cast<uint32_t>(B.hruns.size() - 1), B.corig.as<uint32_t>(),
                  B.slice_rows ? B.res.as<QRes>() : nullptr, B.hits.as<uint64_t>(), B.cpart.as<ReqPartial>(), st);
    B.slice_rows_stale = !B.slice_rows && !B.hchains.empty();
    // sample-free groups: one fused launch, long scans first (range, variantType,
    // general) and point lookups last, so the short waves fill the tail
    std::vector<FusedGroup> fg;
    for (int mode : {MODE_RANGE_N8, MODE_RANGE_N, MODE_VTYPE, MODE_GENERAL, MODE_EXACT})
        for (const auto &g : B.groups)
            if (g.max_words == 0 && g.mode == mode)
                fg.push_back(FusedGroup{B.q.as<QDev>() + g.base, static_cast<uint32_t>(g.idx.size()), g.mode});
    launch_fused(d, fg.data(), static_cast<int>(fg.size()), B.nonneg, B.qbytes.as<uint8_t>(), B.subsets.as<uint64_t>(),
                 B.res.as<QRes>(), B.hits.as<uint64_t>(), st);
    // the sample path ORs words past its register window into samples_out
    // (> 65,536-sample VCFs): start every run from zero
    if (B.samples_out.bytes && std::any_of(B.groups.begin(), B.groups.end(), [](const sb_batch::Group &g) {
            return g.max_words != 0;
        }))
        HIP_OK(hipMemsetAsync(B.samples_out.p, 0, B.samples_out.bytes, st));
    for (const auto &g : B.groups)
        if (g.max_words != 0)
            launch_scan(d, B.q.as<QDev>() + g.base, nullptr, static_cast<uint32_t>(g.idx.size()), B.nonneg,
                        g.max_words, g.mode, B.qbytes.as<uint8_t>(), B.subsets.as<uint64_t>(), B.res.as<QRes>(),
                        B.hits.as<uint64_t>(), B.samples_out.as<uint64_t>(), st);
    // slices whose scan reached a general record (work list filled above)
    launch_general(d, s.g, B.gen_work.as<uint32_t>(), B.gen_grid, B.qbytes.as<uint8_t>(), B.subsets.as<uint64_t>(),
                   B.res.as<QRes>(), B.hits.as<uint64_t>(), B.samples_out.as<uint64_t>(), B.gen_scratch.as<uint8_t>(),
                   B.gen_big_n.as<uint32_t>(), B.gen_big.as<GenBig>(), B.gen_limbs.as<uint32_t>(), B.gen_big_cap, st);
    HIP_OK(hipGetLastError());
}

void sync(sb_batch &B) {
    HIP_OK(hipSetDevice(B.s->device));
    if (B.runs_pending) HIP_OK(hipEventRecord(B.ev[1], B.strm()));
    const bool chk = B.req && B.req->err.p && B.req->err_h.p;
    if (chk) HIP_OK(hipMemcpyAsync(B.req->err_h.p, B.req->err.p, 4, hipMemcpyDeviceToHost, B.strm()));
    HIP_OK(hipStreamSynchronize(B.strm()));
    if (B.runs_pending) {  // device time per run = the span / runs (back-to-back launches)
        float x;
        HIP_OK(hipEventElapsedTime(&x, B.ev[0], B.ev[1]));
        B.last_total_ms = x / static_cast<float>(B.runs_pending);
        B.runs_pending = 0;
    }
    if (B.req && B.req->eval_used) {  // request batches: request_eval_kernel alone, averaged over the passes
        double sum = 0;
        for (size_t k = 0; k < B.req->eval_used; ++k) {
            float x;
            HIP_OK(hipEventElapsedTime(&x, B.req->eval_ev[k][0], B.req->eval_ev[k][1]));
            sum += x;
        }
        B.req->last_eval_ms = sum / static_cast<double>(B.req->eval_used);
        B.req->eval_used = 0;
    }
    if (chk && *static_cast<volatile uint32_t *>(B.req->err_h.p))
        throw Error(SB_EINTERNAL, "request_eval_kernel: the per-chain sums of a pass failed their invariants "
                                  "(chain counts vs the wave's staged hits / exists-slices)");
}

// each query's hit-region offset: chained slices' hits are dense per chain,
// so theirs follow from the n_hits of the chain's earlier slices
const uint64_t *src_offsets(sb_batch &B, hipStream_t st) {
    if (B.hchains.empty()) return B.hoff.as<uint64_t>();
    launch_chain_src(B.chains.as<ChainDev>(), static_cast<uint32_t>(B.hchains.size()), B.corig.as<uint32_t>(),
                     B.res.as<QRes>(), B.srcoff.as<uint64_t>(), st);
    return B.srcoff.as<uint64_t>();
}

sb_result_set *fetch(sb_batch &B) {
    if (B.slice_rows_stale)
        throw Error(SB_EINVAL, "the last run skipped per-slice results (sb_batch_set_slice_results): enable them and run");
    sync(B);
    sb_store &s = *B.s;
    hipStream_t st = B.strm();
    auto R = std::make_unique<sb_result_set>();
    R->s = store_hold(&s);
    const uint32_t nq = B.nq;
    R->res.resize(nq);
    if (nq) HIP_OK(hipMemcpyAsync(R->res.data(), B.res.p, nq * sizeof(QRes), hipMemcpyDeviceToHost, st));
    std::vector<uint64_t> sout(B.samples_words);
    if (!sout.empty()) HIP_OK(hipMemcpyAsync(sout.data(), B.samples_out.p, sout.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (uint32_t i = 0; i < nq; ++i) {
        if (B.host_err[i]) R->res[i].error = B.host_err[i];
        if (!B.chained.empty() && B.chained[i]) R->res[i].n_scanned = B.nscan[i];
    }
    if (B.gen_grid) {  // general slices whose counts need more than 64 bits
        uint32_t nb = 0;
        HIP_OK(hipMemcpy(&nb, B.gen_big_n.p, 4, hipMemcpyDeviceToHost));
        if (nb > B.gen_big_cap)
            throw Error(SB_ENOMEM, "more than " + std::to_string(B.gen_big_cap) +
                                       " slices of one batch have counts past 64 bits: split the batch");
        if (nb) {
            std::vector<GenBig> bl(nb);
            std::vector<uint32_t> limbs(size_t(nb) * 2 * kGenAccMax);
            HIP_OK(hipMemcpy(bl.data(), B.gen_big.p, nb * sizeof(GenBig), hipMemcpyDeviceToHost));
            HIP_OK(hipMemcpy(limbs.data(), B.gen_limbs.p, limbs.size() * 4, hipMemcpyDeviceToHost));
            const uint32_t W = (s.g.acc_limbs + 63) / 64 * 64;
            R->big_limbs = W;
            for (uint32_t k = 0; k < nb; ++k) {
                const uint32_t *p = limbs.data() + size_t(k) * 2 * kGenAccMax;
                std::vector<uint32_t> v(p, p + W);
                v.insert(v.end(), p + kGenAccMax, p + kGenAccMax + W);
                R->big[bl[k].orig] = std::move(v);
            }
        }
    }
    // dense offsets on the host, gather on the device, one D2H
    R->dense_off.assign(size_t(nq) + 1, 0);
    for (uint32_t i = 0; i < nq; ++i) R->dense_off[i + 1] = R->dense_off[i] + (R->res[i].error ? 0 : R->res[i].n_hits);
    const uint64_t total = R->dense_off[nq];
    R->hit.pool = req_pool(s);
    R->hit.n = total;
    if (total) {
        ReqPool &P = *R->hit.pool;
        DevMem doff = P.get_dev((size_t(nq) + 1) * 8), dense = P.get_dev(total * 8);
        R->hit.mem = P.get_pinned(total * 8);
        HIP_OK(hipMemcpyAsync(doff.p, R->dense_off.data(), (size_t(nq) + 1) * 8, hipMemcpyHostToDevice, st));
        const uint64_t *hoff = src_offsets(B, st);
        // queries with an error report n_hits = 0 on the device (host errors are F_EMPTY)
        launch_compact(hoff, doff.as<uint64_t>(), B.res.as<QRes>(), nq, B.hits.as<uint64_t>(), dense.as<uint64_t>(), st);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(R->hit.data(), dense.p, total * 8, hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        P.put_dev(std::move(doff));
        P.put_dev(std::move(dense));
    }
    R->sidx.assign(nq, std::vector<uint32_t>());
    R->emitted = B.emitted;
    R->chrom = B.chrom;
    R->vcf_of = B.vcf;
    R->samples_variant = B.samples_variant;
    uint64_t scanned = 0;
    for (uint32_t i = 0; i < nq; ++i) {
        const QDev &d = B.hq[i];
        scanned += R->res[i].n_scanned;
        if (d.samples_out_off != ~0ull && !R->res[i].error) {
            const uint64_t *w = sout.data() + d.samples_out_off;
            if (B.samples_variant[i]) {
                const auto &em = B.emitted[i];
                for (uint32_t j = 0; j < em.size(); ++j)
                    if ((w[em[j] >> 6] >> (em[j] & 63)) & 1) R->sidx[i].push_back(j);
            } else {
                for (uint32_t h = 0; h < d.n_samples; ++h)
                    if ((w[h >> 6] >> (h & 63)) & 1) R->sidx[i].push_back(h);
            }
        }
    }
    R->vtext.assign(nq, std::string());
    R->ntext.assign(nq, std::string());
    R->vbuilt.assign(nq, 0);
    R->nbuilt.assign(nq, 0);
    R->stats.n_queries = nq;
    R->stats.records_scanned = scanned;
    R->stats.chained_slices = B.chain_members.size();
    R->stats.chains = B.hchains.size();
    R->stats.cand_loaded = B.cand_loaded;
    R->stats.cand_window = B.cand_window;
    R->stats.cand_unique = B.cand_unique;
    R->stats.hits = total;
    R->stats.device_ms = B.last_total_ms;
    return R.release();
}

// virtual offset -> offset in the VCF text stream (block table of the BGZF file)
bool voff_to_stream(const VcfData &v, uint64_t voff, uint64_t *u) {
    const uint64_t co = voff >> 16, uo = voff & 0xffffu;
    auto it = std::lower_bound(v.blk_coff.begin(), v.blk_coff.end(), co);
    if (it == v.blk_coff.end()) {
        if (uo) return false;
        *u = v.stream_len;  // one past the last block
        return true;
    }
    if (*it != co) return false;
    *u = v.blk_ustart[static_cast<size_t>(it - v.blk_coff.begin())] + uo;
    return *u <= v.stream_len;
}

// summariseSlice scratch, kept per store (sb_store::summarise_ws)
struct SumWs {
    DevMem dsl, dbm, dres, dcs, dpart;
};

void summarise(sb_store &s, const sb_slice *sl, size_t n, sb_slice_stats *out, double *device_ms) {
    std::vector<SDev> hs(n);
    std::vector<uint32_t> chunk_slice;  // phase-A chunk -> slice
    std::vector<int32_t> herr(n, 0);
    uint64_t words = 0;
    for (size_t i = 0; i < n; ++i) {
        SDev &d = hs[i];
        d.lo = d.hi = 0;
        d.chunk_lo = static_cast<uint32_t>(chunk_slice.size());
        d.n_chunks = 0;
        d.bitmap_off = words;
        if (sl[i].vcf_id >= s.vcfs.size()) throw Error(SB_ENOSTORE, "slice " + std::to_string(i) + ": unknown vcf id");
        const VcfData &v = s.vcfs[sl[i].vcf_id];
        if (v.blk_coff.empty()) throw Error(SB_EINVAL, "summarise needs a VCF ingested from a BGZF file (virtual offsets)");
        uint64_t u0, u1;
        if (!voff_to_stream(v, sl[i].virtual_start, &u0) || !voff_to_stream(v, sl[i].virtual_end, &u1)) {
            herr[i] = SB_QERR_UNSUPPORTED;  // offset not on a block of this file
            continue;
        }
        if (u1 < u0) u1 = u0;
        const uint32_t rb = v.rec_base;
        uint32_t re = rb;
        for (const auto &sg : v.segments) re = std::max(re, sg.hi);
        auto first = s.h_start.begin() + rb, last = s.h_start.begin() + re;
        const uint32_t lo = rb + static_cast<uint32_t>(std::lower_bound(first, last, u0) - first);
        const uint32_t hi = rb + static_cast<uint32_t>(std::lower_bound(first, last, u1) - first);
        if (hi > lo) {
            // the slice must start on a record and must not cut one (index
            // chunk boundaries are record boundaries); header bytes likewise
            const uint64_t end_last = hi < re ? s.h_start[hi] : v.stream_len;
            if (s.h_start[lo] != u0 || end_last > u1) herr[i] = SB_QERR_UNSUPPORTED;
        } else if (u1 > u0) {
            herr[i] = SB_QERR_UNSUPPORTED;  // a non-empty stretch with no record start
        }
        if (herr[i]) continue;
        d.lo = lo;
        d.hi = hi;
        d.chunk_lo = static_cast<uint32_t>(chunk_slice.size());
        d.n_chunks = (hi - lo + kSumChunk - 1) / kSumChunk;
        chunk_slice.insert(chunk_slice.end(), d.n_chunks, static_cast<uint32_t>(i));
        words += (hi - lo + 63) / 64;
    }
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    if (!s.summarise_ws)
        s.summarise_ws = std::shared_ptr<void>(new SumWs, [](void *w) { delete static_cast<SumWs *>(w); });
    SumWs &W = *static_cast<SumWs *>(s.summarise_ws.get());
    DevMem &dsl = W.dsl, &dbm = W.dbm, &dres = W.dres, &dcs = W.dcs, &dpart = W.dpart;
    dsl.reserve(n * sizeof(SDev));
    dbm.reserve(words * 8);  // every word is written by the chunk kernel
    dres.reserve(n * sizeof(SRes));
    dcs.reserve(chunk_slice.size() * 4);
    dpart.reserve(chunk_slice.size() * sizeof(SPart));
    if (n) HIP_OK(hipMemcpyAsync(dsl.p, hs.data(), n * sizeof(SDev), hipMemcpyHostToDevice, st));
    if (!chunk_slice.empty())
        HIP_OK(hipMemcpyAsync(dcs.p, chunk_slice.data(), chunk_slice.size() * 4, hipMemcpyHostToDevice, st));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, st));
    launch_summarise(s.ds, dsl.as<SDev>(), static_cast<uint32_t>(n), dcs.as<uint32_t>(),
                     static_cast<uint32_t>(chunk_slice.size()), dbm.as<uint64_t>(), dpart.as<SPart>(), dres.as<SRes>(),
                     st);
    HIP_OK(hipEventRecord(e1, st));
    HIP_OK(hipGetLastError());
    std::vector<SRes> r(n);
    if (n) HIP_OK(hipMemcpyAsync(r.data(), dres.p, n * sizeof(SRes), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (device_ms) *device_ms = ms;
    for (size_t i = 0; i < n; ++i) {
        out[i].error = herr[i] ? herr[i] : r[i].error;
        out[i]._pad = 0;
        out[i].num_variants = out[i].error ? 0 : r[i].num_variants;
        out[i].num_calls = out[i].error ? 0 : r[i].num_calls;
        out[i].records = out[i].error ? 0 : r[i].records;
    }
}

// ---------------------------------------------------------- region files
// summariseSlice's region files (lambda/summariseSlice/source/
// write_data_to_s3.h): the reader visits the records of the slice exactly as
// main.cpp:217-237 does (first record; then per record addCounts, seek
// (skipSize), skipPast('\n') — the walk the device summarise kernels
// reproduce), and recordHeader (:150-228) pushes one entry {pos, ref', alt'}
// per ALT of every visited record; a file is closed when a record's POS is
// more than MAX_SLICE_GAP past the buffer's last entry (:191-194) or when the
// buffer holds more than VCF_S3_OUTPUT_SIZE_LIMIT entries (:224-227), and at
// the end of the slice (~writeDataToS3).  File length = sum over entries of
// pos u64 + len u16 + |ref'| + 1 + |alt'| (saveOutputToS3, :39-92).
constexpr uint64_t kMaxSliceGap = 100000;        // main.tf:215 MAX_SLICE_GAP
constexpr uint64_t kOutputSizeLimit = 50000000;  // main.tf:17,216 VCF_S3_OUTPUT_SIZE_LIMIT

uint32_t key_tail_len(const sb_store &s, uint64_t k) {
    const uint64_t t = s.h_dk_tail[k];
    return (t & kTailBlob) ? static_cast<uint32_t>((t >> 40) & 0xffff) : static_cast<uint32_t>(t >> 56);
}

void append_key_entry(const sb_store &s, uint64_t k, std::vector<uint8_t> &out) {
    const uint64_t pos = s.h_dk_pos[k];
    const uint32_t tl = key_tail_len(s, k);
    const uint16_t len = static_cast<uint16_t>(tl);
    const size_t o = out.size();
    out.resize(o + 10 + tl);
    memcpy(out.data() + o, &pos, 8);
    memcpy(out.data() + o + 8, &len, 2);
    const uint64_t t = s.h_dk_tail[k];
    if (t & kTailBlob)
        memcpy(out.data() + o + 10, s.h_dk_blob.data() + (t & ((1ull << 40) - 1)), tl);
    else
        for (uint32_t j = 0; j < tl; ++j) out[o + 10 + j] = static_cast<uint8_t>(t >> (8 * j));
}

// One gzip member of buf (write_data_to_s3.h:51-52,64-65 -> gzip.cpp:19-59):
// deflateInit2(level 9, 16 + MAX_WBITS, memLevel 9), a header named "c"; the
// reference leaves the header's other fields uninitialised, here they are 0.
void gzip_member(const uint8_t *buf, size_t n, std::vector<uint8_t> &out) {
    z_stream zs{};
    if (deflateInit2(&zs, Z_BEST_COMPRESSION, Z_DEFLATED, 16 + MAX_WBITS, 9, Z_DEFAULT_STRATEGY) != Z_OK)
        throw Error(SB_EIO, "deflateInit2 failed");
    gz_header h{};
    static char name[] = "c";
    h.name = reinterpret_cast<Bytef *>(name);
    deflateSetHeader(&zs, &h);
    zs.next_in = const_cast<Bytef *>(buf);
    zs.avail_in = static_cast<uInt>(n);
    uint8_t chunk[1 << 16];
    int ret;
    do {
        zs.next_out = chunk;
        zs.avail_out = sizeof chunk;
        ret = deflate(&zs, Z_FINISH);
        if (ret == Z_STREAM_ERROR) {
            deflateEnd(&zs);
            throw Error(SB_EIO, "deflate failed");
        }
        out.insert(out.end(), chunk, chunk + (sizeof chunk - zs.avail_out));
    } while (zs.avail_out == 0);
    deflateEnd(&zs);
}

// one slice: status (0 / SB_QERR_UNSUPPORTED), files appended to `files`,
// file bytes appended to `data` when non-null (gz: as gzip members)
int32_t slice_region_files(const sb_store &s, uint32_t si, const sb_slice &sl, std::vector<sb_region_file> &files,
                           std::vector<uint8_t> *data, bool gz = false,
                           std::vector<std::vector<uint32_t>> *file_keys = nullptr) {
    if (sl.vcf_id >= s.vcfs.size()) throw Error(SB_ENOSTORE, "slice " + std::to_string(si) + ": unknown vcf id");
    const VcfData &v = s.vcfs[sl.vcf_id];
    if (v.blk_coff.empty()) throw Error(SB_EINVAL, "region files need a VCF ingested from a BGZF file (virtual offsets)");
    uint64_t u0, u1;
    if (!voff_to_stream(v, sl.virtual_start, &u0) || !voff_to_stream(v, sl.virtual_end, &u1)) return SB_QERR_UNSUPPORTED;
    if (u1 < u0) u1 = u0;
    const uint32_t rb = v.rec_base;
    uint32_t re = rb;
    for (const auto &sg : v.segments) re = std::max(re, sg.hi);
    auto first = s.h_start.begin() + rb, last = s.h_start.begin() + re;
    const uint32_t lo = rb + static_cast<uint32_t>(std::lower_bound(first, last, u0) - first);
    const uint32_t hi = rb + static_cast<uint32_t>(std::lower_bound(first, last, u1) - first);
    if (hi <= lo) return u1 > u0 ? SB_QERR_UNSUPPORTED : 0;
    const uint64_t end_last = hi < re ? s.h_start[hi] : v.stream_len;
    if (s.h_start[lo] != u0 || end_last > u1) return SB_QERR_UNSUPPORTED;
    // contig of the slice (one contig per slice: index chunks never cross)
    uint32_t contig = 0;
    for (uint32_t g = 0; g < v.segments.size(); ++g)
        if (lo >= v.segments[g].lo && lo < v.segments[g].hi) contig = g;
    const size_t f0 = files.size();
    const size_t d0 = data ? data->size() : 0;
    sb_region_file cur{si, contig, 0, 0, 0, 0, 0};
    bool open = false;
    // the open file's bytes and, for gzip output, where saveOutputToS3 cuts
    // members: before an entry when bufferLength + ref' + alt' + sizeof(pos)
    // > VCF_S3_OUTPUT_SIZE_LIMIT (write_data_to_s3.h:49)
    std::vector<uint8_t> fbuf;
    std::vector<size_t> cuts;
    size_t member_len = 0;
    std::vector<uint32_t> fkeys;  // the open file's store keys, in entry order (file_keys)
    const size_t k0 = file_keys ? file_keys->size() : 0;
    auto close = [&]() {
        if (open && cur.entries) {
            if (file_keys) file_keys->push_back(fkeys);
            if (data) {
                const size_t at = data->size();
                if (gz) {
                    size_t a = 0;
                    cuts.push_back(fbuf.size());
                    for (size_t c : cuts) {
                        if (c > a) gzip_member(fbuf.data() + a, c - a, *data);
                        a = c;
                    }
                } else {
                    data->insert(data->end(), fbuf.begin(), fbuf.end());
                }
                cur.data_bytes = data->size() - at;
            }
            files.push_back(cur);
        }
        cur = sb_region_file{si, contig, 0, 0, 0, 0, 0};
        open = false;
        fbuf.clear();
        cuts.clear();
        member_len = 0;
        fkeys.clear();
    };
    const uint64_t skip = 2ull * s.h_dcount[lo];
    uint32_t r = lo;
    while (r < hi) {
        if (s.h_sum_bad[r]) {  // the reference throws / reads past the line
            files.resize(f0);
            if (data) data->resize(d0);
            if (file_keys) file_keys->resize(k0);
            return SB_QERR_UNSUPPORTED;
        }
        const uint64_t pos = s.h_pos[r];
        if (open && cur.entries) {
            if (pos < cur.last_pos) throw Error(SB_EINVAL, "unsorted file");  // write_data_to_s3.h:184-188
            if (pos > cur.last_pos + kMaxSliceGap) close();
        }
        for (uint32_t k = s.h_dk_lo[r]; k < s.h_dk_lo[r + 1]; ++k) {
            if (!open || !cur.entries) {
                cur.first_pos = s.h_dk_pos[k];
                open = true;
            }
            cur.last_pos = s.h_dk_pos[k];
            const uint32_t tl = key_tail_len(s, k);
            cur.bytes += 10 + tl;
            ++cur.entries;
            if (data) {
                if (gz && member_len + (tl - 1) + 8 > kOutputSizeLimit) {  // ref' + alt' = tail - '_'
                    cuts.push_back(fbuf.size());
                    member_len = 0;
                }
                append_key_entry(s, k, fbuf);
                member_len += 10 + tl;
            }
            if (file_keys) fkeys.push_back(k);
        }
        if (cur.entries > kOutputSizeLimit) close();
        // next visited record
        if (r == lo) {
            r = lo + 1;  // skipPastAndCountChars('\n') ends the first record's line
        } else if (skip >= s.h_rem[r]) {  // seek(skipSize) lands past this line
            const uint64_t P = s.h_start[r] + s.h_cur[r] + skip;
            r = static_cast<uint32_t>(std::upper_bound(s.h_start.begin() + r + 1, s.h_start.begin() + hi, P) -
                                      s.h_start.begin());
        } else {
            ++r;
        }
    }
    close();
    return 0;
}

// the key string of store key k: decimal(pos) ++ ref'_alt'
std::string key_string(const sb_store &s, uint32_t k) {
    std::string out = std::to_string(s.h_dk_pos[k]);
    const uint64_t t = s.h_dk_tail[k];
    if (t & kTailBlob) {
        const uint64_t off = t & ((1ull << 40) - 1), len = (t >> 40) & 0xffff;
        out.append(reinterpret_cast<const char *>(s.h_dk_blob.data() + off), len);
    } else {
        for (uint64_t j = 0, len = t >> 56; j < len; ++j) out.push_back(static_cast<char>((t >> (8 * j)) & 0xff));
    }
    return out;
}

// dedup scratch, kept per store (sb_store::dedup_ws) and grown on demand
struct DedupWs {
    DevMem dseg, dtiles, tcnt, ke0, ke1, kh0, vh0, kh1, vh1, hist, bsum, counts, coll, ncoll, pe, ph, overflow;
};

void dedup_run(sb_store &s, const std::vector<KSeg> &segs, uint64_t n, size_t nj, uint64_t *unique, int32_t *status,
               sb_dedup_stats *stats, bool force_radix = false, std::vector<KRun> *runs = nullptr);

void dedup(sb_store &s, const sb_dedup_job *jobs, size_t nj, uint64_t *unique, int32_t *status,
           sb_dedup_stats *stats) {
    if (nj > (1u << 20)) throw Error(SB_EINVAL, "more than 2^20 dedup jobs in one call");
    std::vector<KSeg> segs;
    std::vector<KRun> runs;  // parallel to segs (window path)
    uint64_t n = 0;
    for (size_t j = 0; j < nj; ++j) {
        const sb_dedup_job &J = jobs[j];
        status[j] = 0;
        unique[j] = 0;
        if ((!J.vcf_ids && J.n_vcf) || (!J.contig && J.contig_len)) throw Error(SB_EINVAL, "dedup job: NULL array");
        const std::string contig(J.contig ? J.contig : "", J.contig_len);
        std::vector<uint32_t> seen;
        const size_t seg0 = segs.size();
        for (uint32_t t = 0; t < J.n_vcf; ++t) {
            const uint32_t id = J.vcf_ids[t];
            if (id >= s.vcfs.size()) throw Error(SB_ENOSTORE, "dedup job " + std::to_string(j) + ": unknown vcf id");
            if (std::find(seen.begin(), seen.end(), id) != seen.end()) continue;  // a file listed twice adds nothing
            seen.push_back(id);
            const VcfData &v = s.vcfs[id];
            auto it = v.seg_index.find(contig);
            if (it == v.seg_index.end() || J.range_start > J.range_end || J.range_start > 0xffffffffull) continue;
            const Segment &sg = v.segments[it->second];
            const uint32_t rs = static_cast<uint32_t>(J.range_start);
            const uint32_t re = static_cast<uint32_t>(std::min<uint64_t>(J.range_end, 0xffffffffull));
            // records the reference's summariseSlice throws on, inside the range
            auto b0 = std::lower_bound(s.h_dk_bad.begin(), s.h_dk_bad.end(), sg.lo);
            for (auto b = b0; b != s.h_dk_bad.end() && *b < sg.hi; ++b)
                if (s.h_pos[*b] >= rs && s.h_pos[*b] <= re) status[j] = SB_QERR_UNSUPPORTED;
            const auto kb = s.h_dk_pos.begin();
            const uint32_t klo = s.h_dk_lo[sg.lo], khi = s.h_dk_lo[sg.hi];
            const uint32_t a = static_cast<uint32_t>(std::lower_bound(kb + klo, kb + khi, rs) - kb);
            const uint32_t e = static_cast<uint32_t>(std::upper_bound(kb + klo, kb + khi, re) - kb);
            if (e > a) {
                segs.push_back(KSeg{a, n, e - a, static_cast<uint32_t>(j), rs, 0});
                const BucketIndex &bi = v.buckets[it->second];
                runs.push_back(KRun{a, e, s.h_dk_pos[a], s.h_dk_pos[e - 1], sg.lo, sg.hi, bi.base, bi.shift, bi.off,
                                    bi.n, static_cast<uint32_t>(j), 0, 0, {0, 0}});
                n += e - a;
            }
        }
        if (status[j]) {  // drop the job's keys
            for (size_t g = seg0; g < segs.size(); ++g) n -= segs[g].n;
            segs.resize(seg0);
            runs.resize(seg0);
        }
    }
    dedup_run(s, segs, n, nj, unique, status, stats, false, &runs);
}

// ---- window dedup planning (devtypes.hpp KWin / KJob)
// Every key run of a job is POS-sorted: cutting the job's runs at common POS
// boundaries into windows of about kWinTarget keys puts all keys of one
// (string, POS) in one window.  The host only sizes each job (windows =
// its keys / kWinTarget, its leader run, its POS span); dedup_plan_kernel
// finds the cuts.  runs[g] = segs[g]'s KRun (key range, POS span, its
// segment's coarse POS index for the cuts and the twin lookups).
struct WinPlan {
    std::vector<KJob> jobs;
    uint64_t n_wins = 0, n_e = 0;
    const char *why = "";  // why the plan was declined (SBEACON_DEDUP_DEBUG)
};

bool plan_windows(const sb_store &s, std::vector<KRun> &runs, size_t nj, WinPlan &P) {
    uint32_t target = kWinTarget;  // SBEACON_DEDUP_WIN_TARGET (tests): smaller windows
    if (const int k = config().dedup_win_target) target = std::max(1, std::min(static_cast<int>(kWinCap), k));
    if (s.n_keys >= 0x80000000ull) return P.why = "2^31 keys", false;
    std::vector<char> seen(nj, 0);
    for (size_t g0 = 0; g0 < runs.size();) {
        size_t g1 = g0 + 1;
        while (g1 < runs.size() && runs[g1].job == runs[g0].job) ++g1;
        if (seen[runs[g0].job]) return P.why = "job runs not contiguous", false;
        seen[runs[g0].job] = 1;
        if (g1 - g0 > kWinPieces) return P.why = "runs", false;
        KJob J{};
        uint64_t keys = 0;
        size_t lead = g0;
        J.pmin = UINT32_MAX;
        for (size_t g = g0; g < g1; ++g) {
            runs[g].run_lo = static_cast<uint32_t>(g0);
            runs[g].nruns = static_cast<uint32_t>(g1 - g0);
            const uint32_t k = runs[g].key_hi - runs[g].key_lo;
            keys += k;
            if (k > runs[lead].key_hi - runs[lead].key_lo) lead = g;
            J.pmin = std::min(J.pmin, runs[g].pos_lo);
            J.pmax = std::max(J.pmax, runs[g].pos_hi);
        }
        J.lead_lo = runs[lead].key_lo;
        J.lead_n = runs[lead].key_hi - runs[lead].key_lo;
        J.nw = static_cast<uint32_t>(std::min<uint64_t>(std::max<uint64_t>(1, (keys + target - 1) / target), J.lead_n));
        J.w0 = static_cast<uint32_t>(P.n_wins);
        J.run_lo = static_cast<uint32_t>(g0);
        J.nruns = static_cast<uint32_t>(g1 - g0);
        J.eoff = static_cast<uint32_t>(P.n_e);
        P.n_wins += J.nw;
        P.n_e += uint64_t(J.nruns) * (J.nw + 1);
        if (P.n_wins >= 0x7fffffffull || P.n_e >= 0xffffffffull) return P.why = "windows", false;
        P.jobs.push_back(J);
        g0 = g1;
    }
    return true;
}

struct PinnedHost {  // grow-only pinned host staging (hipHostMalloc)
    void *p = nullptr;
    size_t bytes = 0;
    void reserve(size_t n) {
        if (n <= bytes) return;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        HIP_OK(hipHostMalloc(&p, n, hipHostMallocDefault));
        bytes = n;
    }
    ~PinnedHost() {
        if (p) (void)hipHostFree(p);
    }
};

struct WinWs {
    DevMem jobs, wins, e, runs, counts, overflow, list, n_list, wfresh;
    PinnedHost stage;  // jobs | runs for one H2D copy; counts + overflow back
};

// the window path: true when it answered every job (counts in unique[])
bool dedup_window_run(sb_store &s, std::vector<KRun> &runs, uint64_t n, size_t nj, uint64_t *unique,
                      const int32_t *status, sb_dedup_stats *stats) {
    WinPlan P;
    const bool dbg = config().dedup_debug;
    const auto t0 = std::chrono::steady_clock::now();
    auto since = [&]() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
    if (!plan_windows(s, runs, nj, P)) {
        if (dbg) std::fprintf(stderr, "[sbeacon] dedup windows: plan declined (%s)\n", P.why);
        return false;
    }
    const double t_plan = since();
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    if (!s.win_ws) s.win_ws = std::shared_ptr<void>(new WinWs, [](void *w) { delete static_cast<WinWs *>(w); });
    WinWs &W = *static_cast<WinWs *>(s.win_ws.get());
    const uint32_t nw = static_cast<uint32_t>(P.n_wins);
    W.jobs.reserve(std::max<size_t>(P.jobs.size(), 1) * sizeof(KJob));
    W.wins.reserve(std::max<size_t>(nw, 1) * sizeof(KWin));
    W.e.reserve(std::max<size_t>(P.n_e, 1) * 4);
    W.runs.reserve(std::max<size_t>(runs.size(), 1) * sizeof(KRun));
    W.counts.reserve(std::max<size_t>(nj, 1) * 8);
    W.wfresh.reserve(std::max<size_t>(nw, 1) * 4);
    W.overflow.reserve(4);
    // deferred displaced keys (10 POS <= the job's largest POS): a list of a
    // quarter of the keys; a fuller list is an overflow (the sorted path)
    const uint32_t cap = static_cast<uint32_t>(std::min<uint64_t>(n / 4 + 65536, 0xffffffffull));
    W.list.reserve(static_cast<size_t>(cap) * 8);
    W.n_list.reserve(4);
    HIP_OK(hipMemsetAsync(W.n_list.p, 0, 4, st));
    // jobs and runs staged in pinned memory: DMA without a pageable bounce;
    // the previous call's copies have completed (it synchronised)
    const size_t bj = P.jobs.size() * sizeof(KJob), br = runs.size() * sizeof(KRun);
    W.stage.reserve(bj + br + 64 + std::max<size_t>(nj, 1) * 8);
    if (nw) {
        std::memcpy(W.stage.p, P.jobs.data(), bj);
        std::memcpy(static_cast<uint8_t *>(W.stage.p) + bj, runs.data(), br);
        HIP_OK(hipMemcpyAsync(W.jobs.p, W.stage.p, bj, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemcpyAsync(W.runs.p, static_cast<uint8_t *>(W.stage.p) + bj, br, hipMemcpyHostToDevice, st));
    }
    HIP_OK(hipMemsetAsync(W.counts.p, 0, std::max<size_t>(nj, 1) * 8, st));
    HIP_OK(hipMemsetAsync(W.overflow.p, 0, 4, st));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, st));
    launch_window_dedupe(s.dk, W.jobs.as<KJob>(), static_cast<uint32_t>(P.jobs.size()), W.wins.as<KWin>(), nw,
                         W.e.as<uint32_t>(), W.runs.as<KRun>(), W.counts.as<unsigned long long>(), W.list.as<uint2>(),
                         W.n_list.as<uint32_t>(), cap, W.overflow.as<uint32_t>(), W.wfresh.as<uint32_t>(), st);
    HIP_OK(hipEventRecord(e1, st));
    HIP_OK(hipGetLastError());
    std::vector<uint64_t> cnt(std::max<size_t>(nj, 1));
    uint32_t ovf = 0;
    HIP_OK(hipMemcpyAsync(cnt.data(), W.counts.p, cnt.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(&ovf, W.overflow.p, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (dbg)
        std::fprintf(stderr, "[sbeacon] dedup windows: %u windows, plan %.3f ms, all %.3f ms (device %.3f ms)\n", nw,
                     t_plan, since(), ms);
    if (ovf) {
        if (dbg) std::fprintf(stderr, "[sbeacon] dedup windows: device overflow over %u windows\n", nw);
        return false;
    }
    for (size_t j = 0; j < nj; ++j) unique[j] = status[j] ? 0 : cnt[j];
    if (stats) {
        stats->keys = n;
        stats->collisions = 0;
        stats->device_ms = ms;
        stats->path = SB_DEDUP_WINDOWS;
        stats->windows = nw;
    }
    return true;
}

// the device part of duplicateVariantSearch over planned key runs: windows
// (one read of every key), else gather, radix sort, adjacent-unique (+ host
// recount of 64-bit word collisions)
void dedup_run(sb_store &s, const std::vector<KSeg> &segs, uint64_t n, size_t nj, uint64_t *unique, int32_t *status,
               sb_dedup_stats *stats, bool force_radix, std::vector<KRun> *runs) {
    if (n >= 0xffffffffull) throw Error(SB_EINVAL, "dedup batch exceeds 2^32 keys; split it");
    {
        // SBEACON_DEDUP_EXACT=bucket / radix (tests, A/B) skip the window path
        const Config cf = config();
        const bool hash_hook = cf.dedup_hash_bits != 0;
        if (runs && !force_radix && !hash_hook && !cf.dedup_exact &&
            dedup_window_run(s, *runs, n, nj, unique, status, stats))
            return;
    }
    uint32_t job_bits = 0;
    while ((1ull << job_bits) < nj) ++job_bits;
    uint64_t mask = ~0ull;
    if (const int b = config().dedup_hash_bits) {  // test hook: force collisions
        if (b > 0 && b < 64) mask = (1ull << b) - 1;
    }
    // exact-word window: POS - rangeStart of every gathered key fits pos_bits
    uint64_t max_rel = 0;
    for (const KSeg &g : segs) max_rel = std::max<uint64_t>(max_rel, s.h_dk_pos[g.key_lo + g.n - 1] - g.range_start);
    uint32_t pos_bits = 1;
    while (pos_bits < 40 && (max_rel >> pos_bits)) ++pos_bits;
    if (job_bits + pos_bits + 6 > 64 || mask != ~0ull) pos_bits = 0;  // exact stream off (all keys hashed)
    const uint32_t exact_job_shift = pos_bits + 6;
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    std::vector<uint2> tiles;  // gather tiles: (segment, first key offset)
    const uint32_t gt = dedup_gather_tile();
    for (uint32_t g = 0; g < segs.size(); ++g)
        for (uint32_t o = 0; o < segs[g].n; o += gt) tiles.push_back(uint2{g, o});
    const uint32_t ntiles = static_cast<uint32_t>(tiles.size());
    const uint64_t slots = static_cast<uint64_t>(ntiles) * gt;  // sparse gather layout
    const uint64_t maxt = std::max<uint64_t>(ntiles, (n + gt - 1) / gt);
    if (!s.dedup_ws) s.dedup_ws = std::shared_ptr<void>(new DedupWs, [](void *w) { delete static_cast<DedupWs *>(w); });
    DedupWs &W = *static_cast<DedupWs *>(s.dedup_ws.get());
    DevMem &dseg = W.dseg, &dtiles = W.dtiles, &tcnt = W.tcnt, &ke0 = W.ke0, &ke1 = W.ke1, &kh0 = W.kh0, &vh0 = W.vh0,
           &kh1 = W.kh1, &vh1 = W.vh1, &hist = W.hist, &bsum = W.bsum, &counts = W.counts, &coll = W.coll,
           &ncoll = W.ncoll, &pe = W.pe, &ph = W.ph;
    dseg.reserve(segs.size() * sizeof(KSeg));
    dtiles.reserve(tiles.size() * sizeof(uint2));
    tcnt.reserve(2 * static_cast<size_t>(ntiles) * 4);
    ke0.reserve(slots * 8);
    ke1.reserve(n * 8);
    kh0.reserve(slots * 8);
    vh0.reserve(slots * 4);
    kh1.reserve(n * 8);
    vh1.reserve(n * 4);
    hist.reserve(maxt * 256 * 4);
    bsum.reserve(radix_bsum_words(maxt * gt) * 4);
    counts.reserve(std::max<size_t>(nj, 1) * 8);
    coll.reserve(n * 4);
    ncoll.reserve(4);
    if (!segs.empty()) HIP_OK(hipMemcpyAsync(dseg.p, segs.data(), segs.size() * sizeof(KSeg), hipMemcpyHostToDevice, st));
    if (!tiles.empty())
        HIP_OK(hipMemcpyAsync(dtiles.p, tiles.data(), tiles.size() * sizeof(uint2), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(counts.p, 0, std::max<size_t>(nj, 1) * 8, st));
    HIP_OK(hipMemsetAsync(ncoll.p, 0, 4, st));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, st));
    launch_dedup_gather(s.dk, dseg.as<KSeg>(), dtiles.as<uint2>(), ntiles, pos_bits, exact_job_shift, job_bits, mask,
                        ke0.as<uint64_t>(), kh0.as<uint64_t>(), vh0.as<uint32_t>(), tcnt.as<uint32_t>(), st);
    std::vector<uint32_t> htc(2 * static_cast<size_t>(ntiles));
    if (!htc.empty()) HIP_OK(hipMemcpyAsync(htc.data(), tcnt.p, htc.size() * 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    uint64_t ne = 0, nh = 0;
    for (uint32_t t = 0; t < ntiles; ++t) {
        ne += htc[t];
        nh += htc[ntiles + t];
    }
    if (ne + nh != n) throw Error(SB_EHIP, "dedup gather lost keys");
    // exact stream: hash buckets (two radix passes on a mix of the word +
    // an LDS hash set per workgroup; SBEACON_DEDUP_EXACT=radix forces the
    // full sort) or as many 8-bit radix passes as its words have bits + an
    // adjacent-unique pass; the first pass compacts the gather tiles
    const bool bucket = !force_radix && config().dedup_exact != 'r' && ne > 0;
    const uint32_t be = bucket ? 0u : dedup_unique_blocks(ne), bh = bucket ? 0u : dedup_unique_blocks(nh);
    pe.reserve(std::max<uint32_t>(be, 1) * sizeof(uint4));
    ph.reserve(std::max<uint32_t>(bh, 1) * sizeof(uint4));
    W.overflow.reserve(4);
    HIP_OK(hipMemsetAsync(W.overflow.p, 0, 4, st));
    if (bucket) {
        launch_bucket_dedupe(ke0.as<uint64_t>(), nullptr, ke1.as<uint64_t>(), nullptr, ne, s.dk, exact_job_shift,
                             static_cast<uint32_t>(nj), counts.as<unsigned long long>(), W.overflow.as<uint32_t>(),
                             hist.as<uint32_t>(), bsum.as<uint32_t>(), st, tcnt.as<uint32_t>(), ntiles);
    } else {
        const int re = launch_radix_sort(ke0.as<uint64_t>(), nullptr, ke1.as<uint64_t>(), nullptr, ne,
                                         job_bits + pos_bits + 6, hist.as<uint32_t>(), bsum.as<uint32_t>(), st,
                                         tcnt.as<uint32_t>(), ntiles);
        launch_dedup_unique(re ? ke1.as<uint64_t>() : ke0.as<uint64_t>(), nullptr, ne, s.dk, exact_job_shift, false,
                            counts.as<unsigned long long>(), pe.as<uint4>(), coll.as<uint32_t>(), ncoll.as<uint32_t>(),
                            st);
    }
    // hashed stream: (job | hash, key id); hash buckets with equal words
    // confirmed on the strings (any collision: the sorted path below via the
    // overflow rerun), or 8 radix passes + adjacent unique with the exact
    // host recount of collided groups
    const uint32_t hjob_shift = job_bits ? 64 - job_bits : 64;
    int rh = 0;
    if (bucket && nh) {
        rh = launch_bucket_dedupe(kh0.as<uint64_t>(), vh0.as<uint32_t>(), kh1.as<uint64_t>(), vh1.as<uint32_t>(), nh, s.dk,
                                  hjob_shift, static_cast<uint32_t>(nj), counts.as<unsigned long long>(),
                                  W.overflow.as<uint32_t>(), hist.as<uint32_t>(), bsum.as<uint32_t>(), st,
                                  tcnt.as<uint32_t>() + ntiles, ntiles);
    } else {
        rh = launch_radix_sort(kh0.as<uint64_t>(), vh0.as<uint32_t>(), kh1.as<uint64_t>(), vh1.as<uint32_t>(), nh, 64,
                               hist.as<uint32_t>(), bsum.as<uint32_t>(), st, tcnt.as<uint32_t>() + ntiles, ntiles);
        launch_dedup_unique((rh ? kh1 : kh0).as<uint64_t>(), (rh ? vh1 : vh0).as<uint32_t>(), nh, s.dk, hjob_shift,
                            true, counts.as<unsigned long long>(), ph.as<uint4>(), coll.as<uint32_t>(),
                            ncoll.as<uint32_t>(), st);
    }
    DevMem &kh = rh ? kh1 : kh0;
    DevMem &vh = rh ? vh1 : vh0;
    HIP_OK(hipEventRecord(e1, st));
    HIP_OK(hipGetLastError());
    std::vector<uint64_t> cnt(std::max<size_t>(nj, 1));
    uint32_t nc = 0, ovf = 0;
    HIP_OK(hipMemcpyAsync(cnt.data(), counts.p, cnt.size() * 8, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(&nc, ncoll.p, 4, hipMemcpyDeviceToHost, st));
    HIP_OK(hipMemcpyAsync(&ovf, W.overflow.p, 4, hipMemcpyDeviceToHost, st));
    std::vector<uint4> hpe(be), hph(bh);
    if (be) HIP_OK(hipMemcpyAsync(hpe.data(), pe.p, be * sizeof(uint4), hipMemcpyDeviceToHost, st));
    if (bh) HIP_OK(hipMemcpyAsync(hph.data(), ph.p, bh * sizeof(uint4), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (const auto *P : {&hpe, &hph})
        for (const uint4 &q : *P) {  // per-block partials: first and last job of each block
            cnt[q.x] += q.y;
            if (q.z != q.x) cnt[q.z] += q.w;
        }
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (ovf) {  // a workgroup's buckets outgrew its hash set: recount with the full sort
        dedup_run(s, segs, n, nj, unique, status, stats, true);
        return;
    }
    if (nc) {
        // exact recount of every group holding a collision: the device counted
        // 1 + (adjacent string changes) for it; replace that by |distinct|
        const uint64_t n = nh;  // collisions live in the hashed stream
        std::vector<uint64_t> hk(n);
        std::vector<uint32_t> hv(n), ci(nc);
        HIP_OK(hipMemcpy(hk.data(), kh.p, n * 8, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(hv.data(), vh.p, n * 4, hipMemcpyDeviceToHost));
        HIP_OK(hipMemcpy(ci.data(), coll.p, nc * 4, hipMemcpyDeviceToHost));
        std::sort(ci.begin(), ci.end());
        uint64_t done_to = 0;  // groups end before this index
        for (uint32_t i : ci) {
            if (i < done_to) continue;
            uint64_t g0 = i, g1 = i + 1;
            while (g0 > 0 && hk[g0 - 1] == hk[i]) --g0;
            while (g1 < n && hk[g1] == hk[i]) ++g1;
            std::vector<std::string> strs;
            for (uint64_t x = g0; x < g1; ++x) strs.push_back(key_string(s, hv[x]));
            uint64_t adjacent = 1;
            for (size_t x = 1; x < strs.size(); ++x) adjacent += strs[x] != strs[x - 1];
            std::sort(strs.begin(), strs.end());
            const uint64_t exact = static_cast<uint64_t>(std::unique(strs.begin(), strs.end()) - strs.begin());
            const uint32_t job = job_bits ? static_cast<uint32_t>(hk[i] >> (64 - job_bits)) : 0u;
            cnt[job] = cnt[job] - adjacent + exact;
            done_to = g1;
        }
    }
    for (size_t j = 0; j < nj; ++j) unique[j] = status[j] ? 0 : cnt[j];
    if (stats) {
        stats->keys = n;
        stats->collisions = nc;
        stats->device_ms = ms;
        stats->path = bucket ? SB_DEDUP_BUCKETS : SB_DEDUP_RADIX;
        stats->windows = 0;
    }
}

// ------------------------------------------------ reference-exact duplicateVariantSearch
// What ReadVcfData::getVcfData (lambda/duplicateVariantSearch/source/
// readVcfData.cpp:3-71) inserts from one region file depends on when its
// gzip reader (lambda/shared/gzip/gzip.cpp:61-144) reports the end of the
// stream: the loop keeps reading while hasMoreData(), whatever the POS, and
// only inside the last decompressed window stops after the first entry past
// rangeEnd.  So the strict mode reads the region files exactly that way, over
// the gzip members this library writes (sb_slice_region_files with_data = 2):
// a multi-member stream inflated with Z_BLOCK through a 1 KiB input window
// into the reader's 1 KiB buffer, the buffer's unread tail moved to its front
// at every refill.  The entries it would insert are then deduplicated on the
// device like the intended-range mode's.
struct RefThrow {};  // a runtime_error of the reference (the Lambda fails)

class RegionReader {  // gzip.cpp:4-17 (constructor), 61-79, 81-144 (proccesData)
  public:
    RegionReader(const uint8_t *file, uint64_t size, char *buf, uint32_t buf_size)
        : file_(file), size_(static_cast<uint32_t>(size)), buf_(buf), buf_size_(buf_size) {
        if (size > 0xffffffffull) throw RefThrow{};  // gzip.cpp:16
    }
    ~RegionReader() {
        if (live_) inflateEnd(&zs_);
    }
    int start() {
        const int err = inflateInit2(&zs_, 16 + MAX_WBITS);
        live_ = err == Z_OK;
        if (err >= 0) more_ = true;
        return err;
    }
    bool more() const { return more_; }
    uint32_t fill(uint32_t beg, uint32_t end) {
        if (beg > end) throw RefThrow{};  // "gzip Error: proccesData input invalid"
        if (beg < end) memmove(buf_, buf_ + beg, end - beg);
        zs_.avail_out = buf_size_ - (end - beg);
        zs_.next_out = reinterpret_cast<Bytef *>(buf_ + (end - beg));
        for (;;) {
            if (zs_.avail_out == 0) return buf_size_;
            if (zs_.avail_in == 0) {
                zs_.avail_in = std::min<uint32_t>(sizeof window_, size_ - read_);
                zs_.next_in = window_;
                memcpy(window_, file_ + read_, zs_.avail_in);
                read_ += zs_.avail_in;
            }
            int err = inflate(&zs_, Z_BLOCK);
            if (err == Z_STREAM_END) {
                if (zs_.avail_in == 0 && size_ == read_) break;  // end of the file
                stop();  // another member: start the decompression again
                if (start() < 0) break;
            } else if (err < 0 || size_ - read_ + zs_.avail_in <= 8) {
                break;  // an error, or only the gzip footer left
            }
        }
        stop();
        return buf_size_ - zs_.avail_out;
    }

  private:
    void stop() {
        more_ = false;
        if (live_) inflateEnd(&zs_);
        live_ = false;
    }
    const uint8_t *file_;
    uint32_t size_, read_ = 0;
    char *buf_;
    uint32_t buf_size_;
    z_stream zs_{};
    bool more_ = false, live_ = false;
    Bytef window_[1024];
};

// readVcfData.cpp:3-71 over one region file: the file positions (entry
// indices) of the entries getVcfData returns.  false = the reference throws.
bool strict_region_entries(const uint8_t *file, uint64_t size, uint64_t rs, uint64_t re, std::vector<uint32_t> &incl) {
    constexpr size_t kMin = sizeof(uint64_t) + sizeof(uint16_t);  // readVcfData.hpp:8 MIN_DATA_SIZE
    char buf[1024];                                               // readVcfData.hpp:7 BUFFER_SIZE
    size_t pos = 0, len = 0;
    uint64_t vpos = 0;
    uint32_t entry = 0;
    try {
        RegionReader in(file, size, buf, sizeof buf);
        in.start();
        auto avail = [&](size_t need) -> bool {  // checkForAvailableData
            if (len >= pos + need) return true;
            if (!in.more()) return false;
            len = in.fill(static_cast<uint32_t>(pos), static_cast<uint32_t>(len));
            if (len > 0) {
                pos = 0;
                return true;
            }
            return false;
        };
        do {
            if (!avail(kMin)) return false;  // "Invalid File Read - getVcfData()"
            memcpy(&vpos, buf + pos, sizeof vpos);
            pos += sizeof vpos;
            uint16_t sl;
            memcpy(&sl, buf + pos, sizeof sl);
            if (rs <= vpos) {  // readString
                pos += sizeof sl;
                if (!avail(sl)) return false;  // "Invalid File Read - readString()"
                pos += sl;
                incl.push_back(entry);
            } else {
                pos += sl + sizeof sl;  // skipped with no availability check (:27-30)
            }
            ++entry;
        } while ((len != pos && vpos <= re) || in.more());
    } catch (const RefThrow &) {
        return false;
    }
    return true;
}

// The same reader over a whole file, once (every entry read): what a call's
// (rangeStart, rangeEnd) then selects follows in closed form.  Entries are
// POS-sorted in a region file, so getVcfData skips a prefix [0, lo) (POS <
// rangeStart) and reads on; the refills happen at the same entries on the
// read and the skip path except where an entry's string crosses the end of
// the buffer -- a skipped one leaves the read position past the data and the
// next refill throws ("proccesData input invalid").  The loop stops after
// the first entry at or past the final refill (`last`, more() false from
// then on) whose POS exceeds rangeEnd; with no final refill before the last
// entry it runs past the end and throws.
struct FileProfile {
    uint32_t n = 0;                   // entries
    uint32_t last_fill = UINT32_MAX;  // entry during which the stream ended (more() false after it)
    uint32_t fail_at = UINT32_MAX;    // entry at which the all-read walk failed (n: past the last)
    bool sorted = true;               // POS non-decreasing (else: the walk per call)
    bool consec = false;              // the entries' store keys are consecutive
    std::vector<uint32_t> straddle;   // entries whose string crosses a refill
    std::vector<uint64_t> vpos;
};

FileProfile profile_region_file(const uint8_t *file, uint64_t size) {
    constexpr size_t kMin = sizeof(uint64_t) + sizeof(uint16_t);
    char buf[1024];
    size_t pos = 0, len = 0;
    FileProfile P;
    uint32_t entry = 0;
    try {
        RegionReader in(file, size, buf, sizeof buf);
        in.start();
        auto avail = [&](size_t need) -> bool {
            if (len >= pos + need) return true;
            if (!in.more()) return false;
            len = in.fill(static_cast<uint32_t>(pos), static_cast<uint32_t>(len));
            if (!in.more() && P.last_fill == UINT32_MAX) P.last_fill = entry;
            if (len > 0) {
                pos = 0;
                return true;
            }
            return false;
        };
        do {
            if (!avail(kMin)) {
                P.fail_at = entry;
                break;
            }
            uint64_t vpos;
            uint16_t sl;
            memcpy(&vpos, buf + pos, sizeof vpos);
            pos += sizeof vpos;
            memcpy(&sl, buf + pos, sizeof sl);
            pos += sizeof sl;
            if (len < pos + sl) P.straddle.push_back(entry);
            if (!avail(sl)) {
                P.fail_at = entry;
                break;
            }
            pos += sl;
            if (!P.vpos.empty() && vpos < P.vpos.back()) P.sorted = false;
            P.vpos.push_back(vpos);
            ++entry;
        } while (len != pos || in.more());
    } catch (const RefThrow &) {
        P.fail_at = entry;
    }
    P.n = static_cast<uint32_t>(P.vpos.size());
    return P;
}

// the entries [lo, last] getVcfData returns for (rs, re) (none when lo >
// last); false = it throws
bool profile_range(const FileProfile &P, uint64_t rs, uint64_t re, uint32_t &lo, uint32_t &last) {
    const auto b = P.vpos.begin(), e = P.vpos.end();
    lo = static_cast<uint32_t>(std::lower_bound(b, e, rs) - b);
    const bool tail = !(P.last_fill < P.n);  // more() still true after the last entry
    last = P.n ? P.n - 1 : 0;
    if (!tail) {  // the first entry at or after the final refill with POS > re ends the loop
        const uint32_t j = static_cast<uint32_t>(std::upper_bound(b + P.last_fill, e, re) - b);
        if (j < P.n) last = j;
    }
    const uint32_t reach = tail ? P.n : last;  // the last entry the loop starts
    if (P.fail_at != UINT32_MAX && P.fail_at <= reach) return false;
    // a skipped entry whose string crosses the buffer end throws when the next entry starts
    if (!P.straddle.empty() && P.straddle.front() < std::min(lo, reach)) return false;
    return true;
}

// A slice's region files as summariseSlice writes them (gzip members, the
// store key of every entry), kept per store: the reference writes them once
// and every duplicateVariantSearch message reads them, so strict mode
// compresses each slice's files once (level 9 dominates: ~10 MB/s) and then
// only inflates.  Bounded by bytes (cleared when full).
struct SliceFiles {
    int32_t status = 0;
    std::vector<sb_region_file> files;
    std::vector<uint8_t> data;
    std::vector<uint64_t> at;  // each file's first byte in data
    std::vector<std::vector<uint32_t>> keys;
    std::vector<FileProfile> prof;  // per file (profile_region_file)
    size_t bytes() const {
        size_t b = data.size() + files.size() * sizeof(sb_region_file);
        for (const auto &k : keys) b += k.size() * 4;
        for (const auto &f : prof) b += f.vpos.size() * 8 + f.straddle.size() * 4;
        return b;
    }
};
struct RegionCache {
    std::map<std::tuple<uint32_t, uint64_t, uint64_t>, std::shared_ptr<const SliceFiles>> m;
    size_t bytes = 0;
    static constexpr size_t kCap = size_t(8) << 30;
};

void dedup_files(sb_store &s, const sb_dedup_file_job *jobs, size_t nj, uint64_t *unique, int32_t *status,
                 sb_dedup_stats *stats) {
    if (nj > (1u << 20)) throw Error(SB_EINVAL, "more than 2^20 dedup jobs in one call");
    if (!s.region_cache)  // under the store lock (sb_dedup_count_files)
        s.region_cache = std::shared_ptr<void>(new RegionCache, [](void *w) { delete static_cast<RegionCache *>(w); });
    RegionCache &C = *static_cast<RegionCache *>(s.region_cache.get());
    using Key = std::tuple<uint32_t, uint64_t, uint64_t>;
    // every (job, file) pair, and the slices not cached yet
    struct Pair {
        uint32_t job;
        const SliceFiles *sf = nullptr;
        uint32_t file;
        bool ok = true;
        bool walked = false;          // entries listed in incl (an unsorted file)
        uint32_t e_lo = 0, e_hi = 0;  // else the entries [e_lo, e_hi)
        std::vector<uint32_t> incl;
    };
    std::vector<Pair> pairs;
    std::vector<Key> missing;
    std::vector<Key> pkey;
    for (size_t j = 0; j < nj; ++j) {
        const sb_dedup_file_job &J = jobs[j];
        status[j] = 0;
        unique[j] = 0;
        if (!J.files && J.n_files) throw Error(SB_EINVAL, "dedup job: NULL file list");
        for (uint32_t t = 0; t < J.n_files; ++t) {
            const sb_region_ref &F = J.files[t];
            if (F.vcf_id >= s.vcfs.size()) throw Error(SB_ENOSTORE, "dedup job " + std::to_string(j) + ": unknown vcf id");
            const Key key = std::make_tuple(F.vcf_id, F.virtual_start, F.virtual_end);
            if (!C.m.count(key)) missing.push_back(key);
            pairs.push_back(Pair{static_cast<uint32_t>(j), nullptr, F.file, true, false, 0, 0, {}});
            pkey.push_back(key);
        }
    }
    std::sort(missing.begin(), missing.end());
    missing.erase(std::unique(missing.begin(), missing.end()), missing.end());
    // the missing slices' files, in parallel (gzip level 9 is the cost)
    std::vector<std::shared_ptr<SliceFiles>> made(missing.size());
    std::vector<std::unique_ptr<Error>> errs(missing.size());  // raised when a job reaches that file
    parallel_for(missing.size(), [&](size_t i) {
        try {
            auto sf = std::make_shared<SliceFiles>();
            const sb_slice sl{std::get<0>(missing[i]), 0, std::get<1>(missing[i]), std::get<2>(missing[i])};
            sf->status = slice_region_files(s, 0, sl, sf->files, &sf->data, true, &sf->keys);
            uint64_t a = 0;
            for (const auto &f : sf->files) {
                sf->at.push_back(a);
                a += f.data_bytes;
            }
            for (size_t f = 0; f < sf->files.size(); ++f) {
                sf->prof.push_back(profile_region_file(sf->data.data() + sf->at[f], sf->files[f].data_bytes));
                const auto &fk = sf->keys[f];
                bool c = fk.size() == sf->prof.back().n;
                for (size_t k = 1; c && k < fk.size(); ++k) c = fk[k] == fk[k - 1] + 1;
                sf->prof.back().consec = c;
            }
            made[i] = std::move(sf);
        } catch (const Error &e) {
            errs[i] = std::make_unique<Error>(e);
        } catch (const std::exception &e) {
            errs[i] = std::make_unique<Error>(SB_EINVAL, e.what());
        }
    }, 16, 1);
    size_t add = 0;
    for (const auto &m : made)
        if (m) add += m->bytes();
    if (C.bytes + add > RegionCache::kCap) {
        C.m.clear();
        C.bytes = 0;
    }
    // this call's slices stay referenced here even if the cache drops them
    std::map<Key, std::shared_ptr<const SliceFiles>> use;
    std::map<Key, const Error *> failed;
    for (size_t i = 0; i < missing.size(); ++i) {
        if (!made[i]) {
            failed[missing[i]] = errs[i].get();
            continue;
        }
        use[missing[i]] = made[i];
        C.m[missing[i]] = made[i];
        C.bytes += made[i]->bytes();
    }
    for (size_t p = 0; p < pairs.size(); ++p) {
        if (failed.count(pkey[p])) continue;  // sf stays null
        auto it = use.find(pkey[p]);
        if (it == use.end()) it = use.emplace(pkey[p], C.m.at(pkey[p])).first;
        pairs[p].sf = it->second.get();
    }
    // each pair's entries as the reference reader returns them: from the
    // file's profile (two binary searches), or by the walk itself for an
    // unsorted file; SBEACON_STRICT_CHECK=1 (tests) runs both and compares
    const bool check = config().strict_check;
    std::atomic<bool> mismatch{false};
    parallel_for(pairs.size(), [&](size_t p) {
        Pair &P = pairs[p];
        if (!P.sf) return;
        const SliceFiles &sf = *P.sf;
        if (sf.status || P.file >= sf.files.size()) return;  // reported in job order below
        const sb_dedup_file_job &J = jobs[P.job];
        const FileProfile &F = sf.prof[P.file];
        if (F.sorted) {
            uint32_t lo = 0, last = 0;
            P.ok = profile_range(F, J.range_start, J.range_end, lo, last);
            P.e_lo = std::min(lo, F.n);
            P.e_hi = std::max(P.e_lo, std::min(last + 1, F.n));
        }
        if (!F.sorted || check) {
            std::vector<uint32_t> incl;
            const bool ok = strict_region_entries(sf.data.data() + sf.at[P.file], sf.files[P.file].data_bytes,
                                                  J.range_start, J.range_end, incl);
            if (F.sorted) {
                bool same = ok == P.ok;
                if (same && ok) {
                    same = incl.size() == P.e_hi - P.e_lo;
                    for (size_t k = 0; same && k < incl.size(); ++k) same = incl[k] == P.e_lo + k;
                }
                if (!same) mismatch = true;
            } else {
                P.ok = ok;
                P.walked = true;
                P.incl = std::move(incl);
            }
        }
    }, 16, 1);
    if (mismatch) throw Error(SB_EINVAL, "strict dedup: region-file profile disagrees with the reader walk");
    // key runs in job order (consecutive store keys; KRun pieces of the
    // window path: a run is cut where the keys stop being consecutive or
    // leave their contig segment); a job stops at its first failing file
    std::vector<KSeg> segs;
    std::vector<KRun> runs;
    uint64_t n = 0;
    auto add_run = [&](uint32_t vcf, uint32_t a, uint32_t e, uint32_t j, uint32_t rs) {
        const VcfData &v = s.vcfs[vcf];
        while (a < e) {
            uint32_t k = 0;  // the segment holding key a
            while (k < v.segments.size() && !(s.h_dk_lo[v.segments[k].lo] <= a && a < s.h_dk_lo[v.segments[k].hi])) ++k;
            if (k == v.segments.size()) throw Error(SB_EINVAL, "strict dedup: a region-file key outside its VCF");
            const Segment &sg = v.segments[k];
            const uint32_t b = std::min(e, s.h_dk_lo[sg.hi]);
            if (!runs.empty() && runs.back().job == j && runs.back().key_hi == a && runs.back().seg_lo == sg.lo) {
                runs.back().key_hi = b;  // continues the previous run
                runs.back().pos_hi = s.h_dk_pos[b - 1];
                segs.back().n += b - a;
            } else {
                const BucketIndex &bi = v.buckets[k];
                segs.push_back(KSeg{a, n, b - a, j, rs, 0});
                runs.push_back(KRun{a, b, s.h_dk_pos[a], s.h_dk_pos[b - 1], sg.lo, sg.hi, bi.base, bi.shift, bi.off,
                                    bi.n, j, 0, 0, {0, 0}});
            }
            n += b - a;
            a = b;
        }
    };
    for (size_t p = 0; p < pairs.size();) {
        const uint32_t j = pairs[p].job;
        const uint32_t rs = static_cast<uint32_t>(std::min<uint64_t>(jobs[j].range_start, 0xffffffffull));
        const size_t seg0 = segs.size();
        const uint64_t n0 = n;
        for (; p < pairs.size() && pairs[p].job == j; ++p) {
            if (status[j]) continue;
            const Pair &P = pairs[p];
            if (!P.sf) throw *failed.at(pkey[p]);  // the error writing that slice's files raised
            const SliceFiles &sf = *P.sf;
            if (sf.status) {  // that summariseSlice never wrote its files
                status[j] = sf.status;
                continue;
            }
            if (P.file >= sf.files.size())
                throw Error(SB_EINVAL, "dedup job " + std::to_string(j) + ": no region file " + std::to_string(P.file) +
                                           " in that slice");
            if (!P.ok) {
                status[j] = SB_QERR_RUNTIME;
                continue;
            }
            const auto &fk = sf.keys[P.file];
            const uint32_t vcf = std::get<0>(pkey[p]);
            auto key_of = [&](uint32_t k) { return P.walked ? fk[P.incl[k]] : fk[P.e_lo + k]; };
            const uint32_t cnt = P.walked ? static_cast<uint32_t>(P.incl.size()) : P.e_hi - P.e_lo;
            for (uint32_t a = 0; a < cnt;) {  // runs of consecutive store keys
                uint32_t b = a + 1;
                if (!P.walked && sf.prof[P.file].consec) b = cnt;  // every key of the file is consecutive
                else
                    while (b < cnt && key_of(b) == key_of(b - 1) + 1) ++b;
                add_run(vcf, key_of(a), key_of(b - 1) + 1, j, rs);
                a = b;
            }
        }
        if (status[j]) {
            segs.resize(seg0);
            runs.resize(seg0);
            n = n0;
        }
    }
    dedup_run(s, segs, n, nj, unique, status, stats, false, &runs);
}

}  // namespace

extern "C" {

int sb_summarise_slices(sb_store *s, const sb_slice *slices, size_t n, sb_slice_stats *out, double *device_ms) {
    return guard([&] {
        if (!s || (!slices && n) || (!out && n)) throw Error(SB_EINVAL, "NULL argument");
        std::lock_guard<std::mutex> lk(s->mu);
        summarise(*s, slices, n, out, device_ms);
    });
}

struct sb_region_files {
    std::vector<sb_region_file> files;
    std::vector<uint8_t> data;
};

int sb_slice_region_files(sb_store *s, const sb_slice *slices, size_t n, int with_data, int32_t *status,
                          sb_region_files **out) {
    return guard([&] {
        if (!s || (!slices && n) || (!status && n) || !out) throw Error(SB_EINVAL, "NULL argument");
        auto R = std::make_unique<sb_region_files>();
        if (with_data < 0 || with_data > 2) throw Error(SB_EINVAL, "with_data must be 0, 1 or 2");
        for (size_t i = 0; i < n; ++i)
            status[i] = slice_region_files(*s, static_cast<uint32_t>(i), slices[i], R->files,
                                           with_data ? &R->data : nullptr, with_data == 2);
        *out = R.release();
    });
}

int sb_region_files_get(const sb_region_files *r, const sb_region_file **files, size_t *n, const uint8_t **data,
                        size_t *data_len) {
    if (!r || !files || !n) return SB_EINVAL;
    *files = r->files.data();
    *n = r->files.size();
    if (data) *data = r->data.data();
    if (data_len) *data_len = r->data.size();
    return SB_OK;
}

void sb_region_files_free(sb_region_files *r) { delete r; }

int sb_dedup_count(sb_store *s, const sb_dedup_job *jobs, size_t n_jobs, uint64_t *unique, int32_t *status,
                   sb_dedup_stats *stats) {
    return guard([&] {
        if (!s || (n_jobs && (!jobs || !unique || !status))) throw Error(SB_EINVAL, "NULL argument");
        std::lock_guard<std::mutex> lk(s->mu);
        dedup(*s, jobs, n_jobs, unique, status, stats);
    });
}

int sb_dedup_count_files(sb_store *s, const sb_dedup_file_job *jobs, size_t n_jobs, uint64_t *unique, int32_t *status,
                         sb_dedup_stats *stats) {
    return guard([&] {
        if (!s || (n_jobs && (!jobs || !unique || !status))) throw Error(SB_EINVAL, "NULL argument");
        std::lock_guard<std::mutex> lk(s->mu);
        dedup_files(*s, jobs, n_jobs, unique, status, stats);
    });
}

int sb_store_n_contigs(const sb_store *s, uint32_t vcf_id, uint32_t *n) {
    if (!s || !n) return SB_EINVAL;
    if (vcf_id >= s->vcfs.size()) return SB_ENOSTORE;
    *n = static_cast<uint32_t>(s->vcfs[vcf_id].segments.size());
    return SB_OK;
}

int sb_store_contig_name(const sb_store *s, uint32_t vcf_id, uint32_t i, const char **p, size_t *len) {
    if (!s || !p || !len) return SB_EINVAL;
    if (vcf_id >= s->vcfs.size() || i >= s->vcfs[vcf_id].segments.size()) return SB_ENOSTORE;
    const std::string &c = s->vcfs[vcf_id].segments[i].contig;
    *p = c.data();
    *len = c.size();
    return SB_OK;
}

int sb_store_chunk_boundaries(const sb_store *s, uint32_t vcf_id, const char *contig, size_t contig_len,
                              uint32_t stride, uint64_t *voffs, size_t cap, size_t *n) {
    return guard([&] {
        if (!s || !n || (!contig && contig_len) || (!voffs && cap)) throw Error(SB_EINVAL, "NULL argument");
        if (vcf_id >= s->vcfs.size()) throw Error(SB_ENOSTORE, "unknown vcf id");
        const VcfData &v = s->vcfs[vcf_id];
        if (v.blk_coff.empty()) throw Error(SB_EINVAL, "chunk boundaries need a VCF ingested from a BGZF file");
        auto it = v.seg_index.find(std::string(contig ? contig : "", contig_len));
        *n = 0;
        if (it == v.seg_index.end()) return;
        const Segment &sg = v.segments[it->second];
        uint32_t re = v.rec_base;  // end of this vcf's records
        for (const auto &g : v.segments) re = std::max(re, g.hi);
        const uint32_t st = std::max(1u, stride);
        auto voff = [&](uint64_t u) {  // stream offset -> (block coffset << 16 | in-block offset)
            auto b = std::upper_bound(v.blk_ustart.begin(), v.blk_ustart.end(), u);
            size_t i = static_cast<size_t>(b - v.blk_ustart.begin()) - 1;
            while (i + 1 < v.blk_ustart.size() && v.blk_ustart[i + 1] == v.blk_ustart[i]) ++i;  // skip empty blocks
            return (v.blk_coff[i] << 16) | (u - v.blk_ustart[i]);
        };
        size_t k = 0;
        auto put = [&](uint64_t x) {
            if (k < cap) voffs[k] = x;
            ++k;
        };
        for (uint32_t r = sg.lo; r < sg.hi; r += st) put(voff(s->h_start[r]));
        put(voff(sg.hi < re ? s->h_start[sg.hi] : v.stream_len));
        *n = k;
    });
}

int sb_store_vcf_stream(const sb_store *s, uint32_t vcf_id, uint64_t *n_blocks, uint64_t *stream_len) {
    if (!s || vcf_id >= s->vcfs.size()) return SB_EINVAL;
    if (n_blocks) *n_blocks = s->vcfs[vcf_id].blk_coff.size();
    if (stream_len) *stream_len = s->vcfs[vcf_id].stream_len;
    return SB_OK;
}

const char *sb_last_error(void) { return sb::last_error_cstr(); }
int sb_abi_version(void) { return SB_ABI_VERSION; }

int sb_builder_new(const sb_build_opts *opts, sb_builder **out) {
    return guard([&] {
        if (!out) throw Error(SB_EINVAL, "out is NULL");
        auto b = std::make_unique<sb_builder>();
        if (opts) {
            b->opts = *opts;
        } else {
            b->opts.keep_genotypes = 1;
            b->opts.n_threads = 0;
        }
        b->vt.get("N/A");
        *out = b.release();
    });
}

int sb_builder_begin_vcf(sb_builder *b, const char *location, size_t len, uint32_t *vcf_id) {
    return guard([&] {
        if (!b || !location || !vcf_id) throw Error(SB_EINVAL, "NULL argument");
        const std::string loc(location, len);
        for (const auto &v : b->vcfs)
            if (v.location == loc) throw Error(SB_EINVAL, "duplicate vcf location " + loc);
        b->vcfs.emplace_back();
        b->vcfs.back().location = loc;
        *vcf_id = static_cast<uint32_t>(b->vcfs.size() - 1);
    });
}

int sb_builder_add_text(sb_builder *b, uint32_t vcf_id, const char *text, size_t len) {
    return guard([&] {
        if (!b || (!text && len)) throw Error(SB_EINVAL, "NULL argument");
        builder_add_text(*b, vcf_id, text, len);
    });
}

int sb_builder_add_file(sb_builder *b, uint32_t vcf_id, const char *path) {
    return guard([&] {
        if (!b || !path) throw Error(SB_EINVAL, "NULL argument");
        builder_add_file(*b, vcf_id, path);
    });
}

struct sb_vcf_scan {
    VcfScan s;
};

int sb_vcf_scan_file(const char *path, sb_vcf_scan **out) {
    return guard([&] {
        if (!path || !out) throw Error(SB_EINVAL, "NULL argument");
        auto r = std::make_unique<sb_vcf_scan>();
        vcf_scan_file(path, r->s);
        *out = r.release();
    });
}

int sb_vcf_scan_info(const sb_vcf_scan *s, uint64_t *n_records, uint32_t *n_contigs, const uint32_t **pos) {
    if (!s || !n_records || !n_contigs || !pos) return SB_EINVAL;
    *n_records = s->s.pos.size();
    *n_contigs = static_cast<uint32_t>(s->s.contigs.size());
    *pos = s->s.pos.data();
    return SB_OK;
}

int sb_vcf_scan_contig(const sb_vcf_scan *s, uint32_t i, const char **name, size_t *len, uint64_t *lo, uint64_t *hi) {
    if (!s || !name || !len || !lo || !hi || i >= s->s.contigs.size()) return SB_EINVAL;
    const auto &c = s->s.contigs[i];
    *name = c.name.data();
    *len = c.name.size();
    *lo = c.lo;
    *hi = c.hi;
    return SB_OK;
}

void sb_vcf_scan_free(sb_vcf_scan *s) { delete s; }

int sb_builder_set_record_range(sb_builder *b, uint32_t vcf_id, uint64_t lo, uint64_t hi) {
    return guard([&] {
        if (!b) throw Error(SB_EINVAL, "NULL builder");
        if (vcf_id >= b->vcfs.size()) throw Error(SB_ENOSTORE, "unknown vcf id");
        VcfData &v = b->vcfs[vcf_id];
        if (v.lines_seen || v.stream_off) throw Error(SB_EINVAL, "set the record range before adding text");
        if (lo > hi) throw Error(SB_EINVAL, "record range lo > hi");
        v.rec_lo = lo;
        v.rec_hi = hi;
    });
}

int sb_builder_attach_carriers(sb_builder *b, uint32_t vcf_id, const char *const *names, const uint32_t *name_len,
                               uint32_t n_samples, const uint64_t *planes, uint64_t n_rows) {
    return guard([&] {
        if (!b) throw Error(SB_EINVAL, "NULL argument");
        builder_attach_carriers(*b, vcf_id, names, name_len, n_samples, planes, n_rows);
    });
}

int sb_builder_finish(sb_builder *b, int device, sb_store **out) {
    return guard([&] {
        if (!b || !out) throw Error(SB_EINVAL, "NULL argument");
        const bool trace = config().ingest_trace;  // phase times to stderr
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t i = 0; i < b->vcfs.size(); ++i) builder_flush(*b, i);
        const auto t1 = std::chrono::steady_clock::now();
        auto s = std::make_unique<sb_store>();
        s->device = device;
        if (device != SB_HOST_ONLY) {
            int n_dev = 0;
            HIP_OK(hipGetDeviceCount(&n_dev));
            if (device < 0 || device >= n_dev) throw Error(SB_EHIP, "device ordinal out of range");
            HIP_OK(hipSetDevice(device));
            HIP_OK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
        }
        upload_store(*b, *s);
        if (trace)
            std::fprintf(stderr, "[ingest] flush %.2f s, store columns + upload %.2f s\n",
                         std::chrono::duration<double>(t1 - t0).count(),
                         std::chrono::duration<double>(std::chrono::steady_clock::now() - t1).count());
        s->vcfs = std::move(b->vcfs);
        s->vt = std::move(b->vt);
        s->sym = std::move(b->sym);
        for (uint32_t i = 0; i < s->vcfs.size(); ++i) s->vcf_by_location.emplace(s->vcfs[i].location, i);
        b->vcfs.clear();
        b->vt = Dict();
        b->vt.get("N/A");
        b->sym = Dict();
        *out = s.release();
    });
}

void sb_builder_free(sb_builder *b) { delete b; }
void sb_store_close(sb_store *s) {
    if (s) store_release(s);
}

int sb_store_save(sb_store *s, const char *dir) {
    return guard([&] {
        if (!s || !dir) throw Error(SB_EINVAL, "NULL argument");
        std::lock_guard<std::mutex> lk(s->mu);
        store_save(*s, dir);
    });
}

int sb_store_open(const char *path, int device, sb_store **out) {
    return guard([&] {
        if (!path || !out) throw Error(SB_EINVAL, "NULL argument");
        std::string stale;
        sb_store *s = store_open(path, device, &stale);
        if (!s) throw Error(SB_ESTALE, stale);
        *out = s;
    });
}

int sb_store_trim(sb_store *s) {
    return guard([&] {
        if (!s) throw Error(SB_EINVAL, "NULL store");
        if (s->req_pool) static_cast<ReqPool *>(s->req_pool.get())->trim();
    });
}

int sb_store_get_info(const sb_store *s, sb_store_info *out) {
    return guard([&] {
        if (!s || !out) throw Error(SB_EINVAL, "NULL argument");
        out->n_records = s->n_records;
        out->n_alt_rows = s->n_records + s->n_extra;
        out->n_vcfs = static_cast<uint32_t>(s->vcfs.size());
        uint32_t nseg = 0, ms = 0;
        for (const auto &v : s->vcfs) {
            nseg += static_cast<uint32_t>(v.segments.size());
            ms = std::max(ms, static_cast<uint32_t>(v.samples.size()));
        }
        out->n_segments = nseg;
        out->device_bytes = s->device_bytes;
        out->max_samples = ms;
        out->device = s->device;
    });
}

int sb_store_find_vcf(const sb_store *s, const char *location, size_t len, uint32_t *vcf_id) {
    if (!s || !location || !vcf_id) return SB_EINVAL;
    auto it = s->vcf_by_location.find(std::string(location, len));
    if (it == s->vcf_by_location.end()) return SB_ENOSTORE;
    *vcf_id = it->second;
    return SB_OK;
}

int sb_store_n_samples(const sb_store *s, uint32_t vcf_id, uint32_t *n) {
    if (!s || !n || vcf_id >= s->vcfs.size()) return SB_EINVAL;
    *n = static_cast<uint32_t>(s->vcfs[vcf_id].samples.size());
    return SB_OK;
}

int sb_store_sample_name(const sb_store *s, uint32_t vcf_id, uint32_t i, const char **p, size_t *len) {
    if (!s || !p || !len || vcf_id >= s->vcfs.size() || i >= s->vcfs[vcf_id].samples.size()) return SB_EINVAL;
    *p = s->vcfs[vcf_id].samples[i].data();
    *len = s->vcfs[vcf_id].samples[i].size();
    return SB_OK;
}

namespace {

constexpr int64_t kSplitSize = 10000;  // lambda/splitQuery/lambda_function.py:12

// Request batch (sb_requests_prepare): rows = requests.  A request whose
// slices need none of the order-dependent machinery (variantType query with
// referenceBases 'N', include_details, no boolean break, a non-negative-AC
// VCF, no samples, at most kReqChainSlices slices, no VT_SLOW / general
// record in its window) becomes ONE chain answered by request_eval_kernel;
// every other request is cut into its splitQuery slices (split_query_sync,
// lambda/splitQuery/lambda_function.py:74-110) and answered per slice by the
// query kernels (the batch's query part), its row reduced by request_reduce
// and gathered by request_deliver_kernel.
extern "C++" {  // overloads and templates inside the extern "C" block

// Request sources: the sb_request array, or the same requests as columns
// (sb_request_columns: numeric arrays or scalars, string columns as a
// dictionary + a code per request).  src(i) is request i as an sb_request.
struct AosSrc {
    const sb_request *rq;
    sb_request operator()(size_t i) const { return rq[i]; }
};

struct ColSrc {
    const sb_request_columns &c;
    static sb_str pick(const sb_str *dict, const uint32_t *code, size_t i) {
        return dict ? dict[code ? code[i] : 0u] : sb_str{nullptr, 0};
    }
    sb_request operator()(size_t i) const {
        sb_request r{};
        r.vcf_id = c.vcf_id ? c.vcf_id[i] : c.vcf_id_all;
        r.contig = c.contig ? c.contig[i] : c.contig_all;
        r.start_min = c.start_min[i];
        r.start_max = c.start_max[i];
        r.end_min = c.end_min ? c.end_min[i] : c.end_min_all;
        r.end_max = c.end_max ? c.end_max[i] : c.end_max_all;
        const sb_str ref = pick(c.reference_dict, c.reference_code, i), alt = pick(c.alternate_dict, c.alternate_code, i),
                     vt = pick(c.variant_type_dict, c.variant_type_code, i),
                     sn = pick(c.sample_names_dict, c.sample_names_code, i);
        r.reference_bases = ref.p;
        r.reference_len = ref.len;
        r.alternate_bases = alt.p;
        r.alternate_len = alt.len;
        r.variant_type = vt.p;
        r.variant_type_len = vt.len;
        r.variant_min_length = c.variant_min_length ? c.variant_min_length[i] : c.variant_min_length_all;
        r.variant_max_length = c.variant_max_length ? c.variant_max_length[i] : c.variant_max_length_all;
        r.granularity = c.granularity ? c.granularity[i] : c.granularity_all;
        r.include_details = c.include_details ? c.include_details[i] : c.include_details_all;
        r.include_samples = c.include_samples ? c.include_samples[i] : c.include_samples_all;
        r.selected_samples_only = c.selected_samples_only ? c.selected_samples_only[i] : c.selected_samples_only_all;
        r.strict_variant_type = c.strict_variant_type;
        r.sample_names = sn.p;
        r.sample_names_len = sn.len;
        return r;
    }
};

// variantType strings -> (kind, symbolic-ALT LUT offset), each distinct value once
struct VtResolver {
    sb_store &s;
    std::unordered_map<std::string, std::pair<uint32_t, uint32_t>> map;
    std::vector<uint32_t> lut_all;
    std::pair<uint32_t, uint32_t> get(const char *p, size_t len) {
        const std::string vt = p ? std::string(p, len) : std::string("None");
        auto it = map.find(vt);
        if (it == map.end()) {
            const uint32_t kind = !p                    ? VT_OTHER
                                  : vt == "DEL"        ? VT_DEL
                                  : vt == "INS"        ? VT_INS
                                  : vt == "DUP"        ? VT_DUP
                                  : vt == "DUP:TANDEM" ? VT_DUPT
                                  : vt == "CNV"        ? VT_CNV
                                                       : VT_OTHER;
            const auto lut = sym_lut(s, kind, "<" + vt);
            const uint32_t off = static_cast<uint32_t>(lut_all.size());
            lut_all.insert(lut_all.end(), lut.begin(), lut.end());
            it = map.emplace(vt, std::make_pair(kind, off)).first;
        }
        return it->second;
    }
};

// a handful of distinct values in practice: a pointer cache in front of the map
void resolve_vtypes(VtResolver &V, const AosSrc &src, size_t n, std::vector<uint32_t> &vt_of,
                    std::vector<uint32_t> &lut_of) {
    struct VtEnt {
        const char *p;
        size_t len;
        uint32_t kind, lut;
    };
    std::vector<VtEnt> seen;
    for (size_t i = 0; i < n; ++i) {
        const sb_request &x = src.rq[i];
        if (x.alternate_bases) continue;
        const VtEnt *hit = nullptr;
        for (const VtEnt &e : seen)
            if (e.p == x.variant_type && e.len == x.variant_type_len) {
                hit = &e;
                break;
            }
        if (!hit) {
            const auto kl = V.get(x.variant_type, x.variant_type_len);
            if (seen.size() < 16) seen.push_back(VtEnt{x.variant_type, x.variant_type_len, kl.first, kl.second});
            vt_of[i] = kl.first;
            lut_of[i] = kl.second;
        } else {
            vt_of[i] = hit->kind;
            lut_of[i] = hit->lut;
        }
    }
}

// columns: per dictionary entry, then a table lookup per request
void resolve_vtypes(VtResolver &V, const ColSrc &src, size_t n, std::vector<uint32_t> &vt_of,
                    std::vector<uint32_t> &lut_of) {
    const sb_request_columns &c = src.c;
    std::vector<std::pair<uint32_t, uint32_t>> tab;
    if (c.variant_type_dict)
        for (uint32_t d = 0; d < c.n_variant_type; ++d) tab.push_back(V.get(c.variant_type_dict[d].p, c.variant_type_dict[d].len));
    else
        tab.push_back(V.get(nullptr, 0));
    parallel_for(n, [&](size_t i) {
        const auto &kl = tab[c.variant_type_dict && c.variant_type_code ? c.variant_type_code[i] : 0u];
        vt_of[i] = kl.first;
        lut_of[i] = kl.second;
    });
}

void check_columns(const sb_request_columns &c, size_t n) {
    if (n && (!c.start_min || !c.start_max)) throw Error(SB_EINVAL, "start_min / start_max columns are required");
    auto codes = [&](const char *what, const sb_str *dict, const uint32_t *code, uint32_t nd) {
        if (!dict) {
            if (code) throw Error(SB_EINVAL, std::string(what) + ": codes without a dictionary");
            return;
        }
        if (!nd) throw Error(SB_EINVAL, std::string(what) + ": empty dictionary");
        for (uint32_t d = 0; d < nd; ++d)
            if (!dict[d].p && dict[d].len) throw Error(SB_EINVAL, std::string(what) + ": NULL string with a length");
        if (code)
            for (size_t i = 0; i < n; ++i)
                if (code[i] >= nd) throw Error(SB_EINVAL, std::string(what) + ": code out of range at request " + std::to_string(i));
    };
    codes("reference_bases", c.reference_dict, c.reference_code, c.n_reference);
    codes("alternate_bases", c.alternate_dict, c.alternate_code, c.n_alternate);
    codes("variant_type", c.variant_type_dict, c.variant_type_code, c.n_variant_type);
    codes("sample_names", c.sample_names_dict, c.sample_names_code, c.n_sample_names);
}

// The per-slice part of a request batch: splitQuery's slices of the rows
// with cls[i] == 2, in row order (split_query_sync,
// lambda/splitQuery/lambda_function.py:74-110), planned as one slice batch
// (prepare); seg[w] .. seg[w + 1] = row w's queries.
template <class Src>
void slice_part(sb_batch &B, sb_batch::Req &R, const Src &src, size_t n, const std::vector<uint8_t> &cls,
                std::vector<uint32_t> &seg) {
    sb_store &s = *B.s;
    std::vector<sb_query> qs;
    std::vector<uint32_t> owner;
    std::deque<std::string> regions;  // stable storage for the region strings
    for (size_t i = 0; i < n; ++i) {
        if (cls[i] != 2) continue;
        const sb_request x = src(i);
        const std::string &chrom = s.vcfs[x.vcf_id].segments[x.contig].contig;
        for (int64_t a = x.start_min; a <= x.start_max; a += kSplitSize) {
            const int64_t b = std::min(a + kSplitSize - 1, x.start_max);
            regions.push_back(chrom + ":" + std::to_string(a) + "-" + std::to_string(b));
            sb_query q{};
            q.vcf_id = x.vcf_id;
            q.region = regions.back().data();
            q.region_len = regions.back().size();
            q.end_min = x.end_min;
            q.end_max = x.end_max;
            q.reference_bases = x.reference_bases;
            q.reference_len = x.reference_len;
            q.alternate_bases = x.alternate_bases;
            q.alternate_len = x.alternate_len;
            q.variant_type = x.variant_type;
            q.variant_type_len = x.variant_type_len;
            q.variant_min_length = x.variant_min_length;
            q.variant_max_length = x.variant_max_length;
            q.granularity = x.granularity;
            q.include_details = x.include_details;
            q.include_samples = x.include_samples;
            q.selected_samples_only = x.selected_samples_only;
            q.strict_variant_type = x.strict_variant_type;
            q.sample_names = x.sample_names;
            q.sample_names_len = x.sample_names_len;
            qs.push_back(q);
            owner.push_back(static_cast<uint32_t>(i));
            if (a > INT64_MAX - kSplitSize) break;
        }
    }
    B.no_chains = true;
    if (!qs.empty()) {
        prepare(B, qs.data(), qs.size());
        R.slices = true;
    }
    seg.assign(n + 1, 0);
    for (uint32_t o : owner) ++seg[o + 1];
    for (size_t w = 0; w < n; ++w) seg[w + 1] += seg[w];
}

// the per-slice part's row table, host errors and (general records) the
// inexact-row marks on the device
void upload_slice_part(sb_batch &B, sb_batch::Req &R, const std::vector<uint32_t> &seg, size_t n, hipStream_t st) {
    if (!R.slices) return;
    ReqPool &P = *R.pool;
    std::vector<uint8_t> he(std::max<size_t>(B.nq, 1), 0);
    for (uint32_t q = 0; q < B.nq; ++q) he[q] = B.host_err[q] ? 1 : 0;
    R.sseg = P.get_dev(seg.size() * 4);
    R.sherr = P.get_dev(he.size());
    if (B.gen_grid) {  // general records can make a row's counts wider than int64
        R.wide = P.get_dev(std::max<size_t>(B.nq, 1));
        R.row_flag = P.get_dev(std::max<size_t>(n, 1));
    }
    HIP_OK(hipMemcpyAsync(R.sseg.p, seg.data(), seg.size() * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(R.sherr.p, he.data(), he.size(), hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));  // he / seg are freed by the caller
}

// sb_requests_prepare_columns, planned on the device: when the columns that
// decide the chain test are batch-wide scalars (one VCF, referenceBases 'N',
// alternateBases None, include_details, no boolean break, no samples) the
// host only packs each request into a 32-byte ReqIn (one streaming pass on
// 16 threads: window, END / length bounds, kind and LUT, class) and
// request_plan_kernel forms the runs of 64 rows, resolves every chain's
// candidate range from the coarse index and its hit capacity, and packs the
// descriptors; request_stage_scan_kernel lays the runs' staging regions end
// to end.  One readback (chains, slices, staging total) sizes the buffers.
// Returns false when the columns do not qualify: prepare_requests plans on
// the host.  The per-row numbers come from `get` (PackRow: the columns as
// they are, or the Beacon conversion + shard cut of sb_requests_prepare_beacon
// fused into the same pass); `full()` gives columns the per-slice part can
// read (only called when some row goes per slice).
// The calling thread's planning stream on `device`: concurrent preparers
// (pipelined callers) neither queue behind nor wait for each other's uploads
// and planning kernels on the store stream.  Everything planned on it is
// synchronised before prepare returns.
hipStream_t planning_stream(int device) {
    thread_local std::vector<hipStream_t> per_dev;
    if (per_dev.size() <= static_cast<size_t>(device)) per_dev.resize(device + 1, nullptr);
    hipStream_t &st = per_dev[device];
    if (!st) HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    return st;
}
struct PackRow {
    uint32_t contig;
    uint32_t vt;  // variant_type code
    int64_t smin, smax, emin, emax, vmin, vmax;
};
struct ColRows {
    const sb_request_columns &c;
    PackRow operator()(size_t i) const {
        return PackRow{c.contig ? c.contig[i] : c.contig_all,
                       c.variant_type_dict && c.variant_type_code ? c.variant_type_code[i] : 0u,
                       c.start_min[i],
                       c.start_max[i],
                       c.end_min ? c.end_min[i] : c.end_min_all,
                       c.end_max ? c.end_max[i] : c.end_max_all,
                       c.variant_min_length ? c.variant_min_length[i] : c.variant_min_length_all,
                       c.variant_max_length ? c.variant_max_length[i] : c.variant_max_length_all};
    }
};
template <class Get, class Full>
bool prepare_requests_device(sb_batch &B, const sb_request_columns &c, size_t n, const Get &get, const Full &full) {
    sb_store &s = *B.s;
    if (s.device < 0 || n == 0 || n >= (1u << 31) || c.vcf_id || c.vcf_id_all >= s.vcfs.size()) return false;
    const VcfData &v = s.vcfs[c.vcf_id_all];
    auto single = [](const sb_str *d, const uint32_t *code, uint32_t nd) { return d && (!code || nd == 1); };
    if (!v.nonneg || !single(c.reference_dict, c.reference_code, c.n_reference) ||
        c.reference_dict[0].len != 1 || !c.reference_dict[0].p || c.reference_dict[0].p[0] != 'N')
        return false;
    if (c.alternate_dict && !(single(c.alternate_dict, c.alternate_code, c.n_alternate) && !c.alternate_dict[0].p))
        return false;
    if (c.granularity || c.granularity_all == SB_GRAN_BOOLEAN || c.include_details || !c.include_details_all ||
        c.selected_samples_only || c.selected_samples_only_all || c.include_samples || c.strict_variant_type)
        return false;
    const bool collect = (c.granularity_all == SB_GRAN_RECORD || c.granularity_all == SB_GRAN_AGGREGATED) &&
                         c.include_samples_all;
    if (collect && v.words) return false;
    const bool trace = config().prep_trace;
    auto t_last = std::chrono::steady_clock::now();
    auto tick = [&](const char *what) {
        if (!trace) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[prep-dev] %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    auto R = std::make_unique<sb_batch::Req>();
    R->n_rows = static_cast<uint32_t>(n);
    R->run = kReqRun;
    R->pool = req_pool(s);
    ReqPool &P = *R->pool;
    // variantType dictionary -> (kind, LUT offset)
    VtResolver V{s, {}, {}};
    std::vector<std::pair<uint32_t, uint32_t>> tab;
    if (c.variant_type_dict)
        for (uint32_t d = 0; d < c.n_variant_type; ++d) tab.push_back(V.get(c.variant_type_dict[d].p, c.variant_type_dict[d].len));
    else
        tab.push_back(V.get(nullptr, 0));
    std::vector<uint32_t> &lut_all = V.lut_all;
    lut_all.insert(lut_all.end(), 8, 0u);
    // pack
    const uint32_t vid = c.vcf_id_all;
    const auto &slow_pos = s.seg_slow_pos[vid];
    // one pinned block: the packed requests, then the LUT words, then the
    // planner's three counters (one upload of each, one readback, one sync)
    const size_t lut_at = n * sizeof(ReqIn), cnt_at = (lut_at + lut_all.size() * 4 + 15) & ~size_t(15);
    ReqPool::Pinned pin = P.get_pinned(cnt_at + 32);
    ReqIn *pk = static_cast<ReqIn *>(pin.p);
    std::memcpy(static_cast<char *>(pin.p) + lut_at, lut_all.data(), lut_all.size() * 4);
    std::vector<uint8_t> cls(n, 0);
    std::atomic<bool> any_slices{false};
    parallel_for(n, [&](size_t i) {
        const PackRow x = get(i);
        const uint32_t contig = x.contig;
        const int64_t smin = x.smin, smax = x.smax;
        ReqIn o{0, 0, 0, 0, 0, 0, 0, REQ_NONE};
        if (contig < v.segments.size() && smin <= smax) {  // else bcftools emits nothing / no slice
            const int64_t nsl = (smax - smin) / kSplitSize + 1;
            const auto &kl = tab[x.vt];
            bool chain = smin >= 1 && smax <= 0xfffffffell && nsl <= kReqChainSlices && kl.second < kReqLutMax;
            if (chain && !slow_pos[contig].empty()) {  // a VT_SLOW / general record in the window: per slice
                const auto &sp = slow_pos[contig];
                auto a = std::lower_bound(sp.begin(), sp.end(), static_cast<uint32_t>(smin));
                if (a != sp.end() && *a <= static_cast<uint64_t>(smax)) chain = false;
            }
            if (!chain) {
                o.cls = REQ_SLICES;
                cls[i] = 2;
                any_slices.store(true, std::memory_order_relaxed);
            } else {
                const int64_t emin = x.emin, emax = x.emax;
                const bool end_void = emax < 0 || emin > 0xffffffffll || emin > emax;
                o.first = static_cast<uint32_t>(smin);
                o.last = static_cast<uint32_t>(smax);
                o.e0 = emin < 0 ? 0u : static_cast<uint32_t>(emin);
                o.espan = (emax > 0xffffffffll ? 0xffffffffu : static_cast<uint32_t>(emax)) - o.e0;
                const int64_t vmin = x.vmin;
                const int64_t vmax = x.vmax < 0 ? INT64_MAX : x.vmax;
                const int64_t vl = vmin < 0 ? 0 : vmin, vh = vmax > 255 ? 255 : vmax;
                o.bits = req_bits(vh < vl ? 256u : static_cast<uint32_t>(vl), vh < vl ? 0u : static_cast<uint32_t>(vh - vl),
                                  0u, kl.first, end_void);
                o.seg = v.seg_base + contig;
                o.lut_off = kl.second;
                o.cls = REQ_CHAIN | static_cast<uint32_t>(nsl) << 2;
            }
        }
        pk[i] = o;
    });
    tick("pack");
    std::vector<uint32_t> seg;
    if (any_slices.load()) slice_part(B, *R, ColSrc{full()}, n, cls, seg);
    tick("slices");
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = planning_stream(s.device);
    const uint32_t n_runs = static_cast<uint32_t>((n + kRunRows - 1) / kRunRows);
    const size_t chain_bytes = size_t(n_runs) * kReqRun * sizeof(ReqChain), run_bytes = size_t(n_runs) * sizeof(RowRun);
    // rc: per run {capacity, slices << 32 | chains} (request_plan_kernel), then the 3 counters
    DevMem din = P.get_dev(n * sizeof(ReqIn)), rc = P.get_dev(size_t(n_runs) * 16 + 32);
    R->dchains = P.get_dev(chain_bytes + run_bytes);
    R->runs_at = chain_bytes;
    R->n_runs = n_runs;
    unsigned long long *cnt = reinterpret_cast<unsigned long long *>(rc.as<char>() + size_t(n_runs) * 16);
    R->lut = P.get_dev(lut_all.size() * 4);
    R->n_lut = static_cast<uint32_t>(lut_all.size());
    HIP_OK(hipMemcpyAsync(din.p, pk, n * sizeof(ReqIn), hipMemcpyHostToDevice, st));
    HIP_OK(hipMemcpyAsync(R->lut.p, static_cast<char *>(pin.p) + lut_at, lut_all.size() * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(cnt, 0, 32, st));
    launch_request_plan(s.d, din.as<ReqIn>(), static_cast<uint32_t>(n), R->dchains.as<ReqChain>(),
                        reinterpret_cast<RowRun *>(R->dchains.as<char>() + chain_bytes), rc.as<unsigned long long>(),
                        cnt, st);
    HIP_OK(hipGetLastError());
    unsigned long long *hc = reinterpret_cast<unsigned long long *>(static_cast<char *>(pin.p) + cnt_at);
    HIP_OK(hipMemcpyAsync(hc, cnt, 24, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));  // uploads, planning and the counters: one wait
    R->n_chains = hc[0];
    R->n_chain_slices = hc[1];
    const uint64_t stage_total = hc[2];
    tick("plan");
    P.put_pinned(pin);
    R->din = std::move(din);  // kept: sb_requests_set_replan re-plans from them
    R->rcap = std::move(rc);
    R->n_in = static_cast<uint32_t>(n);
    R->cap = B.cap_total + stage_total;
    R->status = P.get_dev(size_t(n_runs) * 8);
    R->tstatus = P.get_dev(size_t(request_tiles(n_runs)) * 8);
    R->stage = P.get_dev(stage_total * 4);
    R->row_src = P.get_dev(R->slices ? n * 8 : 0);
    upload_slice_part(B, *R, seg, n, st);  // (synchronises when there is a per-slice part)
    tick("upload");
    B.req = std::move(R);
    return true;
}

#ifdef SBEACON_CHECKS
// Plan invariants (the sanitizer build, tests/test_host_sanitizers.py): a
// run's slots hold its chain rows once each (those with candidates first,
// each row field inside the run, each range the one planned for the row and
// inside the (segment, kind) pair's candidates); the staging regions are laid
// end to end and each covers every ALT of its chains' ranges.
void check_request_plan(const sb_store &s, const sb_batch::Req &R, const ReqChain *hc, const std::vector<uint8_t> &cls,
                        const std::vector<uint32_t> &clo, const std::vector<uint32_t> &chi, size_t n) {
    auto fail = [](const std::string &m) { throw Error(SB_EINVAL, "request plan check: " + m); };
    uint64_t stage = 0, chains = 0;
    const uint64_t n_cand = s.h_vc_altpre.empty() ? 0 : s.h_vc_altpre.size() - 1;
    for (size_t r = 0; r < R.runs.size(); ++r) {
        const RowRun &run = R.runs[r];
        if (run.row_hi <= run.row_lo || run.row_hi - run.row_lo > kRunRows || run.row_hi > n) fail("run rows");
        if (run.stage != stage) fail("staging regions not end to end");
        std::vector<uint8_t> seen(kRunRows, 0);
        uint64_t cap = 0;
        bool empty_seen = false;
        uint32_t j = 0;
        for (; j < R.run; ++j) {
            const ReqChain &c = hc[r * R.run + j];
            if (c.first == 0) break;
            const uint32_t row = (c.bits >> 17) & 63u;
            if (run.row_lo + row >= run.row_hi || seen[row]++ || cls[run.row_lo + row] != 1) fail("slot row");
            const size_t i = run.row_lo + row;
            if (c.c_lo != clo[i] || c.c_hi != chi[i] || c.c_hi < c.c_lo || c.c_hi > n_cand) fail("slot range");
            if (c.c_hi > c.c_lo && empty_seen) fail("a chain with candidates after an empty one");
            empty_seen |= c.c_hi == c.c_lo;
            cap += s.h_vc_altpre[c.c_hi] - s.h_vc_altpre[c.c_lo];
            ++chains;
        }
        for (uint32_t k = j; k < R.run; ++k)
            if (hc[r * R.run + k].first != 0) fail("a used slot after an empty one");
        for (uint32_t i = run.row_lo; i < run.row_hi; ++i)
            if (cls[i] == 1 && !seen[i - run.row_lo]) fail("a chain row without a slot");
        stage += cap;
    }
    if (chains != R.n_chains) fail("chain count");
}
#endif

template <class Src>
void prepare_requests(sb_batch &B, const Src &src, size_t n) {
    sb_store &s = *B.s;
    if (n >= (1u << 31)) throw Error(SB_EINVAL, "too many requests");
    auto R = std::make_unique<sb_batch::Req>();
    R->n_rows = static_cast<uint32_t>(n);
    // SBEACON_PREP_TRACE=1: host phase times to stderr (bench diagnostics)
    const bool trace = config().prep_trace;
    auto t_last = std::chrono::steady_clock::now();
    auto tick = [&](const char *what) {
        if (!trace) return;
        const auto t = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[prep] %-10s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t_last).count());
        t_last = t;
    };
    // variantType strings -> kind + LUT
    VtResolver V{s, {}, {}};
    std::vector<uint32_t> vt_of(n, 0u), lut_of(n, 0u);
    resolve_vtypes(V, src, n, vt_of, lut_of);
    std::vector<uint32_t> &lut_all = V.lut_all;
    lut_all.insert(lut_all.end(), 8, 0u);
    tick("vtypes");
    // classify: 0 = no slices, 1 = one chain, 2 = per slice (and the slice
    // count of a chain); the first bad request, if any, is reported
    std::vector<uint8_t> cls(n, 0);
    std::vector<uint32_t> nsl_of(n, 0), clo_of(n, 0), chi_of(n, 0);
    std::atomic<size_t> bad{SIZE_MAX};
    parallel_for(n, [&](size_t i) {
        const sb_request x = src(i);
        if (x.vcf_id >= s.vcfs.size() || (!x.reference_bases && x.reference_len)) {
            size_t b = bad.load(std::memory_order_relaxed);
            while (i < b && !bad.compare_exchange_weak(b, i, std::memory_order_relaxed)) {
            }
            return;
        }
        const VcfData &v = s.vcfs[x.vcf_id];
        if (x.contig >= v.segments.size() || x.start_min > x.start_max) return;  // bcftools emits nothing / no slice
        const int64_t nsl = (x.start_max - x.start_min) / kSplitSize + 1;
        const bool collect = (x.granularity == SB_GRAN_RECORD || x.granularity == SB_GRAN_AGGREGATED) &&
                             (x.selected_samples_only || x.include_samples);
        bool chain = !x.alternate_bases && x.reference_bases && x.reference_len == 1 && x.reference_bases[0] == 'N' &&
                     x.include_details && x.granularity != SB_GRAN_BOOLEAN && !x.selected_samples_only &&
                     !x.strict_variant_type && !(collect && v.words) && v.nonneg && nsl <= kReqChainSlices &&
                     x.start_min >= 1 && x.start_max <= 0xfffffffell && lut_of[i] < kReqLutMax;
        if (chain) {  // a VT_SLOW / general record in the window: per slice
            const auto &sp = s.seg_slow_pos[x.vcf_id][x.contig];
            auto a = std::lower_bound(sp.begin(), sp.end(), static_cast<uint32_t>(x.start_min));
            if (a != sp.end() && *a <= static_cast<uint64_t>(x.start_max)) chain = false;
        }
        cls[i] = chain ? 1 : 2;
        if (chain) {
            nsl_of[i] = static_cast<uint32_t>(nsl);
            // the candidate range from the (kind, segment) coarse index (no
            // END can match: none)
            const VcIndex &vi = v.vc_index[x.contig][vt_of[i]];
            auto cb = [&](uint64_t xx, uint32_t up) -> uint32_t {
                if (xx <= vi.base) return vi.c_lo;
                const uint64_t b = (xx - vi.base) >> vi.shift;
                return b >= vi.n ? vi.c_hi : s.h_vc_bucket[vi.off + b + up];
            };
            const int64_t emin = x.end_min, emax = x.end_max;
            const bool end_void = emax < 0 || emin > 0xffffffffll || emin > emax;
            const uint32_t C0 = cb(static_cast<uint64_t>(x.start_min), 0);
            clo_of[i] = C0;
            chi_of[i] = end_void ? C0 : std::max(C0, cb(static_cast<uint64_t>(x.start_max) + 1, 1));
        }
    });
    if (bad.load() != SIZE_MAX) {
        const size_t i = bad.load();
        const sb_request x = src(i);
        if (x.vcf_id >= s.vcfs.size()) throw Error(SB_ENOSTORE, "request " + std::to_string(i) + ": unknown vcf id");
        throw Error(SB_EINVAL, "request " + std::to_string(i) + ": bad REF");
    }
    tick("classify");
    // the per-slice part: splitQuery's slices of the other requests, in row order
    std::vector<uint32_t> seg;
    slice_part(B, *R, src, n, cls, seg);
    tick("slices");
    // runs of consecutive rows (<= kRunRows rows, R->run chains, every chain
    // starting below position kReqStartPos of the run's candidates), formed
    // greedily in blocks of rows on several threads (a block boundary also
    // ends a run)
    R->run = req_run_max();
    const uint32_t run_max = R->run;
    constexpr uint64_t kReqStartPos = 64ull * kReqStartChunks;
    {
        const size_t nb = std::max<size_t>(1, std::min<size_t>(16, n / 65536));
        std::vector<std::vector<RowRun>> part(nb);
        std::vector<uint64_t> part_chains(nb, 0), part_slices(nb, 0);
        parallel_for(nb, [&](size_t k) {
            const uint32_t r0 = static_cast<uint32_t>(n * k / nb), r1 = static_cast<uint32_t>(n * (k + 1) / nb);
            auto &out = part[k];
            out.reserve((r1 - r0) / 16 + 1);
            RowRun cur{r0, r0, 0, 0, 0, 0, kRunSimple};
            uint32_t c = 0;
            uint64_t sl = 0, tpos = 0;  // the run's candidates so far
            for (uint32_t i = r0; i < r1; ++i) {
                const bool ch = cls[i] == 1;
                const uint32_t need = nsl_of[i];
                if (i > cur.row_lo && (i - cur.row_lo == kRunRows ||
                                       (ch && (cur.c_hi - cur.c_lo == run_max || tpos >= kReqStartPos)))) {
                    cur.row_hi = i;
                    out.push_back(cur);
                    cur = RowRun{i, i, c, c, 0, 0, kRunSimple};
                    tpos = 0;
                }
                if (cls[i] == 2) cur.flags &= ~kRunSimple;  // a row answered per slice: gathered row by row
                if (ch) {
                    cur.c_hi = ++c;
                    cur.n_slots += need;
                    sl += need;
                    tpos += chi_of[i] - clo_of[i];
                }
            }
            if (r1 > r0) {
                cur.row_hi = r1;
                out.push_back(cur);
            }
            part_chains[k] = c;
            part_slices[k] = sl;
        }, 16, 1);
        size_t total = 0;
        for (auto &p : part) total += p.size();
        R->runs.reserve(total);
        uint32_t cbase = 0;
        for (size_t k = 0; k < nb; ++k) {  // chain ordinals made batch-wide
            for (RowRun r : part[k]) {
                r.c_lo += cbase;
                r.c_hi += cbase;
                R->runs.push_back(r);
            }
            cbase += static_cast<uint32_t>(part_chains[k]);
            R->n_chain_slices += part_slices[k];
        }
        R->n_chains = cbase;
    }
    tick("runs");
    // chain descriptors straight into pinned staging, kReqRun slots per run
    // (request_eval_kernel loads a run's slots beside its RowRun), the runs
    // after them: one H2D copy from pinned memory
    const size_t n_runs = R->runs.size(), slots = run_max;
    const size_t chain_bytes = n_runs * slots * sizeof(ReqChain), run_bytes = n_runs * sizeof(RowRun);
    R->pool = req_pool(s);
    const bool host_only = s.device < 0;
    ReqPool::Pinned pin = host_only ? ReqPool::Pinned{} : R->pool->get_pinned(chain_bytes + run_bytes);
    if (host_only) {  // no device: the plan is kept in host memory (R->hplan)
        R->hplan.resize(chain_bytes + run_bytes);
        pin.p = R->hplan.data();
    }
    ReqChain *hc = static_cast<ReqChain *>(pin.p);
    RowRun *hr = reinterpret_cast<RowRun *>(static_cast<char *>(pin.p) + chain_bytes);
    std::vector<uint64_t> rcap(n_runs, 0);  // each run's hit capacity (staging slots)
    parallel_for(n_runs, [&](size_t r) {
        const RowRun &run = R->runs[r];
        ReqChain *out = hc + r * slots;
        uint32_t j = 0;
        uint64_t cap = 0;
        // the chains with candidates first (row order: their hits are staged
        // in slot order), then those without
        for (int pass = 0; pass < 2; ++pass)
        for (uint32_t i = run.row_lo; i < run.row_hi; ++i) {
            if (cls[i] != 1 || (chi_of[i] > clo_of[i]) != (pass == 0)) continue;
            const sb_request x = src(i);
            ReqChain &cd = out[j++];
            cd.first = static_cast<uint32_t>(x.start_min);
            cd.last = static_cast<uint32_t>(x.start_max);
            const int64_t emin = x.end_min, emax = x.end_max;
            const bool end_void = emax < 0 || emin > 0xffffffffll || emin > emax;
            cd.e0 = emin < 0 ? 0u : static_cast<uint32_t>(emin);
            cd.espan = (emax > 0xffffffffll ? 0xffffffffu : static_cast<uint32_t>(emax)) - cd.e0;
            const int64_t vmax = x.variant_max_length < 0 ? INT64_MAX : x.variant_max_length;
            const int64_t vl = x.variant_min_length < 0 ? 0 : x.variant_min_length, vh = vmax > 255 ? 255 : vmax;
            cd.bits = req_bits(vh < vl ? 256u : static_cast<uint32_t>(vl), vh < vl ? 0u : static_cast<uint32_t>(vh - vl),
                               i - run.row_lo, vt_of[i], end_void);
            cd.lut_off = lut_of[i];
            // the candidate range (classify); hit capacity: every ALT of it
            cd.c_lo = clo_of[i];
            cd.c_hi = chi_of[i];
            cap += s.h_vc_altpre[cd.c_hi] - s.h_vc_altpre[cd.c_lo];
        }
        std::memset(static_cast<void *>(out + j), 0, (slots - j) * sizeof(ReqChain));  // empty slots: first == 0
        rcap[r] = cap;
    });
    uint64_t stage_total = 0;  // staging slots: every run's chain hit capacity, back to back
    for (size_t r = 0; r < n_runs; ++r) {
        R->runs[r].stage = stage_total;
        stage_total += rcap[r];
    }
    std::memcpy(static_cast<void *>(hr), R->runs.data(), run_bytes);
    R->cap = B.cap_total + stage_total;
    R->n_runs = static_cast<uint32_t>(n_runs);
    R->runs_at = chain_bytes;
    tick("chains");
#ifdef SBEACON_CHECKS
    check_request_plan(s, *R, hc, cls, clo_of, chi_of, n);
#endif
    if (host_only) {
        B.req = std::move(R);
        return;
    }
    // device buffers (pooled per store: a batch returns them when freed)
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = s.stream;
    ReqPool &P = *R->pool;
    R->dchains = P.get_dev(chain_bytes + run_bytes);
    R->status = P.get_dev(n_runs * 8);
    R->tstatus = P.get_dev(size_t(request_tiles(static_cast<uint32_t>(n_runs))) * 8);
    R->stage = P.get_dev(stage_total * 4);
    R->row_src = P.get_dev(R->slices || std::any_of(R->runs.begin(), R->runs.end(),
                                                    [](const RowRun &r) { return !(r.flags & kRunSimple); })
                               ? size_t(n) * 8 : 0);
    R->lut = P.get_dev(lut_all.size() * 4);
    R->n_lut = static_cast<uint32_t>(lut_all.size());
    if (chain_bytes + run_bytes)
        HIP_OK(hipMemcpyAsync(R->dchains.p, pin.p, chain_bytes + run_bytes, hipMemcpyHostToDevice, st));
    R->runs_at = chain_bytes;
    HIP_OK(hipMemcpyAsync(R->lut.p, lut_all.data(), lut_all.size() * 4, hipMemcpyHostToDevice, st));
    upload_slice_part(B, *R, seg, n, st);
    HIP_OK(hipStreamSynchronize(st));
    R->n_runs = static_cast<uint32_t>(n_runs);
    P.put_pinned(pin);
    tick("upload");
    B.req = std::move(R);
}

}  // extern "C++"

void run_requests(sb_batch &B, void *rows, void *hits, void *row_off, uint64_t rec_base) {
    sb_store &s = *B.s;
    sb_batch::Req &R = *B.req;
    if (s.device < 0) throw Error(SB_EHIP, "the store has no device image (SB_HOST_ONLY)");
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = B.strm();
    mark_run(B);
    if (R.slices) {  // the per-slice part, then its rows (chain rows come out zero; the row kernel writes them)
        run_kernels(B);
        if (R.wide.p) {
            HIP_OK(hipMemsetAsync(R.wide.p, 0, B.nq, st));
            mark_wide(B.gen_big_n.as<uint32_t>(), B.gen_big.as<GenBig>(), B.gen_big_cap, R.wide.as<uint8_t>(), st);
        }
        launch_request_reduce(B.res.as<QRes>(), R.sseg.as<uint32_t>(), R.sherr.as<uint8_t>(), R.wide.as<uint8_t>(),
                              R.n_rows, static_cast<ReqPartial *>(rows), R.row_flag.as<uint8_t>(), st);
    }
    if (!R.err.p) {
        R.err = R.pool->get_dev(16);
        R.err_h = R.pool->get_pinned(16);
        HIP_OK(hipMemsetAsync(R.err.p, 0, 16, st));
    }
    if (R.compact && rec_base + s.n_records > kStageCandMask)
        throw Error(SB_EINVAL, "compact request output: record numbers (rec_base + records) reach 2^29");
    if (R.replan) {  // the planning kernels again, from the resident packed requests (same descriptors, same sizes)
        launch_request_plan(s.d, R.din.as<ReqIn>(), R.n_in, R.dchains.as<ReqChain>(),
                            reinterpret_cast<RowRun *>(R.dchains.as<char>() + R.runs_at), R.rcap.as<unsigned long long>(),
                            reinterpret_cast<unsigned long long *>(R.rcap.as<char>() + size_t(R.n_runs) * 16), st);
        HIP_OK(hipGetLastError());
    }
    DStore d = s.d;
    d.sym_lut = R.lut.as<uint32_t>();
    std::array<hipEvent_t, 2> ev{nullptr, nullptr};
    if (R.time_eval) {
        if (R.eval_used == R.eval_ev.size()) {
            std::array<hipEvent_t, 2> p{};
            for (auto &e : p) HIP_OK(hipEventCreate(&e));
            R.eval_ev.push_back(p);
        }
        ev = R.eval_ev[R.eval_used++];
    }
    launch_request_rows(d, R.dchains.as<ReqChain>(), reinterpret_cast<const RowRun *>(R.dchains.as<char>() + R.runs_at),
                        R.n_runs,
                        R.status.as<unsigned long long>(), R.tstatus.as<unsigned long long>(),
                        R.slices ? B.res.as<QRes>() : nullptr,
                        R.sseg.as<uint32_t>(), B.hoff.as<uint64_t>(), R.sherr.as<uint8_t>(), B.hits.as<uint64_t>(),
                        static_cast<ReqPartial *>(rows), static_cast<uint64_t *>(row_off), R.row_src.as<uint64_t>(),
                        R.stage.as<uint32_t>(), static_cast<uint64_t *>(hits), R.n_rows, rec_base, R.n_lut, R.run,
                        R.err.as<unsigned int>(), R.compact, st, ev[0], ev[1]);
    HIP_OK(hipGetLastError());
}

}  // namespace

int sb_requests_prepare(sb_store *s, const sb_request *r, size_t n, sb_batch **out) {
    return guard([&] {
        if (!s || (!r && n) || !out) throw Error(SB_EINVAL, "NULL argument");
        // request batches do not take the store lock: planning reads the
        // store's host columns only, and each batch owns its device buffers
        // (runs on separate streams overlap on the device)
        auto B = std::make_unique<sb_batch>();
        B->s = s;
        prepare_requests(*B, AosSrc{r}, n);
        store_hold(s);
        *out = B.release();
    });
}

int sb_requests_prepare_columns(sb_store *s, const sb_request_columns *c, size_t n, sb_batch **out) {
    return guard([&] {
        if (!s || (!c && n) || !out) throw Error(SB_EINVAL, "NULL argument");
        static const sb_request_columns kNone{};
        const sb_request_columns &cc = c ? *c : kNone;
        check_columns(cc, n);
        auto B = std::make_unique<sb_batch>();
        B->s = s;
        if (!prepare_requests_device(*B, cc, n, ColRows{cc}, [&]() -> const sb_request_columns & { return cc; }))
            prepare_requests(*B, ColSrc{cc}, n);
        store_hold(s);
        *out = B.release();
    });
}

namespace {
// sb_requests_prepare_beacon: row i's SplitQueryPayload numbers
// (search_variants.py:179-197) cut to the shard core (ShardPlan.slice_runs,
// sbeacon/sharding.py): slice k of [start_min, start_max] starts at
// start_min + 10000 k; the core keeps the slices k0 <= k < k1
struct BeaconRows {
    const sb_beacon_requests &q;
    const sb_shard_core *core;
    std::atomic<size_t> *bad;  // first row with a variant_type code out of range
    // first slice index routed at or past key (kc, kp): ceil((kp - smin) / 10000) clipped to [0, nsl]
    static int64_t first_k(uint32_t c, int64_t smin, int64_t nsl, uint32_t kc, int64_t kp) {
        if (c > kc) return 0;
        if (c < kc) return nsl;
        if (kp <= smin) return 0;
        const uint64_t d = static_cast<uint64_t>(kp) - static_cast<uint64_t>(smin);  // > 0, exact in 64 bits
        const uint64_t need = d / kSplitSize + (d % kSplitSize != 0);
        return need >= static_cast<uint64_t>(nsl) ? nsl : static_cast<int64_t>(need);
    }
    PackRow operator()(size_t i) const {
        // the core is cut in the caller's contig codes (the VCF's contig
        // order: a shard store may hold only some of the contigs), then the
        // code is mapped to the store's contig index
        const int64_t code = q.contig[i];
        const uint32_t cc = code >= 0 && code < UINT32_MAX ? static_cast<uint32_t>(code) : UINT32_MAX;
        uint32_t contig = UINT32_MAX;
        if (!q.contig_map) contig = cc;
        else if (cc < q.n_contig_map) contig = q.contig_map[cc];
        const int64_t s0 = q.start[i], e0 = q.end[i];
        int64_t smin = s0, smax, emin, emax;
        if (q.end2) {
            emin = e0;
            emax = q.end2[i];
        } else {
            emin = s0;
            emax = e0;
        }
        smax = q.start2 ? q.start2[i] : emax;
        constexpr int64_t kLim = int64_t(1) << 62;  // past any contig: a row with no slices (no overflow below)
        auto out = [&](int64_t x) { return x < -kLim || x > kLim; };
        if (out(smin) || out(smax) || out(emin) || out(emax)) {
            contig = UINT32_MAX;
            smin = smax = emin = emax = 0;
        }
        ++smin, ++smax, ++emin, ++emax;
        if (core && smin <= smax) {
            const int64_t nsl = (smax - smin) / kSplitSize + 1;
            const int64_t k0 = core->contig_lo == UINT32_MAX ? nsl : first_k(cc, smin, nsl, core->contig_lo, core->pos_lo);
            const int64_t k1 =
                std::max(k0, core->contig_hi == UINT32_MAX ? nsl : first_k(cc, smin, nsl, core->contig_hi, core->pos_hi));
            const int64_t a = smin + kSplitSize * k0;
            smax = k1 > k0 ? std::min(smax, smin + kSplitSize * k1 - 1) : a - 1;
            smin = a;
        }
        uint32_t vt = 0;
        if (q.variant_type_dict && q.variant_type_code) {
            const int64_t v = q.variant_type_code[i];
            if (v < 0 || v >= q.n_variant_type) {
                size_t cur = bad->load(std::memory_order_relaxed);
                while (i < cur && !bad->compare_exchange_weak(cur, i)) {
                }
            } else {
                vt = static_cast<uint32_t>(v);
            }
        }
        return PackRow{contig, vt, smin, smax, emin, emax,
                       q.variant_min_length ? q.variant_min_length[i] : q.variant_min_length_all,
                       q.variant_max_length ? q.variant_max_length[i] : q.variant_max_length_all};
    }
};

// the same rows as sb_request_columns arrays (the host planner and the
// per-slice part read columns)
struct BeaconColumns {
    std::vector<uint32_t> contig, vt;
    std::vector<int64_t> smin, smax, emin, emax, vmin, vmax;
    sb_request_columns c{};
    BeaconColumns(const sb_request_columns &base, const BeaconRows &rows, size_t n)
        : contig(n), vt(n), smin(n), smax(n), emin(n), emax(n), vmin(n), vmax(n), c(base) {
        parallel_for(n, [&](size_t i) {
            const PackRow x = rows(i);
            contig[i] = x.contig;
            vt[i] = x.vt;
            smin[i] = x.smin;
            smax[i] = x.smax;
            emin[i] = x.emin;
            emax[i] = x.emax;
            vmin[i] = x.vmin;
            vmax[i] = x.vmax;
        });
        c.contig = contig.data();
        c.start_min = smin.data();
        c.start_max = smax.data();
        c.end_min = emin.data();
        c.end_max = emax.data();
        c.variant_min_length = vmin.data();
        c.variant_max_length = vmax.data();
        if (c.variant_type_dict) c.variant_type_code = vt.data();
    }
};
}  // namespace

int sb_requests_prepare_beacon(sb_store *s, const sb_beacon_requests *q, size_t n, const sb_shard_core *core,
                               sb_batch **out) {
    return guard([&] {
        if (!s || !q || !out) throw Error(SB_EINVAL, "NULL argument");
        if (n && (!q->contig || !q->start || !q->end)) throw Error(SB_EINVAL, "contig / start / end columns are required");
        if (q->vcf_id >= s->vcfs.size()) throw Error(SB_EINVAL, "vcf_id out of range");
        if (q->variant_type_dict && !q->n_variant_type) throw Error(SB_EINVAL, "variant_type: empty dictionary");
        if (!q->variant_type_dict && q->variant_type_code) throw Error(SB_EINVAL, "variant_type: codes without a dictionary");
        if (q->reference_bases.len && !q->reference_bases.p) throw Error(SB_EINVAL, "reference_bases: NULL with a length");
        if (q->alternate_bases.len && !q->alternate_bases.p) throw Error(SB_EINVAL, "alternate_bases: NULL with a length");
        // the batch-wide values as columns with scalars (the qualification
        // of the device planner reads these)
        sb_request_columns c{};
        c.vcf_id_all = q->vcf_id;
        c.reference_dict = q->reference_bases.p ? &q->reference_bases : nullptr;
        c.n_reference = c.reference_dict ? 1 : 0;
        c.alternate_dict = q->alternate_bases.p ? &q->alternate_bases : nullptr;
        c.n_alternate = c.alternate_dict ? 1 : 0;
        c.variant_type_dict = q->variant_type_dict;
        c.n_variant_type = q->variant_type_dict ? q->n_variant_type : 0;
        c.variant_min_length_all = q->variant_min_length_all;
        c.variant_max_length_all = q->variant_max_length_all;
        c.granularity_all = q->granularity;
        c.include_details_all = q->include_details;
        std::atomic<size_t> bad{SIZE_MAX};
        const BeaconRows rows{*q, core, &bad};
        auto B = std::make_unique<sb_batch>();
        B->s = s;
        std::unique_ptr<BeaconColumns> cols;
        auto full = [&]() -> const sb_request_columns & {
            if (!cols) cols = std::make_unique<BeaconColumns>(c, rows, n);
            return cols->c;
        };
        auto check_codes = [&] {
            if (bad.load() != SIZE_MAX)
                throw Error(SB_EINVAL, "variant_type: code out of range at request " + std::to_string(bad.load()));
        };
        if (!prepare_requests_device(*B, c, n, rows, full)) {
            const sb_request_columns &m = full();
            check_codes();
            prepare_requests(*B, ColSrc{m}, n);
        }
        check_codes();
        store_hold(s);
        *out = B.release();
    });
}

int sb_requests_run(sb_batch *b, void *dev_rows, void *dev_hits, void *dev_row_off, uint64_t rec_base) {
    return guard([&] {
        if (!b) throw Error(SB_EINVAL, "NULL batch");
        if (!b->req) throw Error(SB_EINVAL, "not a request batch (sb_requests_prepare)");
        if ((!dev_rows && b->req->n_rows) || (!dev_hits && b->req->cap) || !dev_row_off)
            throw Error(SB_EINVAL, "NULL argument");
        std::lock_guard<std::mutex> lk(b->mu);  // this batch's buffers only (see sb_requests_prepare)
        run_requests(*b, dev_rows, dev_hits, dev_row_off, rec_base);
    });
}

int sb_requests_inexact_rows(sb_batch *b, uint8_t *flags) {
    return guard([&] {
        if (!b || (!flags && b->req && b->req->n_rows)) throw Error(SB_EINVAL, "NULL argument");
        if (!b->req) throw Error(SB_EINVAL, "not a request batch (sb_requests_prepare)");
        sb_batch::Req &R = *b->req;
        std::lock_guard<std::mutex> lk(b->mu);
        if (!R.row_flag.p) {
            std::memset(flags, 0, R.n_rows);
            return;
        }
        HIP_OK(hipSetDevice(b->s->device));
        HIP_OK(hipStreamSynchronize(b->strm()));
        HIP_OK(hipMemcpy(flags, R.row_flag.p, R.n_rows, hipMemcpyDeviceToHost));
    });
}

int sb_requests_set_compact(sb_batch *b, int on) {
    return guard([&] {
        if (!b || !b->req) throw Error(SB_EINVAL, "not a request batch");
        if (on && b->req->slices)
            throw Error(SB_EINVAL, "sb_requests_set_compact: the batch answers some rows per slice (wide rows only)");
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->runs_pending) throw Error(SB_EINVAL, "sb_requests_set_compact between a run and its sync");
        b->req->compact = on != 0;
    });
}

int sb_requests_set_replan(sb_batch *b, int on) {
    return guard([&] {
        if (!b || !b->req) throw Error(SB_EINVAL, "not a request batch");
        if (on && !b->req->din.p)
            throw Error(SB_EINVAL, "sb_requests_set_replan: the batch was planned on the host (no packed requests on "
                                   "the device)");
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->runs_pending) throw Error(SB_EINVAL, "sb_requests_set_replan between a run and its sync");
        b->req->replan = on != 0;
    });
}

int sb_requests_time_eval(sb_batch *b, int on) {
    return guard([&] {
        if (!b || !b->req) throw Error(SB_EINVAL, "not a request batch");
        sync(*b);
        b->req->time_eval = on != 0;
        b->req->last_eval_ms = 0;
    });
}

int sb_batch_prepare(sb_store *s, const sb_query *q, size_t nq, sb_batch **out) {
    return guard([&] {
        if (!s || (!q && nq) || !out) throw Error(SB_EINVAL, "NULL argument");
        std::lock_guard<std::mutex> lk(s->mu);
        auto B = std::make_unique<sb_batch>();
        B->s = s;
        prepare(*B, q, nq);
        store_hold(s);
        *out = B.release();
    });
}

int sb_batch_run(sb_batch *b) {
    return guard([&] {
        if (!b) throw Error(SB_EINVAL, "NULL batch");
        if (b->req) throw Error(SB_EINVAL, "a request batch runs through sb_requests_run");
        std::lock_guard<std::mutex> lk(b->s->mu);
        run(*b);
    });
}

int sb_batch_sync(sb_batch *b) {
    return guard([&] {
        if (!b) throw Error(SB_EINVAL, "NULL batch");
        sync(*b);
    });
}

int sb_batch_last_timing(const sb_batch *b, double *total_ms, double *scan_ms, double *bounds_ms) {
    if (!b) return SB_EINVAL;
    // the query step is one launch: bounds are found inside the scan kernel;
    // request batches with eval timing on: scan = request_eval_kernel alone
    if (total_ms) *total_ms = b->last_total_ms;
    if (scan_ms) *scan_ms = (b->req && b->req->time_eval && b->req->last_eval_ms > 0) ? b->req->last_eval_ms
                                                                                      : b->last_total_ms;
    if (bounds_ms) *bounds_ms = 0.0;
    return SB_OK;
}

int sb_batch_get_stats(const sb_batch *b, sb_batch_stats *out) {
    if (!b || !out) return SB_EINVAL;
    out->n_queries = b->nq;
    out->records_scanned = 0;
    for (uint32_t i = 0; i < b->nq && !b->chained.empty(); ++i)
        if (b->chained[i]) out->records_scanned += b->nscan[i];
    out->chained_slices = b->chain_members.size();
    out->chains = b->hchains.size();
    out->cand_loaded = b->cand_loaded;
    out->cand_window = b->cand_window;
    out->cand_unique = b->cand_unique;
    out->hits = b->cap_total;
    out->device_ms = b->last_total_ms;
    if (b->req) {  // request batch: the rows' output capacity and its chains
        out->hits = b->req->cap;
        out->chains = b->req->n_chains;
        out->chained_slices = b->req->n_chain_slices;
    }
    return SB_OK;
}

static_assert(sizeof(ReqPartial) == sizeof(sb_request_partial), "sb_request_partial layout");

int sb_batch_set_owners(sb_batch *b, const uint32_t *owner, size_t nq, uint32_t n_rows) {
    return guard([&] {
        if (!b || (!owner && nq)) throw Error(SB_EINVAL, "NULL argument");
        if (nq != b->nq) throw Error(SB_EINVAL, "owner array length differs from the batch's query count");
        std::vector<uint32_t> seg(size_t(n_rows) + 1, 0);
        for (size_t i = 0; i < nq; ++i) {
            if (owner[i] >= n_rows) throw Error(SB_EINVAL, "owner " + std::to_string(owner[i]) + " >= n_rows");
            if (i && owner[i] < owner[i - 1]) throw Error(SB_EINVAL, "owners must be non-decreasing in query order");
            ++seg[owner[i] + 1];
        }
        for (uint32_t w = 0; w < n_rows; ++w) seg[w + 1] += seg[w];
        // rows as pieces when every chain lies in one row: a chain is listed at
        // its first slice, unchained queries one by one, in query order
        std::vector<uint32_t> chain_of(b->chained.empty() ? 0 : nq, UINT32_MAX);
        bool pieces_ok = true;
        {
            size_t m = 0;
            for (uint32_t c = 0; c < b->hchains.size(); ++c)
                for (uint32_t j = 0; j < b->hchains[c].n; ++j, ++m) {
                    const uint32_t i = b->chain_members[m];
                    chain_of[i] = c;
                    if (owner[i] != owner[b->chain_members[m - j]]) pieces_ok = false;
                }
        }
        std::vector<uint32_t> poff(size_t(n_rows) + 1, 0), piece;
        if (pieces_ok) {
            std::vector<uint8_t> listed(b->hchains.size(), 0);
            for (size_t i = 0; i < nq; ++i) {
                const uint32_t c = chain_of.empty() ? UINT32_MAX : chain_of[i];
                if (c == UINT32_MAX) {
                    piece.push_back(static_cast<uint32_t>(i));
                } else if (!listed[c]) {
                    listed[c] = 1;
                    piece.push_back(c | (1u << 31));
                } else {
                    continue;
                }
                ++poff[owner[i] + 1];
            }
            for (uint32_t w = 0; w < n_rows; ++w) poff[w + 1] += poff[w];
        }
        std::vector<uint8_t> he(std::max<size_t>(nq, 1), 0);
        for (size_t i = 0; i < nq; ++i) he[i] = b->host_err[i] ? 1 : 0;
        std::lock_guard<std::mutex> lk(b->s->mu);
        // per-slice rows off (sb_batch_set_slice_results(0)) needs every chain in
        // one row: a split chain's slices would have no QRes rows to reduce
        if (!pieces_ok && !b->slice_rows)
            throw Error(SB_EINVAL, "a chain of slices spans request rows while per-slice results are off "
                                   "(sb_batch_set_slice_results(b, 1) first)");
        HIP_OK(hipSetDevice(b->s->device));
        hipStream_t st = b->s->stream;
        b->seg.alloc(seg.size() * 4);
        b->herr.alloc(he.size());
        HIP_OK(hipMemcpyAsync(b->seg.p, seg.data(), seg.size() * 4, hipMemcpyHostToDevice, st));
        HIP_OK(hipMemcpyAsync(b->herr.p, he.data(), he.size(), hipMemcpyHostToDevice, st));
        b->row_pieces = pieces_ok;
        if (pieces_ok) {
            b->rowsrc.alloc(std::max<size_t>(n_rows, 1) * 16);
            b->poff.alloc(poff.size() * 4);
            b->piece.alloc(std::max<size_t>(piece.size(), 1) * 4);
            HIP_OK(hipMemcpyAsync(b->poff.p, poff.data(), poff.size() * 4, hipMemcpyHostToDevice, st));
            if (!piece.empty())
                HIP_OK(hipMemcpyAsync(b->piece.p, piece.data(), piece.size() * 4, hipMemcpyHostToDevice, st));
            // each single-piece row's hit region (static for the batch): the
            // deliver gather reads it instead of a per-run rowsrc
            std::vector<uint64_t> rowout(std::max<size_t>(n_rows, 1), ~0ull);
            for (uint32_t w = 0; w < n_rows; ++w) {
                if (poff[w + 1] == poff[w]) rowout[w] = 0;
                if (poff[w + 1] != poff[w] + 1) continue;
                const uint32_t p = piece[poff[w]];
                rowout[w] = (p & (1u << 31)) ? b->hchains[p & ~(1u << 31)].out : b->hq[p].hit_off;
            }
            b->rowout.alloc(rowout.size() * 8);
            HIP_OK(hipMemcpyAsync(b->rowout.p, rowout.data(), rowout.size() * 8, hipMemcpyHostToDevice, st));
        }
        HIP_OK(hipStreamSynchronize(st));
        b->n_rows = n_rows;
    });
}

int sb_batch_reduce_requests(sb_batch *b, void *dev_out) {
    return guard([&] {
        if (!b || (!dev_out && b->n_rows)) throw Error(SB_EINVAL, "NULL argument");
        if (!b->seg.p && b->n_rows) throw Error(SB_EINVAL, "sb_batch_set_owners was not called");
        std::lock_guard<std::mutex> lk(b->s->mu);
        if (!b->row_pieces && b->slice_rows_stale)
            throw Error(SB_EINVAL, "the last run skipped per-slice results that a per-query reduction needs");
        HIP_OK(hipSetDevice(b->s->device));
        if (b->row_pieces)
            launch_row_reduce(b->cpart.as<ReqPartial>(), b->chains.as<ChainDev>(), b->hoff.as<uint64_t>(),
                              b->res.as<QRes>(), b->herr.as<uint8_t>(), b->poff.as<uint32_t>(),
                              b->piece.as<uint32_t>(), b->n_rows, static_cast<ReqPartial *>(dev_out),
                              b->rowsrc.as<ulonglong2>(), b->strm());
        else
            launch_request_reduce(b->res.as<QRes>(), b->seg.as<uint32_t>(), b->herr.as<uint8_t>(), nullptr,
                                  b->n_rows, static_cast<ReqPartial *>(dev_out), nullptr, b->strm());
        HIP_OK(hipGetLastError());
    });
}

int sb_batch_deliver(sb_batch *b, void *dev_rows, void *dev_hits, void *dev_row_off, uint64_t rec_base) {
    if (b && b->row_pieces) {
        return guard([&] {
            if ((!dev_rows && b->n_rows) || (!dev_hits && b->cap_total) || !dev_row_off)
                throw Error(SB_EINVAL, "NULL argument");
            std::lock_guard<std::mutex> lk(b->s->mu);
            HIP_OK(hipSetDevice(b->s->device));
            b->tsum.reserve(hit_scan_words(b->n_rows) * 8);
            b->nvs.reserve(std::max<size_t>(b->n_rows, 1) * 8);
            launch_row_deliver(b->cpart.as<ReqPartial>(), b->chains.as<ChainDev>(), b->hoff.as<uint64_t>(),
                               b->res.as<QRes>(), b->herr.as<uint8_t>(), b->poff.as<uint32_t>(),
                               b->piece.as<uint32_t>(), b->n_rows, static_cast<ReqPartial *>(dev_rows),
                               b->rowsrc.as<ulonglong2>(),
                               config().no_rowout ? nullptr : b->rowout.as<uint64_t>(),  // A/B knob
                               b->nvs.as<int64_t>(), b->tsum.as<uint64_t>(),
                               b->hits.as<uint64_t>(), rec_base, static_cast<uint64_t *>(dev_row_off),
                               static_cast<uint64_t *>(dev_hits), b->strm());
            HIP_OK(hipGetLastError());
        });
    }
    const int rc = sb_batch_reduce_requests(b, dev_rows);
    return rc != SB_OK ? rc : sb_batch_compact_hits(b, dev_rows, dev_hits, dev_row_off, rec_base);
}

int sb_batch_set_stream(sb_batch *b, void *stream) {
    return guard([&] {
        if (!b) throw Error(SB_EINVAL, "NULL batch");
        std::lock_guard<std::mutex> lk(b->s->mu);
        if (b->runs_pending) throw Error(SB_EINVAL, "sb_batch_set_stream between a run and its sync");
        b->stream = static_cast<hipStream_t>(stream);
    });
}

int sb_batch_set_slice_results(sb_batch *b, int on) {
    return guard([&] {
        if (!b) throw Error(SB_EINVAL, "NULL batch");
        std::lock_guard<std::mutex> lk(b->s->mu);
        if (b->runs_pending) throw Error(SB_EINVAL, "sb_batch_set_slice_results between a run and its sync");
        if (!on && !b->hchains.empty() && !b->row_pieces)
            throw Error(SB_EINVAL, "per-slice results are needed unless every chain lies in one request row "
                                   "(sb_batch_set_owners)");
        b->slice_rows = on != 0;
    });
}

int sb_batch_compact_hits(sb_batch *b, const void *dev_rows, void *dev_hits, void *dev_row_off, uint64_t rec_base) {
    return guard([&] {
        if (!b || (!dev_hits && b->cap_total) || !dev_row_off) throw Error(SB_EINVAL, "NULL argument");
        if (!b->seg.p) throw Error(SB_EINVAL, "sb_batch_set_owners was not called");
        std::lock_guard<std::mutex> lk(b->s->mu);
        if (!b->row_pieces && b->slice_rows_stale)
            throw Error(SB_EINVAL, "the last run skipped per-slice results that per-query hit lists need");
        HIP_OK(hipSetDevice(b->s->device));
        hipStream_t st = b->strm();
        if (b->row_pieces) {  // over rows and pieces (chains as one contiguous copy each)
            const ReqPartial *rows = static_cast<const ReqPartial *>(dev_rows);
            if (!rows) {  // (the reduction also leaves rowsrc for the gather)
                b->rows_scratch.reserve(std::max<size_t>(b->n_rows, 1) * sizeof(ReqPartial));
                launch_row_reduce(b->cpart.as<ReqPartial>(), b->chains.as<ChainDev>(), b->hoff.as<uint64_t>(),
                                  b->res.as<QRes>(), b->herr.as<uint8_t>(), b->poff.as<uint32_t>(),
                                  b->piece.as<uint32_t>(), b->n_rows, b->rows_scratch.as<ReqPartial>(),
                                  b->rowsrc.as<ulonglong2>(), st);
                rows = b->rows_scratch.as<ReqPartial>();
            }
            b->tsum.reserve(hit_scan_words(b->n_rows) * 8);
            launch_row_hit_lists(rows, b->rowsrc.as<ulonglong2>(), b->poff.as<uint32_t>(), b->piece.as<uint32_t>(),
                                 b->n_rows, b->chains.as<ChainDev>(), b->cpart.as<ReqPartial>(), b->res.as<QRes>(),
                                 b->hoff.as<uint64_t>(), b->hits.as<uint64_t>(), rec_base, b->tsum.as<uint64_t>(),
                                 static_cast<uint64_t *>(dev_row_off), static_cast<uint64_t *>(dev_hits), st);
        } else {  // over queries
            b->tsum.reserve(hit_scan_words(b->nq) * 8);
            b->dense.reserve((size_t(b->nq) + 1) * 8);
            const uint64_t *src = src_offsets(*b, st);
            launch_hit_lists(b->res.as<QRes>(), b->nq, src, b->hits.as<uint64_t>(), rec_base, b->seg.as<uint32_t>(),
                             b->n_rows, b->tsum.as<uint64_t>(), b->dense.as<uint64_t>(),
                             static_cast<uint64_t *>(dev_hits), static_cast<uint64_t *>(dev_row_off), st);
        }
        HIP_OK(hipGetLastError());
    });
}

int sb_batch_fetch(sb_batch *b, sb_result_set **out) {
    return guard([&] {
        if (!b || !out) throw Error(SB_EINVAL, "NULL argument");
        std::lock_guard<std::mutex> lk(b->s->mu);
        *out = fetch(*b);
    });
}

void sb_batch_free(sb_batch *b) {
    if (!b) return;
    sb_store *s = b->s;
    if (s->device >= 0) (void)hipSetDevice(s->device);
    delete b;
    store_release(s);  // every batch handed out holds its store
}

int sb_query_batch(sb_store *s, const sb_query *q, size_t nq, uint32_t flags, sb_result_set **out) {
    (void)flags;
    return guard([&] {
        if (!s || (!q && nq) || !out) throw Error(SB_EINVAL, "NULL argument");
        std::lock_guard<std::mutex> lk(s->mu);
        static const bool trace = config().wire_trace;  // phase times (bench diagnostics)
        auto t0 = std::chrono::steady_clock::now();
        auto tick = [&](const char *what) {
            if (!trace) return;
            const auto t = std::chrono::steady_clock::now();
            std::fprintf(stderr, "[query] %-8s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
            t0 = t;
        };
        sb_batch B;
        B.s = s;
        prepare(B, q, nq);
        tick("prepare");
        run(B);
        tick("run");
        *out = fetch(B);
        tick("fetch");
    });
}

int sb_result_get(const sb_result_set *r, size_t i, sb_result_view *out) {
    if (!r || !out || i >= r->res.size()) return SB_EINVAL;
    std::call_once(r->tmp_once, [r] {  // the record / ALT views of every hit
        const size_t total = r->hit.size();
        r->tmp_rec.resize(total);
        r->tmp_alt.resize(total);
        parallel_for(total, [r](size_t h) {
            r->tmp_rec[h] = static_cast<uint32_t>(r->hit[h]);
            r->tmp_alt[h] = static_cast<uint32_t>(r->hit[h] >> kHitAltShift);
        }, 16, 1 << 16);
    });
    return sb::result_view(r, i, out);
}
}  // extern "C"

namespace sb {
// sb_result_get without the hit views (the wire formatter)
int result_view(const sb_result_set *r, size_t i, sb_result_view *out) {
    if (!r || !out || i >= r->res.size()) return SB_EINVAL;
    const QRes &q = r->res[i];
    out->error = q.error;
    out->exists = q.exists;
    out->call_count = q.call_count;
    out->all_alleles_count = q.all_alleles_count;
    const uint64_t a = r->dense_off[i], b = r->dense_off[i + 1];
    out->n_variants = q.error ? 0 : b - a;
    const bool views = r->tmp_rec.size() == r->hit.size();  // sb_result_get split them
    out->hit_record = views ? r->tmp_rec.data() + a : nullptr;
    out->hit_alt = views ? r->tmp_alt.data() + a : nullptr;
    out->n_sample_indices = r->sidx[i].size();
    out->sample_indices = r->sidx[i].data();
    out->big_limbs = 0;
    out->_pad = 0;
    out->big_call_count = out->big_all_alleles_count = nullptr;
    if (!r->big.empty()) {
        auto it = r->big.find(static_cast<uint32_t>(i));
        if (it != r->big.end() && !q.error) {
            out->big_limbs = r->big_limbs;
            out->big_call_count = it->second.data();
            out->big_all_alleles_count = it->second.data() + r->big_limbs;
        }
    }
    return SB_OK;
}
}  // namespace sb

extern "C" {
int sb_result_get_all(const sb_result_set *r, sb_result_view *out, size_t n) {
    if (!r || (!out && n) || n > r->res.size()) return SB_EINVAL;
    for (size_t i = 0; i < n; ++i) sb_result_get(r, i, out + i);
    return SB_OK;
}

namespace {
// f'{chrom}\t{position}\t{reference}\t{alts[i]}\t{variant_type}' (search_variants.py:210)
void append_variant(std::string &o, const sb_store &s, const std::string &chrom, uint64_t hit) {
    const uint32_t rec = static_cast<uint32_t>(hit);
    const uint32_t k = static_cast<uint32_t>(hit >> kHitAltShift);
    char num[16];
    o += chrom;
    o.push_back('\t');
    {  // decimal POS (no snprintf: millions of variant strings per batch)
        uint32_t v = s.h_pos[rec];
        char *e = num + sizeof num, *q = e;
        do {
            *--q = static_cast<char>('0' + v % 10);
            v /= 10;
        } while (v);
        o.append(q, static_cast<size_t>(e - q));
    }
    o.push_back('\t');
    o.append(reinterpret_cast<const char *>(s.h_blob.data() + s.h_ref_off[rec]), s.h_end[rec] - s.h_pos[rec] + 1);
    o.push_back('\t');
    if (k == 0) {
        o.append(reinterpret_cast<const char *>(s.h_blob.data() + s.h_a0_off[rec]), s.h_a0_len[rec]);
    } else {
        const uint32_t x = s.h_x_lo[rec] + k - 1;
        o.append(reinterpret_cast<const char *>(s.h_blob.data() + s.h_x_off[x]), s.h_x_len[x]);
    }
    o.push_back('\t');
    o += s.vt.items[s.h_vt[rec]];
}
}  // namespace

}  // extern "C"

namespace sb {
// The wire formatter's per-store cache: for every ALT row (record rec's ALT
// 0 = row rec, its extra ALT x = row n_records + x) the JSON-escaped tail of
// its variant string, "\\t" POS "\\t" REF "\\t" ALT "\\t" VT
// (search_variants.py:210), built once on first use (parallel): a response's
// variant list is then its chrom and one copy per hit.  A row whose text is
// not UTF-8 has no entry (bad): its events take the Python handler.
struct VarText {
    std::vector<uint64_t> off;  // rows + 1
    std::vector<char> text;
    std::vector<uint8_t> bad;
};

const VarText &var_text(sb_store &s) {
    std::call_once(s.var_text_once, [&] {
        auto V = std::make_shared<VarText>();
        const size_t nr = s.n_records, rows = nr + s.n_extra;
        std::vector<std::string> vt(s.vt.items.size());
        std::vector<uint8_t> vt_bad(vt.size(), 0);
        for (size_t k = 0; k < vt.size(); ++k)
            if (!json_escape_append(vt[k], s.vt.items[k].data(), s.vt.items[k].size())) vt_bad[k] = 1;
        std::vector<uint32_t> xrec(s.n_extra);  // extra ALT row -> its record
        for (size_t r = 0; r < nr; ++r) {
            const uint32_t nx = (r + 1 < nr ? s.h_x_lo[r + 1] : static_cast<uint32_t>(s.n_extra)) - s.h_x_lo[r];
            for (uint32_t j = 0; j < nx; ++j) xrec[s.h_x_lo[r] + j] = static_cast<uint32_t>(r);
        }
        const char *blob = reinterpret_cast<const char *>(s.h_blob.data());
        auto parts = [&](size_t row, const char *&alt, size_t &al, uint32_t &rec) {
            if (row < nr) {
                rec = static_cast<uint32_t>(row);
                alt = blob + s.h_a0_off[rec];
                al = s.h_a0_len[rec];
            } else {
                const size_t x = row - nr;
                rec = xrec[x];
                alt = blob + s.h_x_off[x];
                al = s.h_x_len[x];
            }
        };
        // pass 1: each row's escaped length (0 + bad mark where not UTF-8)
        std::vector<uint32_t> len(rows, 0);
        V->bad.assign(rows, 0);
        parallel_for(rows, [&](size_t row) {
            const char *alt;
            size_t al;
            uint32_t rec;
            parts(row, alt, al, rec);
            const size_t rl = s.h_end[rec] - s.h_pos[rec] + 1;
            thread_local std::string tmp;
            tmp.clear();
            bool ok = json_escape_append(tmp, blob + s.h_ref_off[rec], rl) && json_escape_append(tmp, alt, al) &&
                      !vt_bad[s.h_vt[rec]];
            uint32_t digits = 1;
            for (uint32_t v = s.h_pos[rec]; v >= 10; v /= 10) ++digits;
            if (!ok) V->bad[row] = 1;
            else len[row] = static_cast<uint32_t>(8 + digits + tmp.size() + vt[s.h_vt[rec]].size());
        });
        V->off.assign(rows + 1, 0);
        for (size_t r = 0; r < rows; ++r) V->off[r + 1] = V->off[r] + len[r];
        V->text.resize(V->off[rows]);
        // pass 2: the text
        parallel_for(rows, [&](size_t row) {
            if (V->bad[row]) return;
            const char *alt;
            size_t al;
            uint32_t rec;
            parts(row, alt, al, rec);
            char *p = V->text.data() + V->off[row];
            *p++ = '\\';
            *p++ = 't';
            char num[16];
            uint32_t v = s.h_pos[rec];
            char *e = num + sizeof num, *q = e;
            do {
                *--q = static_cast<char>('0' + v % 10);
                v /= 10;
            } while (v);
            std::memcpy(p, q, static_cast<size_t>(e - q));
            p += e - q;
            *p++ = '\\';
            *p++ = 't';
            p = json_escape_to(p, blob + s.h_ref_off[rec], s.h_end[rec] - s.h_pos[rec] + 1);
            *p++ = '\\';
            *p++ = 't';
            p = json_escape_to(p, alt, al);
            *p++ = '\\';
            *p++ = 't';
            const std::string &t = vt[s.h_vt[rec]];
            std::memcpy(p, t.data(), t.size());
        });
        s.var_text = V;
    });
    return *static_cast<const VarText *>(s.var_text.get());
}

void result_prepare_json(sb_result_set *r) {
    if (!r->vt_json.empty()) return;
    (void)var_text(*r->s);
    const auto &items = r->s->vt.items;
    r->vt_json.resize(items.size());
    for (size_t k = 0; k < items.size(); ++k)
        if (!json_escape_append(r->vt_json[k], items[k].data(), items[k].size())) r->vt_json[k] = std::string("\x01");
    // sample names: the reference joins the selected names with ',' and the
    // response lists the pieces of splitting that text on ',' -- per name,
    // the pieces of the name split on ','
    r->names_json.assign(r->s->vcfs.size(), {});
    std::vector<uint8_t> need(r->s->vcfs.size(), 0);
    for (size_t i = 0; i < r->res.size(); ++i)
        if (!r->sidx[i].empty()) need[r->vcf_of[i]] = 1;
    for (size_t f = 0; f < need.size(); ++f) {
        if (!need[f]) continue;
        const auto &names = r->s->vcfs[f].samples;
        auto &out = r->names_json[f];
        out.resize(names.size());
        for (size_t h = 0; h < names.size(); ++h) {
            const std::string &nm = names[h];
            std::string &o = out[h];
            size_t a = 0;
            for (size_t k = 0; k <= nm.size(); ++k)
                if (k == nm.size() || nm[k] == ',') {
                    if (a) o += ", ";
                    o.push_back('"');
                    if (!json_escape_append(o, nm.data() + a, k - a)) {
                        o = std::string("\x01");
                        break;
                    }
                    o.push_back('"');
                    a = k + 1;
                }
        }
    }
}

namespace {
// query i's chrom, JSON-escaped (in buf when it fits); false: not UTF-8
struct ChromText {
    char buf[256];
    std::string lng;
    const char *p = nullptr;
    size_t n = 0;
    bool make(const std::string &cs) {
        if (6 * cs.size() <= sizeof buf) {
            char *e = json_escape_to(buf, cs.data(), cs.size());
            if (!e) return false;
            p = buf;
            n = static_cast<size_t>(e - buf);
        } else {
            if (!json_escape_append(lng, cs.data(), cs.size())) return false;
            p = lng.data();
            n = lng.size();
        }
        return true;
    }
};
uint64_t variant_row(const sb_store &s, uint64_t hit) {
    const uint32_t rec = static_cast<uint32_t>(hit);
    const uint32_t k = static_cast<uint32_t>(hit >> kHitAltShift);
    return k == 0 ? rec : s.n_records + s.h_x_lo[rec] + k - 1;
}
}  // namespace

bool result_variants_len(const sb_result_set *r, size_t i, size_t *need) {
    const sb_store &s = *r->s;
    const uint64_t a = r->dense_off[i], b = r->res[i].error ? a : r->dense_off[i + 1];
    *need = 0;
    if (b == a) return true;
    const VarText &V = *static_cast<const VarText *>(s.var_text.get());  // result_prepare_json built it
    ChromText c;
    if (!c.make(r->chrom[i])) return false;
    size_t n = 0;
    for (uint64_t h = a; h < b; ++h) {
        const uint64_t row = variant_row(s, r->hit[h]);
        if (V.bad[row]) return false;  // not UTF-8: the Python handler
        n += 4 + c.n + (V.off[row + 1] - V.off[row]);
    }
    *need = n - 2;  // no ", " before the first
    return true;
}

void result_variants_write(const sb_result_set *r, size_t i, char *p) {
    const sb_store &s = *r->s;
    const uint64_t a = r->dense_off[i], b = r->res[i].error ? a : r->dense_off[i + 1];
    if (b == a) return;
    const VarText &V = *static_cast<const VarText *>(s.var_text.get());
    ChromText c;
    c.make(r->chrom[i]);  // (result_variants_len accepted it)
    for (uint64_t h = a; h < b; ++h) {
        const uint64_t row = variant_row(s, r->hit[h]);
        if (h > a) {
            *p++ = ',';
            *p++ = ' ';
        }
        *p++ = '"';
        std::memcpy(p, c.p, c.n);
        p += c.n;
        const size_t n = V.off[row + 1] - V.off[row];
        std::memcpy(p, V.text.data() + V.off[row], n);
        p += n;
        *p++ = '"';
    }
}

bool result_variants_json(const sb_result_set *r, size_t i, std::string &o) {
    size_t need;
    if (!result_variants_len(r, i, &need)) return false;
    const size_t o0 = o.size();
    o.resize(o0 + need);
    result_variants_write(r, i, &o[o0]);
    return true;
}

bool result_sample_names_len(const sb_result_set *r, size_t i, size_t *need) {
    const auto &ix = r->sidx[i];
    const auto &nj = r->names_json[r->vcf_of[i]];
    size_t n = ix.empty() ? 0 : 2 * (ix.size() - 1);
    for (size_t j = 0; j < ix.size(); ++j) {
        const std::string &x = nj[r->samples_variant[i] ? r->emitted[i][ix[j]] : ix[j]];
        if (x.size() == 1 && x[0] == '\x01') return false;  // not UTF-8
        n += x.size();
    }
    *need = n;
    return true;
}

void result_sample_names_write(const sb_result_set *r, size_t i, char *p) {
    const auto &ix = r->sidx[i];
    const auto &nj = r->names_json[r->vcf_of[i]];
    for (size_t j = 0; j < ix.size(); ++j) {
        const std::string &x = nj[r->samples_variant[i] ? r->emitted[i][ix[j]] : ix[j]];
        if (j) {
            *p++ = ',';
            *p++ = ' ';
        }
        std::memcpy(p, x.data(), x.size());
        p += x.size();
    }
}

bool result_sample_names_json(const sb_result_set *r, size_t i, std::string &o) {
    size_t need;
    if (!result_sample_names_len(r, i, &need)) return false;
    const size_t o0 = o.size();
    o.resize(o0 + need);
    result_sample_names_write(r, i, &o[o0]);
    return true;
}
}  // namespace sb

extern "C" {

int sb_result_variants_text(sb_result_set *r, size_t i, const char **p, size_t *len) {
    if (!r || !p || !len || i >= r->res.size()) return SB_EINVAL;
    if (!r->vbuilt[i]) {
        std::string &o = r->vtext[i];
        const uint64_t a = r->dense_off[i], b = r->res[i].error ? a : r->dense_off[i + 1];
        for (uint64_t h = a; h < b; ++h) {
            if (h > a) o.push_back('\n');
            append_variant(o, *r->s, r->chrom[i], r->hit[h]);
        }
        r->vbuilt[i] = 1;
    }
    *p = r->vtext[i].data();
    *len = r->vtext[i].size();
    return SB_OK;
}

int sb_result_distinct_variants(sb_result_set *r, const uint32_t *queries, size_t n, const char **p, size_t *len,
                                uint64_t *count) {
    return guard([&] {
        if (!r || !p || !len || !count || (n && !queries)) throw Error(SB_EINVAL, "NULL argument");
        // (chrom string, record, alt) first, then the formatted strings: two
        // records (or two VCFs naming the contig alike) can print the same line
        std::unordered_map<std::string, uint32_t> chrom_id;
        std::unordered_set<uint64_t> seen_hit;
        std::unordered_set<std::string> seen_text;
        std::string &o = r->distinct;
        o.clear();
        uint64_t c = 0;
        std::string line;
        for (size_t j = 0; j < n; ++j) {
            const uint32_t i = queries[j];
            if (i >= r->res.size()) throw Error(SB_EINVAL, "query index out of range");
            if (r->res[i].error) continue;
            const uint32_t cid = chrom_id.emplace(r->chrom[i], static_cast<uint32_t>(chrom_id.size())).first->second;
            for (uint64_t h = r->dense_off[i]; h < r->dense_off[i + 1]; ++h) {
                // hit = rec | alt << kHitAltShift; rec < 2^32, alt < 64: fold the chrom id above both
                const uint64_t key = r->hit[h] ^ (static_cast<uint64_t>(cid) << 40);
                if (!seen_hit.insert(key).second) continue;
                line.clear();
                append_variant(line, *r->s, r->chrom[i], r->hit[h]);
                if (!seen_text.insert(line).second) continue;
                if (c++) o.push_back('\n');
                o += line;
            }
        }
        *p = o.data();
        *len = o.size();
        *count = c;
    });
}

int sb_result_sample_names_text(sb_result_set *r, size_t i, const char **p, size_t *len) {
    if (!r || !p || !len || i >= r->res.size()) return SB_EINVAL;
    if (!r->nbuilt[i]) {
        std::string &o = r->ntext[i];
        const VcfData &v = r->s->vcfs[r->vcf_of[i]];
        const auto &ix = r->sidx[i];
        for (size_t j = 0; j < ix.size(); ++j) {
            const uint32_t h = r->samples_variant[i] ? r->emitted[i][ix[j]] : ix[j];
            if (j) o.push_back(',');
            o += v.samples[h];
        }
        r->nbuilt[i] = 1;
    }
    *p = r->ntext[i].data();
    *len = r->ntext[i].size();
    return SB_OK;
}

int sb_result_stats(const sb_result_set *r, sb_batch_stats *out) {
    if (!r || !out) return SB_EINVAL;
    *out = r->stats;
    return SB_OK;
}

void sb_result_free(sb_result_set *r) { delete r; }

}  // extern "C"
