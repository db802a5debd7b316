// internal.hpp — internals shared by the C ABI's translation units
// (api.cpp: store, builder, query batches; requests.cpp: request batches;
// summarise.cpp: summariseSlice and duplicateVariantSearch; results.cpp:
// result sets and their text).  Included by those files only.
#pragma once

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
inline ParsedRegion parse_region(const char *p, size_t n) {
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

inline bool starts(const std::string &s, const char *pre) { return s.compare(0, strlen(pre), pre) == 0; }

// Host-side evaluation of the symbolic-ALT predicates of :101-166 for one
// variantType string over the store's symbolic dictionary.
inline std::vector<uint32_t> sym_lut(const sb_store &s, uint32_t kind, const std::string &vprefix) {
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

sb_store *store_hold(sb_store *s);
void store_release(sb_store *s);

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

}  // namespace sb

using namespace sb;

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

inline std::shared_ptr<ReqPool> req_pool(sb_store &s) {
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
        bool plan_fused = false;  // the last pass planned inside request_eval_kernel (sb_requests_plan_fused)
        uint64_t stage_stride = 0;  // staging slots per run when fixed (re-planning skips the staging scan); 0: packed
        int compact = 0;  // sb_requests_set_compact: 0 wide, SB_COMPACT_ALL, SB_COMPACT_HITS
        // request_eval_kernel's invariant word (sticky; checked at sync: SB_EINTERNAL)
        DevMem err;
        ReqPool::Pinned err_h;
        // rows whose counts are not exact in int64 (sb_requests_inexact_rows):
        // per-slice wide marks + one flag per row (batches with general records)
        DevMem wide, row_flag;
        // compact outputs' escapes (devtypes.hpp ReqEsc): the wide rows of
        // escaped rows (SB_COMPACT_ALL; also the per-slice part's reduced rows)
        // and the ALT index of escaped hit labels; escapes = what the passes
        // since the last sync wrote (bit 0 rows, bit 1 hits)
        DevMem xrows, xlab;
        uint32_t escapes = 0;
        std::vector<char> hplan;  // host-only stores: the descriptors + runs (as dchains would hold them)
        size_t runs_at = 0;
        uint32_t run = kReqRun;        // chain slots per run (request_eval_kernel: one lane each)
        std::shared_ptr<ReqPool> pool;  // where the device buffers go back when the batch is freed
        bool slices = false;           // some rows answered per slice (the batch's query part)
        void give_back() {
            for (DevMem *m : {&dchains, &status, &tstatus, &stage, &row_src, &lut, &sseg, &sherr, &wide, &row_flag, &din,
                              &rcap, &err, &xrows, &xlab})
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
    // a second stream for the sample-free groups of a batch that also has
    // sample-path groups (run_kernels): fork / join events on the batch stream
    hipStream_t aux = nullptr;
    std::array<hipEvent_t, 2> fork{};
    size_t runs_pending = 0;
    float last_total_ms = 0;
    std::mutex mu;  // request batches: one pass at a time per batch
    ~sb_batch() {
        for (auto e : ev)
            if (e) (void)hipEventDestroy(e);
        if ((req && req->pool) || pool) (void)hipStreamSynchronize(strm());  // a pass may still be in flight
        if (aux) {  // (its work is joined into strm() by every run; waited for again here)
            (void)hipStreamSynchronize(aux);
            (void)hipStreamDestroy(aux);
        }
        for (auto e : fork)
            if (e) (void)hipEventDestroy(e);
        if (req && req->pool) req->give_back();
        if (pool)
            for (DevMem *m : {&q, &hoff, &qbytes, &subsets, &lut, &res, &hits, &samples_out, &chains, &runs, &corig,
                              &srcoff, &cpart, &gen_work, &gen_scratch, &gen_big_n, &gen_big, &gen_limbs})
                if (m->p) pool->put_dev(std::move(*m));
    }
};

// a batch buffer: from the batch's pool when it has one
inline void palloc(sb_batch &B, DevMem &m, size_t n) {
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
namespace sb {
// the query batch (api.cpp), shared with the request batches (requests.cpp)
void prepare(sb_batch &B, const sb_query *qs, size_t nq);
void mark_run(sb_batch &B);
void run_kernels(sb_batch &B);
void sync(sb_batch &B);
}  // namespace sb
