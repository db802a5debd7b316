// requests.cpp — request batches (sb_requests_*): one row per beacon
// request, answered by the request pass (query_kernels.hip).
#include "internal.hpp"

extern "C" {

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
// a packed request written with non-temporal stores: the pinned block is
// read by the DMA engine, never again by this CPU, so its lines need no
// read-for-ownership (a third less host memory traffic in the pack)
inline void stream_store(ReqIn *dst, const ReqIn &v) {
    typedef long long v2i __attribute__((vector_size(16)));
    const v2i *src = reinterpret_cast<const v2i *>(&v);
    v2i *d = reinterpret_cast<v2i *>(dst);
    __builtin_nontemporal_store(src[0], d);
    __builtin_nontemporal_store(src[1], d + 1);
}
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
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = planning_stream(s.device);
    DevMem din = P.get_dev(n * sizeof(ReqIn));
    // an exception past the first queued upload leaves by way of a stream
    // wait: no DMA still reading the pinned block or writing `din` when they
    // go back to the pool (on the normal path the stream is idle by then)
    struct Drain {
        hipStream_t s;
        ~Drain() { (void)hipStreamSynchronize(s); }
    } drain{st};
    auto pack_row = [&](size_t i) {
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
        stream_store(pk + i, o);
    };
    // packed in pieces, each piece's upload queued as soon as it is packed:
    // the DMA of piece j (pinned source, the planning stream) runs while the
    // host packs piece j + 1, so the upload hides behind the pack but for
    // the last piece
    const size_t pieces = n >= (size_t(1) << 18) ? 4 : 1;
    for (size_t j = 0; j < pieces; ++j) {
        const size_t a = n * j / pieces, b = n * (j + 1) / pieces;
        const size_t m = b - a, parts = std::min<size_t>(16, std::max<size_t>(1, m / 4096));
        parallel_for(
            parts,
            [&](size_t k) {
                for (size_t i = a + m * k / parts, e = a + m * (k + 1) / parts; i < e; ++i) pack_row(i);
                __builtin_ia32_sfence();  // this thread's streaming stores drained before the upload is queued
            },
            16, 1);
        HIP_OK(hipMemcpyAsync(din.as<char>() + a * sizeof(ReqIn), pk + a, (b - a) * sizeof(ReqIn),
                              hipMemcpyHostToDevice, st));
    }
    tick("pack");
    std::vector<uint32_t> seg;
    if (any_slices.load()) slice_part(B, *R, ColSrc{full()}, n, cls, seg);
    tick("slices");
    const uint32_t n_runs = static_cast<uint32_t>((n + kRunRows - 1) / kRunRows);
    const size_t chain_bytes = size_t(n_runs) * kReqRun * sizeof(ReqChain), run_bytes = size_t(n_runs) * sizeof(RowRun);
    // rc: per run {capacity, slices << 32 | chains} (request_plan_kernel), then the 3 counters
    DevMem rc = P.get_dev(request_plan_words(n_runs) * 8);
    R->dchains = P.get_dev(chain_bytes + run_bytes);
    R->runs_at = chain_bytes;
    R->n_runs = n_runs;
    unsigned long long *cnt = reinterpret_cast<unsigned long long *>(rc.as<char>() + size_t(n_runs) * 16);
    R->lut = P.get_dev(lut_all.size() * 4);
    R->n_lut = static_cast<uint32_t>(lut_all.size());
    HIP_OK(hipMemcpyAsync(R->lut.p, static_cast<char *>(pin.p) + lut_at, lut_all.size() * 4, hipMemcpyHostToDevice, st));
    HIP_OK(hipMemsetAsync(cnt, 0, 32, st));
    launch_request_plan(s.d, din.as<ReqIn>(), static_cast<uint32_t>(n), R->dchains.as<ReqChain>(),
                        reinterpret_cast<RowRun *>(R->dchains.as<char>() + chain_bytes), rc.as<unsigned long long>(),
                        cnt, st);
    HIP_OK(hipGetLastError());
    unsigned long long *hc = reinterpret_cast<unsigned long long *>(static_cast<char *>(pin.p) + cnt_at);
    HIP_OK(hipMemcpyAsync(hc, cnt, 32, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));  // uploads, planning and the counters: one wait
    R->n_chains = hc[0];
    R->n_chain_slices = hc[1];
    const uint64_t stage_total = hc[2];
    // staging at a fixed stride per run (the largest run capacity) when that
    // costs at most twice the packed size or 64 MiB: a re-planning pass then
    // needs no staging scan (w x stride) -- HBM traded for a launch
    uint64_t stage_alloc = stage_total;
    {
        const uint64_t stride = std::max<uint64_t>((hc[3] + 15) & ~uint64_t(15), 16);
        const uint64_t fixed = stride * n_runs;
        if (fixed <= std::max<uint64_t>(2 * stage_total, (64ull << 20) / 4)) {
            R->stage_stride = stride;
            stage_alloc = fixed;  // (the packed offsets of this first plan fit inside it)
        }
    }
    tick("plan");
    P.put_pinned(pin);
    R->din = std::move(din);  // kept: sb_requests_set_replan re-plans from them
    R->rcap = std::move(rc);
    R->n_in = static_cast<uint32_t>(n);
    R->cap = B.cap_total + stage_total;
    R->status = P.get_dev(size_t(n_runs) * 8);
    R->tstatus = P.get_dev(request_tstatus_words(n_runs) * 8);
    R->stage = P.get_dev(stage_alloc * 4);
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
    R->tstatus = P.get_dev(request_tstatus_words(static_cast<uint32_t>(n_runs)) * 8);
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

// a record with 8 ALTs (VtHot: 7 extra ALTs, the 3-bit field's most): the
// only way a chain's staged hit carries the ALT label 7, which the compact
// hit form escapes (request_deliver_kernel checks for it only then)
bool store_has_label7(sb_store &s) {
    std::call_once(s.label7_once, [&s] {
        const size_t n = s.n_records;
        for (size_t r = 0; r < n && !s.label7; ++r) {
            const uint32_t nx = (r + 1 < n ? s.h_x_lo[r + 1] : static_cast<uint32_t>(s.n_extra)) - s.h_x_lo[r];
            if (nx >= VT_MAX_NX) s.label7 = true;
        }
    });
    return s.label7;
}

void run_requests(sb_batch &B, void *rows, void *hits, void *row_off, uint64_t rec_base) {
    sb_store &s = *B.s;
    sb_batch::Req &R = *B.req;
    if (s.device < 0) throw Error(SB_EHIP, "the store has no device image (SB_HOST_ONLY)");
    // every argument check before the run is marked or anything is queued: a
    // refused run leaves the batch as it was (no run pending)
    if (R.compact && rec_base + s.n_records > kStageCandMask)
        throw Error(SB_EINVAL, "compact request output: record numbers (rec_base + records) reach 2^29");
    HIP_OK(hipSetDevice(s.device));
    hipStream_t st = B.strm();
    // the compact forms' escape buffers (devtypes.hpp ReqEsc), once per batch
    if (R.compact == SB_COMPACT_ALL && !R.xrows.p) R.xrows = R.pool->get_dev(std::max<size_t>(R.n_rows, 1) * sizeof(ReqPartial));
    if (R.compact && !R.xlab.p) R.xlab = R.pool->get_dev(std::max<uint64_t>(R.cap, 1) * sizeof(uint16_t));
    mark_run(B);
    if (R.slices) {  // the per-slice part, then its rows (chain rows come out zero; the row kernel writes them)
        run_kernels(B);
        if (R.wide.p) {
            HIP_OK(hipMemsetAsync(R.wide.p, 0, B.nq, st));
            mark_wide(B.gen_big_n.as<uint32_t>(), B.gen_big.as<GenBig>(), B.gen_big_cap, R.wide.as<uint8_t>(), st);
        }
        // (compact rows: the wide sums go to xrows; request_eval_kernel
        // narrows each row or marks it escaped)
        launch_request_reduce(B.res.as<QRes>(), R.sseg.as<uint32_t>(), R.sherr.as<uint8_t>(), R.wide.as<uint8_t>(),
                              R.n_rows,
                              R.compact == SB_COMPACT_ALL ? R.xrows.as<ReqPartial>() : static_cast<ReqPartial *>(rows),
                              R.row_flag.as<uint8_t>(), st);
    }
    if (!R.err.p) {
        R.err = R.pool->get_dev(16);
        R.err_h = R.pool->get_pinned(16);
        HIP_OK(hipMemsetAsync(R.err.p, 0, 16, st));
    }
    const Config cfg = config();  // (once per pass: each call reads every SBEACON_* variable)
    const bool rec_staged = s.n_records <= kStageCandMask && !cfg.req_index_stage;
    // a fixed-stride batch re-planning with record staging and no per-slice
    // part: each eval wave plans its own run (request_eval_kernel PLAN)
    const bool fuse = R.replan && R.stage_stride && !R.slices && rec_staged && !cfg.req_plan_apart;
    R.plan_fused = fuse;
    if (R.replan && !fuse) {  // the planning kernels again, from the resident packed requests (same descriptors, same sizes)
        launch_request_plan(s.d, R.din.as<ReqIn>(), R.n_in, R.dchains.as<ReqChain>(),
                            reinterpret_cast<RowRun *>(R.dchains.as<char>() + R.runs_at), R.rcap.as<unsigned long long>(),
                            reinterpret_cast<unsigned long long *>(R.rcap.as<char>() + size_t(R.n_runs) * 16), st,
                            R.stage_stride, R.err.as<unsigned int>());
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
    launch_request_rows(d, R.dchains.as<ReqChain>(), reinterpret_cast<RowRun *>(R.dchains.as<char>() + R.runs_at),
                        R.n_runs,
                        R.status.as<unsigned long long>(), R.tstatus.as<unsigned long long>(),
                        R.slices ? B.res.as<QRes>() : nullptr,
                        R.sseg.as<uint32_t>(), B.hoff.as<uint64_t>(), R.sherr.as<uint8_t>(), B.hits.as<uint64_t>(),
                        static_cast<ReqPartial *>(rows), static_cast<uint64_t *>(row_off), R.row_src.as<uint64_t>(),
                        R.stage.as<uint32_t>(), static_cast<uint64_t *>(hits), R.n_rows, rec_base, R.n_lut, R.run,
                        R.err.as<unsigned int>(), R.compact, rec_staged, st, ev[0], ev[1],
                        fuse ? R.din.as<ReqIn>() : nullptr, R.n_in, R.stage_stride, cfg.req_inject,
                        cfg.req_tile_scan, ReqEsc{R.xrows.as<ReqPartial>(), R.row_flag.as<uint8_t>(), R.xlab.as<uint16_t>()},
                        R.compact && store_has_label7(s));
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
        if (on != 0 && on != SB_COMPACT_ALL && on != SB_COMPACT_HITS)
            throw Error(SB_EINVAL, "sb_requests_set_compact: mode 0, SB_COMPACT_ALL or SB_COMPACT_HITS");
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->runs_pending) throw Error(SB_EINVAL, "sb_requests_set_compact between a run and its sync");
        b->req->compact = on;
    });
}

int sb_requests_escapes(sb_batch *b, int *rows, int *hits) {
    return guard([&] {
        if (!b || !b->req || !rows || !hits) throw Error(SB_EINVAL, "not a request batch");
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->runs_pending) throw Error(SB_EINVAL, "sb_requests_escapes between a run and its sync");
        *rows = b->req->escapes & 1u ? 1 : 0;
        *hits = b->req->escapes & 2u ? 1 : 0;
    });
}

extern "C++" {
// n entries of `width` bytes at the given indexes of a device buffer: one
// copy each when few, else the whole buffer once
template <class Idx>
void gather_down(const DevMem &m, size_t width, size_t count, const Idx *idx, size_t n, void *out, hipStream_t st) {
    if (!n) return;
    for (size_t i = 0; i < n; ++i)
        if (static_cast<uint64_t>(idx[i]) >= count) throw Error(SB_EINVAL, "index past the batch's output");
    char *o = static_cast<char *>(out);
    if (n <= 64) {
        for (size_t i = 0; i < n; ++i)
            HIP_OK(hipMemcpyAsync(o + i * width, m.as<char>() + static_cast<uint64_t>(idx[i]) * width, width,
                                  hipMemcpyDeviceToHost, st));
        HIP_OK(hipStreamSynchronize(st));
        return;
    }
    std::vector<char> all(count * width);
    HIP_OK(hipMemcpyAsync(all.data(), m.p, all.size(), hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    for (size_t i = 0; i < n; ++i) std::memcpy(o + i * width, all.data() + static_cast<uint64_t>(idx[i]) * width, width);
}
}  // extern "C++"

int sb_requests_wide_rows(sb_batch *b, const uint32_t *rows, size_t n, sb_request_partial *out) {
    return guard([&] {
        if (!b || !b->req || ((!rows || !out) && n)) throw Error(SB_EINVAL, "NULL argument");
        sb_batch::Req &R = *b->req;
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->runs_pending) throw Error(SB_EINVAL, "sb_requests_wide_rows between a run and its sync");
        if (!R.xrows.p) throw Error(SB_EINVAL, "sb_requests_wide_rows: no SB_COMPACT_ALL pass on this batch");
        HIP_OK(hipSetDevice(b->s->device));
        gather_down(R.xrows, sizeof(ReqPartial), R.n_rows, rows, n, out, b->strm());
    });
}

int sb_requests_hit_labels(sb_batch *b, const uint64_t *pos, size_t n, uint32_t *out) {
    return guard([&] {
        if (!b || !b->req || ((!pos || !out) && n)) throw Error(SB_EINVAL, "NULL argument");
        sb_batch::Req &R = *b->req;
        std::lock_guard<std::mutex> lk(b->mu);
        if (b->runs_pending) throw Error(SB_EINVAL, "sb_requests_hit_labels between a run and its sync");
        if (!R.xlab.p) throw Error(SB_EINVAL, "sb_requests_hit_labels: no compact pass on this batch");
        HIP_OK(hipSetDevice(b->s->device));
        std::vector<uint16_t> lab(n);
        gather_down(R.xlab, sizeof(uint16_t), std::max<uint64_t>(R.cap, 1), pos, n, lab.data(), b->strm());
        for (size_t i = 0; i < n; ++i) out[i] = lab[i];
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

int sb_requests_plan_fused(sb_batch *b, int *fused) {
    return guard([&] {
        if (!b || !b->req || !fused) throw Error(SB_EINVAL, "not a request batch");
        std::lock_guard<std::mutex> lk(b->mu);
        *fused = b->req->plan_fused ? 1 : 0;
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

}  // extern "C"
