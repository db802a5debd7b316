// summarise.cpp — summariseSlice (sb_summarise_slices) and
// duplicateVariantSearch over region files (sb_region_files, sb_dedup_*).
#include "internal.hpp"

#include <zlib.h>

namespace {

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
    uint64_t n_wins = 0;
    uint32_t rec_words = kWinRecHead;  // window record: header + 2 words per run of the call's largest job
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
        P.n_wins += J.nw;
        P.rec_words = std::max(P.rec_words, (kWinRecHead + 2 * J.nruns + 3) / 4 * 4);
        if (P.n_wins >= 0x7fffffffull) return P.why = "windows", false;
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
    DevMem jobs, rec, runs, counts, overflow, list, n_list, wfresh;
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
    W.rec.reserve(std::max<size_t>(nw, 1) * P.rec_words * 4);
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
    launch_window_dedupe(s.dk, W.jobs.as<KJob>(), static_cast<uint32_t>(P.jobs.size()), W.rec.as<uint32_t>(), P.rec_words,
                         nw, W.runs.as<KRun>(), W.counts.as<unsigned long long>(), W.list.as<uint2>(),
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

}  // extern "C"
