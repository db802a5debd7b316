// api.cpp — the C ABI (include/sbeacon.h): builder, HBM store, query batches.
// Request batches live in requests.cpp, summarise / dedup in summarise.cpp,
// result sets in results.cpp; what they share is internal.hpp.
//
// The query path mirrors one splitQuery fan-out (lambda/splitQuery/
// lambda_function.py:74-110) handed to the device as ONE batch: every
// PerformQueryPayload becomes a QDev; the host plans each query's output
// region from the store's coarse POS index (an upper bound on its hits), so
// a query step is a single kernel launch (query_kernels.hip).  Result strings
// are formatted on the host from the store's allele blob in the reference's
// exact format.
#include "internal.hpp"

#include <zlib.h>

namespace sb {
void builder_add_text(sb_builder &b, uint32_t vcf_id, const char *text, size_t len);
void builder_add_file(sb_builder &b, uint32_t vcf_id, const char *path);
void builder_flush(sb_builder &b, uint32_t vcf_id);
void vcf_scan_file(const char *path, VcfScan &out);
void builder_attach_carriers(sb_builder &b, uint32_t vcf_id, const char *const *names, const uint32_t *name_len,
                             uint32_t n_samples, const uint64_t *planes, uint64_t n_rows);

namespace {
thread_local std::string g_last_error;
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

// the query batch (sb_batch_*); prepare / mark_run / run_kernels / sync are
// the request batches' too (requests.cpp)
namespace sb {

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

#ifndef SBEACON_PAR_GROUPS
#define SBEACON_PAR_GROUPS 1
#endif
constexpr bool kParGroups = SBEACON_PAR_GROUPS != 0;

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
    // with sample-path groups too, the fused launch runs on a second stream
    // beside them (disjoint results and hit regions; both may append to the
    // general-record work list, atomically): a short scan-bound launch and a
    // long carrier-row-bound one share the device instead of queueing
    const bool scans = std::any_of(B.groups.begin(), B.groups.end(), [](const sb_batch::Group &g) {
        return g.max_words != 0 && !g.idx.empty();
    });
    // (not on the legacy default stream: an event recorded on hipStreamLegacy
    // and waited for on another stream crashed the HIP runtime in
    // hipStreamWaitEvent -- the request batches' tests found it)
    const bool split = kParGroups && scans && !fg.empty() && st != hipStreamLegacy;
    hipStream_t fs = st;
    if (split) {
        if (!B.aux) {
            HIP_OK(hipStreamCreateWithFlags(&B.aux, hipStreamNonBlocking));
            for (auto &e : B.fork) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        HIP_OK(hipEventRecord(B.fork[0], st));
        HIP_OK(hipStreamWaitEvent(B.aux, B.fork[0], 0));
        fs = B.aux;
    }
    launch_fused(d, fg.data(), static_cast<int>(fg.size()), B.nonneg, B.qbytes.as<uint8_t>(), B.subsets.as<uint64_t>(),
                 B.res.as<QRes>(), B.hits.as<uint64_t>(), fs);
    if (split) HIP_OK(hipEventRecord(B.fork[1], B.aux));
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
    if (split) HIP_OK(hipStreamWaitEvent(st, B.fork[1], 0));  // join before the general records and the next run
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
    const uint32_t e = chk ? *static_cast<volatile uint32_t *>(B.req->err_h.p) : 0u;
    if (e) {  // reported once: the next pass of this batch (e.g. answered wide after an error) starts clean
        HIP_OK(hipMemsetAsync(B.req->err.p, 0, 4, B.strm()));
        HIP_OK(hipStreamSynchronize(B.strm()));
        *static_cast<volatile uint32_t *>(B.req->err_h.p) = 0u;
    }
    if (chk) B.req->escapes = (e & kErrRowEscapes ? 1u : 0u) | (e & kErrHitEscapes ? 2u : 0u);
    if (e & 1u)
        throw Error(SB_EINTERNAL, "request_eval_kernel: the per-chain sums of a pass failed their invariants "
                                  "(chain counts, call counts or AN sums vs the wave's own totals)");
    if (e & 2u)
        throw Error(SB_EINVAL, "compact request output (SB_COMPACT_ALL): the hit offsets pass 32 bits (more "
                               "than 2^32 hits in the batch); answer this batch with wide rows");
    if (e & 4u)
        throw Error(SB_EINVAL, "compact request hits: a per-slice hit has an ALT index past 65,535, which the "
                               "label escape cannot hold; answer this batch with wide hits");
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

}  // namespace sb

extern "C" {

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

int sb_store_candidates(const sb_store *s, uint64_t *n, uint64_t *bytes) {
    return guard([&] {
        if (!s || !n || !bytes) throw Error(SB_EINVAL, "NULL argument");
        *n = s->h_vc_altpre.empty() ? 0 : s->h_vc_altpre.size() - 1;
        *bytes = *n * (sizeof(VcQ) + sizeof(uint32_t));  // the VcQ word + the record id request_eval_kernel loads
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

}  // extern "C"
