// persist.cpp — a store on disk: sb_store_save / sb_store_open.
//
// The reference keeps its ingest state between invocations: each VCF's
// region files in S3 (lambda/summariseSlice/source/write_data_to_s3.h:39-92)
// and the per-dataset toUpdate bookkeeping in DynamoDB
// (lambda/summariseSlice/source/main.cpp:360-438), so a performQuery never
// re-reads VCF text.  Here the finished store itself is saved: every device
// buffer (copied back from HBM), the host columns the planners and
// formatters read, and the VCF metadata, plus a fingerprint of every source
// file (size, mtime, a hash of its first and last 64 KiB).  sb_store_open
// re-allocates the buffers, streams them up from the file (no re-parse, no
// column rebuild) and remaps the device pointers the store's kernel views
// hold.  A source that changed since the save makes sb_store_open fail with
// SB_ESTALE naming it; the caller re-ingests that store only (stores are per
// VCF group: sbeacon.catalog.StoreCatalog rebuilds just the stale ones).
//
//   <dir>/manifest.json  version, sources with fingerprints, sizes (text)
//   <dir>/host.bin       host columns + VCF metadata + kernel views
//   <dir>/device.bin     the device buffers, back to back (4 KiB aligned)
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <functional>
#include <chrono>
#include <memory>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "jsonesc.hpp"
#include "store.hpp"

namespace sb {

constexpr uint64_t kMagic = 0x3150544f5453424full;  // "OBSTOTP1"
constexpr uint32_t kFormat = 4;  // 2: dedup class words carry tail ids; 3: VcIndex::xinfo; 4: view sizes + pointer table

// FNV-1a over the first and last 64 KiB (with the size and mtime, a change
// detector -- not a content address)
SourceFile fingerprint(const std::string &path) {
    SourceFile f;
    f.path = path;
    struct stat st {};
    if (stat(path.c_str(), &st) != 0) return f;
    f.size = static_cast<uint64_t>(st.st_size);
    f.mtime_ns = static_cast<int64_t>(st.st_mtim.tv_sec) * 1000000000ll + st.st_mtim.tv_nsec;
    FILE *fp = fopen(path.c_str(), "rb");
    if (!fp) return f;
    uint64_t h = 1469598103934665603ull;
    std::vector<uint8_t> buf(65536);
    auto eat = [&](long at) {
        if (fseek(fp, at, SEEK_SET) != 0) return;
        const size_t n = fread(buf.data(), 1, buf.size(), fp);
        for (size_t i = 0; i < n; ++i) h = (h ^ buf[i]) * 1099511628211ull;
    };
    eat(0);
    if (f.size > buf.size()) eat(static_cast<long>(f.size - buf.size()));
    fclose(fp);
    f.sample_hash = h;
    return f;
}

namespace {

void pread_all(int fd, void *dst, size_t n, uint64_t off, const char *what) {
    size_t got = 0;
    while (got < n) {
        const ssize_t r = pread(fd, static_cast<uint8_t *>(dst) + got, n - got, static_cast<off_t>(off + got));
        if (r <= 0) throw Error(SB_EIO, std::string("persisted store: truncated ") + what);
        got += static_cast<size_t>(r);
    }
}

// run jobs on up to nt threads, largest first; the first error is rethrown
void run_jobs(std::vector<std::pair<size_t, std::function<void()>>> &jobs, unsigned nt) {
    std::sort(jobs.begin(), jobs.end(), [](const auto &a, const auto &b) { return a.first > b.first; });
    std::atomic<size_t> next{0};
    std::vector<std::string> errs(nt);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            try {
                for (size_t q; (q = next.fetch_add(1)) < jobs.size();) jobs[q].second();
            } catch (const std::exception &e) {
                errs[t] = e.what();
            }
        });
    for (auto &x : th) x.join();
    for (const std::string &e : errs)
        if (!e.empty()) throw Error(SB_EIO, e);
}

struct Writer {
    FILE *f = nullptr;
    uint64_t at = 0;
    std::string path;
    explicit Writer(const std::string &p) : path(p) {
        f = fopen(path.c_str(), "wb");
        if (!f) throw Error(SB_EIO, "cannot write " + path);
    }
    ~Writer() {
        if (f) fclose(f);  // (an error path: close() reports the normal one)
    }
    // flush + close, every failure an SB_EIO (ENOSPC in the final flush included)
    void close() {
        const bool ok = fflush(f) == 0 && fsync(fileno(f)) == 0;
        const int rc = fclose(f);
        f = nullptr;
        if (!ok || rc != 0) throw Error(SB_EIO, "cannot finish writing " + path);
    }
    void raw(const void *p, size_t n) {
        if (n && fwrite(p, 1, n, f) != n) throw Error(SB_EIO, "short write");
        at += n;
    }
    template <class T>
    void pod(const T &v) {
        static_assert(std::is_trivially_copyable<T>::value, "pod");
        raw(&v, sizeof v);
    }
    template <class T>
    void vec(const std::vector<T> &v) {
        static_assert(std::is_trivially_copyable<T>::value, "vec of pod");
        pod<uint64_t>(v.size());
        raw(v.data(), v.size() * sizeof(T));
    }
    void str(const std::string &s) {
        pod<uint64_t>(s.size());
        raw(s.data(), s.size());
    }
    void strs(const std::vector<std::string> &v) {
        pod<uint64_t>(v.size());
        for (const auto &s : v) str(s);
    }
    void pad(uint64_t align) {
        static const uint8_t z[4096] = {};
        while (at % align) raw(z, std::min<uint64_t>(align - at % align, sizeof z));
    }
};

// host.bin is parsed from a read-only mapping; columns of 1 MiB or more are
// not copied during the parse but become jobs (resize + pread into the
// column) that threads run beside the device image upload
struct Reader {
    const uint8_t *b = nullptr;
    size_t size = 0, at = 0;
    int fd = -1;
    std::vector<std::pair<size_t, std::function<void()>>> *defer = nullptr;  // (bytes, job)
    void need(size_t n) const {
        if (at + n > size) throw Error(SB_EIO, "persisted store: truncated host.bin");
    }
    void raw(void *p, size_t n) {
        need(n);
        if (n) std::memcpy(p, b + at, n);
        at += n;
    }
    template <class T>
    T pod() {
        T v;
        raw(&v, sizeof v);
        return v;
    }
    template <class T>
    void vec(std::vector<T> &v) {
        const uint64_t n = pod<uint64_t>();
        const size_t bytes = n * sizeof(T);
        need(bytes);
        if (defer && bytes >= (size_t(1) << 20)) {
            const size_t off = at;
            const int f = fd;
            defer->emplace_back(bytes, [&v, n, off, f] {
                v.resize(n);
                pread_all(f, v.data(), n * sizeof(T), off, "host.bin");
            });
            at += bytes;
        } else {
            v.resize(n);
            raw(v.data(), bytes);
        }
    }
    std::string str() {
        const uint64_t n = pod<uint64_t>();
        need(n);
        std::string s(reinterpret_cast<const char *>(b + at), n);
        at += n;
        return s;
    }
    std::vector<std::string> strs() {
        std::vector<std::string> v(pod<uint64_t>());
        for (auto &s : v) s = str();
        return v;
    }
};

// a read-only mapping of a whole file
struct Mapped {
    int fd = -1;
    const uint8_t *p = nullptr;
    size_t n = 0;
    explicit Mapped(const std::string &path) {
        fd = ::open(path.c_str(), O_RDONLY);
        if (fd < 0) throw Error(SB_EIO, "cannot open " + path);
        struct stat st{};
        if (fstat(fd, &st) != 0) {
            ::close(fd);
            throw Error(SB_EIO, "cannot stat " + path);
        }
        n = static_cast<size_t>(st.st_size);
        if (n) {
            void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
            if (m == MAP_FAILED) {
                ::close(fd);
                throw Error(SB_EIO, "cannot map " + path);
            }
            p = static_cast<const uint8_t *>(m);
        }
    }
    ~Mapped() {
        if (p) munmap(const_cast<uint8_t *>(p), n);
        if (fd >= 0) ::close(fd);
    }
    Mapped(const Mapped &) = delete;
    Mapped &operator=(const Mapped &) = delete;
};

void put_sources(Writer &w, const std::vector<SourceFile> &v) {
    w.pod<uint64_t>(v.size());
    for (const SourceFile &f : v) {
        w.str(f.path);
        w.pod(f.size);
        w.pod(f.mtime_ns);
        w.pod(f.sample_hash);
    }
}

std::vector<SourceFile> get_sources(Reader &r) {
    std::vector<SourceFile> v(r.pod<uint64_t>());
    for (SourceFile &f : v) {
        f.path = r.str();
        f.size = r.pod<uint64_t>();
        f.mtime_ns = r.pod<int64_t>();
        f.sample_hash = r.pod<uint64_t>();
    }
    return v;
}

// a finished store's VCF metadata (its columns were moved into the store)
void put_vcf(Writer &w, const VcfData &v) {
    w.str(v.location);
    put_sources(w, v.sources);
    w.pod(v.rec_lo);
    w.pod(v.rec_hi);
    w.pod(v.lines_seen);
    w.strs(v.samples);
    w.pod(v.words);
    w.pod<uint8_t>(v.header_seen);
    w.pod<uint64_t>(v.segments.size());
    for (const Segment &g : v.segments) {
        w.str(g.contig);
        w.pod(g.lo);
        w.pod(g.hi);
    }
    w.vec(v.buckets);
    w.vec(v.vc_index);
    w.pod(v.seg_base);
    w.pod(v.stream_off);
    w.vec(v.blk_coff);
    w.vec(v.blk_ustart);
    w.pod(v.stream_len);
    w.pod(v.rec_base);
    w.pod(v.x_base);
    w.pod(v.plane0_base);
    w.pod(v.planex_base);
    w.pod<uint8_t>(v.nonneg);
    w.pod<uint8_t>(v.has_planes);
    w.pod<uint8_t>(v.range8);
    w.pod(v.an_default);
}

void get_vcf(Reader &r, VcfData &v) {
    v.location = r.str();
    v.sources = get_sources(r);
    v.rec_lo = r.pod<uint64_t>();
    v.rec_hi = r.pod<uint64_t>();
    v.lines_seen = r.pod<uint64_t>();
    v.samples = r.strs();
    v.words = r.pod<uint32_t>();
    v.header_seen = r.pod<uint8_t>() != 0;
    v.segments.resize(r.pod<uint64_t>());
    for (Segment &g : v.segments) {
        g.contig = r.str();
        g.lo = r.pod<uint32_t>();
        g.hi = r.pod<uint32_t>();
    }
    r.vec(v.buckets);
    r.vec(v.vc_index);
    v.seg_base = r.pod<uint32_t>();
    v.stream_off = r.pod<uint64_t>();
    r.vec(v.blk_coff);
    r.vec(v.blk_ustart);
    v.stream_len = r.pod<uint64_t>();
    v.rec_base = r.pod<uint32_t>();
    v.x_base = r.pod<uint32_t>();
    v.plane0_base = r.pod<uint64_t>();
    v.planex_base = r.pod<uint64_t>();
    v.nonneg = r.pod<uint8_t>() != 0;
    v.has_planes = r.pod<uint8_t>() != 0;
    v.range8 = r.pod<uint8_t>() != 0;
    v.an_default = r.pod<int32_t>();
    v.seg_index.clear();
    for (uint32_t i = 0; i < v.segments.size(); ++i) v.seg_index.emplace(v.segments[i].contig, i);
    v.sample_pos.clear();
    for (uint32_t k = 0; k < v.samples.size(); ++k) v.sample_pos[v.samples[k]].push_back(k);
}

// every host column of the store, in one order for save and open
template <class F>
void host_columns(sb_store &s, F &&f) {
    f(s.h_pos), f(s.h_end), f(s.h_a0_len), f(s.h_x_lo), f(s.h_x_len), f(s.h_bucket);
    f(s.h_vt), f(s.h_vt_slow), f(s.h_vc_pos), f(s.h_vc_bucket), f(s.h_vc_altpre);
    f(s.h_ref_off), f(s.h_a0_off), f(s.h_x_off), f(s.h_blob), f(s.h_start);
    f(s.h_rem), f(s.h_cur), f(s.h_dcount), f(s.h_sum_bad);
    f(s.h_dk_pos), f(s.h_dk_lo), f(s.h_dk_bad), f(s.h_dk_tail), f(s.h_dk_blob);
}

// the store's kernel views, as 8-byte words (their pointers are remapped)
template <class T>
uint64_t *words(T &v) {
    static_assert(sizeof(T) % 8 == 0, "views are 8-byte multiples");
    return reinterpret_cast<uint64_t *>(&v);
}
template <class T>
const uint64_t *words(const T &v) {
    return reinterpret_cast<const uint64_t *>(&v);
}

// The views' pointer words, classified once at save: (view, word, buffer,
// offset) for every word that points into -- or one past the end of -- a
// device buffer (strict containment wins over an end pointer).  Open remaps
// exactly these words; no word is guessed at from its value on open.
struct RemapEntry {
    uint32_t view, word, buf, pad;
    uint64_t off;
};
std::vector<RemapEntry> remap_table(const sb_store &s) {
    std::vector<RemapEntry> out;
    auto scan = [&](uint32_t view, const uint64_t *w, size_t n) {
        for (size_t i = 0; i < n; ++i) {
            if (!w[i]) continue;
            int end_hit = -1;
            bool done = false;
            for (size_t b = 0; b < s.bufs.size() && !done; ++b) {
                const uint64_t base = reinterpret_cast<uint64_t>(s.bufs[b].p), bytes = s.bufs[b].bytes;
                if (w[i] >= base && w[i] < base + bytes) {
                    out.push_back(RemapEntry{view, static_cast<uint32_t>(i), static_cast<uint32_t>(b), 0, w[i] - base});
                    done = true;
                } else if (w[i] == base + bytes && end_hit < 0) {
                    end_hit = static_cast<int>(b);
                }
            }
            if (!done && end_hit >= 0)
                out.push_back(RemapEntry{view, static_cast<uint32_t>(i), static_cast<uint32_t>(end_hit), 0,
                                         s.bufs[end_hit].bytes});
        }
    };
    scan(0, words(s.d), sizeof(DStore) / 8);
    scan(1, words(s.ds), sizeof(SStore) / 8);
    scan(2, words(s.dk), sizeof(KStore) / 8);
    scan(3, words(s.g), sizeof(GStore) / 8);
    return out;
}
// the views' layout as saved: sizes (a changed struct without a kFormat bump
// is refused instead of misread)
constexpr uint64_t kViewSizes[4] = {sizeof(DStore), sizeof(SStore), sizeof(KStore), sizeof(GStore)};

std::string manifest_text(const sb_store &s, uint64_t host_bytes, uint64_t device_bytes) {
    std::string o = "{\n  \"format\": " + std::to_string(kFormat) + ",\n  \"abi\": " + std::to_string(SB_ABI_VERSION) +
                    ",\n  \"records\": " + std::to_string(s.n_records) + ",\n  \"host_bytes\": " +
                    std::to_string(host_bytes) + ",\n  \"device_bytes\": " + std::to_string(device_bytes) +
                    ",\n  \"vcfs\": [";
    for (size_t i = 0; i < s.vcfs.size(); ++i) {
        const VcfData &v = s.vcfs[i];
        o += i ? ",\n    {" : "\n    {";
        o += "\"location\": \"";
        if (!json_escape_append(o, v.location.data(), v.location.size())) o += "?";
        o += "\"";
        o += ", \"sources\": [";
        for (size_t k = 0; k < v.sources.size(); ++k) {
            const SourceFile &f = v.sources[k];
            if (k) o += ", ";
            o += "{\"path\": \"";
            if (!json_escape_append(o, f.path.data(), f.path.size())) o += "?";
            o += "\", \"size\": " + std::to_string(f.size) + ", \"mtime_ns\": " + std::to_string(f.mtime_ns) +
                 ", \"sample_hash\": \"" + std::to_string(f.sample_hash) + "\"}";
        }
        o += "]}";
    }
    o += "\n  ]\n}\n";
    return o;
}

}  // namespace

namespace {
void save_files(sb_store &s, const std::string &dir);
// the names a save directory holds (save_files): only such a directory is
// ever removed -- a user's own DIR.tmp / DIR.old is left alone (the save fails)
bool save_name(const char *n) {
    // (sbeacon.json: the Python layer's side file, sbeacon/engine.py Store.save)
    return !std::strcmp(n, "manifest.json") || !std::strcmp(n, "host.bin") || !std::strcmp(n, "device.bin") ||
           !std::strcmp(n, "sbeacon.json");
}
// remove a save directory (plain files named as save_files names them);
// absent: nothing; anything else in it: SB_EIO, nothing removed
void remove_tree(const std::string &d) {
    DIR *x = opendir(d.c_str());
    if (!x) {
        struct stat st {};
        if (lstat(d.c_str(), &st) == 0) throw Error(SB_EIO, "cannot replace " + d + ": not a store directory");
        return;
    }
    std::vector<std::string> names;
    bool foreign = false;
    while (const dirent *e = readdir(x)) {
        if (!std::strcmp(e->d_name, ".") || !std::strcmp(e->d_name, "..")) continue;
        if (!save_name(e->d_name)) foreign = true;
        names.emplace_back(e->d_name);
    }
    closedir(x);
    if (foreign) throw Error(SB_EIO, "refusing to remove " + d + ": it holds files a store save does not write");
    for (const auto &n : names) (void)unlink((d + "/" + n).c_str());
    (void)rmdir(d.c_str());
}
// the directory entry of `path` made durable (its parent fsynced)
void sync_parent(const std::string &path) {
    const size_t k = path.find_last_of('/');
    const std::string parent = k == std::string::npos ? "." : k == 0 ? "/" : path.substr(0, k);
    const int fd = open(parent.c_str(), O_RDONLY | O_DIRECTORY);
    if (fd < 0) return;
    (void)fsync(fd);
    close(fd);
}
}  // namespace

// The three files are written into `dir.tmp` and the directory renamed into
// place: a crash mid-save leaves the previous save, as `dir` or (between the
// two renames) as `dir.old`, which store_open takes when `dir` is missing --
// never a new device.bin beside an old host.bin.
void store_save(sb_store &s, const std::string &dir_in) {
    std::string dir = dir_in;
    while (dir.size() > 1 && dir.back() == '/') dir.pop_back();
    const std::string tmp = dir + ".tmp", prev = dir + ".old";
    remove_tree(tmp);
    if (mkdir(tmp.c_str(), 0755) != 0) throw Error(SB_EIO, "cannot create " + tmp);
    try {
        save_files(s, tmp);
    } catch (...) {
        remove_tree(tmp);
        throw;
    }
    struct stat st {};
    const bool had = stat(dir.c_str(), &st) == 0;
    remove_tree(prev);
    if (had && rename(dir.c_str(), prev.c_str()) != 0) throw Error(SB_EIO, "cannot replace " + dir);
    if (rename(tmp.c_str(), dir.c_str()) != 0) {
        if (had) (void)rename(prev.c_str(), dir.c_str());
        throw Error(SB_EIO, "cannot move " + tmp + " to " + dir);
    }
    sync_parent(dir);
    if (had) remove_tree(prev);
}

namespace {
void save_files(sb_store &s, const std::string &dir) {
    if (s.device >= 0) {
        HIP_OK(hipSetDevice(s.device));
        HIP_OK(hipStreamSynchronize(s.stream));
    }
    // device buffers, back to back: copied down through a pinned bounce (a
    // host-only store (SB_HOST_ONLY) has none)
    uint64_t dev_bytes = 0;
    if (s.device >= 0) {
        Writer w(dir + "/device.bin");
        void *pin = nullptr;
        const size_t chunk = size_t(64) << 20;
        HIP_OK(hipHostMalloc(&pin, chunk, hipHostMallocDefault));
        try {
            for (const DeviceBuffer &b : s.bufs) {
                for (size_t o = 0; o < b.bytes; o += chunk) {
                    const size_t n = std::min(chunk, b.bytes - o);
                    HIP_OK(hipMemcpy(pin, static_cast<const uint8_t *>(b.p) + o, n, hipMemcpyDeviceToHost));
                    w.raw(pin, n);
                }
                w.pad(4096);
            }
        } catch (...) {
            (void)hipHostFree(pin);
            throw;
        }
        (void)hipHostFree(pin);
        dev_bytes = w.at;
        w.close();
    } else {
        Writer w(dir + "/device.bin");  // empty: no device image
        w.close();
    }
    uint64_t host_bytes = 0;
    {
        Writer w(dir + "/host.bin");
        w.pod(kMagic);
        w.pod(kFormat);
        w.pod<uint64_t>(s.n_records);
        w.pod<uint64_t>(s.n_extra);
        w.pod<uint32_t>(s.max_words);
        w.pod<uint64_t>(s.n_keys);
        host_columns(s, [&](auto &v) { w.vec(v); });
        w.pod<uint64_t>(s.seg_slow_pos.size());
        for (const auto &per_vcf : s.seg_slow_pos) {
            w.pod<uint64_t>(per_vcf.size());
            for (const auto &seg : per_vcf) w.vec(seg);
        }
        w.strs(s.vt.items);
        w.strs(s.sym.items);
        w.pod<uint64_t>(s.vcfs.size());
        for (const VcfData &v : s.vcfs) put_vcf(w, v);
        // kernel views (their sizes first), the buffers their pointers index
        // and the pointer words (remap_table)
        for (uint64_t z : kViewSizes) w.pod(z);
        w.pod(s.d);
        w.pod(s.ds);
        w.pod(s.dk);
        w.pod(s.g);
        w.pod<uint64_t>(s.bufs.size());
        for (const DeviceBuffer &b : s.bufs) {
            w.pod<uint64_t>(reinterpret_cast<uint64_t>(b.p));
            w.pod<uint64_t>(b.bytes);
        }
        w.vec(s.device >= 0 ? remap_table(s) : std::vector<RemapEntry>{});
        w.pod(kMagic);
        host_bytes = w.at;
        w.close();
    }
    const std::string m = manifest_text(s, host_bytes, dev_bytes);
    Writer w(dir + "/manifest.json");
    w.raw(m.data(), m.size());
    w.close();
}
}  // namespace

// dir of a manifest path (or the directory itself)
std::string store_dir(const std::string &p) {
    const std::string tail = "/manifest.json";
    if (p.size() >= tail.size() && p.compare(p.size() - tail.size(), tail.size(), tail) == 0)
        return p.substr(0, p.size() - tail.size());
    if (p == "manifest.json") return ".";
    return p;
}

sb_store *store_open(const std::string &path, int device, std::string *stale) {
    const std::string dir = store_dir(path);
    {  // a save interrupted between its two renames left the previous save as dir.old
        struct stat st {};
        const std::string prev = dir + ".old";
        if (stat(dir.c_str(), &st) != 0 && stat((prev + "/manifest.json").c_str(), &st) == 0 &&
            rename(prev.c_str(), dir.c_str()) == 0)
            sync_parent(dir);
    }
    Mapped hm(dir + "/host.bin");
    std::vector<std::pair<size_t, std::function<void()>>> host_jobs;
    Reader r;
    r.b = hm.p;
    r.size = hm.n;
    r.fd = hm.fd;
    r.defer = &host_jobs;
    if (r.pod<uint64_t>() != kMagic || r.pod<uint32_t>() != kFormat)
        throw Error(SB_EIO, "persisted store: not a store file of this format (" + dir + ")");
    auto s = std::make_unique<sb_store>();
    s->n_records = r.pod<uint64_t>();
    s->n_extra = r.pod<uint64_t>();
    s->max_words = r.pod<uint32_t>();
    s->n_keys = r.pod<uint64_t>();
    host_columns(*s, [&](auto &v) { r.vec(v); });
    s->seg_slow_pos.resize(r.pod<uint64_t>());
    for (auto &per_vcf : s->seg_slow_pos) {
        per_vcf.resize(r.pod<uint64_t>());
        for (auto &seg : per_vcf) r.vec(seg);
    }
    for (const std::string &x : r.strs()) s->vt.get(x);
    for (const std::string &x : r.strs()) s->sym.get(x);
    s->vcfs.resize(r.pod<uint64_t>());
    for (VcfData &v : s->vcfs) get_vcf(r, v);
    // sources changed since the save: the caller re-ingests this store
    for (const VcfData &v : s->vcfs)
        for (const SourceFile &f : v.sources) {
            const SourceFile now = fingerprint(f.path);
            if (now.size != f.size || now.mtime_ns != f.mtime_ns || now.sample_hash != f.sample_hash) {
                if (stale) *stale += (stale->empty() ? "" : "\n") + f.path;
            }
        }
    if (stale && !stale->empty()) return nullptr;
    for (uint64_t z : kViewSizes)
        if (r.pod<uint64_t>() != z) throw Error(SB_EIO, "persisted store: kernel view layout differs (" + dir + ")");
    s->d = r.pod<DStore>();
    s->ds = r.pod<SStore>();
    s->dk = r.pod<KStore>();
    s->g = r.pod<GStore>();
    std::vector<DeviceBuffer> old(r.pod<uint64_t>());
    for (DeviceBuffer &b : old) {
        b.p = reinterpret_cast<void *>(r.pod<uint64_t>());
        b.bytes = r.pod<uint64_t>();
    }
    std::vector<RemapEntry> rmap;
    r.vec(rmap);
    if (r.pod<uint64_t>() != kMagic) throw Error(SB_EIO, "persisted store: corrupt host.bin");
    for (uint32_t i = 0; i < s->vcfs.size(); ++i) s->vcf_by_location.emplace(s->vcfs[i].location, i);
    if (device == SB_HOST_ONLY) {  // the host side only (planning, region files, index)
        s->device = SB_HOST_ONLY;
        s->d = DStore{};
        s->ds = SStore{};
        s->dk = KStore{};
        s->g = GStore{};
        run_jobs(host_jobs, 8);
        return s.release();
    }
    if (old.empty() && s->n_records)
        throw Error(SB_EINVAL, "persisted store: saved from a host-only store (no device image); open it SB_HOST_ONLY");
    // device image: the buffers re-allocated in order, streamed up
    int n_dev = 0;
    HIP_OK(hipGetDeviceCount(&n_dev));
    if (device < 0 || device >= n_dev) throw Error(SB_EHIP, "device ordinal out of range");
    s->device = device;
    HIP_OK(hipSetDevice(device));
    HIP_OK(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    // the buffers re-allocated in order; their bytes cut into 32 MiB pieces
    // that 8 threads read (pread, page cache) into their own pinned pair and
    // copy up on their own streams
    struct Piece {
        uint64_t file_off;
        void *dst;
        size_t n;
    };
    std::vector<Piece> pieces;
    {
        const size_t chunk = size_t(32) << 20;
        uint64_t at = 0;
        for (const DeviceBuffer &o : old) {
            DeviceBuffer b;
            b.bytes = o.bytes;
            HIP_OK(hipMalloc(&b.p, b.bytes));
            s->bufs.push_back(b);
            s->device_bytes += b.bytes;
            for (size_t off = 0; off < b.bytes; off += chunk)
                pieces.push_back(Piece{at + off, static_cast<uint8_t *>(b.p) + off, std::min(chunk, b.bytes - off)});
            at = (at + b.bytes + 4095) / 4096 * 4096;
        }
    }
    const int fd = ::open((dir + "/device.bin").c_str(), O_RDONLY);
    if (fd < 0) throw Error(SB_EIO, "cannot open " + dir + "/device.bin");
    // the host columns load beside the device image
    std::string host_err;
    std::thread host_loader([&] {
        try {
            run_jobs(host_jobs, 6);
        } catch (const std::exception &e) {
            host_err = e.what();
        }
    });
    const unsigned nt = static_cast<unsigned>(std::min<size_t>(8, std::max<size_t>(1, pieces.size())));
    std::vector<std::string> errs(nt);
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
        th.emplace_back([&, t] {
            std::array<void *, 2> pin{nullptr, nullptr};
            std::array<hipEvent_t, 2> done{nullptr, nullptr};
            hipStream_t st = nullptr;
            try {
                HIP_OK(hipSetDevice(device));
                HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
                for (int k = 0; k < 2; ++k) {
                    HIP_OK(hipHostMalloc(&pin[k], size_t(32) << 20, hipHostMallocDefault));
                    HIP_OK(hipEventCreate(&done[k]));
                }
                int k = 0;
                for (size_t q = t; q < pieces.size(); q += nt) {  // double-buffered: read n + 1 while n copies
                    const Piece &pc = pieces[q];
                    HIP_OK(hipEventSynchronize(done[k]));
                    size_t got = 0;
                    while (got < pc.n) {
                        const ssize_t r = pread(fd, static_cast<uint8_t *>(pin[k]) + got, pc.n - got,
                                                static_cast<off_t>(pc.file_off + got));
                        if (r <= 0) throw Error(SB_EIO, "persisted store: truncated device.bin");
                        got += static_cast<size_t>(r);
                    }
                    HIP_OK(hipMemcpyAsync(pc.dst, pin[k], pc.n, hipMemcpyHostToDevice, st));
                    HIP_OK(hipEventRecord(done[k], st));
                    k ^= 1;
                }
                HIP_OK(hipStreamSynchronize(st));
            } catch (const std::exception &e) {
                errs[t] = e.what();
                if (st) (void)hipStreamSynchronize(st);
            }
            for (int k = 0; k < 2; ++k) {
                if (pin[k]) (void)hipHostFree(pin[k]);
                if (done[k]) (void)hipEventDestroy(done[k]);
            }
            if (st) (void)hipStreamDestroy(st);
        });
    for (auto &x : th) x.join();
    host_loader.join();
    ::close(fd);
    for (const std::string &e : errs)
        if (!e.empty()) throw Error(SB_EIO, "persisted store: " + e);
    if (!host_err.empty()) throw Error(SB_EIO, host_err);
    // remap exactly the pointer words the save classified (remap_table)
    uint64_t *views[4] = {words(s->d), words(s->ds), words(s->dk), words(s->g)};
    for (const RemapEntry &e : rmap) {
        if (e.view >= 4 || e.word >= kViewSizes[e.view] / 8 || e.buf >= s->bufs.size() || e.off > old[e.buf].bytes)
            throw Error(SB_EIO, "persisted store: corrupt pointer table (" + dir + ")");
        views[e.view][e.word] = reinterpret_cast<uint64_t>(s->bufs[e.buf].p) + e.off;
    }
    return s.release();
}

}  // namespace sb
