// jsonout.hpp -- the JSON-lines output of the batched handlers
// (sb_perform_query_events in wire.cpp, sb_route_bodies in routes.cpp):
// one big host buffer on 2 MB pages, an offset per item and a status byte.
#pragma once
#include <sys/mman.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/sbeacon.h"

namespace sb {
// large host buffers backed by 2 MB pages where the kernel allows it (the
// response text runs to hundreds of MB: 4 KB first-touch faults were a third
// of the formatting time)
struct FreeDel {
    void operator()(char *p) const { std::free(p); }
};
// one released output buffer is kept for the next call (freeing and
// re-faulting ~200 MB of response text cost ~10 ms per call)
inline std::mutex g_spare_mu;
inline std::unique_ptr<char, FreeDel> g_spare;
inline size_t g_spare_sz = 0;

inline std::unique_ptr<char, FreeDel> big_alloc(size_t n, size_t *cap) {
    constexpr size_t kHuge = size_t(2) << 20;
    const size_t sz = (std::max<size_t>(n, 1) + kHuge - 1) / kHuge * kHuge;
    {
        std::lock_guard<std::mutex> lk(g_spare_mu);
        if (g_spare && g_spare_sz >= sz && g_spare_sz <= 2 * sz + (size_t(64) << 20)) {
            *cap = g_spare_sz;
            g_spare_sz = 0;
            return std::move(g_spare);
        }
    }
    char *p = static_cast<char *>(std::aligned_alloc(kHuge, sz));
    if (!p) throw std::bad_alloc();
    (void)madvise(p, sz, MADV_HUGEPAGE);
    *cap = sz;
    return std::unique_ptr<char, FreeDel>(p);
}

inline void big_release(std::unique_ptr<char, FreeDel> &b, size_t cap) {
    if (!b) return;
    std::lock_guard<std::mutex> lk(g_spare_mu);
    if (cap > g_spare_sz) {  // keep the larger one
        g_spare = std::move(b);
        g_spare_sz = cap;
    }
}
}  // namespace sb

struct sb_json_out {
    std::unique_ptr<char, sb::FreeDel> buf;  // n bytes (uninitialised storage: filled in parallel)
    uint64_t n = 0;
    size_t cap = 0;  // buf's allocation (kept for the next call when released)
    std::vector<uint64_t> off;    // n + 1
    std::vector<uint8_t> status;  // per item: 0 answered; else the function's own code (no text)
};
