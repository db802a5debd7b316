// common.hpp — host helpers shared by ingest and the C ABI.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/sbeacon.h"

namespace sb {

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string &m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string &msg);

inline uint8_t upc(uint8_t c) { return (c >= 'a' && c <= 'z') ? static_cast<uint8_t>(c - 32) : c; }

// Python int(str) over the ASCII forms a VCF carries (whitespace, sign,
// digits, single '_' between digits) — the parse the reference applies to
// INFO/AC and INFO/AN (search_variants.py:199,206).
inline bool py_int(const char *p, size_t n, int64_t *out) {
    size_t i = 0, j = n;
    auto sp = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; };
    while (i < j && sp(p[i])) ++i;
    while (j > i && sp(p[j - 1])) --j;
    if (i == j) return false;
    bool neg = false;
    if (p[i] == '+' || p[i] == '-') {
        neg = p[i] == '-';
        ++i;
    }
    if (i == j || p[i] < '0' || p[i] > '9') return false;
    int64_t v = 0;
    for (size_t k = i; k < j; ++k) {
        const char c = p[k];
        if (c == '_') {
            if (k + 1 >= j || p[k + 1] < '0' || p[k + 1] > '9' || p[k - 1] < '0' || p[k - 1] > '9') return false;
            continue;
        }
        if (c < '0' || c > '9') return false;
        if (v > (INT64_MAX - 9) / 10) return false;  // beyond int64: not representable in the store
        v = v * 10 + (c - '0');
    }
    *out = neg ? -v : v;
    return true;
}

// CPython's str -> int digit limit (Python >= 3.10.7 / 3.9.14; the Lambda
// python3.9 runtime too): int() of a string with more digits raises ValueError
constexpr size_t kPyMaxStrDigits = 4300;

// py_int with the rest of Python's range: 0 = *out holds the value, 1 = a
// valid int() beyond int64 (py_int_limbs has it), -1 = int() raises
// ValueError (syntax, or more than kPyMaxStrDigits digits).
inline int py_int_ex(const char *p, size_t n, int64_t *out) {
    size_t i = 0, j = n;
    auto sp = [](char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; };
    while (i < j && sp(p[i])) ++i;
    while (j > i && sp(p[j - 1])) --j;
    if (i == j) return -1;
    bool neg = false;
    if (p[i] == '+' || p[i] == '-') {
        neg = p[i] == '-';
        ++i;
    }
    if (i == j || p[i] < '0' || p[i] > '9') return -1;
    uint64_t v = 0;
    bool over = false;
    size_t digits = 0;
    for (size_t k = i; k < j; ++k) {
        const char c = p[k];
        if (c == '_') {
            if (k + 1 >= j || p[k + 1] < '0' || p[k + 1] > '9' || p[k - 1] < '0' || p[k - 1] > '9') return -1;
            continue;
        }
        if (c < '0' || c > '9') return -1;
        ++digits;
        if (!over) {
            if (v > (UINT64_MAX - 9) / 10) over = true;
            else v = v * 10 + static_cast<uint64_t>(c - '0');
        }
    }
    if (digits > kPyMaxStrDigits) return -1;
    if (over || v > (neg ? uint64_t(INT64_MAX) + 1 : uint64_t(INT64_MAX))) return 1;
    *out = neg ? static_cast<int64_t>(0 - v) : static_cast<int64_t>(v);
    return 0;
}

// the value of a string py_int_ex accepted, as two's complement u32 limbs
// (little-endian, shortest form with at least 2 limbs)
inline void py_int_limbs(const char *p, size_t n, std::vector<uint32_t> &limbs) {
    limbs.assign(2, 0u);
    bool neg = false;
    for (size_t k = 0; k < n; ++k) {
        const char c = p[k];
        if (c == '-') neg = true;
        if (c < '0' || c > '9') continue;
        uint64_t carry = static_cast<uint64_t>(c - '0');
        for (auto &l : limbs) {
            carry += static_cast<uint64_t>(l) * 10u;
            l = static_cast<uint32_t>(carry);
            carry >>= 32;
        }
        if (carry) limbs.push_back(static_cast<uint32_t>(carry));
    }
    limbs.push_back(0u);  // room for the sign bit of the magnitude
    if (neg) {
        uint64_t c = 1;
        for (auto &l : limbs) {
            c += static_cast<uint32_t>(~l);
            l = static_cast<uint32_t>(c);
            c >>= 32;
        }
    }
    while (limbs.size() > 2) {  // drop limbs that only repeat the sign
        const uint32_t s = (limbs[limbs.size() - 2] >> 31) ? 0xffffffffu : 0u;
        if (limbs.back() != s) break;
        limbs.pop_back();
    }
}
inline void i64_limbs(int64_t v, std::vector<uint32_t> &limbs) {
    limbs.assign({static_cast<uint32_t>(static_cast<uint64_t>(v)), static_cast<uint32_t>(static_cast<uint64_t>(v) >> 32)});
}

// 64-bit allele key.  Alleles of <= 8 printable-ASCII bytes are packed
// verbatim (exact, bit 63 clear); anything else is a 63-bit hash with bit 63
// set, and equal keys are confirmed byte-for-byte on the device.
inline uint64_t allele_key(const uint8_t *p, size_t n, bool to_upper, bool *hashed) {
    if (n <= 8) {
        uint64_t k = 0;
        bool ok = true;
        for (size_t i = 0; i < n; ++i) {
            const uint8_t c = to_upper ? upc(p[i]) : p[i];
            if (c == 0 || c >= 0x80) ok = false;
            k |= static_cast<uint64_t>(c) << (8 * i);
        }
        if (ok) {
            *hashed = false;
            return k;
        }
    }
    uint64_t h = 0xcbf29ce484222325ull ^ (static_cast<uint64_t>(n) * 0x9E3779B97F4A7C15ull);
    for (size_t i = 0; i < n; ++i) {
        h ^= to_upper ? upc(p[i]) : p[i];
        h *= 0x100000001b3ull;
    }
    h ^= h >> 31;
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 29;
    *hashed = true;
    return h | (1ull << 63);
}

}  // namespace sb
