// nfgpu_guidmap.hpp — NFGUID -> index hash table shared by libnfgpu.so and the C++ plugin (an
// internal helper, not part of the C-ABI).
#pragma once
#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

#include "nfgpu_hugealloc.hpp"

namespace nfgpu_detail {

// NFGUID -> object index (the reference's NFMapEx<NFGUID, NFIObject> lookup, KM:323): open
// addressing, linear probing, backward-shift deletion; every SetProperty / schedule call does one
// lookup, so this is the host's per-call cost
class GuidMap {
public:
    int32_t find(int64_t h, int64_t d) const {
        if (cap_ == 0) return -1;
        for (size_t i = slot(h, d);; i = (i + 1) & (cap_ - 1)) {
            const E& e = t_[i];
            if (e.v < 0) return -1;
            if (e.h == h && e.d == d) return e.v;
        }
    }
    bool count(int64_t h, int64_t d) const { return find(h, d) >= 0; }
    // n lookups with the home slots of the lookups kPre ahead prefetched (a batch of calls is
    // bound by the table's cache misses, not by the probing)
    void find_many(int32_t n, const int64_t* h, const int64_t* d, int32_t* out) const {
        constexpr int32_t kPre = 32;
        if (cap_ == 0) {
            for (int32_t i = 0; i < n; i++) out[i] = -1;
            return;
        }
        for (int32_t i = 0; i < n && i < kPre; i++) __builtin_prefetch(&t_[slot(h[i], d[i])]);
        for (int32_t i = 0; i < n; i++) {
            if (i + kPre < n) __builtin_prefetch(&t_[slot(h[i + kPre], d[i + kPre])]);
            out[i] = find(h[i], d[i]);
        }
    }
    void insert(int64_t h, int64_t d, int32_t v) {
        if ((n_ + 1) * 2 > cap_) rehash(std::max<size_t>(64, cap_ * 2));
        size_t i = slot(h, d);
        for (; t_[i].v >= 0; i = (i + 1) & (cap_ - 1))
            if (t_[i].h == h && t_[i].d == d) {
                t_[i].v = v;
                logged(i);
                return;
            }
        t_[i] = E{h, d, v};
        logged(i);
        n_++;
    }
    void erase(int64_t h, int64_t d) {
        if (cap_ == 0) return;
        size_t i = slot(h, d);
        for (;; i = (i + 1) & (cap_ - 1)) {
            if (t_[i].v < 0) return;
            if (t_[i].h == h && t_[i].d == d) break;
        }
        // backward shift: pull later members of the probe run into the hole
        for (size_t j = (i + 1) & (cap_ - 1);; j = (j + 1) & (cap_ - 1)) {
            if (t_[j].v < 0) break;
            const size_t home = slot(t_[j].h, t_[j].d);
            if (((j - home) & (cap_ - 1)) >= ((j - i) & (cap_ - 1))) {
                t_[i] = t_[j];
                logged(i);
                i = j;
            }
        }
        t_[i].v = -1;
        logged(i);
        n_--;
    }

    // A mirror of the table elsewhere (the world's device copy, nfgpu_host.hip find_many_dev)
    // follows it through a log of the entries every insert / erase wrote, and a rewrite flag set
    // when the table was rebuilt at a new capacity.
    struct E {
        int64_t h, d;
        int32_t v = -1;
    };
    void set_log(std::vector<uint32_t>* log) { log_ = log; }
    bool take_rebuilt() {
        const bool r = rebuilt_;
        rebuilt_ = false;
        return r;
    }
    const E* entries() const { return t_.data(); }
    size_t capacity() const { return cap_; }
    size_t size() const { return n_; }
    // the home entry of a GUID (the device mirror's lookups hash the same way)
    static size_t home(int64_t h, int64_t d, size_t mask) {
        uint64_t x = (uint64_t)h * 0x9E3779B97F4A7C15ull ^ (uint64_t)d;
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        return (size_t)x & mask;
    }

private:
    size_t slot(int64_t h, int64_t d) const { return home(h, d, cap_ - 1); }
    void logged(size_t i) {
        if (log_ && !rebuilt_) log_->push_back((uint32_t)i);
    }
    void rehash(size_t c) {
        std::vector<E, HugeAlloc<E>> old;
        old.swap(t_);
        t_.assign(c, E{});
        cap_ = c;
        n_ = 0;
        rebuilt_ = true;  // (the mirror is rewritten whole; the log restarts)
        if (log_) log_->clear();
        for (const E& e : old)
            if (e.v >= 0) insert(e.h, e.d, e.v);
    }
    std::vector<E, HugeAlloc<E>> t_;
    size_t cap_ = 0, n_ = 0;
    std::vector<uint32_t>* log_ = nullptr;
    bool rebuilt_ = false;
};

}  // namespace nfgpu_detail
