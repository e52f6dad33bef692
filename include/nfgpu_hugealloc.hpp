// nfgpu_hugealloc.hpp — std::allocator replacement for the host tables the frame reads at random
// (the NFGUID table, the per-(object, kind) functor slots and pool, the object NFGUIDs): a block of
// 2 MB or more is allocated 2 MB-aligned and advised for transparent huge pages (MADV_HUGEPAGE;
// the hosts run THP in "madvise" mode), so a random read of a 100 MB table costs a cache miss, not a
// cache miss and a page walk.  NFGPU_HUGEPAGES=0 turns the advice off (plain allocations).
#pragma once
#include <sys/mman.h>

#include <cstddef>
#include <cstdlib>
#include <new>

namespace nfgpu_detail {

inline bool huge_pages_on() {
    static const bool on = [] {
        const char* e = std::getenv("NFGPU_HUGEPAGES");
        return !(e && e[0] == '0');
    }();
    return on;
}

template <class T>
struct HugeAlloc {
    using value_type = T;
    static constexpr size_t kHuge = size_t(2) << 20;
    HugeAlloc() = default;
    template <class U>
    HugeAlloc(const HugeAlloc<U>&) {}
    // (the same size test on both sides: allocate and deallocate see the same n)
    static bool huge(size_t n) { return n * sizeof(T) >= kHuge && huge_pages_on(); }
    T* allocate(size_t n) {
        if (!huge(n)) return static_cast<T*>(::operator new(n * sizeof(T)));
        const size_t bytes = (n * sizeof(T) + kHuge - 1) & ~(kHuge - 1);
        void* p = nullptr;
        if (posix_memalign(&p, kHuge, bytes) != 0) throw std::bad_alloc();
        madvise(p, bytes, MADV_HUGEPAGE);  // (advice only: a refusal leaves ordinary pages)
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t n) {
        if (!huge(n)) ::operator delete(p);
        else std::free(p);
    }
};
template <class T, class U>
bool operator==(const HugeAlloc<T>&, const HugeAlloc<U>&) { return true; }
template <class T, class U>
bool operator!=(const HugeAlloc<T>&, const HugeAlloc<U>&) { return false; }

}  // namespace nfgpu_detail
