// host_pool.h — host memory for the ILU analysis' large arrays.
//
// The analysis builds a few hundred MB of host arrays per pattern (levels,
// plans, the downloaded pattern and symbolic data) and frees them when it
// returns. With glibc's defaults every array of >= 32 MiB (and most of the
// smaller ones) is a fresh anonymous mapping, so each analysis pays one page
// fault + zeroing per 4 KiB on first touch. Measured on the MI355X box
// (config 3, 21 matrices, 3rd of 3 reps): 490 ms as is, 317 ms with
// GLIBC_TUNABLES=glibc.malloc.hugetlb=1, 290 ms with freed memory kept in the
// heap (mmap/trim thresholds raised) — the library cannot set either for its
// caller's process, so it keeps its own blocks:
//
//   * blocks of >= kPoolMin bytes come from a process-wide cache of 2-MiB
//     aligned blocks (transparent huge pages requested with madvise: one
//     fault per 2 MiB when a block is first touched) and go back to it when
//     freed, so the next array of that size class is already mapped;
//   * the cache keeps at most RSP_HOST_POOL_MB (default 1024) of free blocks;
//     beyond that a freed block is returned to the system;
//   * smaller blocks use the global operator new.
//
// Thread-safe (one mutex: the analysis allocates from its worker threads).
#ifndef RSP_HOST_POOL_H
#define RSP_HOST_POOL_H

#include <stddef.h>

#include <new>
#include <type_traits>
#include <vector>

namespace rsp_an {

void *pool_get(size_t bytes);            // >= kPoolMin bytes; throws std::bad_alloc
void pool_put(void *p, size_t bytes);    // bytes as given to pool_get
constexpr size_t kPoolMin = 1u << 20;

template <typename T>
struct PoolAlloc {
    using value_type = T;
    PoolAlloc() noexcept = default;
    template <typename U>
    PoolAlloc(const PoolAlloc<U> &) noexcept {}
    // elements added by resize() / a size constructor are value-initialised
    // (zeroed), unless resize_uninit (below) is on the stack of this thread
    template <typename U, typename... A>
    void construct(U *p, A &&...a) {
        ::new ((void *)p) U(static_cast<A &&>(a)...);
    }
    template <typename U>
    void construct(U *p) {
        if (uninit_scope())
            ::new ((void *)p) U;
        else
            ::new ((void *)p) U();
    }
    static bool &uninit_scope() {
        static thread_local bool on = false;
        return on;
    }
    T *allocate(size_t n) {
        const size_t b = n * sizeof(T);
        if (b >= kPoolMin) return static_cast<T *>(pool_get(b));
        return static_cast<T *>(::operator new(b));
    }
    void deallocate(T *p, size_t n) noexcept {
        const size_t b = n * sizeof(T);
        if (b >= kPoolMin)
            pool_put(p, b);
        else
            ::operator delete(p);
    }
    template <typename U>
    bool operator==(const PoolAlloc<U> &) const noexcept { return true; }
    template <typename U>
    bool operator!=(const PoolAlloc<U> &) const noexcept { return false; }
};

// the analysis' vectors
template <typename T>
using hvec = std::vector<T, PoolAlloc<T>>;

// v.resize(n) without zeroing the new elements (trivial T only): for arrays
// that a transfer or a loop overwrites whole right after (round 6: zeroing
// the downloaded pattern, update pointers and stages cost ~3 x 4 B per
// stored entry of serial memset per analysis)
template <typename T>
void resize_uninit(hvec<T> &v, size_t n) {
    static_assert(std::is_trivially_default_constructible<T>::value, "trivial types only");
    bool &on = PoolAlloc<T>::uninit_scope();
    on = true;
    try {
        v.resize(n);
    } catch (...) {
        on = false;
        throw;
    }
    on = false;
}

}  // namespace rsp_an

#endif
