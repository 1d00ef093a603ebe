// Small-block allocator for the interpreter's byte vectors (script stack elements, script codes,
// witness programs).  A P2WPKH spend makes about 20 such allocations in the reference-shaped
// interpreter (stack copies, pushes, OP_DUP / OP_HASH160 results); through malloc they were the
// largest single cost of the host pass.  Blocks of four size classes (32 / 80 / 128 / 544 bytes:
// MAX_SCRIPT_ELEMENT_SIZE 520 fits the last) come from per-thread free lists; a thread refills
// from, and at exit returns its lists to, a global reservoir, so the engine's short-lived worker
// threads do not leak.  Larger requests go to operator new.  Blocks are never returned to the OS.
#pragma once
#include <cstddef>
#include <cstdint>
#include <new>

namespace bcc {
namespace host {

void* pool_alloc(size_t bytes);
void pool_free(void* p, size_t bytes);
size_t pool_chunks();  // 64 KiB chunks carved so far (tests: the reservoir bounds the growth)

template <class T>
struct PoolAlloc {
    using value_type = T;
    PoolAlloc() noexcept = default;
    template <class U>
    PoolAlloc(const PoolAlloc<U>&) noexcept {}
    T* allocate(size_t n) { return static_cast<T*>(pool_alloc(n * sizeof(T))); }
    void deallocate(T* p, size_t n) noexcept { pool_free(p, n * sizeof(T)); }
    template <class U>
    bool operator==(const PoolAlloc<U>&) const noexcept { return true; }
    template <class U>
    bool operator!=(const PoolAlloc<U>&) const noexcept { return false; }
};

}  // namespace host
}  // namespace bcc
