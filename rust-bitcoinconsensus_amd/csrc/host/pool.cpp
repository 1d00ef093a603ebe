// Small-block allocator of the interpreter (pool.h).
#include "pool.h"

#include <cstdlib>
#include <mutex>

namespace bcc {
namespace host {
namespace {

constexpr int NCLASS = 4;
constexpr size_t CLASS_BYTES[NCLASS] = {32, 80, 128, 544};
constexpr size_t CHUNK_BYTES = 64 << 10;
constexpr int REFILL = 128;  // blocks a thread takes from the reservoir at a time

struct Block {
    Block* next;
};

int size_class(size_t bytes) {
    for (int c = 0; c < NCLASS; c++)
        if (bytes <= CLASS_BYTES[c]) return c;
    return -1;
}

std::mutex g_mu;
Block* g_free[NCLASS] = {};  // the reservoir (guarded by g_mu)
size_t g_chunks = 0;         // chunks carved so far (guarded by g_mu)

struct Cache {
    Block* head[NCLASS] = {};
    ~Cache() {  // thread exit: hand every block back to the reservoir
        std::lock_guard<std::mutex> lk(g_mu);
        for (int c = 0; c < NCLASS; c++) {
            while (Block* b = head[c]) {
                head[c] = b->next;
                b->next = g_free[c];
                g_free[c] = b;
            }
        }
    }
};
thread_local Cache tl_cache;

void refill(Cache& pc, int c) {
    std::lock_guard<std::mutex> lk(g_mu);
    for (int k = 0; k < REFILL && g_free[c]; k++) {
        Block* b = g_free[c];
        g_free[c] = b->next;
        b->next = pc.head[c];
        pc.head[c] = b;
    }
    if (pc.head[c]) return;
    // carve a new chunk into blocks of this class (never freed: bounded by the peak live count)
    char* m = static_cast<char*>(std::malloc(CHUNK_BYTES));
    if (!m) throw std::bad_alloc();
    g_chunks++;
    const size_t sz = CLASS_BYTES[c];
    for (size_t off = 0; off + sz <= CHUNK_BYTES; off += sz) {
        Block* b = reinterpret_cast<Block*>(m + off);
        b->next = pc.head[c];
        pc.head[c] = b;
    }
}

}  // namespace

size_t pool_chunks() {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_chunks;
}

void* pool_alloc(size_t bytes) {
    const int c = size_class(bytes);
    if (c < 0) return ::operator new(bytes);
    Cache& pc = tl_cache;
    if (!pc.head[c]) refill(pc, c);
    Block* b = pc.head[c];
    pc.head[c] = b->next;
    return b;
}

void pool_free(void* p, size_t bytes) {
    if (!p) return;
    const int c = size_class(bytes);
    if (c < 0) {
        ::operator delete(p);
        return;
    }
    Cache& pc = tl_cache;
    Block* b = static_cast<Block*>(p);
    b->next = pc.head[c];
    pc.head[c] = b;
}

}  // namespace host
}  // namespace bcc
