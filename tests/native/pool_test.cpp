// tests/native/pool_test.cpp — TEST ONLY: the interpreter's small-block allocator
// (rust-bitcoinconsensus_amd/csrc/host/pool.cpp) under the engine's usage pattern: many short-lived
// threads allocating, growing, copying and freeing byte vectors of every size class.
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "../../rust-bitcoinconsensus_amd/csrc/host/pool.h"

using Bytes = std::vector<uint8_t, bcc::host::PoolAlloc<uint8_t>>;

// one round of T threads, each running `ops` random stack operations with content checks;
// returns the number of content mismatches
extern "C" long pool_stress(int T, int ops, unsigned seed) {
    std::vector<long> bad(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
            std::mt19937 rng(seed * 131 + t);
            std::vector<Bytes> stack;
            std::vector<uint8_t> tag;  // expected fill byte per element
            for (int i = 0; i < ops; i++) {
                const unsigned r = rng() % 8;
                if (r < 4 || stack.empty()) {
                    const size_t n = (size_t)(rng() % 4 == 0 ? rng() % 1200 : rng() % 90);
                    const uint8_t v = (uint8_t)rng();
                    stack.emplace_back(n, v);
                    tag.push_back(v);
                } else if (r < 6) {
                    const Bytes& b = stack.back();
                    for (uint8_t c : b) bad[t] += c != tag.back();
                    stack.pop_back();
                    tag.pop_back();
                } else if (r == 6) {
                    stack.push_back(stack.back());  // OP_DUP-like copy
                    tag.push_back(tag.back());
                } else {
                    Bytes& b = stack.back();  // growth across size classes
                    b.insert(b.end(), (size_t)(rng() % 200), tag.back());
                }
            }
            for (size_t k = 0; k < stack.size(); k++)
                for (uint8_t c : stack[k]) bad[t] += c != tag[k];
        });
    for (auto& x : th) x.join();
    long s = 0;
    for (long b : bad) s += b;
    return s;
}

extern "C" size_t pool_chunk_count() { return bcc::host::pool_chunks(); }
