// Host-side hash functions used by the script interpreter (OP_SHA256 / OP_HASH160 / ...), by the
// sighash preimage builders and by the synthetic-workload generator.
// Restates crypto/sha256.cpp, crypto/sha1.cpp, crypto/ripemd160.cpp (standard FIPS 180-4 /
// RIPEMD-160 algorithms) and hash.h's CHash256 / CHash160 compositions.
#pragma once
#include <cstddef>
#include <cstdint>

namespace bcc {
namespace host {

struct Sha256 {
    uint32_t s[8];
    uint8_t buf[64];
    uint64_t bytes;
    Sha256();
    Sha256& write(const uint8_t* p, size_t n);
    void finalize(uint8_t out[32]);
};

void sha256(const uint8_t* p, size_t n, uint8_t out[32]);
void sha256d(const uint8_t* p, size_t n, uint8_t out[32]);              // CHash256
void sha1(const uint8_t* p, size_t n, uint8_t out[20]);
void ripemd160(const uint8_t* p, size_t n, uint8_t out[20]);
bool sha256_uses_shani();                                                 // x86 SHA extensions in use
void hash160(const uint8_t* p, size_t n, uint8_t out[20]);              // RIPEMD160(SHA256(x))
// hash160 of count messages (eight at a time: RIPEMD-160 of the digests on AVX2 when present)
void hash160_batch(const uint8_t* const* p, const size_t* n, uint8_t* const* out, size_t count);

}  // namespace host
}  // namespace bcc
