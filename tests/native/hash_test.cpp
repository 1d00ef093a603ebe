// TEST ONLY: C exports of the engine's host hash functions (csrc/host/hashes.cpp) for
// tests/test_host_hashes.py.
#include "../../rust-bitcoinconsensus_amd/csrc/host/hashes.h"
#include "../../rust-bitcoinconsensus_amd/csrc/sha256_device.h"

extern "C" {
void th_sha256(const unsigned char* p, unsigned long n, unsigned char* out) { bcc::host::sha256(p, n, out); }
void th_sha1(const unsigned char* p, unsigned long n, unsigned char* out) { bcc::host::sha1(p, n, out); }
void th_ripemd160(const unsigned char* p, unsigned long n, unsigned char* out) { bcc::host::ripemd160(p, n, out); }
void th_hash160(const unsigned char* p, unsigned long n, unsigned char* out) { bcc::host::hash160(p, n, out); }
// the device-side key HASH160 (sha256_device.h key_hash160, run here as host code) of the key
// tag || x (|| y)
void th_key_hash160(unsigned tag, const unsigned char* x, const unsigned char* y, unsigned char* out) {
    uint32_t xw[8], yw[8], h[5];
    for (int i = 0; i < 8; i++) {
        xw[i] = (uint32_t)x[4 * i] << 24 | (uint32_t)x[4 * i + 1] << 16 | (uint32_t)x[4 * i + 2] << 8 | x[4 * i + 3];
        yw[i] = (uint32_t)y[4 * i] << 24 | (uint32_t)y[4 * i + 1] << 16 | (uint32_t)y[4 * i + 2] << 8 | y[4 * i + 3];
    }
    bcc::key_hash160(tag, xw, yw, h);
    for (int i = 0; i < 20; i++) out[i] = (unsigned char)(h[i / 4] >> (8 * (i % 4)));
}
int th_shani() { return bcc::host::sha256_uses_shani() ? 1 : 0; }
// hash160_batch over count messages packed back to back (lengths in n), digests to out[20 * i]
void th_hash160_batch(const unsigned char* blob, const unsigned long* n, unsigned long count,
                      unsigned char* out) {
    const unsigned char* ptr[64];
    size_t len[64];
    unsigned char* o[64];
    size_t at = 0;
    for (unsigned long i = 0; i < count && i < 64; i++) {
        ptr[i] = blob + at;
        len[i] = n[i];
        o[i] = out + 20 * i;
        at += n[i];
    }
    bcc::host::hash160_batch(ptr, len, o, count < 64 ? count : 64);
}
}
