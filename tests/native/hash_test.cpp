// TEST ONLY: C exports of the engine's host hash functions (csrc/host/hashes.cpp) for
// tests/test_host_hashes.py.
#include "../../rust-bitcoinconsensus_amd/csrc/host/hashes.h"

extern "C" {
void th_sha256(const unsigned char* p, unsigned long n, unsigned char* out) { bcc::host::sha256(p, n, out); }
void th_sha1(const unsigned char* p, unsigned long n, unsigned char* out) { bcc::host::sha1(p, n, out); }
void th_ripemd160(const unsigned char* p, unsigned long n, unsigned char* out) { bcc::host::ripemd160(p, n, out); }
void th_hash160(const unsigned char* p, unsigned long n, unsigned char* out) { bcc::host::hash160(p, n, out); }
int th_shani() { return bcc::host::sha256_uses_shani() ? 1 : 0; }
}
