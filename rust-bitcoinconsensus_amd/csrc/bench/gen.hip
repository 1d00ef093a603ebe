// Synthetic-workload kernels (bench / tests only — not on the verification path):
//   keygen_kernel  Q = d*G   -> affine x, y (big-endian)
//   sign_kernel    (r, s) = ECDSA-sign(d, m, k), low-S
//   schnorr_sign_kernel  BIP340 sig64 + x-only key for (d, m, nonce k)
// Both reuse the verify engine's field/group code and LDS-staged G tables.
#include "ecdsa_lane.h"
#include "gpu_common.h"

namespace bcc {

namespace {

struct GTableLDS {
    const fe* xy;
    __device__ void get(int tab, int i, fe& x, fe& y) const {
        x = xy[(tab * GTAB + i) * 2 + 0];
        y = xy[(tab * GTAB + i) * 2 + 1];
    }
};

__device__ void load_sc(sc& r, const uint8_t* p) {
    fe t;
    fe_from_be_bytes(t, p);
    for (int i = 0; i < 8; i++) r.v[i] = t.v[i];
}
__device__ void store_sc(uint8_t* p, const sc& a) {
    fe t;
    for (int i = 0; i < 8; i++) t.v[i] = a.v[i];
    fe_to_be_bytes(p, t);
}

__global__ __launch_bounds__(256) void keygen_kernel(const uint8_t* __restrict__ d32,
                                                     uint8_t* __restrict__ x32,
                                                     uint8_t* __restrict__ y32,
                                                     uint8_t* __restrict__ ok, const fe* gtab,
                                                     size_t n) {
    __shared__ fe g[2 * GTAB * 2];
    for (int i = threadIdx.x; i < 2 * GTAB * 2; i += blockDim.x) g[i] = gtab[i];
    __syncthreads();
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sc d;
    load_sc(d, d32 + 32 * i);
    fe x, y;
    GTableLDS gt{g};
    bool good = ecmult_gen_lane(d, x, y, gt);
    fe_to_be_bytes(x32 + 32 * i, x);
    fe_to_be_bytes(y32 + 32 * i, y);
    ok[i] = good;
}

__global__ __launch_bounds__(256) void sign_kernel(const uint8_t* __restrict__ d32,
                                                   const uint8_t* __restrict__ m32,
                                                   const uint8_t* __restrict__ k32,
                                                   uint8_t* __restrict__ r32,
                                                   uint8_t* __restrict__ s32,
                                                   uint8_t* __restrict__ ok, const fe* gtab,
                                                   size_t n) {
    __shared__ fe g[2 * GTAB * 2];
    for (int i = threadIdx.x; i < 2 * GTAB * 2; i += blockDim.x) g[i] = gtab[i];
    __syncthreads();
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sc d, m, k, r, s;
    load_sc(d, d32 + 32 * i);
    load_sc(m, m32 + 32 * i);
    load_sc(k, k32 + 32 * i);
    GTableLDS gt{g};
    bool good = ecdsa_sign_lane(d, m, k, r, s, gt);
    store_sc(r32 + 32 * i, r);
    store_sc(s32 + 32 * i, s);
    ok[i] = good;
}

__global__ __launch_bounds__(256) void schnorr_sign_kernel(const uint8_t* __restrict__ d32,
                                                           const uint8_t* __restrict__ m32,
                                                           const uint8_t* __restrict__ k32,
                                                           uint8_t* __restrict__ sig64,
                                                           uint8_t* __restrict__ xonly32,
                                                           uint8_t* __restrict__ ok,
                                                           const fe* gtab, size_t n) {
    __shared__ fe g[2 * GTAB * 2];
    for (int i = threadIdx.x; i < 2 * GTAB * 2; i += blockDim.x) g[i] = gtab[i];
    __syncthreads();
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    sc d, m, k, s;
    load_sc(d, d32 + 32 * i);
    load_sc(m, m32 + 32 * i);
    load_sc(k, k32 + 32 * i);
    fe rx, px;
    GTableLDS gt{g};
    bool good = schnorr_sign_lane(d, m, k, rx, s, px, gt);
    fe_to_be_bytes(sig64 + 64 * i, rx);
    store_sc(sig64 + 64 * i + 32, s);
    fe_to_be_bytes(xonly32 + 32 * i, px);
    ok[i] = good;
}

const std::vector<fe>& gtab_host() {
    static std::vector<fe> t;
    static std::once_flag once;
    std::call_once(once, [] {
        t.resize(2 * GTAB * 2);
        build_g_tables(t.data());
    });
    return t;
}

}  // namespace

}  // namespace bcc

using namespace bcc;

extern "C" {

// Q_i = d_i * G for n big-endian scalars; x32/y32 receive the affine coordinates, ok[i] = 1
// unless d_i == 0 mod n.  Host buffers; synchronous on `device`.
int mi_gen_pubkeys(const uint8_t* d32, size_t n, uint8_t* x32, uint8_t* y32, uint8_t* ok,
                   int device) {
    if (n == 0) return 0;
    BCC_HIP_TRY(hipSetDevice(device));
    const auto& g = gtab_host();
    uint8_t* buf = nullptr;
    size_t gbytes = g.size() * sizeof(fe);
    BCC_HIP_TRY(hipMalloc(&buf, gbytes + 97 * n + 256));
    fe* dg = (fe*)buf;
    uint8_t *dd = buf + gbytes, *dx = dd + 32 * n, *dy = dx + 32 * n, *dok = dy + 32 * n;
    int rc = 0;
    if ((rc = (int)hipMemcpy(dg, g.data(), gbytes, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(dd, d32, 32 * n, hipMemcpyHostToDevice))) {
        (void)hipFree(buf);
        return rc;
    }
    hipLaunchKernelGGL(keygen_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dd, dx,
                       dy, dok, dg, n);
    if ((rc = (int)hipGetLastError()) || (rc = (int)hipDeviceSynchronize()) ||
        (rc = (int)hipMemcpy(x32, dx, 32 * n, hipMemcpyDeviceToHost)) ||
        (rc = (int)hipMemcpy(y32, dy, 32 * n, hipMemcpyDeviceToHost)) ||
        (rc = (int)hipMemcpy(ok, dok, n, hipMemcpyDeviceToHost))) {
    }
    (void)hipFree(buf);
    return rc;
}

// ECDSA signatures (r, s) for n (d, m, k) triples (big-endian), low-S normalised.
int mi_gen_sign(const uint8_t* d32, const uint8_t* m32, const uint8_t* k32, size_t n,
                uint8_t* r32, uint8_t* s32, uint8_t* ok, int device) {
    if (n == 0) return 0;
    BCC_HIP_TRY(hipSetDevice(device));
    const auto& g = gtab_host();
    uint8_t* buf = nullptr;
    size_t gbytes = g.size() * sizeof(fe);
    BCC_HIP_TRY(hipMalloc(&buf, gbytes + 161 * n + 256));
    fe* dg = (fe*)buf;
    uint8_t *dd = buf + gbytes, *dm = dd + 32 * n, *dk = dm + 32 * n, *dr = dk + 32 * n,
            *ds = dr + 32 * n, *dok = ds + 32 * n;
    int rc = 0;
    if ((rc = (int)hipMemcpy(dg, g.data(), gbytes, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(dd, d32, 32 * n, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(dm, m32, 32 * n, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(dk, k32, 32 * n, hipMemcpyHostToDevice))) {
        (void)hipFree(buf);
        return rc;
    }
    hipLaunchKernelGGL(sign_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dd, dm,
                       dk, dr, ds, dok, dg, n);
    if ((rc = (int)hipGetLastError()) || (rc = (int)hipDeviceSynchronize()) ||
        (rc = (int)hipMemcpy(r32, dr, 32 * n, hipMemcpyDeviceToHost)) ||
        (rc = (int)hipMemcpy(s32, ds, 32 * n, hipMemcpyDeviceToHost)) ||
        (rc = (int)hipMemcpy(ok, dok, n, hipMemcpyDeviceToHost))) {
    }
    (void)hipFree(buf);
    return rc;
}

// BIP340 signatures sig64 = x(R) || s for n (d, m, k) triples (big-endian scalars, k the nonce)
// and the signers' x-only keys.  ok[i] = 0 when d or k is 0 mod n.
int mi_gen_schnorr_sign(const uint8_t* d32, const uint8_t* m32, const uint8_t* k32, size_t n,
                        uint8_t* sig64, uint8_t* xonly32, uint8_t* ok, int device) {
    if (n == 0) return 0;
    BCC_HIP_TRY(hipSetDevice(device));
    const auto& g = gtab_host();
    uint8_t* buf = nullptr;
    size_t gbytes = g.size() * sizeof(fe);
    BCC_HIP_TRY(hipMalloc(&buf, gbytes + 193 * n + 256));
    fe* dg = (fe*)buf;
    uint8_t *dd = buf + gbytes, *dm = dd + 32 * n, *dk = dm + 32 * n, *dsig = dk + 32 * n,
            *dx = dsig + 64 * n, *dok = dx + 32 * n;
    int rc = 0;
    if ((rc = (int)hipMemcpy(dg, g.data(), gbytes, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(dd, d32, 32 * n, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(dm, m32, 32 * n, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(dk, k32, 32 * n, hipMemcpyHostToDevice))) {
        (void)hipFree(buf);
        return rc;
    }
    hipLaunchKernelGGL(schnorr_sign_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0,
                       dd, dm, dk, dsig, dx, dok, dg, n);
    if ((rc = (int)hipGetLastError()) || (rc = (int)hipDeviceSynchronize()) ||
        (rc = (int)hipMemcpy(sig64, dsig, 64 * n, hipMemcpyDeviceToHost)) ||
        (rc = (int)hipMemcpy(xonly32, dx, 32 * n, hipMemcpyDeviceToHost)) ||
        (rc = (int)hipMemcpy(ok, dok, n, hipMemcpyDeviceToHost))) {
    }
    (void)hipFree(buf);
    return rc;
}

}  // extern "C"
