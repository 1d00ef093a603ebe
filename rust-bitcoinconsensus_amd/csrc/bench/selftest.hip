// Field-arithmetic self-test entry point (tests/test_field_gpu.py): runs one device field
// operation over caller-supplied operands so the inline-asm carry chains -- including their
// rare wave-uniform fold branches -- are checked against Python big integers.
#include "gpu_common.h"
#include "secp256k1_device.h"

namespace bcc {

__global__ __launch_bounds__(256) void fe_selftest_kernel(int op, const u32* __restrict__ a,
                                                          const u32* __restrict__ b,
                                                          u32* __restrict__ out, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    fe x, y, r;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        x.v[j] = a[i * 8 + j];
        y.v[j] = b[i * 8 + j];
    }
    r = fe_zero();
    switch (op) {
        case 0: fe_add(r, x, y); break;
        case 1: fe_sub(r, x, y); break;
        case 2: fe_mul(r, x, y); break;
        case 3: fe_sqr(r, x); break;
        case 4: fe_shl<1>(r, x); break;
        case 5: fe_shl<2>(r, x); break;
        case 6: fe_shl<3>(r, x); break;
        case 7: fe_neg(r, x); break;
        case 8: r.v[0] = fe_is_zero(x) ? 1u : 0u; break;
        case 9: r = x; fe_normalize(r); break;
        case 10: fe_inv(r, x); break;  // weak input, normalized inverse
        case 11: {                     // scalar inverse of x < n
            sc xs, rs;
#pragma unroll
            for (int j = 0; j < 8; j++) xs.v[j] = x.v[j];
            sc_inv(rs, xs);
#pragma unroll
            for (int j = 0; j < 8; j++) r.v[j] = rs.v[j];
            break;
        }
        default: break;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) out[i * 8 + j] = r.v[j];
}

}  // namespace bcc

extern "C" {

// a, b, out: n x 8 little-endian u32 limbs (host memory).  op: 0 add, 1 sub, 2 mul, 3 sqr,
// 4/5/6 shift left by 1/2/3, 7 neg, 8 is_zero (out[0]), 9 normalize, 10 fe_inv, 11 sc_inv (a < n).
// 0 on success.
int mi_fe_selftest(int op, const uint32_t* a, const uint32_t* b, uint32_t* out, size_t n) {
    using namespace bcc;
    if (n == 0) return 0;
    size_t bytes = n * 32;
    u32 *da = nullptr, *db = nullptr, *dout = nullptr;
    BCC_HIP_TRY(hipMalloc(&da, bytes));
    BCC_HIP_TRY(hipMalloc(&db, bytes));
    BCC_HIP_TRY(hipMalloc(&dout, bytes));
    BCC_HIP_TRY(hipMemcpy(da, a, bytes, hipMemcpyHostToDevice));
    BCC_HIP_TRY(hipMemcpy(db, b, bytes, hipMemcpyHostToDevice));
    unsigned grid = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(fe_selftest_kernel, dim3(grid), dim3(256), 0, 0, op, da, db, dout, n);
    BCC_HIP_TRY(hipGetLastError());
    BCC_HIP_TRY(hipMemcpy(out, dout, bytes, hipMemcpyDeviceToHost));
    (void)hipFree(da);
    (void)hipFree(db);
    (void)hipFree(dout);
    return 0;
}

}  // extern "C"
