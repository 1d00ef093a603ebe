// Integer-ALU microbenchmarks for gfx950: the measured peak that roofline.peak is quoted
// against (achieved = verifies/s * 144,448 / peak v_mad_u64_u32 per second).
// Each kernel runs 8 independent dependency chains per lane so issue rate, not latency, binds.
#include "gpu_common.h"

namespace bcc {

template <int OP>
__global__ __launch_bounds__(256) void ubench_kernel(uint32_t* out, int iters, uint32_t seed) {
    uint32_t a = seed ^ threadIdx.x, b = seed * 7u + blockIdx.x;
    uint64_t acc[8];
    uint32_t acc32[8];
    double accd[8];
    const double bd = 1.0 + 1e-9 * (double)b;
#pragma unroll
    for (int k = 0; k < 8; k++) {
        acc[k] = (uint64_t)(a + k) << 7;
        acc32[k] = a + 3 * k;
        accd[k] = (double)(a + k);
    }
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (OP == 0) {  // v_mad_u64_u32
                asm volatile("v_mad_u64_u32 %0, s[0:1], %1, %2, %0" : "+v"(acc[k]) : "v"(a), "v"(b) : "s0", "s1");
            } else if (OP == 1) {  // v_mul_lo_u32
                asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
            } else if (OP == 2) {  // v_mul_hi_u32
                asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
            } else if (OP == 3) {  // v_add_co_u32 (VOP3, carry out to SGPR)
                asm volatile("v_add_co_u32 %0, s[0:1], %0, %1" : "+v"(acc32[k]) : "v"(b) : "s0", "s1");
            } else if (OP == 4) {  // v_addc_co_u32 (carry in + out)
                asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(acc32[k]) : "v"(b) : "vcc");
            } else if (OP == 5) {  // v_mad_u32_u24
                asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc32[k]) : "v"(b));
            } else if (OP == 6) {  // v_lshl_add_u64
                asm volatile("v_lshl_add_u64 %0, %0, 1, %1" : "+v"(acc[k]) : "v"((uint64_t)b));
            } else if (OP == 7) {  // v_fma_f64 (reference for an FP-limb design)
                asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(accd[k]) : "v"(bd));
            } else if (OP == 8) {  // v_add_u32 (plain full-rate reference)
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
            } else if (OP == 9) {  // v_add3_u32
                asm volatile("v_add3_u32 %0, %0, %1, %0" : "+v"(acc32[k]) : "v"(b));
            } else if (OP == 10) {  // v_mul_u32_u24
                asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
            } else if (OP == 11) {  // v_mul_hi_u32_u24
                asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
            } else if (OP == 12) {  // v_alignbit_b32
                asm volatile("v_alignbit_b32 %0, %0, %1, 29" : "+v"(acc32[k]) : "v"(b));
            } else if (OP == 13) {  // v_lshrrev_b64
                asm volatile("v_lshrrev_b64 %0, 3, %0" : "+v"(acc[k]));
            } else if (OP == 14) {  // v_add_co_u32_e32 (VOP2, carry to VCC)
                asm volatile("v_add_co_u32_e32 %0, vcc, %0, %1" : "+v"(acc32[k]) : "v"(b) : "vcc");
            } else if (OP == 15) {  // v_cndmask_b32 (VCC select)
                asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(acc32[k]) : "v"(b) : "vcc");
            } else if (OP == 16) {  // v_mad_u64_u32 + v_addc_co_u32 pairs (rate per instruction)
                asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                             : "+v"(acc[k]), "+v"(acc32[k]) : "v"(a), "v"(b) : "vcc");
            } else if (OP == 17) {  // v_mul_lo_u32 + v_mul_hi_u32 pairs (rate per instruction)
                asm volatile("v_mul_lo_u32 %0, %0, %2\n\tv_mul_hi_u32 %1, %1, %2"
                             : "+v"(acc32[k]), "+v"(*((uint32_t*)&acc[k])) : "v"(b));
            } else if (OP == 18) {  // v_mad_u64_u32 + v_add_u32 pairs (full-rate filler)
                asm volatile("v_mad_u64_u32 %0, s[0:1], %2, %3, %0\n\tv_add_u32 %1, %1, %3"
                             : "+v"(acc[k]), "+v"(acc32[k]) : "v"(a), "v"(b) : "s0", "s1");
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++)
        r ^= (uint32_t)acc[k] ^ (uint32_t)(acc[k] >> 32) ^ acc32[k] ^ (uint32_t)(int64_t)accd[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

}  // namespace bcc

using namespace bcc;

extern "C" {

// Runs microbenchmark `op` (see ubench_kernel; 0..18) and returns lane-instructions per second
// in *rate. Synchronous, on the current device.
int mi_microbench(int op, int iters, double* rate) {
    int dev = 0, cus = 0;
    BCC_HIP_TRY(hipGetDevice(&dev));
    BCC_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int block = 256, grid = cus * 8;
    uint32_t* out = nullptr;
    BCC_HIP_TRY(hipMalloc(&out, (size_t)grid * block * 4));
    hipEvent_t e0, e1;
    BCC_HIP_TRY(hipEventCreate(&e0));
    BCC_HIP_TRY(hipEventCreate(&e1));
#define BCC_UB_CASE(K) \
    case K: hipLaunchKernelGGL(ubench_kernel<K>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
    auto launch = [&](int it) {
        switch (op) {
            BCC_UB_CASE(0) BCC_UB_CASE(1) BCC_UB_CASE(2) BCC_UB_CASE(3) BCC_UB_CASE(4)
            BCC_UB_CASE(5) BCC_UB_CASE(6) BCC_UB_CASE(7) BCC_UB_CASE(9) BCC_UB_CASE(10)
            BCC_UB_CASE(11) BCC_UB_CASE(12) BCC_UB_CASE(13) BCC_UB_CASE(14) BCC_UB_CASE(15)
            BCC_UB_CASE(16) BCC_UB_CASE(17) BCC_UB_CASE(18)
            default: hipLaunchKernelGGL(ubench_kernel<8>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
        }
    };
#undef BCC_UB_CASE
    launch(16);  // warm-up
    BCC_HIP_TRY(hipDeviceSynchronize());
    BCC_HIP_TRY(hipEventRecord(e0, 0));
    launch(iters);
    BCC_HIP_TRY(hipEventRecord(e1, 0));
    BCC_HIP_TRY(hipEventSynchronize(e1));
    float ms = 0;
    BCC_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    const int per = (op == 16 || op == 17 || op == 18) ? 16 : 8;  // instructions per iteration
    *rate = (double)grid * block * iters * per / (ms * 1e-3);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(out);
    return 0;
}

}  // extern "C"
