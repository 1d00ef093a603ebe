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
#pragma unroll
    for (int k = 0; k < 8; k++) {
        acc[k] = (uint64_t)(a + k) << 7;
        acc32[k] = a + 3 * k;
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
                double d = (double)acc[k];
                asm volatile("v_fma_f64 %0, %0, %1, %0" : "+v"(d) : "v"((double)b));
                acc[k] = (uint64_t)d;
            } else if (OP == 8) {  // v_add_u32 (plain full-rate reference)
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc32[k]) : "v"(b));
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++) r ^= (uint32_t)acc[k] ^ (uint32_t)(acc[k] >> 32) ^ acc32[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

}  // namespace bcc

using namespace bcc;

extern "C" {

// Runs microbenchmark `op` (see ubench_kernel) and returns lane-instructions per second in
// *rate. Synchronous, on the current device.
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
    auto launch = [&](int it) {
        switch (op) {
            case 0: hipLaunchKernelGGL(ubench_kernel<0>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
            case 1: hipLaunchKernelGGL(ubench_kernel<1>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
            case 2: hipLaunchKernelGGL(ubench_kernel<2>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
            case 3: hipLaunchKernelGGL(ubench_kernel<3>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
            case 4: hipLaunchKernelGGL(ubench_kernel<4>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
            case 5: hipLaunchKernelGGL(ubench_kernel<5>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
            case 6: hipLaunchKernelGGL(ubench_kernel<6>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
            case 7: hipLaunchKernelGGL(ubench_kernel<7>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
            default: hipLaunchKernelGGL(ubench_kernel<8>, dim3(grid), dim3(block), 0, 0, out, it, 1u); break;
        }
    };
    launch(16);  // warm-up
    BCC_HIP_TRY(hipDeviceSynchronize());
    BCC_HIP_TRY(hipEventRecord(e0, 0));
    launch(iters);
    BCC_HIP_TRY(hipEventRecord(e1, 0));
    BCC_HIP_TRY(hipEventSynchronize(e1));
    float ms = 0;
    BCC_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    *rate = (double)grid * block * iters * 8 / (ms * 1e-3);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(out);
    return 0;
}

}  // extern "C"
