// Dev tool: field-multiply variant microbenchmark + cross-check (not part of the library).
// hipcc --offload-arch=gfx950 -O3 -shared -fPIC -I rust-bitcoinconsensus_amd/csrc -I tools tools/fe_bench.hip -o tools/_build/fe_bench.so
#include "ecdsa_lane.h"
#include "fe_asm.h"
#include "fe_asm_gen.h"
#include "fe29.h"
#include "gpu_common.h"

using namespace bcc;

__device__ __forceinline__ void mul_v(int v, fe& r, const fe& a, const fe& b) {
    u32 t[16];
#if defined(__HIP_DEVICE_COMPILE__)
    if (v == 1) { mul_256x256_asm(t, a.v, b.v); fe_reduce512_asm(r.v, t); return; }
    if (v == 2) { mul_256x256_col(t, a.v, b.v); fe_reduce512_asm(r.v, t); return; }
#endif
    mul_256x256(t, a.v, b.v);
    fe_reduce512(r, t);
}
__device__ __forceinline__ void sqr_v(int v, fe& r, const fe& a) {
    u32 t[16];
#if defined(__HIP_DEVICE_COMPILE__)
    if (v == 1) { sqr_256_asm(t, a.v); fe_reduce512_asm(r.v, t); return; }
    if (v == 2) { sqr_256_col(t, a.v); fe_reduce512_asm(r.v, t); return; }
#endif
    sqr_256(t, a.v);
    fe_reduce512(r, t);
}

template <int V, int SQ>
__global__ __launch_bounds__(256) void k_fe(fe* io, int iters) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (V == 3) {  // radix 2^29
        fe9 a9, b9, c9;
        fe9_from_fe(a9, io[2 * g]);
        fe9_from_fe(b9, io[2 * g + 1]);
        c9 = b9;
        for (int i = 0; i < iters; i++) {
            if (SQ) {
                fe9_sqr(a9, a9);
                fe9_sqr(c9, c9);
            } else {
                fe9_mul(a9, a9, b9);
                fe9_mul(c9, c9, b9);
            }
        }
        fe a, c;
        fe9_to_fe(a, a9);
        fe9_to_fe(c, c9);
        io[2 * g] = a;
        io[2 * g + 1] = c;
        return;
    }
    fe a = io[2 * g], b = io[2 * g + 1], c = b;
    for (int i = 0; i < iters; i++) {
        if (SQ) {
            sqr_v(V, a, a);
            sqr_v(V, c, c);
        } else {
            mul_v(V, a, a, b);
            mul_v(V, c, c, b);
        }
    }
    fe_normalize(a);
    fe_normalize(c);
    io[2 * g] = a;
    io[2 * g + 1] = c;
}

extern "C" int fe_bench(int variant, int sq, int iters, const void* in, void* out, int nblocks,
                        double* ops_per_s) {
    size_t lanes = (size_t)nblocks * 256, bytes = lanes * 2 * sizeof(fe);
    fe* d;
    BCC_HIP_TRY(hipMalloc(&d, bytes));
    BCC_HIP_TRY(hipMemcpy(d, in, bytes, hipMemcpyHostToDevice));
    auto launch = [&]() {
        if (variant == 3 && sq) hipLaunchKernelGGL((k_fe<3, 1>), dim3(nblocks), dim3(256), 0, 0, d, iters);
        else if (variant == 3) hipLaunchKernelGGL((k_fe<3, 0>), dim3(nblocks), dim3(256), 0, 0, d, iters);
        else if (variant == 2 && sq) hipLaunchKernelGGL((k_fe<2, 1>), dim3(nblocks), dim3(256), 0, 0, d, iters);
        else if (variant == 2) hipLaunchKernelGGL((k_fe<2, 0>), dim3(nblocks), dim3(256), 0, 0, d, iters);
        else if (variant == 1 && sq) hipLaunchKernelGGL((k_fe<1, 1>), dim3(nblocks), dim3(256), 0, 0, d, iters);
        else if (variant == 1) hipLaunchKernelGGL((k_fe<1, 0>), dim3(nblocks), dim3(256), 0, 0, d, iters);
        else if (sq) hipLaunchKernelGGL((k_fe<0, 1>), dim3(nblocks), dim3(256), 0, 0, d, iters);
        else hipLaunchKernelGGL((k_fe<0, 0>), dim3(nblocks), dim3(256), 0, 0, d, iters);
    };
    hipEvent_t e0, e1;
    BCC_HIP_TRY(hipEventCreate(&e0));
    BCC_HIP_TRY(hipEventCreate(&e1));
    BCC_HIP_TRY(hipEventRecord(e0, 0));
    launch();
    BCC_HIP_TRY(hipEventRecord(e1, 0));
    BCC_HIP_TRY(hipEventSynchronize(e1));
    float ms;
    BCC_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    *ops_per_s = (double)lanes * iters * 2 / (ms * 1e-3);
    BCC_HIP_TRY(hipMemcpy(out, d, bytes, hipMemcpyDeviceToHost));
    (void)hipFree(d);
    return 0;
}
