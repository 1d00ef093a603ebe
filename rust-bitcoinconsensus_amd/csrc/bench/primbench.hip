// Per-primitive cost of the ladder's building blocks on gfx950 (the decomposition of
// twist_ladder_kernel's issue time): each kernel loops ONE primitive (field
// multiply / square / add / sub / shift, Jacobian doubling, mixed addition) over random operands
// at the ladder's occupancy (4 waves per SIMD, 256-lane groups) and stamps every wave with
// s_memtime so the SIMD cycles per primitive per wave are measured, not inferred.  The loop
// bodies are the same inlined code the ladder runs; tools/isa/isa_blocks.py counts their
// instruction classes from the assembly listing.
#include <algorithm>
#include <vector>

#include "gpu_common.h"
#include "secp256k1_device.h"

namespace bcc {

template <int P>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void prim_kernel(
    u32* io, int iters, unsigned long long* stamps) {
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    u32* p = io + t * 24;
    fe a, b, c;
    for (int j = 0; j < 8; j++) {
        a.v[j] = p[j];
        b.v[j] = p[8 + j];
        c.v[j] = p[16 + j];
    }
    gej g{a, b, c};
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int it = 0; it < iters; it++) {
        if constexpr (P == 0) fe_mul(a, a, b);
        if constexpr (P == 1) fe_sqr(a, a);
        if constexpr (P == 2) fe_add(a, a, b);
        if constexpr (P == 3) fe_sub(a, a, b);
        if constexpr (P == 4) fe_shl<1>(a, a);
        if constexpr (P == 5) {
            gej r;
            gej_double(r, g);
            g = r;
        }
        if constexpr (P == 6) {  // mixed addition of a fixed affine point (never H == 0 here)
            gej r;
            bool inf;
            gej_add_zinv(r, inf, g, a, b, c, false);
            g = r;
        }
    }
    const unsigned long long dc = __builtin_amdgcn_s_memtime() - c0;
    if (P >= 5) a = g.x;
    for (int j = 0; j < 8; j++) p[j] = a.v[j];
    if (stamps && (threadIdx.x & 63) == 0) stamps[t / 64] = dc;
}

}  // namespace bcc

using namespace bcc;

extern "C" {

// Primitive `prim` (0 fe_mul, 1 fe_sqr, 2 fe_add, 3 fe_sub, 4 fe_shl<1>, 5 gej_double,
// 6 gej_add_zinv mixed) looped `iters` times per lane over random operands, 4 waves per SIMD
// on every CU, after `warm` untimed launches.  *cycles = median over waves of the SIMD cycles
// per primitive per wave (s_memtime delta / iters; 4 waves share a SIMD, so the SIMD spends
// cycles / 4 on each wave's primitive when issue-bound), *ms = the launch time.
int mi_primbench(int prim, int iters, int warm, double* cycles, double* ms_out) {
    int dev = 0, cus = 0;
    BCC_HIP_TRY(hipGetDevice(&dev));
    BCC_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (prim < 0 || prim > 6 || iters < 1) return -1;
    const int block = 256, grid = cus * 4;
    const size_t lanes = (size_t)grid * block, nwaves = lanes / 64;
    std::vector<u32> h(lanes * 24);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (auto& w : h) {  // xorshift: random limbs (fe ops accept any 256-bit input)
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        w = (u32)x;
    }
    u32* io = nullptr;
    unsigned long long* stamps = nullptr;
    BCC_HIP_TRY(hipMalloc(&io, h.size() * 4));
    BCC_HIP_TRY(hipMalloc(&stamps, nwaves * 8));
    BCC_HIP_TRY(hipMemcpy(io, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    BCC_HIP_TRY(hipEventCreate(&e0));
    BCC_HIP_TRY(hipEventCreate(&e1));
    float ms = 0;
    for (int r = 0; r <= warm; r++) {
        BCC_HIP_TRY(hipEventRecord(e0, 0));
        switch (prim) {
#define BCC_PB(K) \
    case K: hipLaunchKernelGGL(prim_kernel<K>, dim3(grid), dim3(block), 0, 0, io, iters, stamps); break;
            BCC_PB(0) BCC_PB(1) BCC_PB(2) BCC_PB(3) BCC_PB(4) BCC_PB(5) BCC_PB(6)
#undef BCC_PB
        }
        BCC_HIP_TRY(hipEventRecord(e1, 0));
        BCC_HIP_TRY(hipEventSynchronize(e1));
        BCC_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    }
    std::vector<unsigned long long> st(nwaves);
    BCC_HIP_TRY(hipMemcpy(st.data(), stamps, nwaves * 8, hipMemcpyDeviceToHost));
    std::nth_element(st.begin(), st.begin() + nwaves / 2, st.end());
    *cycles = (double)st[nwaves / 2] / iters;
    if (ms_out) *ms_out = ms;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(io);
    (void)hipFree(stamps);
    return 0;
}

}  // extern "C"
