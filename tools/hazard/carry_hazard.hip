// Dev tool: does gfx950 need wait states between a VALU carry-out write of VCC and the next
// VALU carry-in read (hipcc inserts `s_nop 1` there)?  Runs 256-bit additions as back-to-back
// carry chains in inline asm WITHOUT nops, in three forms, and compares with the host.
//   hipcc -O3 --offload-arch=gfx950 carry_hazard.hip -o carry_hazard && ./carry_hazard
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <vector>

// form 0: VOP2 chain (implicit VCC), no wait states
// form 1: VOP3 (e64) chain with explicit vcc, no wait states
// form 2: v_mad_u64_u32 (sdst vcc) -> v_addc_e64 pairs: r = a*b + c, carries summed into hi
__global__ void kadd(const uint32_t* __restrict__ A, const uint32_t* __restrict__ B,
                     uint32_t* __restrict__ R, int form, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t a[8], b[8], r[9];
    for (int k = 0; k < 8; k++) { a[k] = A[8 * i + k]; b[k] = B[8 * i + k]; }
    if (form == 0) {
        asm volatile(
            "v_add_co_u32_e32 %0, vcc, %9, %17\n\t"
            "v_addc_co_u32_e32 %1, vcc, %10, %18, vcc\n\t"
            "v_addc_co_u32_e32 %2, vcc, %11, %19, vcc\n\t"
            "v_addc_co_u32_e32 %3, vcc, %12, %20, vcc\n\t"
            "v_addc_co_u32_e32 %4, vcc, %13, %21, vcc\n\t"
            "v_addc_co_u32_e32 %5, vcc, %14, %22, vcc\n\t"
            "v_addc_co_u32_e32 %6, vcc, %15, %23, vcc\n\t"
            "v_addc_co_u32_e32 %7, vcc, %16, %24, vcc\n\t"
            "v_addc_co_u32_e64 %8, vcc, 0, 0, vcc"
            : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]),
              "=&v"(r[6]), "=&v"(r[7]), "=&v"(r[8])
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),
              "v"(a[7]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]),
              "v"(b[6]), "v"(b[7])
            : "vcc");
    } else if (form == 1) {
        asm volatile(
            "v_add_co_u32_e64 %0, vcc, %9, %17\n\t"
            "v_addc_co_u32_e64 %1, vcc, %10, %18, vcc\n\t"
            "v_addc_co_u32_e64 %2, vcc, %11, %19, vcc\n\t"
            "v_addc_co_u32_e64 %3, vcc, %12, %20, vcc\n\t"
            "v_addc_co_u32_e64 %4, vcc, %13, %21, vcc\n\t"
            "v_addc_co_u32_e64 %5, vcc, %14, %22, vcc\n\t"
            "v_addc_co_u32_e64 %6, vcc, %15, %23, vcc\n\t"
            "v_addc_co_u32_e64 %7, vcc, %16, %24, vcc\n\t"
            "v_addc_co_u32_e64 %8, vcc, 0, 0, vcc"
            : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]), "=&v"(r[5]),
              "=&v"(r[6]), "=&v"(r[7]), "=&v"(r[8])
            : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]),
              "v"(a[7]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]), "v"(b[4]), "v"(b[5]),
              "v"(b[6]), "v"(b[7])
            : "vcc");
    } else {
        // sum of a[k]*b[k] over k with a 64-bit accumulator and a carry word
        uint64_t acc = 0;
        uint32_t nh = 0;
#pragma unroll
        for (int k = 0; k < 8; k++)
            asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e64 %1, vcc, 0, %1, vcc"
                         : "+v"(acc), "+v"(nh) : "v"(a[k]), "v"(b[k]) : "vcc");
        r[0] = (uint32_t)acc; r[1] = (uint32_t)(acc >> 32); r[2] = nh;
        for (int k = 3; k < 9; k++) r[k] = 0;
    }
    for (int k = 0; k < 9; k++) R[9 * i + k] = r[k];
}

int main() {
    const int n = 1 << 22;
    std::vector<uint32_t> A(8 * (size_t)n), B(8 * (size_t)n), R(9 * (size_t)n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)(s >> 11); };
    for (size_t k = 0; k < A.size(); k++) {
        // bias towards long carry chains: many 0xFFFFFFFF limbs
        A[k] = (rnd() & 3) ? 0xFFFFFFFFu : rnd();
        B[k] = (rnd() & 7) ? 0xFFFFFFFFu - (rnd() & 1) : rnd();
    }
    uint32_t *dA, *dB, *dR;
    hipMalloc(&dA, A.size() * 4); hipMalloc(&dB, B.size() * 4); hipMalloc(&dR, R.size() * 4);
    hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
    for (int form = 0; form < 3; form++) {
        for (int rep = 0; rep < 3; rep++) {
            hipLaunchKernelGGL(kadd, dim3(n / 256), dim3(256), 0, 0, dA, dB, dR, form, n);
            hipMemcpy(R.data(), dR, R.size() * 4, hipMemcpyDeviceToHost);
            size_t bad = 0;
            for (int i = 0; i < n; i++) {
                uint32_t e[9];
                if (form < 2) {
                    uint64_t c = 0;
                    for (int k = 0; k < 8; k++) { c += (uint64_t)A[8 * (size_t)i + k] + B[8 * (size_t)i + k]; e[k] = (uint32_t)c; c >>= 32; }
                    e[8] = (uint32_t)c;
                } else {
                    unsigned __int128 acc = 0;
                    for (int k = 0; k < 8; k++) acc += (unsigned __int128)((uint64_t)A[8 * (size_t)i + k] * B[8 * (size_t)i + k]);
                    e[0] = (uint32_t)acc; e[1] = (uint32_t)(acc >> 32); e[2] = (uint32_t)(acc >> 64);
                    for (int k = 3; k < 9; k++) e[k] = 0;
                }
                for (int k = 0; k < 9; k++) if (e[k] != R[9 * (size_t)i + k]) { bad++; break; }
            }
            printf("form %d rep %d: %zu / %d mismatches\n", form, rep, bad, n);
        }
    }
    return 0;
}
