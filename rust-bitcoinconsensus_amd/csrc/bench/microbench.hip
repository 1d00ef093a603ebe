// Integer-ALU microbenchmarks for gfx950: the measured peak that roofline.peak is quoted
// against (achieved = verifies/s * 144,448 / peak v_mad_u64_u32 per second).
// Each kernel runs 8 independent dependency chains per lane so issue rate, not latency, binds
// (ops 20-21: ONE dependent chain per lane, the latency-bound case of a carry chain).
// mi_microbench_sustained runs launches of >= 10 ms back to back for >= 1 s before timing (the
// clock the chip holds under a sustained integer load, MI355X_MICROARCH.md "DVFS give-back") and
// stamps every wave with s_memtime / s_memrealtime so the clock of the timed launches is known.
#include <algorithm>
#include <vector>

#include "gpu_common.h"

namespace bcc {

template <int OP>
__global__ __launch_bounds__(256) void ubench_kernel(uint32_t* out, int iters, uint32_t seed,
                                                     unsigned long long* stamps) {
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
    const unsigned long long w0 = __builtin_amdgcn_s_memrealtime();
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
            } else if (OP == 19) {  // v_mov_b32
                asm volatile("v_mov_b32 %0, %1" : "=v"(acc32[k]) : "v"(acc32[(k + 1) & 7]));
            } else if (OP == 20) {  // ONE dependent v_addc_co_u32 chain per lane (k == 0 only)
                if (k == 0)
                    asm volatile("v_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\tv_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\t"
                                 "v_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\tv_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\t"
                                 "v_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\tv_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\t"
                                 "v_addc_co_u32_e32 %0, vcc, %0, %1, vcc\n\tv_addc_co_u32_e32 %0, vcc, %0, %1, vcc"
                                 : "+v"(acc32[0]) : "v"(b) : "vcc");
            } else if (OP == 21) {  // ONE dependent mad_u64_u32 + addc chain per lane (k == 0 only)
                if (k == 0)
                    asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
                                 "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
                                 "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"
                                 "v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                                 : "+v"(acc[0]), "+v"(acc32[0]) : "v"(a), "v"(b) : "vcc");
            } else if (OP == 22) {  // v_cndmask_b32_e64 with an SGPR-pair mask
                asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[2:3]" : "+v"(acc32[k]) : "v"(b) : "s2", "s3");
            } else if (OP == 23) {  // v_subb_co_u32 (borrow chain link, VCC)
                asm volatile("v_subb_co_u32_e32 %0, vcc, %0, %1, vcc" : "+v"(acc32[k]) : "v"(b) : "vcc");
            } else if (OP == 25 && k == 0) {  // 8 x v_mad_u64_u32, distinct SGPR carry pairs, one asm block
                asm volatile(
                    "v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n\tv_mad_u64_u32 %1, s[42:43], %8, %9, %1\n\t"
                    "v_mad_u64_u32 %2, s[44:45], %8, %9, %2\n\tv_mad_u64_u32 %3, s[46:47], %8, %9, %3\n\t"
                    "v_mad_u64_u32 %4, s[48:49], %8, %9, %4\n\tv_mad_u64_u32 %5, s[50:51], %8, %9, %5\n\t"
                    "v_mad_u64_u32 %6, s[52:53], %8, %9, %6\n\tv_mad_u64_u32 %7, s[54:55], %8, %9, %7"
                    : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
                      "+v"(acc[6]), "+v"(acc[7])
                    : "v"(a), "v"(b)
                    : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51",
                      "s52", "s53", "s54", "s55");
            } else if (OP == 26 && k == 0) {  // 8 independent v_addc_co_u32_e64 chains (own SGPR carry pairs)
                asm volatile(
                    "v_addc_co_u32_e64 %0, s[40:41], %0, %8, s[40:41]\n\tv_addc_co_u32_e64 %1, s[42:43], %1, %8, s[42:43]\n\t"
                    "v_addc_co_u32_e64 %2, s[44:45], %2, %8, s[44:45]\n\tv_addc_co_u32_e64 %3, s[46:47], %3, %8, s[46:47]\n\t"
                    "v_addc_co_u32_e64 %4, s[48:49], %4, %8, s[48:49]\n\tv_addc_co_u32_e64 %5, s[50:51], %5, %8, s[50:51]\n\t"
                    "v_addc_co_u32_e64 %6, s[52:53], %6, %8, s[52:53]\n\tv_addc_co_u32_e64 %7, s[54:55], %7, %8, s[54:55]"
                    : "+v"(acc32[0]), "+v"(acc32[1]), "+v"(acc32[2]), "+v"(acc32[3]), "+v"(acc32[4]),
                      "+v"(acc32[5]), "+v"(acc32[6]), "+v"(acc32[7])
                    : "v"(b)
                    : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51",
                      "s52", "s53", "s54", "s55");
            } else if (OP == 27 && k == 0) {  // 4 x (mad -> VCC -> addc) pairs, one asm block (the column pattern)
                asm volatile(
                    "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_addc_co_u32_e32 %4, vcc, 0, %4, vcc\n\t"
                    "v_mad_u64_u32 %1, vcc, %8, %9, %1\n\tv_addc_co_u32_e32 %5, vcc, 0, %5, vcc\n\t"
                    "v_mad_u64_u32 %2, vcc, %8, %9, %2\n\tv_addc_co_u32_e32 %6, vcc, 0, %6, vcc\n\t"
                    "v_mad_u64_u32 %3, vcc, %8, %9, %3\n\tv_addc_co_u32_e32 %7, vcc, 0, %7, vcc"
                    : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc32[0]), "+v"(acc32[1]),
                      "+v"(acc32[2]), "+v"(acc32[3])
                    : "v"(a), "v"(b)
                    : "vcc");
            } else if (OP == 28 && k == 0) {  // 8 x v_add_u32, one asm block (full-rate reference)
                asm volatile(
                    "v_add_u32 %0, %0, %8\n\tv_add_u32 %1, %1, %8\n\tv_add_u32 %2, %2, %8\n\tv_add_u32 %3, %3, %8\n\t"
                    "v_add_u32 %4, %4, %8\n\tv_add_u32 %5, %5, %8\n\tv_add_u32 %6, %6, %8\n\tv_add_u32 %7, %7, %8"
                    : "+v"(acc32[0]), "+v"(acc32[1]), "+v"(acc32[2]), "+v"(acc32[3]), "+v"(acc32[4]),
                      "+v"(acc32[5]), "+v"(acc32[6]), "+v"(acc32[7])
                    : "v"(b));
            } else if (OP == 29 && k == 0) {  // 8 x v_addc_co_u32_e32, ONE VCC carry chain (fe_add's chain)
                asm volatile(
                    "v_addc_co_u32_e32 %0, vcc, %0, %8, vcc\n\tv_addc_co_u32_e32 %1, vcc, %1, %8, vcc\n\t"
                    "v_addc_co_u32_e32 %2, vcc, %2, %8, vcc\n\tv_addc_co_u32_e32 %3, vcc, %3, %8, vcc\n\t"
                    "v_addc_co_u32_e32 %4, vcc, %4, %8, vcc\n\tv_addc_co_u32_e32 %5, vcc, %5, %8, vcc\n\t"
                    "v_addc_co_u32_e32 %6, vcc, %6, %8, vcc\n\tv_addc_co_u32_e32 %7, vcc, %7, %8, vcc"
                    : "+v"(acc32[0]), "+v"(acc32[1]), "+v"(acc32[2]), "+v"(acc32[3]), "+v"(acc32[4]),
                      "+v"(acc32[5]), "+v"(acc32[6]), "+v"(acc32[7])
                    : "v"(b)
                    : "vcc");
            } else if (OP == 30 && k == 0) {  // 8 x v_mad_u64_u32 with carry to VCC, one asm block
                asm volatile(
                    "v_mad_u64_u32 %0, vcc, %8, %9, %0\n\tv_mad_u64_u32 %1, vcc, %8, %9, %1\n\t"
                    "v_mad_u64_u32 %2, vcc, %8, %9, %2\n\tv_mad_u64_u32 %3, vcc, %8, %9, %3\n\t"
                    "v_mad_u64_u32 %4, vcc, %8, %9, %4\n\tv_mad_u64_u32 %5, vcc, %8, %9, %5\n\t"
                    "v_mad_u64_u32 %6, vcc, %8, %9, %6\n\tv_mad_u64_u32 %7, vcc, %8, %9, %7"
                    : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
                      "+v"(acc[6]), "+v"(acc[7])
                    : "v"(a), "v"(b)
                    : "vcc");
            } else if (OP == 24) {  // mad_u64_u32 + addc pair with the s_nop 1 hipcc puts between carry links
                asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\ts_nop 1\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                             : "+v"(acc[k]), "+v"(acc32[k]) : "v"(a), "v"(b) : "vcc");
            }
        }
    }
    uint32_t r = 0;
#pragma unroll
    for (int k = 0; k < 8; k++)
        r ^= (uint32_t)acc[k] ^ (uint32_t)(acc[k] >> 32) ^ acc32[k] ^ (uint32_t)(int64_t)accd[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (stamps && (threadIdx.x & 63) == 0) {
        const size_t wv = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        stamps[2 * wv] = __builtin_amdgcn_s_memtime() - c0;
        stamps[2 * wv + 1] = __builtin_amdgcn_s_memrealtime() - w0;
    }
}

// Instructions per loop iteration of op (per lane)
static int ubench_per_iter(int op) {
    switch (op) {
        case 16: case 17: case 18: case 24: return 16;
        case 20: return 8;
        case 21: return 8;
        default: return 8;
    }
}

#define BCC_UB_CASE(K)                                                                          \
    case K:                                                                                     \
        hipLaunchKernelGGL(ubench_kernel<K>, dim3(grid), dim3(block), 0, 0, out, it, 1u, stamps); \
        break;
static void ubench_launch(int op, int grid, int block, uint32_t* out, int it,
                          unsigned long long* stamps) {
    switch (op) {
        BCC_UB_CASE(0) BCC_UB_CASE(1) BCC_UB_CASE(2) BCC_UB_CASE(3) BCC_UB_CASE(4)
        BCC_UB_CASE(5) BCC_UB_CASE(6) BCC_UB_CASE(7) BCC_UB_CASE(9) BCC_UB_CASE(10)
        BCC_UB_CASE(11) BCC_UB_CASE(12) BCC_UB_CASE(13) BCC_UB_CASE(14) BCC_UB_CASE(15)
        BCC_UB_CASE(16) BCC_UB_CASE(17) BCC_UB_CASE(18) BCC_UB_CASE(19) BCC_UB_CASE(20)
        BCC_UB_CASE(21) BCC_UB_CASE(22) BCC_UB_CASE(23) BCC_UB_CASE(24) BCC_UB_CASE(25)
        BCC_UB_CASE(26) BCC_UB_CASE(27) BCC_UB_CASE(28) BCC_UB_CASE(29) BCC_UB_CASE(30)
        default: BCC_UB_CASE(8)
    }
}
#undef BCC_UB_CASE

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
    auto launch = [&](int it) { ubench_launch(op, grid, block, out, it, nullptr); };
    launch(16);  // warm-up
    BCC_HIP_TRY(hipDeviceSynchronize());
    BCC_HIP_TRY(hipEventRecord(e0, 0));
    launch(iters);
    BCC_HIP_TRY(hipEventRecord(e1, 0));
    BCC_HIP_TRY(hipEventSynchronize(e1));
    float ms = 0;
    BCC_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
    *rate = (double)grid * block * iters * ubench_per_iter(op) / (ms * 1e-3);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(out);
    return 0;
}

// Sustained form: waves_per_simd waves of `op` per SIMD (256-lane workgroups), the iteration count
// calibrated so one launch takes about target_ms (>= 10 ms), launches back to back for >= warm_s
// seconds, then `reps` timed launches.  *rate = median lane-instructions per second, *clock_ghz =
// median over waves of the in-kernel clock (delta s_memtime / delta s_memrealtime x the
// realtime counter's rate) of the timed launches, *ms = median launch time.
int mi_microbench_sustained(int op, int waves_per_simd, double target_ms, double warm_s, int reps,
                            double* rate, double* clock_ghz, double* ms_out) {
    int dev = 0, cus = 0, wclk_khz = 0;
    BCC_HIP_TRY(hipGetDevice(&dev));
    BCC_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    BCC_HIP_TRY(hipDeviceGetAttribute(&wclk_khz, hipDeviceAttributeWallClockRate, dev));
    if (waves_per_simd < 1 || waves_per_simd > 8 || reps < 1 || op < 0 || op > 30) return -1;
    const int block = 256, grid = cus * waves_per_simd;  // 4 waves per group, one per SIMD
    const size_t nwaves = (size_t)grid * (block / 64);
    uint32_t* out = nullptr;
    unsigned long long* stamps = nullptr;
    BCC_HIP_TRY(hipMalloc(&out, (size_t)grid * block * 4));
    BCC_HIP_TRY(hipMalloc(&stamps, nwaves * 16));
    hipEvent_t e0, e1;
    BCC_HIP_TRY(hipEventCreate(&e0));
    BCC_HIP_TRY(hipEventCreate(&e1));
    auto timed = [&](int it, unsigned long long* st, float* ms) -> int {
        BCC_HIP_TRY(hipEventRecord(e0, 0));
        ubench_launch(op, grid, block, out, it, st);
        BCC_HIP_TRY(hipEventRecord(e1, 0));
        BCC_HIP_TRY(hipEventSynchronize(e1));
        BCC_HIP_TRY(hipEventElapsedTime(ms, e0, e1));
        return 0;
    };
    // calibrate: grow the iteration count until one launch takes >= target_ms / 4, then scale
    int it = 256;
    float ms = 0;
    for (;;) {
        if (int e = timed(it, nullptr, &ms)) return e;
        if (ms >= target_ms / 4 || it >= (1 << 26)) break;
        it *= 4;
    }
    it = (int)std::min<double>((double)it * target_ms / std::max(ms, 1e-3f), (double)(1 << 28));
    double warm = 0;
    while (warm < warm_s * 1e3) {
        if (int e = timed(it, nullptr, &ms)) return e;
        warm += ms;
    }
    std::vector<double> mss, clks;
    std::vector<unsigned long long> h(2 * nwaves);
    for (int r = 0; r < reps; r++) {
        if (int e = timed(it, stamps, &ms)) return e;
        mss.push_back(ms);
        BCC_HIP_TRY(hipMemcpy(h.data(), stamps, h.size() * 8, hipMemcpyDeviceToHost));
        std::vector<double> c;
        c.reserve(nwaves);
        for (size_t w = 0; w < nwaves; w++)
            if (h[2 * w + 1]) c.push_back((double)h[2 * w] / (double)h[2 * w + 1] * wclk_khz * 1e-6);
        std::nth_element(c.begin(), c.begin() + c.size() / 2, c.end());
        clks.push_back(c.empty() ? 0 : c[c.size() / 2]);
    }
    std::sort(mss.begin(), mss.end());
    std::sort(clks.begin(), clks.end());
    const double med = mss[mss.size() / 2];
    *rate = (double)grid * block * it * ubench_per_iter(op) / (med * 1e-3);
    *clock_ghz = clks[clks.size() / 2];
    if (ms_out) *ms_out = med;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(out);
    (void)hipFree(stamps);
    return 0;
}

}  // extern "C"
