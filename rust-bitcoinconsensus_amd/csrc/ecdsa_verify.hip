// ECDSA verify kernel for gfx950 (stage (c) of the hot path, plus stage (b) pubkey
// decompression fused in front).  One lane = one tuple; the per-lane algorithm is
// ecdsa_lane.h.  Inputs are the reference's b32 convention: big-endian 32-byte values.
//
// HBM layout (all device-resident):
//   tag[n]            u8   pubkey header byte (0 = rejected by the host length filter)
//   x[n][32], y[n][32]     pubkey coordinates, big-endian (y unused for 02/03)
//   r[n][32], s[n][32]     signature scalars after lax-DER (zero on overflow)
//   m[n][32]               sighash (raw SHA-256d bytes == big-endian integer)
//   verdict[n]        u8   1 = valid
// Each lane reads its 32-byte rows with two 16-byte loads; across a wave the union is one
// contiguous 2 KiB span per row array, so the loads are fully coalesced.
#include "ecdsa_lane.h"
#include "gpu_common.h"

namespace bcc {

// Per-lane Q table in global memory, lane-interleaved: word (entry i, field f, limb j) of lane L
// is at base[((i*3 + f)*8 + j) * stride + L] -> every table access of a wave is one coalesced
// 256-byte transaction per limb.
struct QTableGlobal {
    u32* base;
    size_t stride;
    __device__ void put(int i, int f, const fe& a) {
        u32* p = base + (size_t)((i * 3 + f) * 8) * stride;
#pragma unroll
        for (int j = 0; j < 8; j++) p[(size_t)j * stride] = a.v[j];
    }
    __device__ void get(int i, int f, fe& a) const {
        const u32* p = base + (size_t)((i * 3 + f) * 8) * stride;
#pragma unroll
        for (int j = 0; j < 8; j++) a.v[j] = p[(size_t)j * stride];
    }
};

// G tables staged in LDS (16 KiB per workgroup).
struct GTableLDS {
    const fe* xy;
    __device__ void get(int tab, int i, fe& x, fe& y) const {
        x = xy[(tab * GTAB + i) * 2 + 0];
        y = xy[(tab * GTAB + i) * 2 + 1];
    }
};

__device__ __forceinline__ void load_be32(fe& r, const uint8_t* p) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    u32 w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    fe_from_be_words(r, w);
}

__global__ __launch_bounds__(256) void ecdsa_verify_kernel(
    const uint8_t* __restrict__ tag, const uint8_t* __restrict__ px, const uint8_t* __restrict__ py,
    const uint8_t* __restrict__ pr, const uint8_t* __restrict__ ps, const uint8_t* __restrict__ pm,
    uint8_t* __restrict__ verdict, u32* __restrict__ qscratch, const fe* __restrict__ gtab,
    size_t n) {
    __shared__ fe g_lds[2 * GTAB * 2];
    for (int i = threadIdx.x; i < 2 * GTAB * 2; i += blockDim.x) g_lds[i] = gtab[i];
    __syncthreads();
    const size_t lanes = (size_t)gridDim.x * blockDim.x;
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    QTableGlobal qt{qscratch + gid, lanes};
    GTableLDS gt{g_lds};
    for (size_t i = gid; i < n; i += lanes) {
        fe x, y, t;
        sc r, s, m;
        load_be32(x, px + 32 * i);
        load_be32(y, py + 32 * i);
        load_be32(t, pr + 32 * i);
        for (int k = 0; k < 8; k++) r.v[k] = t.v[k];
        load_be32(t, ps + 32 * i);
        for (int k = 0; k < 8; k++) s.v[k] = t.v[k];
        load_be32(t, pm + 32 * i);
        for (int k = 0; k < 8; k++) m.v[k] = t.v[k];
        verdict[i] = (uint8_t)ecdsa_verify_lane(tag[i], x, y, r, s, m, qt, gt);
    }
}

// ------------------------------------------------------------------------------------------
// per-device state: G tables + Q scratch
// ------------------------------------------------------------------------------------------
static constexpr int VERIFY_BLOCK = 256;

struct EcdsaDeviceState {
    fe* d_gtab = nullptr;
    u32* d_qscratch = nullptr;
    int grid = 0;
};

static std::mutex g_state_mu;
static EcdsaDeviceState g_state[64];

static const std::vector<fe>& host_gtab() {
    static std::vector<fe> t;
    static std::once_flag once;
    std::call_once(once, [] {
        t.resize(2 * GTAB * 2);
        build_g_tables(t.data());
    });
    return t;
}

static int ensure_state(int dev, EcdsaDeviceState** out) {
    std::lock_guard<std::mutex> lk(g_state_mu);
    EcdsaDeviceState& st = g_state[dev];
    if (!st.d_gtab) {
        BCC_HIP_TRY(hipSetDevice(dev));
        const auto& h = host_gtab();
        BCC_HIP_TRY(hipMalloc(&st.d_gtab, h.size() * sizeof(fe)));
        BCC_HIP_TRY(hipMemcpy(st.d_gtab, h.data(), h.size() * sizeof(fe), hipMemcpyHostToDevice));
        int cus = 0;
        BCC_HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        st.grid = cus * 4;  // 4 resident 256-thread blocks per CU (VGPR-limited), grid-stride
        size_t lanes = (size_t)st.grid * VERIFY_BLOCK;
        BCC_HIP_TRY(hipMalloc(&st.d_qscratch, lanes * QTAB * 3 * 8 * sizeof(u32)));
    }
    *out = &st;
    return 0;
}

}  // namespace bcc

using namespace bcc;

extern "C" {

// Device-pointer entry: all buffers already resident on the current device; launches on
// `stream` (hipStream_t, may be null). Returns 0 on success, else a hipError_t value.
int mi_ecdsa_verify_device(const uint8_t* d_tag, const uint8_t* d_x, const uint8_t* d_y,
                           const uint8_t* d_r, const uint8_t* d_s, const uint8_t* d_m,
                           uint8_t* d_verdict, size_t n, void* stream) {
    if (n == 0) return 0;
    int dev = 0;
    BCC_HIP_TRY(hipGetDevice(&dev));
    EcdsaDeviceState* st = nullptr;
    if (int e = ensure_state(dev, &st)) return e;
    int blocks = (int)std::min<size_t>((n + VERIFY_BLOCK - 1) / VERIFY_BLOCK, (size_t)st->grid);
    // The Q scratch is sized for st->grid blocks; the kernel strides by its own grid, so a
    // smaller grid simply uses a prefix of it.
    hipLaunchKernelGGL(ecdsa_verify_kernel, dim3(blocks), dim3(VERIFY_BLOCK), 0,
                       (hipStream_t)stream, d_tag, d_x, d_y, d_r, d_s, d_m, d_verdict,
                       st->d_qscratch, st->d_gtab, n);
    BCC_HIP_TRY(hipGetLastError());
    return 0;
}

}  // extern "C"

extern "C" {

// Host-buffer entry (the inner C ABI of SURVEY §8b): pub65[n] = header byte || x || y (y ignored
// for 02/03; header 0 = rejected by the caller's CPubKey length filter), msg32/r32/s32 big-endian.
// Copies in, verifies on `device`, copies verdicts out. Synchronous.
int mi_ecdsa_verify_tuples(const uint8_t* pub65, const uint8_t* msg32, const uint8_t* r32,
                           const uint8_t* s32, uint8_t* verdict, size_t n, int device) {
    if (n == 0) return 0;
    BCC_HIP_TRY(hipSetDevice(device));
    std::vector<uint8_t> tag(n), xy(n * 64);
    for (size_t i = 0; i < n; i++) {
        tag[i] = pub65[65 * i];
        memcpy(&xy[64 * i], pub65 + 65 * i + 1, 64);
    }
    uint8_t* d = nullptr;
    // layout: tag | x | y | r | s | m | verdict  (32-byte rows 16-byte aligned)
    size_t tag_bytes = (n + 255) & ~(size_t)255;
    size_t row = 32 * n;
    size_t total = tag_bytes + 5 * row + tag_bytes;
    BCC_HIP_TRY(hipMalloc(&d, total));
    uint8_t *d_tag = d, *d_x = d + tag_bytes, *d_y = d_x + row, *d_r = d_y + row, *d_s = d_r + row,
            *d_m = d_s + row, *d_v = d_m + row;
    std::vector<uint8_t> xs(row), ys(row);
    for (size_t i = 0; i < n; i++) {
        memcpy(&xs[32 * i], &xy[64 * i], 32);
        memcpy(&ys[32 * i], &xy[64 * i + 32], 32);
    }
    int rc = 0;
    if ((rc = (int)hipMemcpy(d_tag, tag.data(), n, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(d_x, xs.data(), row, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(d_y, ys.data(), row, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(d_r, r32, row, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(d_s, s32, row, hipMemcpyHostToDevice)) ||
        (rc = (int)hipMemcpy(d_m, msg32, row, hipMemcpyHostToDevice)) ||
        (rc = mi_ecdsa_verify_device(d_tag, d_x, d_y, d_r, d_s, d_m, d_v, n, nullptr)) ||
        (rc = (int)hipDeviceSynchronize()) ||
        (rc = (int)hipMemcpy(verdict, d_v, n, hipMemcpyDeviceToHost))) {
        fprintf(stderr, "[bcc] mi_ecdsa_verify_tuples failed: %d\n", rc);
    }
    (void)hipFree(d);
    return rc;
}

}  // extern "C"
