// Experiment kernels for the 1024^2 CSR SpMV (A u, apply.py:72) -- NOT product code.  Built into a standalone
// libspmv_lab.so by tools/spmv_lab.py and driven from Python on the matrices the product library assembles.
//
//   * streaming-read calibration: the same byte count as the SpMV read once, in order (what the box's HBM does);
//   * read + write calibration: the SpMV's exact stream shape without the x gathers (9 KB read and 512 B written
//     per 64-row wave);
//   * the uniform-wave CSR kernel (k_csr_wave's table path) with the staging / cache-policy alternatives:
//       MODE 0: register staging (the product's form), 1: LDS-DMA staging (global_load_lds_dwordx4);
//       NT: nontemporal matrix loads.
//   * a cache flush (a 512 MiB write) for cold-cache timings.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const i32x4 ci32x4;

template <bool NT, class T>
__device__ inline T ldg(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

__device__ inline int xcd_swizzle(int b, int nb) {
    const int full = nb & ~7;
    if (b >= full) return b;
    const int per = full >> 3;
    return (b & 7) * per + (b >> 3);
}

// one workgroup reads 16 KiB (256 lanes x 4 x 16 B) in order
template <bool NT>
__global__ void __launch_bounds__(256) k_read(const f64x2* __restrict__ p, int64_t n16, double* sink) {
    const int64_t base = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 1024 + threadIdx.x;
    f64x2 acc = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t i = base + 256 * j;
        if (i < n16) acc += ldg<NT>(p + i);
    }
    if (acc.x == 1234.5678 && acc.y == -1.0) sink[threadIdx.x] = acc.x;   // never true for the data used
}

// per 64-lane wave: read 9 KiB (9 x 16 B per lane) and write 64 doubles -- the SpMV's shape for 12-entry rows
template <bool NT>
__global__ void __launch_bounds__(256) k_readwrite(const f64x2* __restrict__ p, int64_t nwaves, double* y) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t wv = (int64_t)xcd_swizzle(blockIdx.x, gridDim.x) * 4 + w;
    if (wv >= nwaves) return;
    const f64x2* q = p + wv * 576;
    f64x2 acc = {0.0, 0.0};
#pragma unroll
    for (int j = 0; j < 9; ++j) acc += ldg<NT>(q + lane + 64 * j);
    __builtin_nontemporal_store(acc.x + acc.y, y + wv * 64 + lane);
}

__global__ void k_fill(double* p, int64_t n, double v) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The uniform-wave CSR product (every wave of the table flagged uniform: 64 rows of LEN entries from an even entry
// offset), y = A x, sums left to right in CSR order (bit-identical to the product kernel).
template <int LEN, int MODE, bool NT, int AUX = 2>
__device__ inline void wave_rows(const double* __restrict__ va, const int32_t* __restrict__ ci,
                                 const double* __restrict__ x, int32_t ncols, int32_t s, int lane, double2* vs, int2* cs,
                                 int32_t r, double* __restrict__ y) {
    constexpr int P = LEN / 2;
    if constexpr (MODE == 0) {
        f64x2 v[P];
        i32x2 cc[P];
#pragma unroll
        for (int j = 0; j < P; ++j) {
            const int32_t k = s + 2 * (lane + 64 * j);
            v[j] = ldg<NT>(reinterpret_cast<const f64x2*>(va + k));
            cc[j] = ldg<NT>(reinterpret_cast<const i32x2*>(ci + k));
        }
#pragma unroll
        for (int j = 0; j < P; ++j) {
            vs[lane + 64 * j] = make_double2(v[j].x, v[j].y);
            cs[lane + 64 * j] = make_int2(cc[j].x, cc[j].y);
        }
    } else {
        // LDS-DMA: the wave's chunk copied lane-linearly (16 B per lane per instruction) -- the same image
        constexpr int aux = NT ? AUX : 0;
#pragma unroll
        for (int j = 0; j < P; ++j)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(va + s + 2 * (lane + 64 * j)),
                                             (__attribute__((address_space(3))) void*)(vs + 64 * j),
                                             16, 0, aux);
#pragma unroll
        for (int j = 0; j < P / 2; ++j)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(ci + s + 4 * (lane + 64 * j)),
                                             (__attribute__((address_space(3))) void*)(cs + 128 * j),
                                             16, 0, aux);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    wave_lds_sync();
    const int p0 = lane * P;
    int2 c[P];
#pragma unroll
    for (int i = 0; i < P; ++i) c[i] = cs[p0 + i];
    const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(x), (short)0, ncols * 8, 0x00020000);
    double x0[P], x1[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
        x0[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, c[i].x * 8, 0, 0));
        x1[i] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(xr, c[i].y * 8, 0, 0));
    }
    double acc = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const double2 q = vs[p0 + i];
        acc += q.x * x0[i];
        acc += q.y * x1[i];
    }
    __builtin_nontemporal_store(acc, y + r);
}

template <int MODE, bool NT, bool SW = true, int AUX = 2>
__global__ void __launch_bounds__(256) k_csr_uniform(const double* __restrict__ va, const int32_t* __restrict__ ci,
                                                     const double* __restrict__ x, int32_t ncols,
                                                     const int32_t* __restrict__ table, int nblocks,
                                                     double* __restrict__ y) {
    __shared__ double2 vstage[4][384];
    __shared__ int2 cstage[4][384];
    const int b = SW ? xcd_swizzle(blockIdx.x, nblocks) : (int)blockIdx.x;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const i32x4 t0 = ((ci32x4*)table)[2 * b], t1 = ((ci32x4*)table)[2 * b + 1];
    const int32_t ra = t0.x + 64 * w;
    if (ra >= t0.y) return;
    const int len = (t1.w >> (8 * w)) & 255;
    const int32_t s = w == 0 ? t0.z : w == 1 ? t0.w : w == 2 ? t1.x : t1.y;
    const int32_t r = ra + lane;
    if (len == 12) wave_rows<12, MODE, NT, AUX>(va, ci, x, ncols, s, lane, vstage[w], cstage[w], r, y);
    else if (len == 10) wave_rows<10, MODE, NT, AUX>(va, ci, x, ncols, s, lane, vstage[w], cstage[w], r, y);
    else if (len == 8) wave_rows<8, MODE, NT, AUX>(va, ci, x, ncols, s, lane, vstage[w], cstage[w], r, y);
}

extern "C" {

int lab_read(const void* p, int64_t bytes, int nt, double* sink, void* stream) {
    const int64_t n16 = bytes / 16;
    const int grid = (int)((n16 + 1023) / 1024);
    if (nt) k_read<true><<<grid, 256, 0, (hipStream_t)stream>>>((const f64x2*)p, n16, sink);
    else k_read<false><<<grid, 256, 0, (hipStream_t)stream>>>((const f64x2*)p, n16, sink);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int lab_readwrite(const void* p, int64_t nwaves, int nt, double* y, void* stream) {
    const int grid = (int)((nwaves + 3) / 4);
    if (nt) k_readwrite<true><<<grid, 256, 0, (hipStream_t)stream>>>((const f64x2*)p, nwaves, y);
    else k_readwrite<false><<<grid, 256, 0, (hipStream_t)stream>>>((const f64x2*)p, nwaves, y);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int lab_fill(double* p, int64_t n, double v, void* stream) {
    k_fill<<<4096, 256, 0, (hipStream_t)stream>>>(p, n, v);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int lab_csr(int mode, int nt, const double* va, const int32_t* ci, const double* x, int32_t ncols,
            const int32_t* table, int nblocks, double* y, void* stream) {
    const hipStream_t st = (hipStream_t)stream;
#define L(...) k_csr_uniform<__VA_ARGS__><<<nblocks, 256, 0, st>>>(va, ci, x, ncols, table, nblocks, y)
    if (mode == 0 && nt) L(0, true);
    else if (mode == 0) L(0, false);
    else if (mode == 1 && nt) L(1, true);
    else if (mode == 1) L(1, false);
    else if (mode == 2) L(1, true, false);          // glds nt, blocks in launch order (no XCD swizzle)
    else if (mode == 3) L(1, true, true, 3);        // glds, aux 3
    else if (mode == 4) L(1, true, true, 1);        // glds, aux 1
    else return -2;
#undef L
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // extern "C"
