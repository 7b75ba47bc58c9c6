// gk_common.hpp -- definitions shared by the kernel translation units
// (gk_api.hip: everything but the Chebyshev pass; gk_cheb.hip: the pass).
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

namespace gk {

constexpr int TPB = 256;          // threads per workgroup (4 wave64)
constexpr int WAVES = TPB / 64;
constexpr int UNR = 4;            // double2 per thread per trip in the streaming kernels
constexpr int NPMAX = 4096;       // max partials in a slab

typedef long long i64;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

// Deterministic block sum; result returned to every thread.
__device__ __forceinline__ double block_sum(double v, double *sm) {
    v = wave_sum(v);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sm[wid] = v;
    __syncthreads();
    double r = sm[0];
#pragma unroll
    for (int k = 1; k < WAVES; ++k) r += sm[k];
    return r;
}

// Fixed-order reduction of a partial slab (length np <= NPMAX).
__device__ __forceinline__ double reduce_slab(const double *__restrict__ p, int np, double *sm) {
    double s = 0.0;
    for (int k = threadIdx.x; k < np; k += TPB) s += p[k];
    return block_sum(s, sm);
}

typedef double d2v __attribute__((ext_vector_type(2)));

// Load policy for the Krylov-basis columns: plain, or non-temporal (`nt`) so
// the once-per-launch V stream does not displace w from the Infinity Cache.
template <bool NT>
__device__ __forceinline__ double2 ldv(const double2 *p) {
    if constexpr (NT) {
        const d2v t = __builtin_nontemporal_load(reinterpret_cast<const d2v *>(p));
        return double2{t.x, t.y};
    } else {
        return *p;
    }
}

// A plain (default-policy) load through an address-space-1 pointer: where the compiler
// cannot prove a pointer global (pointers selected per pass from small arrays) it emits
// FLAT loads, and waited for each before issuing the next inside an unrolled batch.
__device__ __forceinline__ double2 ldg(const double2 *p) {
    const d2v t = *(const __attribute__((address_space(1))) d2v *)p;
    return double2{t.x, t.y};
}

// Fused reductions of a pass: none, <y, vdot>, or <y, y>.
enum { ACC_NONE = 0, ACC_DOT = 1, ACC_NORM = 2 };

}  // namespace gk
