// mall_probe.hip -- does the Infinity Cache (MALL, 256 MiB) serve the second
// read of a Krylov column in the MGS access pattern?  Pass p reads columns
// A = V_a(p) and B = V_b(p) (134 MB each at 4096^2, fp64) and reduces <A,B>
// per workgroup.  Pattern "mgs": a(p) = p, b(p) = p+1 -- B of pass p is A of
// pass p+1 (the resident step's V_q -> V_i reuse).  Pattern "fresh": b(p) =
// p+48 -- no column is read twice within 48 passes.  Policies: A non-temporal
// or default; B default or non-temporal (does a non-temporal load still leave
// the line in the Infinity Cache for the next pass?).  Pattern "one": only A
// (single-stream bandwidth).
// Prints microseconds per pass (median of the timed passes) and GB/s.
//   hipcc --offload-arch=gfx950 -O3 tools/mall_probe.hip -o tools/mall_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e = (x);                                                            \
        if (e != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld_nt(const double2 *p) {
    const d2v t = __builtin_nontemporal_load(reinterpret_cast<const d2v *>(p));
    return double2{t.x, t.y};
}

template <bool NT_A, bool NT_B, bool TWO>
__global__ __launch_bounds__(256) void k_pass(const double2 *__restrict__ A, const double2 *__restrict__ B,
                                              long long n2, double *__restrict__ out) {
    double acc = 0.0;
    const long long stride = (long long)gridDim.x * 256;
    for (long long e0 = (long long)blockIdx.x * 256 + threadIdx.x; e0 < n2; e0 += 8 * stride) {
        double2 a[8], b[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const long long e = e0 + u * stride;
            if (e < n2) {
                a[u] = NT_A ? ld_nt(A + e) : A[e];
                b[u] = TWO ? (NT_B ? ld_nt(B + e) : B[e]) : double2{1.0, 1.0};
            } else {
                a[u] = b[u] = double2{0.0, 0.0};
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += a[u].x * b[u].x + a[u].y * b[u].y;
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = acc;
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 4096;
    const int ncol = 96, passes = 40, blocks = 2048;
    const long long n = (long long)N * N, n2 = n / 2;
    double2 *V = nullptr;
    double *out = nullptr;
    CK(hipMalloc(&V, sizeof(double2) * n2 * ncol));
    CK(hipMalloc(&out, sizeof(double) * blocks * 4));
    CK(hipMemset(V, 0x11, sizeof(double2) * n2 * ncol));  // non-zero data
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct Case {
        const char *name;
        int reuse;  // b = a + reuse
        bool nt, ntb, two;
    } cases[] = {{"mgs_ntA", 1, true, false, true},     {"mgs_ntAB", 1, true, true, true},
                 {"mgs_defA", 1, false, false, true},   {"fresh_ntA", 48, true, false, true},
                 {"fresh_ntAB", 48, true, true, true},  {"fresh_defA", 48, false, false, true},
                 {"one_nt", 0, true, false, false},     {"one_def", 0, false, false, false}};
    for (const Case &c : cases) {
        std::vector<float> t;
        for (int p = 0; p < passes; ++p) {
            const double2 *A = V + (long long)(p % ncol) * n2;
            const double2 *B = V + (long long)((p + c.reuse) % ncol) * n2;
            CK(hipEventRecord(e0, 0));
            if (c.two) {
                if (c.nt && c.ntb) k_pass<true, true, true><<<blocks, 256>>>(A, B, n2, out);
                else if (c.nt) k_pass<true, false, true><<<blocks, 256>>>(A, B, n2, out);
                else k_pass<false, false, true><<<blocks, 256>>>(A, B, n2, out);
            } else {
                if (c.nt) k_pass<true, false, false><<<blocks, 256>>>(A, B, n2, out);
                else k_pass<false, false, false><<<blocks, 256>>>(A, B, n2, out);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (p >= 4) t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double us = 1e3 * t[t.size() / 2];
        const double bytes = (c.two ? 2.0 : 1.0) * 16.0 * n2;
        std::printf("{\"case\": \"%s\", \"N\": %d, \"us_per_pass\": %.2f, \"GBps\": %.1f}\n", c.name, N, us,
                    bytes / us / 1e3);
    }
    CK(hipFree(V));
    CK(hipFree(out));
    return 0;
}
