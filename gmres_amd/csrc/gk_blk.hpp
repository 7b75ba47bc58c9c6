// gk_blk.hpp -- interface of the blocked-projection MGS-R step (opt-in,
// GK_TUNE_RES_BLOCK = S; kernel and launcher in gk_blk.hip, its own translation
// unit).
//
// The strict MGS-R step (gmres_mgsr.f90:341-360) runs 2j dependent projections,
// each closed by one in-launch all-gather of its dot -- the all-gather is 18 % of
// a projection at 4096^2 and nearly all of it at 1024^2.  The
// blocked step groups the projections of each sweep into blocks of S consecutive
// columns -- {V_1}, {V_2..V_{S+1}}, {V_{S+2}..}, ... (1-based) -- and takes the
// dots of a whole block in ONE pass and ONE all-gather:
//
//   z_k = <w, V_{c_k}>,   L_kl = <V_{c_l}, V_{c_k}>  (l < k, the block's Gram terms)
//   h_1 = z_1,   h_k = z_k - sum_{l<k} h_l L_kl     (in l order)
//   w   = ((w - h_1 V_{c_1}) - h_2 V_{c_2}) - ...   (element-wise, MGS's AXPY order)
//
// which are MGS's values in exact arithmetic (h_k = <w - sum_{l<k} h_l V_{c_l},
// V_{c_k}>).  A block never straddles the two sweeps, so the second sweep still
// sees w after the whole first sweep (the reorthogonalisation "twice is enough",
// gmres_mgsr.f90:339-341).  Per step 2 * (1 + ceil((j-1)/S)) all-gathers instead of
// 2j.  Gram terms are computed once per cycle: the block holding the newest column
// V_j carries <V_{c_l}, V_j> as extra values of its all-gather; the others come
// from the cycle's Gram table (ResArgs::gm, written by workgroup 0).
#pragma once
#include "gk_common.hpp"

namespace gk {

struct ResArgs;

// All-gathers of one blocked step j (the host's sequence-number and tag budget).
__host__ __device__ constexpr int blk_sweep(int j, int S) { return 1 + (j - 1 + S - 1) / S; }
__host__ __device__ constexpr int blk_exchanges(int j, int S) { return 2 * blk_sweep(j, S); }

// Instantiations (two-wave 512-thread workgroups unless noted); chunk = NT double2
// per thread.  blk_variant picks by the chunks per thread a slab needs.
enum { BLK_R4 = 0, BLK_R8 = 1, BLK_R16 = 2, BLK_R32 = 3, BLK_WONLY = 4, BLK_NVAR = 5 };
struct BlkGeom {
    int rw, lw, rx, lx, nt;  // w chunks in registers / LDS, cached column chunks in registers / LDS, threads
    int pfx;                 // chunks of the next pass's dot block prefetched into LDS (small slabs)
};
BlkGeom blk_geom(int var, int S);
int blk_variant(long long chunks512);  // chunks per thread at 512 threads; BLK_WONLY past 32

// Launch step j's blocked MGS-R launch: G workgroups of blk_geom(var, S).nt threads,
// `lds` bytes of dynamic LDS; returns a hipError_t (hipErrorInvalidValue for an
// unsupported S / variant).
int blk_launch(int var, int S, const ResArgs &a, int G, int lds, int dev, hipStream_t st);

}  // namespace gk
