// gk_cheb.hpp -- interface of the temporal-blocked Chebyshev(k) pass
// (kernel and launcher in gk_cheb.hip, its own translation unit).
#pragma once
#include "gk_common.hpp"

namespace gk {

// --------------------------------------------------------------------------
// Temporal blocking of the Chebyshev(k) sweeps: L sweeps of
//   res' = res - A d ;  d' = c1 d + c2 res' ;  z' = z + d'
// in ONE pass.  A workgroup is one wave owning a 128-point window of the fast
// index i (two points per lane) and marching down grid lines with an L-level
// register pipeline: each time step one input line enters; level l consumes
// the line level l-1 emitted in the same step and emits its own middle line,
// one line behind.  Per point the arithmetic is exactly the per-sweep
// kernel's (bit-identical), only the schedule differs: the pass moves z in and
// the result out instead of 48 B per unknown per sweep.
//
// Layout of the windows (N >= 128): window 0 starts at i = 0 and window gx-1
// ends at i = N, so the physical W / E boundaries fall on lane 0 / lane 63;
// the others keep 128 - 2H points between H-point halos that are recomputed.
// The W / E neighbours come from the adjacent lane by DPP wave shifts whose
// shifted-in value is 0 -- exactly the boundary's missing neighbour on the
// edge windows, and a fake boundary inside the halo elsewhere (its error
// travels one point per level and never reaches the kept points, H >= L).
// So no point of a window needs a select; rows outside the grid are handled
// per level by uniform branches (their d is zero), and levels whose row does
// not reach the kept rows are skipped.  Grids narrower than one window
// (N < 128, tests) run the SMALL variant: one window, the lanes beyond N held
// at zero by a select on the emitted d.
//
// Register state per level and point: d of three lines (S, C and the incoming
// N), res and z of two (C and the incoming).  The step loop is unrolled by 6
// = lcm(3, 2), so the incoming line of a level is written by the level above
// straight into the slot its dead S line held: rotations are renamings, never
// moves.  Across a step boundary 4 doubles per point and level are live.
// --------------------------------------------------------------------------
constexpr int CF_W = 64;           // lanes per window (one wave)
constexpr int CF_PTS = CF_W * 2;   // points per window (2 per lane)
constexpr int CF_LMAX = 8;         // Chebyshev(8) = ONE pass
constexpr int CF_HMAX = CF_LMAX + 1;  // deepest halo: a pass with the fused stencil stage

struct CFArgs {
    const double *din;   // FIRST: z (the residual r); else d entering the pass
    const double *rin;   // !FIRST: residual entering the pass
    const double *zin;   // !FIRST: running sum entering the pass
    double *dout, *rout, *zout;  // !LAST outputs
    double *out;         // LAST output (the preconditioned vector)
    const double *vdot;  // ACC_DOT partner
    double *part;
    double theta;        // FIRST: d0 = r / theta
    double c1[CF_LMAX], c2[CF_LMAX];
    int N, nlines, JT;
    // Row-block slabs (deep halo): L grid lines of each input from the slab
    // neighbours -- lo[*] = rows -L..-1, hi[*] = rows nlines..nlines+L-1 --
    // or nullptr at the physical boundary.  Index 0: din, 1: rin, 2: zin.
    const double *lo[3], *hi[3];
};

// Windows across a grid of side N for halo H (host and device agree).
__host__ __device__ constexpr int cf_halo(int L) { return L + (L & 1); }
__host__ __device__ inline int cf_windows(int N, int L) {
    const int H = cf_halo(L), KI = CF_PTS - 2 * H, E = CF_PTS - H;
    if (N <= CF_PTS) return 1;
    const int rest = N - 2 * E;
    return 2 + (rest > 0 ? (rest + KI - 1) / KI : 0);
}

// Launch one pass of L <= CF_LMAX sweeps (FIRST: from r, d0 = r / theta; LAST:
// writes the result, fused reduction ACC into a.part).  The grid is
// cf_windows(N, L) windows x ceil(lines / JT) line tiles, JT chosen from the
// kernel's occupancy on `cus` CUs; grids narrower than one window run the
// SMALL variant.  Returns 0, GK_CF_ESLOT when the partial count would exceed a
// reduction slot, GK_CF_ESPILL when the kernel uses scratch (a build issue,
// refused), else the hipError_t of the launch; *np = partials written.
struct CFLaunch {
    int L;
    bool first, last;
    int acc;
    bool sten;  // first pass takes v and forms z = A v itself (ACC_DOT, N >= CF_PTS; deep halo L + 1)
    int lines;  // grid lines the tiles are sized for (the largest slab on N ranks)
    int cus;    // CUs the pass may fill
    int dev;
    hipStream_t st;
};
constexpr int GK_CF_ESLOT = -1;
constexpr int GK_CF_ESPILL = -2;  // the build spilled the pass's registers to scratch
constexpr int GK_CF_ESTEN = -3;   // a fused-stencil pass asked for outside its variants
int cheb_launch(const CFLaunch &q, CFArgs &a, i64 *np);

}  // namespace gk
